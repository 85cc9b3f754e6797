// Chain v4 of the persistent Cholesky (k_chol_persistent<4>): the chain workgroup's 64-block
// step as a pipeline of four 16-column leaves.  Included by bb_kernels.hip inside namespace bb,
// after the v1 helpers it uses (v4d, kNB, CholFlags, SpinGuard, ld_sc1, st_sc1, fast_rcp).
//
// Reference op: chol(U, VInv, 'U') + the two triangular solves, Code/C/BridgeRegression.cpp:
// 559-565 (the Woodbury n x n system and the p <= n p x p system alike).
//
// Step k of the blocked factorisation A = U'U holds the diagonal block D_k (all updates of the
// earlier steps applied) and must deliver W_k = U_kk^-T (for the owners and the backward solve),
// U_{k,k+1} = W_k S_k (S_k = A_{k,k+1}, the owners' hand-off) and the next diagonal block
// D_{k+1} = Q_k - U_{k,k+1}' U_{k,k+1} (Q_k = A_{k+1,k+1}, hand-off).  v1 eliminates the 64
// pivots of D_k with all eight waves, then forms U_{k,k+1} and D_{k+1} -- ~17 us per step,
// 11 of them in the elimination.  Here the step is right-looking over 16 x 16
// leaves inside the workgroup, and only the leaf chain is serial:
//   wave 0 (the leaf wave) factors leaf t: lane x of every 16-lane DPP row holds column x of
//     D_tt (the multipliers) and DPP row g a right-hand block -- g = 0 the identity, g >= 1 the
//     block D_{t,t+g} -- so the 16 pivots (v_fmac_f64 with a row_newbcast:c source, one
//     instruction per row per pivot, no readlane, no LDS) turn them into diag(sqrt p) W_tt and
//     diag(sqrt p) U_{t,t+g} at once; the lane's own pivot gives 1/sqrt p, DPP broadcasts scale
//     the rows, and W_tt and every U_{t,b} are stored together; then the next leaf's diagonal
//     block D_{t+1,t+1} -= U_{t,t+1}' U_{t,t+1} (fp64 MFMA) and on to leaf t+1;
//   waves 1-2 (the D stream) apply the other updates inside D_k (D_ab -= U_ta' U_tb), the
//     blocks the next leaf reads first, assemble W_k's off-diagonal blocks
//     W_tb = -W_tt sum_{b<=s<t} U_st' W_sb, release W_k, and then form the next diagonal
//     block's (0, 2) / (0, 3) from the S buffer;
//   waves 3, 5-7 (the S stream) form U_{k,k+1} by blocked forward substitution, column block c
//     of U_{k,k+1} on one wave (U_S,t = W_tt S_t, then S_a -= U_ta' U_S,t for a > t), sum
//     U_{k,k+1}' U_{k,k+1} block by block as the rows appear ((c, c), and (0, 1) on column 1;
//     wave 4 takes (1, 2), (1, 3), (2, 3)) and finish D_{k+1} = Q_k - sum, Q_k loaded into
//     registers ahead of the last leaf.
// The next step's first leaf waits only for D_{k+1}'s block row 0.  Waves synchronise through
// LDS counters (no workgroup barrier after the start): every counter has a single writer or is
// an atomic count, and its values grow over the whole factorisation (4k + 1 + updates for a
// block of step k), so nothing is reset between steps.  The owners' protocol is v1's: the chain
// reads the hand-off tiles (k, k+1) and (k+1, k+1) (flags R) and publishes W_k (flag W[k]) and
// U_{k,k+1} (tile (k, k+1) of A, flag P[k][k+1]).  What bounds a step now (tools/bench_chol_ab.py
// stamps, m = 2048, ~14 us): the four leaves end ~9.8 us in, and S_k arrives ~6.5 us in, one
// owner hop (merge of U_{k-1,k}, 1.7 us of MFMA on one CU) plus two write-through hand-offs
// after U_{k-1,k} is released, so the S stream finishes ~3 us after the last leaf.

constexpr int kC4Ld = 65;
// LDS blocks in the LDS address space, so that every access is a ds_read / ds_write (through
// generic pointers the compiler emitted flat accesses, serialised behind their own waits)
typedef __attribute__((address_space(3))) double C4Row[kC4Ld];
typedef C4Row *C4Blk;

struct C4Sync {
    int ver[4][4];   // D_ab of the current step: 4k + 1 + updates applied (a <= b)
    int sver[4][4];  // S_ac: 4k + 1 + updates applied
    int urdy[4][4];  // U_{t,b} (t < b) stored in place of D_tb: k + 1
    int usr[4][4];   // U_S,t column block c stored in place of S_tc: k + 1
    int wrdy[4][4];  // W_tb (t > b) in the W buffer: k + 1
    int leaf;        // leaves factored: 4k + t + 1
    int t5done;      // S-buffer readers finished (10 per step)
    int upub, wpub;  // drained global stores of U_{k,k+1} (4 per step) and of W_k (2 per step)
    int wread;       // D-stream waves done reading the W buffer (2 per step)
};

typedef volatile __attribute__((address_space(3))) int c4_lds_int;

// wait until an LDS counter reaches v (bounded like every wait of the launch: SpinGuard's 2 s,
// or at once when another wait has given up -- error bit 16)
__device__ __forceinline__ void c4_wait(const int *p, int v, uint32_t *err) {
    c4_lds_int *q = (c4_lds_int *)p;
    if (*q < v) {
        for (SpinGuard sg; *q < v;) {
            __builtin_amdgcn_s_sleep(1);
            if (sg.expired(err)) break;
        }
    }
    asm volatile("" ::: "memory");
}

// single-writer LDS counter: this wave's LDS data writes complete first
__device__ __forceinline__ void c4_set(int *p, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) *(c4_lds_int *)p = v;
    asm volatile("" ::: "memory");
}

// multi-writer LDS count: returns the value before the add (wave-uniform)
__device__ __forceinline__ int c4_add(int *p) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int old = 0;
    if ((threadIdx.x & 63) == 0)
        old = __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(old);
}

// wait for a global flag (an owner's hand-off) set to the factorisation's epoch
__device__ __forceinline__ void c4_gwait(const unsigned int *f, unsigned int ep, uint32_t *err) {
    for (SpinGuard sg;;) {
        const unsigned int v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane((int)(v == ep))) break;
        __builtin_amdgcn_s_sleep(2);
        if (sg.expired(err)) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- 16 x 16 block products (fp64 MFMA 16x16x4, K = 16).  A block in "accumulator layout"
// (registers) is the MFMA output layout: lane (j = lane & 15, g = lane >> 4), register r holds
// element (4r + g, j).  As an A operand of X'(.) and as a B operand of (.)Y such a block is
// used as it stands (register kk is the K step's fragment).
// acc += op(A_blk) op(B_blk), A_blk = LA[16ar.., 16ac..] (transposed if AT), likewise B
template <bool AT, bool BT, bool NEG = false>
__device__ __forceinline__ void c4_mm(v4d &acc, C4Blk LA, int ar, int ac, C4Blk LB, int br, int bc) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int s = 4 * kk + g;
        double a = AT ? LA[16 * ar + s][16 * ac + i] : LA[16 * ar + i][16 * ac + s];
        if (NEG) a = -a;
        const double b = BT ? LB[16 * br + i][16 * bc + s] : LB[16 * br + s][16 * bc + i];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
}
// acc += (+-X') Y, both in registers
template <bool NEG = false>
__device__ __forceinline__ void c4_mm_rr(v4d &acc, const v4d &x, const v4d &y) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -x[kk] : x[kk], y[kk], acc, 0, 0, 0);
}
// acc += X' B_blk, X in registers
__device__ __forceinline__ void c4_mm_rl(v4d &acc, const v4d &x, C4Blk LB, int br, int bc) {
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[kk], LB[16 * br + 4 * kk + g][16 * bc + j], acc,
                                                   0, 0, 0);
}
// acc += (+-op(A_blk)) Y, Y in registers
template <bool AT, bool NEG = false>
__device__ __forceinline__ void c4_mm_lr(v4d &acc, C4Blk LA, int ar, int ac, const v4d &y) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int s = 4 * kk + g;
        double a = AT ? LA[16 * ar + s][16 * ac + i] : LA[16 * ar + i][16 * ac + s];
        if (NEG) a = -a;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, y[kk], acc, 0, 0, 0);
    }
}
__device__ __forceinline__ v4d c4_ld(C4Blk L, int a, int b) {
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    v4d v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = L[16 * a + 4 * r + g][16 * b + j];
    return v;
}
__device__ __forceinline__ void c4_st(C4Blk L, int a, int b, const v4d &v) {
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) L[16 * a + 4 * r + g][16 * b + j] = v[r];
}
// write-through store of a register block into column-major global memory at (row0, col0)
__device__ __forceinline__ void c4_gst(double *G, size_t ld, int row0, int col0, const v4d &v) {
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) st_sc1(&G[(size_t)(row0 + 4 * r + g) + (size_t)(col0 + j) * ld], v[r]);
}
constexpr v4d kC4Zero = {0.0, 0.0, 0.0, 0.0};

// ---- the leaf: 16 pivots of [D | I] in registers ----
// a += bcast_C(src) * mul, bcast_C = lane C of the lane's 16-lane row (DPP row_newbcast)
template <int C>
__device__ __forceinline__ void c4_fmac_bc(double &acc, double src, double mul) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "n"(C));
}
template <int C>
__device__ __forceinline__ void c4_fmac_bc_self(double &acc, double mul) {
    asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(mul), "n"(C));
}
// Pivot C: p = D[C][C] (lane C's register C, broadcast), the scaled pivot row -D[C][x] / p is
// the lane's own register; rows i > C take D[i][C] from lane C: D[i][x] -= D[i][C] D[C][x] / p
// and likewise for the identity part E.  (The hazard recogniser does not see the asm's VALU
// writes: the broadcast of a[C], written by the previous pivot's asm, carries its own two wait
// states; the other DPP reads come several instructions after the write of their source.)
template <int C>
__device__ __forceinline__ void c4_pivot(double (&a)[16], double (&e)[16], double (&pv)[16],
                                         double &md) {
    double p;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "=v"(p) : "v"(a[C]), "n"(C));
    pv[C] = p;
    if ((threadIdx.x & 15) == C) md = p;  // lane x keeps pivot x
    if constexpr (C < 15) {
        const double inv = fast_rcp(p);
        const double na = -a[C] * inv, ne = -e[C] * inv;
#pragma unroll
        for (int i = C + 1; i < 16; ++i) {
            c4_fmac_bc<C>(e[i], a[i], ne);  // reads D[i][C] before row i's update below
            c4_fmac_bc_self<C>(a[i], na);
        }
    }
}
template <int C>
__device__ __forceinline__ void c4_pivots(double (&a)[16], double (&e)[16], double (&pv)[16],
                                          double &md) {
    c4_pivot<C>(a, e, pv, md);
    if constexpr (C < 15) c4_pivots<C + 1>(a, e, pv, md);
}
// val[i] = e[i] * (lane i's r), i = 0 .. 15 (DPP broadcast within each 16-lane row)
template <int I>
__device__ __forceinline__ void c4_scale_rows(double (&val)[16], const double (&e)[16], double r) {
    double ri;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "=v"(ri) : "v"(r), "n"(I));
    val[I] = e[I] * ri;
    if constexpr (I < 15) c4_scale_rows<I + 1>(val, e, r);
}

// trace slots per step (bb_bench_chol, tools/bench_chol_ab.py): 0 leaf 0 start, 1 leaf 3 done,
// 2 W_k released, 3 S_k acquired, 4 U_{k,k+1} released, 5 D_{k+1}(0, 0) ready, 6 leaf 1
// start, 7 leaf 2 start; leaf t: 8 + 4t pivots done, + 1 W_tt stored, + 2 X formed, + 3 the
// next leaf updated; 30 / 27 / 25 / 24 S columns 0 / 1 / 2 / 3 U'U done, 26 S stream free to
// load S_k; 28 / 29 S column 0's U_S,0 / U_S,3 formed, 31 wave 4's U'U done
#define C4_TS(slot)                                                                          \
    do {                                                                                     \
        if (trace && (threadIdx.x & 63) == 0)                                                \
            trace[(size_t)k * 32 + (slot)] = __builtin_amdgcn_s_memrealtime();               \
    } while (0)

__device__ void chol_chain_v4(double *A, int lda, int nblk, int ncb, double *Wd,
                              const CholFlags &F, uint32_t *err, unsigned long long *trace,
                              double *L) {
    __shared__ C4Sync sy;
    C4Blk Lb = (C4Blk)L;
    C4Blk Dm[2] = {Lb, Lb + 64};
    C4Blk Sm = Lb + 2 * 64;
    C4Blk Wm = Lb + 3 * 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int j16 = lane & 15;
    if (tid < (int)(sizeof(C4Sync) / sizeof(int))) ((int *)&sy)[tid] = 0;
    __syncthreads();
    // roles (waves pair up on SIMDs as w, w + 4): leaf wave 0; D stream 1, 2; S stream
    // columns 0..3 on waves 5, 6, 7, 3; the extra U'U blocks on wave 4
    const int scol = wid == 5 ? 0 : wid == 6 ? 1 : wid == 7 ? 2 : wid == 3 ? 3 : -1;
    const size_t lda_ = (size_t)lda;
    auto Aat = [&](int row, int col) -> double * { return A + (size_t)row + (size_t)col * lda_; };

    // ---------------- S stream: the initial diagonal block D_0 = A_00 (mirrored) ----------------
    if (scol >= 0) {
        const int c = scol;
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int y = 16 * c + (lane & 15), x = 4 * q + (lane >> 4);
            v[q] = ld_sc1(y <= x ? Aat(y, x) : Aat(x, y));
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) Dm[0][16 * c + (lane & 15)][4 * q + (lane >> 4)] = v[q];
        for (int b = c; b < 4; ++b) c4_set(&sy.ver[c][b], 1);
    }

    if (wid == 0) {
        // =============================== the leaf wave ===============================
        __builtin_amdgcn_s_setprio(3);
        for (int k = 0; k < nblk; ++k) {
            C4Blk D = (k & 1) ? Dm[1] : Dm[0];
            const int base = 4 * k + 1;
            const int g = lane >> 4;
            for (int t = 0; t < 4; ++t) {
                // leaf t needs block row t of D_k with the updates of leaves 0 .. t-1 (its own
                // diagonal block from the previous leaf's update, the others from the D
                // stream; at t = 0 all four from the S stream's D_{k+1} of step k-1)
                for (int b = t + (t > 0); b < 4; ++b) c4_wait(&sy.ver[t][b], base + t, err);
                if (t == 0) C4_TS(0);
                else if (t == 1) C4_TS(6);
                else if (t == 2) C4_TS(7);
                // the W buffer's block (t, t) is free once every reader of step k - 1 is done
                // (read now, checked after the pivots)
                int wfree = 1;
                if (k > 0) {
                    c4_lds_int *us = (c4_lds_int *)&sy.usr[t][0];
                    wfree = (int)(us[0] >= k) & (int)(us[1] >= k) & (int)(us[2] >= k) & (int)(us[3] >= k);
                    if (t == 0) wfree &= (int)(*(c4_lds_int *)&sy.wread >= 2 * k);
                }
                // [D_tt | I | D_t,t+1 | D_t,t+2 | D_t,t+3]: every 16-lane DPP row holds D_tt
                // (the multipliers) and row g its own right-hand block: g = 0 the identity,
                // g >= 1 the block D_{t,t+g} (zero past the last block).  The same row
                // operations that reduce D_tt turn them into U_tt' L^-1 = diag(sqrt p) W_tt and
                // diag(sqrt p) U_{t,t+g}, one instruction per row per pivot for all of them.
                const int rb = t + g;
                // (branch-free: a select here became a branch with a wait per load)
                const double msk = (g > 0 && rb < 4) ? 1.0 : 0.0;
                double a[16], e[16], pv[16], md = 0.0;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    a[i] = D[16 * t + i][16 * t + j16];
                    const double dv = D[16 * t + i][16 * (rb < 4 ? rb : 3) + j16];
                    e[i] = __builtin_fma(dv, msk, (g == 0 && i == j16) ? 1.0 : 0.0);
                }
                c4_pivots<0>(a, e, pv, md);
                C4_TS(8 + 4 * t);
                if (!wfree) {
                    if (t == 0) c4_wait(&sy.wread, 2 * k, err);
                    for (int c = 0; c < 4; ++c) c4_wait(&sy.usr[t][c], k, err);
                }
                // 1/sqrt(p) of the lane's own pivot (v_rsq_f64 + two Newton steps), then row i
                // scaled by lane i's value (DPP broadcast): W_tt on row 0, U_{t,t+g} on row g
                double r = __builtin_amdgcn_rsq(md);
                r = r * __builtin_fma(-0.5 * md * r, r, 1.5);
                r = r * __builtin_fma(-0.5 * md * r, r, 1.5);
                double val[16];
                c4_scale_rows<0>(val, e, r);
                if (g == 0) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) Wm[16 * t + i][16 * t + j16] = val[i];
                } else if (rb < 4) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) D[16 * t + i][16 * rb + j16] = val[i];
                }
                if (lane == 0) {
                    bool bad = false;
#pragma unroll
                    for (int i = 0; i < 16; ++i) bad |= !(pv[i] > 0.0);
                    if (bad) atomicOr(err, 8u);
                }
                c4_set(&sy.leaf, 4 * k + t + 1);
                for (int b = t + 1; b < 4; ++b) c4_set(&sy.urdy[t][b], k + 1);
                C4_TS(9 + 4 * t);
                if (t == 3) {
                    C4_TS(1);
                    break;
                }
                C4_TS(10 + 4 * t);
                // the next leaf's diagonal block D_{t+1,t+1} -= U_{t,t+1}' U_{t,t+1}
                c4_wait(&sy.ver[t + 1][t + 1], base + t, err);
                v4d cc = c4_ld(D, t + 1, t + 1);
                c4_mm<true, false, true>(cc, D, t, t + 1, D, t, t + 1);
                c4_st(D, t + 1, t + 1, cc);
                c4_set(&sy.ver[t + 1][t + 1], base + t + 1);
                C4_TS(11 + 4 * t);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        return;
    }

    if (wid == 1 || wid == 2) {
        // =============================== the D stream ===============================
        const bool d0 = wid == 1;
        for (int k = 0; k < nblk; ++k) {
            C4Blk D = (k & 1) ? Dm[1] : Dm[0];
            const int base = 4 * k + 1;
            const int kr = k + 1;
            double *Wg = Wd + (size_t)k * kNB * kNB;  // W_k, column-major 64 x 64
            auto leafw = [&](int t) { c4_wait(&sy.leaf, 4 * k + t + 1, err); };
            // W_tt and the zero blocks right of it to global memory
            auto tw = [&](int t) {
                c4_gst(Wg, kNB, 16 * t, 16 * t, c4_ld(Wm, t, t));
                for (int b = t + 1; b < 4; ++b) c4_gst(Wg, kNB, 16 * t, 16 * b, kC4Zero);
            };
            // D_ab -= U_ta' U_tb (U_{t,*} stored in place of D_{t,*} by leaf t)
            auto t3 = [&](int t, int a, int b) {
                c4_wait(&sy.urdy[t][a], kr, err);
                c4_wait(&sy.urdy[t][b], kr, err);
                c4_wait(&sy.ver[a][b], base + t, err);
                v4d c = c4_ld(D, a, b);
                c4_mm<true, false, true>(c, D, t, a, D, t, b);
                c4_st(D, a, b, c);
                c4_set(&sy.ver[a][b], base + t + 1);
            };
            // W_tb = -W_tt P (P = sum_s U_st' W_sb, in registers)
            auto wpost = [&](int t, int b, const v4d &P, bool keep) {
                v4d w = kC4Zero;
                c4_mm_lr<false, true>(w, Wm, t, t, P);
                if (keep) {
                    c4_st(Wm, t, b, w);
                    c4_set(&sy.wrdy[t][b], kr);
                }
                c4_gst(Wg, kNB, 16 * t, 16 * b, w);
            };
            // the blocks leaf t + 1 reads, (t + 1, b > t + 1), first: d0 (1, 2), d1 (1, 3)
            // after leaf 0, d0 (2, 3) after leaf 1
            leafw(0);
            if (d0) {
                t3(0, 1, 2);
                t3(0, 2, 2);
                t3(0, 3, 3);
                leafw(1);
                t3(1, 2, 3);
                c4_wait(&sy.wrdy[1][0], kr, err);
                v4d P = kC4Zero;
                c4_mm<true, false>(P, D, 0, 2, Wm, 0, 0);
                c4_mm<true, false>(P, D, 1, 2, Wm, 1, 0);
                leafw(2);
                wpost(2, 0, P, true);
                c4_wait(&sy.urdy[2][3], kr, err);
                P = kC4Zero;
                c4_mm<true, false>(P, D, 0, 3, Wm, 0, 0);
                c4_mm<true, false>(P, D, 1, 3, Wm, 1, 0);
                c4_mm<true, false>(P, D, 2, 3, Wm, 2, 0);
                leafw(3);
                wpost(3, 0, P, false);
            } else {
                t3(0, 1, 3);
                t3(0, 2, 3);
                tw(0);
                c4_wait(&sy.urdy[0][1], kr, err);
                v4d P = kC4Zero;
                c4_mm<true, false>(P, D, 0, 1, Wm, 0, 0);
                leafw(1);
                wpost(1, 0, P, true);
                tw(1);
                t3(1, 3, 3);
                c4_wait(&sy.urdy[1][2], kr, err);
                P = kC4Zero;
                c4_mm<true, false>(P, D, 1, 2, Wm, 1, 1);
                leafw(2);
                wpost(2, 1, P, true);
                tw(2);
                c4_wait(&sy.urdy[2][3], kr, err);
                P = kC4Zero;
                c4_mm<true, false>(P, D, 1, 3, Wm, 1, 1);
                c4_mm<true, false>(P, D, 2, 3, Wm, 2, 1);
                v4d P2 = kC4Zero;
                c4_mm<true, false>(P2, D, 2, 3, Wm, 2, 2);
                leafw(3);
                wpost(3, 1, P, false);
                wpost(3, 2, P2, false);
                tw(3);
            }
            c4_add(&sy.wread);
            // W_k released once both waves' stores have drained
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (c4_add(&sy.wpub) == 2 * k + 1) {
                if (lane == 0) __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                C4_TS(2);
            }
            // then the next diagonal block's (0, 2) (d0) or (0, 3) (d1): U_{k,k+1}'U_{k,k+1}
            // from the S buffer as the column waves store U_S,t (their SIMD 3 pair runs two
            // column waves; this takes a product per t off each of them)
            if (k + 1 < nblk) {
                const int cb = d0 ? 2 : 3;
                const int cs = (k + 1) * kNB;
                // Q_{0,cb} of the (k+1, k+1) hand-off, loaded while the products run
                c4_gwait(&F.R[2 * (k + 1)], F.ep, err);
                v4d q;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    q[r] = ld_sc1(Aat(cs + 4 * r + (lane >> 4), cs + 16 * cb + j16));
                v4d acc = kC4Zero;
                for (int t = 0; t < 4; ++t) {
                    c4_wait(&sy.usr[t][0], kr, err);
                    c4_wait(&sy.usr[t][cb], kr, err);
                    c4_mm<true, false>(acc, Sm, t, 0, Sm, t, cb);
                }
                c4_add(&sy.t5done);
                C4Blk Dn = (k & 1) ? Dm[0] : Dm[1];
                c4_st(Dn, 0, cb, q - acc);
                c4_set(&sy.ver[0][cb], 4 * (k + 1) + 1);
            }
        }
        return;
    }

    // =============================== the S stream ===============================
    for (int k = 0; k + 1 < nblk; ++k) {
        C4Blk D = (k & 1) ? Dm[1] : Dm[0];
        C4Blk Dn = (k & 1) ? Dm[0] : Dm[1];
        const int base = 4 * k + 1;
        const int kr = k + 1;
        const int nbase = 4 * (k + 1) + 1;
        const unsigned int *fS = &F.R[2 * k + 1], *fQ = &F.R[2 * (k + 1)];
        const int r0 = k * kNB, cs = (k + 1) * kNB;  // tile (k, k+1): rows r0.., cols cs..
        // D_{k+1} block (a, b) = Q_ab - acc (Q: the (k+1, k+1) hand-off; diagonal blocks
        // mirrored from its upper triangle).  Q arrives early in the step: its blocks are
        // loaded into registers before the last leaf (tq_ld) and only subtracted at the end.
        auto tq_ld = [&](int a, int b) {
            v4d q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 4 * r + (lane >> 4);
                int y = 16 * a + i, x = 16 * b + j16;
                if (a == b && i > j16) {
                    y = 16 * a + j16;
                    x = 16 * a + i;
                }
                q[r] = ld_sc1(Aat(cs + y, cs + x));
            }
            return q;
        };
        auto tq = [&](int a, int b, const v4d &q, const v4d &acc) {
            c4_st(Dn, a, b, q - acc);
            c4_set(&sy.ver[a][b], nbase);
        };
        if (scol >= 0) {
            const int c = scol;
            // row block c of S_k into the S buffer, once step k-1's readers are done
            c4_wait(&sy.t5done, 10 * k, err);
            if (c == 0) C4_TS(26);
            c4_gwait(fS, F.ep, err);
            if (c == 0) C4_TS(3);
            {
                double v[16];
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    v[q] = ld_sc1(Aat(r0 + 16 * c + (lane & 15), cs + 4 * q + (lane >> 4)));
#pragma unroll
                for (int q = 0; q < 16; ++q) Sm[16 * c + (lane & 15)][4 * q + (lane >> 4)] = v[q];
            }
            for (int b = 0; b < 4; ++b) c4_set(&sy.sver[c][b], base);
            // U'U blocks (c, c) and, for c >= 1, (0, c): the next step's leaf 0 reads block
            // row 0 of D_{k+1}, one block from each column wave
            const bool own0 = c == 1;  // (0, 1) here; (0, 2), (0, 3) on the D stream
            v4d accd = kC4Zero, acc0 = kC4Zero, qd = kC4Zero, q0 = kC4Zero;
            for (int t = 0; t < 4; ++t) {
                // U_S,t column block c = W_tt S_tc (in place; also tile (k, k+1) of A)
                c4_wait(&sy.leaf, 4 * k + t + 1, err);
                if (t == 3) {
                    c4_gwait(fQ, F.ep, err);
                    qd = tq_ld(c, c);
                    if (own0) q0 = tq_ld(0, c);
                }
                c4_wait(&sy.sver[t][c], base + t, err);
                v4d us = kC4Zero;
                c4_mm<false, false>(us, Wm, t, t, Sm, t, c);
                c4_st(Sm, t, c, us);
                c4_gst(A, lda_, r0 + 16 * t, cs + 16 * c, us);
                c4_set(&sy.usr[t][c], kr);
                if (c == 0 && t == 0) C4_TS(28);
                if (c == 0 && t == 3) C4_TS(29);
                // S_ac -= U_ta' U_S,t for the rows below
                for (int a = t + 1; a < 4; ++a) {
                    c4_wait(&sy.urdy[t][a], kr, err);
                    c4_wait(&sy.sver[a][c], base + t, err);
                    v4d s = c4_ld(Sm, a, c);
                    c4_mm_lr<true, true>(s, D, t, a, us);
                    c4_st(Sm, a, c, s);
                    c4_set(&sy.sver[a][c], base + t + 1);
                }
                if (own0) {
                    c4_wait(&sy.usr[t][0], kr, err);
                    c4_mm_lr<true>(acc0, Sm, t, 0, us);
                }
                c4_mm_rr(accd, us, us);
            }
            if (c == 0) C4_TS(30);
            if (c == 1) C4_TS(27);
            if (c == 2) C4_TS(25);
            if (c == 3) C4_TS(24);
            c4_add(&sy.t5done);
            if (own0) c4_add(&sy.t5done);
            // the next diagonal block first (block row 0 for the next step's leaf 0), then
            // U_{k,k+1} released once the four column waves' stores have drained
            if (own0) tq(0, c, q0, acc0);
            tq(c, c, qd, accd);
            if (c == 0) C4_TS(5);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (c4_add(&sy.upub) == 4 * k + 3) {
                if (lane == 0)
                    __hip_atomic_store(&F.P[(size_t)k * F.ncb + k + 1], F.ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                C4_TS(4);
            }
        } else {
            // wave 4: U'U blocks (1, 2), (1, 3), (2, 3) from the S buffer
            v4d a12 = kC4Zero, a13 = kC4Zero, a23 = kC4Zero, q12, q13, q23;
            for (int t = 0; t < 4; ++t) {
                if (t == 3) {
                    c4_gwait(fQ, F.ep, err);
                    q12 = tq_ld(1, 2);
                    q13 = tq_ld(1, 3);
                    q23 = tq_ld(2, 3);
                }
                c4_wait(&sy.usr[t][1], kr, err);
                c4_wait(&sy.usr[t][2], kr, err);
                c4_mm<true, false>(a12, Sm, t, 1, Sm, t, 2);
                c4_wait(&sy.usr[t][3], kr, err);
                c4_mm<true, false>(a13, Sm, t, 1, Sm, t, 3);
                c4_mm<true, false>(a23, Sm, t, 2, Sm, t, 3);
            }
            C4_TS(31);
            c4_add(&sy.t5done);
            c4_add(&sy.t5done);
            c4_add(&sy.t5done);
            tq(1, 2, q12, a12);
            tq(1, 3, q13, a13);
            tq(2, 3, q23, a23);
        }
    }
}
#undef C4_TS
