// bb_sparse.hip -- gfx950 kernels of the sparse-design Woodbury sweep (bb_sparse.h).
//
// Replaces, for a CSC design, the three passes over X of the beta | rest draw
// (Code/C/BridgeRegression.cpp:552-575 in its Woodbury form):
//   Gram     X diag(D) X'  -> k_sp_gram_col (with the diagonal and X u), or for rows
//                             denser than kSpColMaxRow k_sp_gram + k_sp_rows<true>
//   X u, X b               -> k_sp_rows (X u inside k_sp_gram_col)
//   X' w                   -> k_sp_beta (fused into the beta update)
// and, once at setup, the pair list the Gram streams (k_sp_count, k_sp_build).
//
// Every sum has a fixed order (lane-strided partial sums, then a fixed xor tree), so a
// sweep is bitwise reproducible.  No atomics touch floating-point data.
#include <hip/hip_runtime.h>

#include "bb_sparse.h"

namespace bb {

namespace {

__device__ __forceinline__ double readlane_dbl(double v, int lane) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffu), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

template <int W>
__device__ __forceinline__ double group_sum(double v) {
    // xor tree inside aligned groups of W lanes; every lane of the group gets the sum
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace

// ---------------------------------------------------------------------------
// setup: pair list
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sp_count(const int *__restrict__ rowptr,
                                                  const int *__restrict__ colidx,
                                                  const int *__restrict__ cpos,
                                                  const int *__restrict__ colptr, int n_pad,
                                                  unsigned long long *__restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= n_pad) return;
    unsigned long long s = 0;
    for (int k = rowptr[c] + lane; k < rowptr[c + 1]; k += 64)
        s += (unsigned long long)(cpos[k] - colptr[colidx[k]]);  // entries of column j above c
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) cnt[c] = s;
}

void launch_sp_count(hipStream_t s, const int *rowptr, const int *colidx, const int *cpos,
                     const int *colptr, int n_pad, unsigned long long *cnt) {
    k_sp_count<<<(n_pad + 3) / 4, 256, 0, s>>>(rowptr, colidx, cpos, colptr, n_pad, cnt);
}

// One workgroup per output column c (= row c of X).  The per-row counts of the pairs
// (r, c), r < c, are formed in LDS, scanned into segment starts, and wave 0 then places
// the pairs walking row c's CSR entries in column order: a column's rows are distinct, so
// the LDS cursor updates of one instruction never collide, and within an entry's segment
// the pairs end up sorted by j.
__global__ __launch_bounds__(256) void k_sp_build(
    const int *__restrict__ rowptr, const int *__restrict__ colidx, const int *__restrict__ cpos,
    const double *__restrict__ rval, const int *__restrict__ colptr,
    const int *__restrict__ rowidx, const double *__restrict__ cval,
    const unsigned long long *__restrict__ base, unsigned *__restrict__ estart,
    double *__restrict__ prod, int *__restrict__ pj, unsigned short *__restrict__ pidx) {
    extern __shared__ unsigned cur[];  // c words: count, then cursor, per row r < c
    __shared__ unsigned part[257];
    const int tid = threadIdx.x, lane = tid & 63;
    const int c = blockIdx.x;
    for (int r = tid; r < c; r += 256) cur[r] = 0u;
    __syncthreads();
    const int k0 = rowptr[c], k1 = rowptr[c + 1];
    for (int k = k0 + tid; k < k1; k += 256) {
        const int j = colidx[k];
        for (int q = colptr[j]; q < cpos[k]; ++q) atomicAdd(&cur[rowidx[q]], 1u);
    }
    __syncthreads();
    // exclusive scan over r in [0, c): one contiguous chunk per thread
    const int chunk = (c + 255) / 256;
    const int r0 = min(c, tid * chunk), r1 = min(c, r0 + chunk);
    unsigned s = 0;
    for (int r = r0; r < r1; ++r) s += cur[r];
    part[tid] = s;
    __syncthreads();
    if (tid == 0) {
        unsigned run = 0;
        for (int i = 0; i < 256; ++i) {
            const unsigned v = part[i];
            part[i] = run;
            run += v;
        }
        part[256] = run;
    }
    __syncthreads();
    const unsigned long long b = base[c];
    const size_t e0 = tri_index(0, c);
    unsigned run = part[tid];
    for (int r = r0; r < r1; ++r) {
        const unsigned v = cur[r];
        cur[r] = run;
        estart[e0 + r] = (unsigned)(b + run);
        run += v;
    }
    if (tid == 0) estart[e0 + c] = (unsigned)(b + part[256]);  // empty diagonal segment
    __syncthreads();
    if (tid >= 64) return;
    for (int kb = k0; kb < k1; kb += 64) {
        const int k = kb + lane;
        const bool ok = k < k1;
        const int jl = ok ? colidx[k] : 0;
        const int q0l = ok ? colptr[jl] : 0;
        const int q1l = ok ? cpos[k] : 0;
        const double xl = ok ? rval[k] : 0.0;
        const int nb = min(64, k1 - kb);
        for (int l = 0; l < nb; ++l) {
            const int j = __builtin_amdgcn_readlane(jl, l);
            const int q0 = __builtin_amdgcn_readlane(q0l, l);
            const int q1 = __builtin_amdgcn_readlane(q1l, l);
            const double xc = readlane_dbl(xl, l);
            for (int q = q0 + lane; q < q1; q += 64) {
                const int r = rowidx[q];
                const unsigned pos = cur[r];
                cur[r] = pos + 1u;
                const size_t o = (size_t)(b + pos);
                prod[o] = cval[q] * xc;
                if (pidx)
                    pidx[o] = (unsigned short)(kb + l - k0);  // position of j in row c
                else
                    pj[o] = j;
            }
        }
    }
}

void launch_sp_build(hipStream_t s, const int *rowptr, const int *colidx, const int *cpos,
                     const double *rval, const int *colptr, const int *rowidx,
                     const double *cval, int n_pad, const unsigned long long *base,
                     unsigned *estart, double *prod, int *pj, unsigned short *pidx) {
    k_sp_build<<<n_pad, 256, (size_t)n_pad * sizeof(unsigned), s>>>(
        rowptr, colidx, cpos, rval, colptr, rowidx, cval, base, estart, prod, pj, pidx);
}

// ---------------------------------------------------------------------------
// per sweep
// ---------------------------------------------------------------------------
// Gram off-diagonal: kSpLpe lanes per packed entry; lane q sums the entry's pairs
// q, q + kSpLpe, ... in order (two in flight), then a fixed xor tree.  A wave covers
// 64 / kSpLpe consecutive entries, i.e. one contiguous stretch of the pair arrays.
constexpr int kSpLpe = 4;

__global__ __launch_bounds__(256) void k_sp_gram(const unsigned *__restrict__ estart,
                                                 const double *__restrict__ prod,
                                                 const int *__restrict__ pj,
                                                 const double *__restrict__ D, size_t nent,
                                                 double *__restrict__ out, const int *gate) {
    if (gated(gate)) return;
    const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t e = gid / kSpLpe;
    const unsigned q = (unsigned)(gid % kSpLpe);
    double s = 0.0;
    if (e < nent) {
        const unsigned en = estart[e + 1];
        unsigned k = estart[e] + q;
        for (; k + kSpLpe < en; k += 2 * kSpLpe) {
            const double p0 = prod[k], p1 = prod[k + kSpLpe];
            const int j0 = pj[k], j1 = pj[k + kSpLpe];
            s += p0 * D[j0];
            s += p1 * D[j1];
        }
        if (k < en) s += prod[k] * D[pj[k]];
    }
    s = group_sum<kSpLpe>(s);
    if (q == 0 && e < nent) out[e] = s;
}

void launch_sp_gram(hipStream_t s, const unsigned *estart, const double *prod, const int *pj,
                    const double *D, int n_pad, double *out, const int *gate) {
    const size_t nent = tri_count(n_pad);
    const size_t threads = nent * kSpLpe;
    note_launch(KF_GRAM, (const void *)k_sp_gram);
    k_sp_gram<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(estart, prod, pj, D, nent, out, gate);
}

// Gram by output column (used when every row of X has at most kSpColMaxRow non-zeros;
// k_sp_gram_flat below is the default form).  All pairs of the entries (r, c), r < c, share row c of X, so
// their columns j lie in row c's support J_c: the workgroup stages D[J_c] in LDS once and
// the pairs carry 16-bit positions into J_c instead of 32-bit column indices -- the
// per-pair D gathers become LDS reads and the pair stream shrinks to 10 bytes.  The same
// pass forms the diagonal sum_j X_cj^2 D_j and (X u)_c.  kSpColLpe lanes per entry, lane q
// sums pairs q, q + kSpColLpe, ... in order, kSpDepth pairs per lane in flight, then a fixed
// xor tree.  Heaviest columns (largest c) launch first.  Measured at C5 (~20 pairs per
// entry): 8 lanes x 4 deep 0.74 ms, 8 x 2..16 0.74-0.77, 4 x 8 (the first version) 0.80,
// 16 x 4 0.84, 2 x 16 1.10 ms.
constexpr int kSpColLpe = 8;
constexpr int kSpDepth = 4;

template <bool NTL>
__global__ __launch_bounds__(256) void k_sp_gram_col(
    const int *__restrict__ rowptr, const int *__restrict__ colidx,
    const double *__restrict__ rval, const unsigned *__restrict__ estart,
    const double *__restrict__ prod, const unsigned short *__restrict__ pidx,
    const double *__restrict__ D, const double *__restrict__ u, int n_pad,
    double *__restrict__ tri, double *__restrict__ xu, const int *gate) {
    if (gated(gate)) return;
    extern __shared__ double Dl[];  // D over row c's support
    __shared__ double red[2][4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = n_pad - 1 - (int)blockIdx.x;
    const int k0 = rowptr[c], nk = rowptr[c + 1] - k0;
    double sd = 0.0, su = 0.0;
    for (int l = tid; l < nk; l += 256) {
        const int j = colidx[k0 + l];
        const double x = rval[k0 + l], d = D[j];
        Dl[l] = d;
        sd += x * x * d;
        if (u) su += x * u[j];
    }
    sd = group_sum<64>(sd);
    su = group_sum<64>(su);
    if (lane == 0) {
        red[0][wid] = sd;
        red[1][wid] = su;
    }
    __syncthreads();
    if (tid == 0) {
        tri[tri_index(c, c)] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        if (xu) xu[c] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
    const size_t e0 = tri_index(0, c);
    const int g = tid / kSpColLpe, q = tid % kSpColLpe;
    for (int r0 = 0; r0 < c; r0 += 256 / kSpColLpe) {
        const int r = r0 + g;
        double s = 0.0;
        if (r < c) {
            const unsigned en = estart[e0 + r + 1];
            for (unsigned k = estart[e0 + r] + q; k < en; k += kSpDepth * kSpColLpe) {
                double pv[kSpDepth];
                unsigned short iv[kSpDepth];
#pragma unroll
                for (int i = 0; i < kSpDepth; ++i) {
                    const unsigned kk = k + i * kSpColLpe;
                    if constexpr (NTL) {  // the pair list is streamed once per sweep
                        pv[i] = kk < en ? __builtin_nontemporal_load(prod + kk) : 0.0;
                        iv[i] = kk < en ? __builtin_nontemporal_load(pidx + kk) : (unsigned short)0;
                    } else {
                        pv[i] = kk < en ? prod[kk] : 0.0;
                        iv[i] = kk < en ? pidx[kk] : (unsigned short)0;
                    }
                }
#pragma unroll
                for (int i = 0; i < kSpDepth; ++i)
                    if (k + i * kSpColLpe < en) s += pv[i] * Dl[iv[i]];
            }
        }
        s = group_sum<kSpColLpe>(s);
        if (q == 0 && r < c) tri[e0 + r] = s;
    }
}

// The same Gram with the pair stream read flat (the production kernel since round 3):
// the workgroup of column c walks its pair range [estart(0, c), estart(c, c)) in chunks of
// 256 x kSpFlatV pairs, lane t loading pairs t, t + 256, ... (full-width coalesced loads;
// the next chunk is requested as soon as the current one is staged), stages the products
// prod_k D[J_c(idx_k)] in LDS, and one thread per entry intersecting the chunk sums its
// pairs left to right, an entry that runs past the chunk carrying its partial sum into the
// next one.  Deterministic: every entry is a plain left-to-right sum of its pairs.
// Measured at C5 (`tools/sp_nt_ab.py`, same box, alternating): 16 pairs per lane 0.66-0.69
// ms against 0.71-0.74 for k_sp_gram_col, 8 per lane 0.70-0.73; two chunks in flight per
// workgroup no faster, and 4 consecutive pairs per lane (16-byte loads) 0.75.
template <int kSpFlatV>
__global__ __launch_bounds__(256) void k_sp_gram_flat(
    const int *__restrict__ rowptr, const int *__restrict__ colidx,
    const double *__restrict__ rval, const unsigned *__restrict__ estart,
    const double *__restrict__ prod, const unsigned short *__restrict__ pidx,
    const double *__restrict__ D, const double *__restrict__ u, int n_pad,
    double *__restrict__ tri, double *__restrict__ xu, const int *gate) {
    if (gated(gate)) return;
    extern __shared__ double Dl[];  // D over row c's support
    constexpr int kSpFlatCap = 256 * kSpFlatV;
    __shared__ double vals[kSpFlatCap];
    __shared__ double red[2][4];
    __shared__ double carry_s[2];
    __shared__ int next_s[2];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = n_pad - 1 - (int)blockIdx.x;
    const int k0 = rowptr[c], nk = rowptr[c + 1] - k0;
    double sd = 0.0, su = 0.0;
    // row c's support, 4 entries per thread in flight (the same per-thread sum order)
    for (int l0 = tid; l0 < nk; l0 += 4 * 256) {
        int jv[4];
        double xv[4], dv[4], uv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int l = l0 + q * 256;
            jv[q] = l < nk ? colidx[k0 + l] : 0;
            xv[q] = l < nk ? rval[k0 + l] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            dv[q] = l0 + q * 256 < nk ? D[jv[q]] : 0.0;
            uv[q] = u && l0 + q * 256 < nk ? u[jv[q]] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (l0 + q * 256 < nk) {
                Dl[l0 + q * 256] = dv[q];
                sd += xv[q] * xv[q] * dv[q];
                if (u) su += xv[q] * uv[q];
            }
        }
    }
    sd = group_sum<64>(sd);
    su = group_sum<64>(su);
    if (lane == 0) {
        red[0][wid] = sd;
        red[1][wid] = su;
    }
    __syncthreads();
    if (tid == 0) {
        tri[tri_index(c, c)] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        if (xu) xu[c] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
    const size_t e0 = tri_index(0, c);
    const unsigned P0 = estart[e0], P1 = estart[e0 + c];
    // the next chunk is requested as soon as this one is staged
    double pv[kSpFlatV];
    unsigned short iv[kSpFlatV];
#pragma unroll
    for (int q = 0; q < kSpFlatV; ++q) {
        const unsigned k = P0 + q * 256 + tid;
        pv[q] = k < P1 ? prod[k] : 0.0;
        iv[q] = k < P1 ? pidx[k] : (unsigned short)0;
    }
    int ra = 0, par = 0;
    double carry = 0.0;
    unsigned pa = P0;
    if (tid == 0) next_s[0] = next_s[1] = c;  // (every chunk overwrites its slot)
    while (pa < P1) {
        const unsigned pb = min(pa + (unsigned)kSpFlatCap, P1);
#pragma unroll
        for (int q = 0; q < kSpFlatV; ++q)
            vals[q * 256 + tid] = pa + q * 256 + tid < pb ? pv[q] * Dl[iv[q]] : 0.0;
#pragma unroll
        for (int q = 0; q < kSpFlatV; ++q) {
            const unsigned k = pa + kSpFlatCap + q * 256 + tid;
            pv[q] = k < P1 ? prod[k] : 0.0;
            iv[q] = k < P1 ? pidx[k] : (unsigned short)0;
        }
        __syncthreads();
        for (int r = ra + tid; r < c; r += 256) {
            const unsigned st = estart[e0 + r];
            if (st >= pb) break;
            const unsigned en = estart[e0 + r + 1];
            const unsigned lo = st < pa ? pa : st, hi = en < pb ? en : pb;
            double s = st < pa ? carry : 0.0;
            unsigned k = lo;
            for (; k + 4 <= hi; k += 4) {  // 4 LDS reads in flight, adds in order
                const double v0 = vals[k - pa], v1 = vals[k + 1 - pa], v2 = vals[k + 2 - pa],
                             v3 = vals[k + 3 - pa];
                s += v0;
                s += v1;
                s += v2;
                s += v3;
            }
            for (; k < hi; ++k) s += vals[k - pa];
            if (en <= pb) tri[e0 + r] = s;
            if (en >= pb) {  // the chunk's last entry (exactly one: st < pb <= en)
                next_s[par] = en > pb ? r : r + 1;  // it runs on: carry its partial sum
                carry_s[par] = s;
            }
        }
        __syncthreads();  // (parity slots: the ones written here were last read two chunks ago)
        carry = carry_s[par];  // used only if entry ra continues (starts before pb)
        ra = next_s[par];
        pa = pb;
        par ^= 1;
    }
    for (int r = ra + tid; r < c; r += 256) tri[e0 + r] = 0.0;  // empty entries past P1
}

int sp_col_max_row() { return kSpColMaxRow; }

// sparse Gram variant (bb_set_tuning key 3): 0 lanes per entry (k_sp_gram_col), 1 the same
// with non-temporal pair-list loads, 2 / 3 (the default) the flat chunked stream
// (k_sp_gram_flat) with 8 / 16 pairs per lane per chunk
int g_sp_nt = 3;

void launch_sp_gram_col(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                        const unsigned *estart, const double *prod, const unsigned short *pidx,
                        const double *D, const double *u, int n_pad, int max_row, double *tri,
                        double *xu, const int *gate) {
    const size_t lds = (size_t)(max_row > 0 ? max_row : 1) * sizeof(double);
    if (g_sp_nt >= 2) {
        auto kern = g_sp_nt == 2 ? k_sp_gram_flat<8> : k_sp_gram_flat<16>;
        note_launch(KF_GRAM, (const void *)kern);
        kern<<<n_pad, 256, lds, s>>>(rowptr, colidx, rval, estart, prod, pidx, D, u, n_pad, tri,
                                     xu, gate);
    } else if (g_sp_nt)
        k_sp_gram_col<true><<<n_pad, 256, lds, s>>>(rowptr, colidx, rval, estart, prod, pidx, D,
                                                    u, n_pad, tri, xu, gate);
    else
        k_sp_gram_col<false><<<n_pad, 256, lds, s>>>(rowptr, colidx, rval, estart, prod, pidx, D,
                                                     u, n_pad, tri, xu, gate);
}

// One wave per row c of X (CSR), lanes strided over the row's entries, fixed tree.  (Four
// independent accumulators, or a workgroup per row, measured slower at C5: 53 against 45 us.)
template <bool DIAG>
__global__ __launch_bounds__(256) void k_sp_rows(const int *__restrict__ rowptr,
                                                 const int *__restrict__ colidx,
                                                 const double *__restrict__ rval, int n_pad,
                                                 const double *__restrict__ v,
                                                 const double *__restrict__ D,
                                                 double *__restrict__ xv,
                                                 double *__restrict__ tri, const int *gate) {
    if (gated(gate)) return;
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= n_pad) return;
    double s = 0.0, d = 0.0;
    for (int k = rowptr[c] + lane; k < rowptr[c + 1]; k += 64) {
        const int j = colidx[k];
        const double x = rval[k];
        s += x * v[j];
        if (DIAG) d += x * x * D[j];
    }
    s = group_sum<64>(s);
    if (DIAG) d = group_sum<64>(d);
    if (lane == 0) {
        xv[c] = s;
        if (DIAG) tri[tri_index(c, c)] = d;
    }
}

void launch_sp_rows(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                    int n_pad, const double *v, const double *D, double *xv, double *tri, const int *gate) {
    const int blocks = (n_pad + 3) / 4;
    if (D)
        k_sp_rows<true><<<blocks, 256, 0, s>>>(rowptr, colidx, rval, n_pad, v, D, xv, tri, gate);
    else
        k_sp_rows<false><<<blocks, 256, 0, s>>>(rowptr, colidx, rval, n_pad, v, D, xv, tri, gate);
}

// 16 lanes per column of the CSC: s = X_j . w, beta_j = u_j + D_j s / sig.
constexpr int kSpBetaLanes = 16;

__global__ __launch_bounds__(256) void k_sp_beta(const int *__restrict__ colptr,
                                                 const int *__restrict__ rowidx,
                                                 const double *__restrict__ cval, int p_loc,
                                                 const double *__restrict__ w,
                                                 const double *__restrict__ u,
                                                 const double *__restrict__ D,
                                                 const DevScalars *sc, double *__restrict__ beta,
                                                 double *__restrict__ trace) {
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const int j = (int)(gid / kSpBetaLanes);
    const int q = (int)(gid % kSpBetaLanes);
    double s = 0.0;
    if (j < p_loc)
        for (int k = colptr[j] + q; k < colptr[j + 1]; k += kSpBetaLanes) s += cval[k] * w[rowidx[k]];
    s = group_sum<kSpBetaLanes>(s);
    if (q == 0 && j < p_loc) {
        const double sig = sqrt(sc->sig2);
        const double b = u[j] + D[j] * s / sig;
        beta[j] = b;
        if (trace) trace[j] = b;
    }
}

void launch_sp_beta(hipStream_t s, const int *colptr, const int *rowidx, const double *cval,
                    int p_loc, const double *w, const double *u, const double *D,
                    const DevScalars *sc, double *beta, double *beta_trace) {
    const long threads = (long)p_loc * kSpBetaLanes;
    note_launch(KF_BETA, (const void *)k_sp_beta);
    k_sp_beta<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(colptr, rowidx, cval, p_loc, w, u,
                                                                D, sc, beta, beta_trace);
}

}  // namespace bb
