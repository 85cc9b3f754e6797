// bb_ozaki.hip -- fp64-accurate Woodbury Gram X diag(D) X' on the int8 matrix cores of gfx950
// (Ozaki scheme II: exact int8 GEMMs modulo pairwise coprime moduli + CRT).  See bb_ozaki.h
// for the arithmetic; DESIGN.md s5 for the roofline.  Replaces the fp64 MFMA k_gram on the
// p > n beta step (the reference's Gram is BridgeRegression.cpp:24, X'X, for its p x p path).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "bb_kernels.h"
#include "bb_ozaki.h"

namespace bb {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// Host constants.
// ---------------------------------------------------------------------------
static constexpr int kMods[kOzMods] = {247, 245, 244, 243, 241, 239, 233, 229,
                                       227, 223, 211, 199, 197, 193, 191, 181};

// Compile-time Garner tables: the CRT kernel folds them into instruction literals (as
// kernel arguments they spill out of SGPRs and are re-fetched by scalar loads per element).
struct OzTab {
    int m[kOzMods];
    int invP[kOzMods];
    int Pmod[kOzMods][kOzMods];
    float inv_mf[kOzMods];
    double inv_md[kOzMods];
    double Wh[kOzMods], Wl[kOzMods];  // mixed-radix weights prod_{i<k} m_i = Wh + Wl
};

constexpr long long cx_inv_mod(long long a, long long m) {
    long long g = m, x = 0, x1 = 1, a1 = ((a % m) + m) % m;
    while (a1) {
        long long q = g / a1, t = g - q * a1;
        g = a1;
        a1 = t;
        t = x - q * x1;
        x = x1;
        x1 = t;
    }
    return ((x % m) + m) % m;
}

constexpr OzTab oz_make_tab() {
    OzTab t{};
    for (int k = 0; k < kOzMods; ++k) {
        t.m[k] = kMods[k];
        t.inv_mf[k] = 1.0f / (float)kMods[k];
        long long P = 1;
        for (int j = 0; j < k; ++j) {
            t.Pmod[j][k] = (int)P;
            P = (P * kMods[j]) % kMods[k];
        }
        t.invP[k] = k ? (int)cx_inv_mod(P, kMods[k]) : 1;
        t.inv_md[k] = 1.0 / (double)kMods[k];
    }
    __int128 W = 1;  // < 2^125: exact in 128 bits
    for (int k = 0; k < kOzMods; ++k) {
        t.Wh[k] = (double)W;
        t.Wl[k] = (double)(W - (__int128)t.Wh[k]);
        W *= kMods[k];
    }
    return t;
}

constexpr OzTab kOzTab = oz_make_tab();

static long long inv_mod(long long a, long long m) {
    long long g = m, x = 0, x1 = 1, a1 = ((a % m) + m) % m;
    while (a1) {
        long long q = g / a1, t = g - q * a1;
        g = a1;
        a1 = t;
        t = x - q * x1;
        x = x1;
        x1 = t;
    }
    return ((x % m) + m) % m;
}

const OzConsts &oz_consts() {
    static OzConsts c = [] {
        OzConsts o{};
        o.log2M = 0.0;
        for (int k = 0; k < kOzMods; ++k) {
            o.m[k] = kMods[k];
            o.inv_m[k] = 1.0 / kMods[k];
            o.inv_mf[k] = 1.0f / (float)kMods[k];
            o.log2M += std::log2((double)kMods[k]);
            long long P = 1;  // prod_{i<k} m_i mod m_k
            for (int j = 0; j < k; ++j) {
                o.Pmod[j][k] = (int)P;
                P = (P * kMods[j]) % kMods[k];
            }
            o.invP[k] = k ? (int)inv_mod(P, kMods[k]) : 1;
        }
        return o;
    }();
    return c;
}

int oz_bits_for(int K) {
    const double l = oz_consts().log2M - 1.0 - std::log2((double)(K > 1 ? K : 1)) - 1e-6;
    int b = (int)std::floor(l / 2.0);
    return b > 53 ? 53 : b;
}

int oz_rows(int n_pad) { return (n_pad + kOzT - 1) / kOzT * kOzT; }

// 2^31 / (123^2 * 64) = 2217.9: chunks per split with exact int32 accumulation
constexpr int kOzMaxSplitChunks = 2217;

int oz_splits_for(int n_oz, int nkc) {
    const int nt = n_oz / kOzT;
    const int nper = nt * (nt - 1) / 2 + (nt + 1) / 2;  // workgroups per (modulus, split) unit
    // the persistent GEMM runs one workgroup per CU over kOzMods * S units: take the fewest
    // K splits (each adds a partial plane per modulus for the GEMM to write and the CRT to
    // read) that give every CU a workgroup, at most 4 (the CRT's specialisations) and with
    // >= 16 chunks per split
    int S = 1;
    while (S < 4 && nper * kOzMods * S < 256 && nkc / (2 * S) >= 16) S *= 2;
    // exactness: a split's int32 sums of products of balanced residues (|r| <= 123) must stay
    // below 2^31, i.e. at most kOzMaxSplitChunks 64-deep chunks per split
    while ((nkc + S - 1) / S > kOzMaxSplitChunks) S *= 2;
    return S;
}

size_t oz_residue_bytes(int n_oz, int p_pad) { return (size_t)kOzMods * n_oz * p_pad; }

size_t oz_partial_bytes(int n_oz, int nsplit) {
    const int nt = n_oz / kOzT;
    return (size_t)nsplit * kOzMods * (nt * (nt + 1) / 2) * kOzT * kOzT;
}

// ---------------------------------------------------------------------------
// Setup: per-(64-column chunk, row) max |X|.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_oz_xmax(const double *__restrict__ X, int ldx, int n_pad,
                                                 int n_oz, double *__restrict__ xmax) {
    const int c = blockIdx.x;
    const int i = blockIdx.y * 256 + threadIdx.x;
    double m = 0.0;
    if (i < n_pad)
        for (int j = 0; j < kOzKC; ++j) m = fmax(m, fabs(X[(size_t)i + (size_t)(c * kOzKC + j) * ldx]));
    xmax[(size_t)c * n_oz + i] = m;
}

void launch_oz_xmax(hipStream_t s, const double *X, int ldx, int n_pad, int n_oz, int p_pad,
                    double *xmax) {
    dim3 grid(p_pad / kOzKC, n_oz / 256);
    k_oz_xmax<<<grid, 256, 0, s>>>(X, ldx, n_pad, n_oz, xmax);
}

// ---------------------------------------------------------------------------
// Per sweep: chunk maxima of sqrt(D), then row exponents.
// ---------------------------------------------------------------------------
// Two stages, no atomics.  k_oz_bound: workgroup = (256 rows, kOzBoundChunks chunks); each
// wave forms the chunk maxima of sqrt(D) of four of the chunks (wave reductions), then each
// thread (one row) takes max_c xmax[c][i] * sdm[c] over the group's chunks into
// part[group][i] (coalesced).  k_oz_finalize takes the max over the groups (max is exact and
// order-independent, so the result is deterministic) and turns it into the row exponents.
// (The first version folded every (64 rows, 16 chunks) wave into rowbits[i] with a 64-bit
// atomicMax: 20 us at C3 for 12.8 MB of xmax, the sqrt maxima recomputed per row block.)
constexpr int kOzBoundChunks = 16;

int oz_bound_groups(int p_pad) { return (p_pad / kOzKC + kOzBoundChunks - 1) / kOzBoundChunks; }

__global__ __launch_bounds__(256) void k_oz_bound(const double *__restrict__ D, int nkc,
                                                  const double *__restrict__ xmax, int n_oz,
                                                  double *__restrict__ part, const int *gate) {
    if (gated(gate)) return;
    __shared__ double sdm[kOzBoundChunks];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cg = blockIdx.y * kOzBoundChunks;
    const int i = blockIdx.x * 256 + threadIdx.x;
    double xm[kOzBoundChunks];  // this row's chunk maxima, in flight during the sqrt maxima
#pragma unroll
    for (int q = 0; q < kOzBoundChunks; ++q)
        xm[q] = cg + q < nkc ? xmax[(size_t)(cg + q) * n_oz + i] : 0.0;
#pragma unroll
    for (int q = w; q < kOzBoundChunks; q += 4) {
        const int c = cg + q;
        double v = c < nkc ? sqrt(D[(size_t)c * kOzKC + lane]) : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
        if (lane == 0) sdm[q] = v;
    }
    __syncthreads();
    double m = 0.0;
#pragma unroll
    for (int q = 0; q < kOzBoundChunks; ++q) m = fmax(m, xm[q] * sdm[q]);
    part[(size_t)blockIdx.y * n_oz + i] = m;
}

// 16 lanes per row, each over every 16th group, then a max across the 16 lanes
__global__ __launch_bounds__(256) void k_oz_finalize(const double *__restrict__ part, int ng,
                                                     int n_oz, int b, double *__restrict__ rscale,
                                                     int *__restrict__ escale, const int *gate) {
    if (gated(gate)) return;
    const int i = blockIdx.x * 16 + (threadIdx.x >> 4), l = threadIdx.x & 15;
    double m = 0.0;
    if (i < n_oz)
        for (int g = l; g < ng; g += 16) m = fmax(m, part[(size_t)g * n_oz + i]);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 16));
    if (i >= n_oz || l != 0) return;
    int e = 0;
    if (m > 0.0) (void)frexp(m, &e);  // m < 2^e
    if (e < -960) e = -960;
    rscale[i] = ldexp(1.0, b - e);
    escale[i] = e - b;
}

void launch_oz_scale(hipStream_t s, const double *D, int p_pad, const double *xmax, int n_oz,
                     int b, double *part, double *rscale, int *escale, const int *gate) {
    const int nkc = p_pad / kOzKC;
    const int ng = oz_bound_groups(p_pad);
    k_oz_bound<<<dim3(n_oz / 256, ng), 256, 0, s>>>(D, nkc, xmax, n_oz, part, gate);
    k_oz_finalize<<<(n_oz + 15) / 16, 256, 0, s>>>(part, ng, n_oz, b, rscale, escale, gate);
}

// ---------------------------------------------------------------------------
// Residues.  Wave = (64 rows, one 64-column chunk); lane = row.  Each lane rounds its 64
// scaled values once, then emits 64 bytes per modulus: r = v - m rint(v/m) via the
// 1.5*2^52 magic constant (|v| <= 2^53, m <= 247 => |r| <= 125, int8), the byte taken from
// the low word of r + magic.  Stores: four 16-byte units per lane into the blocked layout
// (16 consecutive lanes write one contiguous 256 B run), 4 KB per wave and modulus.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double oz_readlane_d(double v, int lane) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)bits, lane);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

constexpr int kOzResCols = 32;   // columns per wave (half a chunk): keeps occupancy >= 4
constexpr int kOzResChunks = 4;  // 64-column chunks per workgroup, at most (oz_res_cpw)

// Workgroup = cpw (<= kOzResChunks) 64-column chunks x 256 rows (8 waves: 4 row slices x 2 column
// halves), so the X reads are 2 KB contiguous per column and each modulus plane is written
// as one 16 KB contiguous block per chunk.  The same pass over X also forms the X.u partial
// sums of the Woodbury draw (u = sqrt(D) z): part[g][row] over the cpw * 64 columns of group g,
// summed per lane in column order, then the two column halves -- so the separate X.u pass
// (k_xv) disappears from the Ozaki sweep.
template <bool NT, bool NTL>
__global__ __launch_bounds__(512) void k_oz_residues(const double *__restrict__ X, int ldx,
                                                     int n_pad, int n_oz, int nkc,
                                                     const double *__restrict__ D,
                                                     const double *__restrict__ rscale,
                                                     int8_t *__restrict__ R, OzConsts C,
                                                     const double *__restrict__ u,
                                                     double *__restrict__ xu_part, int cpw, const int *gate) {
    if (gated(gate)) return;
    __shared__ double xu_half[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int half = w & 1;
    const int row = blockIdx.y * 256 + (w >> 1) * 64 + lane;
    const double rs = rscale[row];
    // rows >= n_pad (tile padding) load a valid row and are zeroed through rs = 0
    const double rsl = row < n_pad ? rs : 0.0;
    double xu = 0.0;
    for (int cc = 0; cc < cpw; ++cc) {
        const int kc = blockIdx.x * cpw + cc;
        if (kc >= nkc) break;
        const int col0 = kc * kOzKC + half * kOzResCols;
        const int cl = col0 + (lane & (kOzResCols - 1));
        const double sdl = sqrt(D[cl]);
        const double ul = u ? u[cl] : 0.0;
        const double *xp = X + (size_t)min(row, n_pad - 1) + (size_t)col0 * ldx;
        double v[kOzResCols];
#pragma unroll
        for (int j = 0; j < kOzResCols; ++j)
            v[j] = NTL ? __builtin_nontemporal_load(xp + (size_t)j * ldx) : xp[(size_t)j * ldx];
        if (u) {
#pragma unroll
            for (int j = 0; j < kOzResCols; ++j) xu += v[j] * oz_readlane_d(ul, j);
        }
#pragma unroll
        for (int j = 0; j < kOzResCols; ++j) v[j] = rint(v[j] * oz_readlane_d(sdl, j) * rsl);
        // low 32 bits of each integer x (|x| <= 2^53): x = xh 2^32 + xl, 0 <= xl < 2^32
        unsigned int xl[kOzResCols];
#pragma unroll
        for (int j = 0; j < kOzResCols; ++j) {
            const double xh = floor(v[j] * 2.3283064365386963e-10);  // 2^-32
            xl[j] = (unsigned int)__builtin_fma(-xh, 4294967296.0, v[j]);
        }
        const double magic = 6755399441055744.0;  // 1.5 * 2^52
#pragma unroll 1
        for (int k = 0; k < kOzMods; ++k) {
            // q = rint(x / m) sits in the low word of fma(x, 1/m, 1.5*2^52) (two's
            // complement); r = x - q m is the balanced residue (|r| <= 125), and its byte is
            // (xl + q (256 - m)) mod 256 -- one fp64 FMA and one v_mad_u32_u24 per element
            const double im = C.inv_m[k];
            const unsigned int cm = 256u - (unsigned int)C.m[k];
            // plane (k, kc) is [16-row block][unit 0..3][row in block][16 B]: one store
            // instruction writes the 64 rows' 16-byte unit as four 256-B runs, and one GEMM
            // LDS-DMA instruction (16 rows x 4 units) reads one 1 KB block
            int8_t *dst = R + ((size_t)k * nkc + kc) * n_oz * kOzKC + (size_t)(row >> 4) * 1024 +
                          (size_t)(row & 15) * 16 + (size_t)(2 * half) * 256;
#pragma unroll
            for (int q = 0; q < kOzResCols / 16; ++q) {
                unsigned int wd[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    unsigned int b4[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = q * 16 + d * 4 + e;
                        const unsigned int ql =
                            (unsigned int)__double_as_longlong(__builtin_fma(v[j], im, magic));
                        b4[e] = __umul24(ql, cm) + xl[j];
                    }
                    const unsigned int lo = __builtin_amdgcn_perm(b4[1], b4[0], 0x0c0c0400u);
                    const unsigned int hi = __builtin_amdgcn_perm(b4[3], b4[2], 0x0c0c0400u);
                    wd[d] = lo | (hi << 16);
                }
                const v4i val = (v4i){(int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]};
                if constexpr (NT) __builtin_nontemporal_store(val, (v4i *)(dst + q * 256));
                else *(v4i *)(dst + q * 256) = val;
            }
        }
    }
    if (!u) return;
    if (half == 1) xu_half[w >> 1][lane] = xu;
    __syncthreads();
    if (half == 0 && row < n_pad)
        xu_part[(size_t)blockIdx.x * n_pad + row] = xu + xu_half[w >> 1][lane];
}

// Chunks per workgroup: kOzResChunks, halved (down to 1) until the launch has >= 1024
// workgroups -- at C2 (K = 5120, 1024 rows) four chunks gave 80 workgroups
static int oz_res_cpw(int nkc, int n_oz) {
    int c = kOzResChunks;
    while (c > 1 && (long)((nkc + c - 1) / c) * (n_oz / 256) < 1024) c >>= 1;
    return c;
}

int oz_xu_parts(int p_pad, int n_oz) {
    const int nkc = p_pad / kOzKC, c = oz_res_cpw(nkc, n_oz);
    return (nkc + c - 1) / c;
}

// residue-plane stores and X loads (round 3, tools/res_nt_ab.py, C3 ozprep on three boxes):
// 0 ordinary, 1 non-temporal stores, 2 (the default) non-temporal stores and X loads.
// Box A: 0.68 / 0.53 / -- ms (ordinary stores slow there); box B: 0.457 / 0.463 / 0.405 ms;
// box C: 0.458 / 0.465 / 0.461 ms.  bb_set_tuning(1, v) for A/B
int g_oz_res_nt = 2;

void launch_oz_residues(hipStream_t s, const double *X, int ldx, int n_pad, int n_oz, int p_pad,
                        const double *D, const double *rscale, int8_t *R, const double *u,
                        double *xu_part, const int *gate) {
    const int nkc = p_pad / kOzKC, cpw = oz_res_cpw(nkc, n_oz);
    dim3 grid((nkc + cpw - 1) / cpw, n_oz / 256);
    if (g_oz_res_nt == 2)
        k_oz_residues<true, true><<<grid, 512, 0, s>>>(X, ldx, n_pad, n_oz, nkc, D, rscale, R,
                                                       oz_consts(), u, xu_part, cpw, gate);
    else if (g_oz_res_nt)
        k_oz_residues<true, false><<<grid, 512, 0, s>>>(X, ldx, n_pad, n_oz, nkc, D, rscale, R,
                                                        oz_consts(), u, xu_part, cpw, gate);
    else
        k_oz_residues<false, false><<<grid, 512, 0, s>>>(X, ldx, n_pad, n_oz, nkc, D, rscale,
                                                         R, oz_consts(), u, xu_part, cpw, gate);
}

// ---------------------------------------------------------------------------
// int8 GEMM per (modulus, lower tile, K split): C = R_I R_K' (exact int32), stored mod m.
// 256 threads = 4 waves; one workgroup per CU.  Staging: a 4-stage LDS ring (32 KB per
// stage: A then B, 256 rows x 64 B each) filled by global_load_lds_dwordx4 three chunks
// ahead; one wave-instruction moves one 1 KB block of 16 rows, lane-linearly (the residue
// image is stored in that [16-row block][unit][row][16 B] order, so fragment reads need no
// swizzle).  Per chunk: counted s_waitcnt vmcnt (two stages stay in flight), raw s_barrier,
// MFMAs interleaved with the next chunk's fragment reads and the refill pieces.
// XCD grouping: block b runs on XCD b % 8; all tiles of one (modulus, split) unit are given
// to one XCD so that their shared row blocks stay in that XCD's L2.
// ---------------------------------------------------------------------------
constexpr int kOzStages = 4;
constexpr int kOzOpBytes = kOzT * kOzKC;          // 16 KB per operand per stage
constexpr int kOzStageBytes = 2 * kOzOpBytes;     // 32 KB

__device__ __forceinline__ void oz_glds(const int8_t *src, int8_t *lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}

// ---------------------------------------------------------------------------
// The tile on v_mfma_i32_16x16x64_i8: one K step is a whole
// 64-byte chunk, and a 16-row operand fragment (lane l: row l & 15, unit l >> 4) is exactly
// one 1 KB block of the residue image, read lane-linearly.  Per wave 8 x 8 accumulator
// blocks of 16 x 16 (256 registers), 64 MFMAs of 16 cycles per chunk.  The MFMA is issued
// as B x A' (C/D map: col = l & 15 on the A side, row = 4 (l >> 4) + reg on the B side), so
// each lane's 4 results are 4 consecutive output bytes.
// ---------------------------------------------------------------------------
// v_mfma_i32_16x16x64_i8 with the accumulator pinned to AGPRs (the builtin lets the register
// allocator shuttle 64 four-register accumulators between the files every K step).  Every
// accumulator is re-used only 64 MFMAs later; the epilogue waits out the last writes.
__device__ __forceinline__ void oz_mfma16(v4i &acc, const v4i &a, const v4i &b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// s_waitcnt vmcnt(N) (expcnt, lgkmcnt left open): every piece older than the newest N landed
template <int N>
__device__ __forceinline__ void oz_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// Diagonal tiles, two per workgroup.  A diagonal tile (I, I) needs only its lower half:
// the off-diagonal quadrant (rows 128..255 x cols 0..127, 64 blocks) and the lower halves
// of its two diagonal quadrants (36 + 36 blocks, the diagonal blocks whole).  Its two
// operands are the same 256-row block, so one 16 KB operand slot per stage feeds a tile:
// slot 0 = tile (I1, I1), slot 1 = tile (I2, I2).  Waves 0, 1 take the off-diagonal
// quadrant of tile wid (64 MFMAs per chunk), waves 2, 3 the diagonal quadrants of tile
// wid - 2 (72 MFMAs: D1 lower blocks in acc[i][j], i >= j; D2 strictly lower in acc[j][i];
// D2's diagonal blocks in 8 VGPR accumulators).  Every wave reads the same 16 fragments of
// its slot per chunk (blocks 8..15 as the A side, 0..7 as the K side).  The DMA ring and
// the per-chunk protocol are oz_full_pass's.  The grid is tiles / 2 instead of tiles
// workgroups for the diagonal band.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void oz_mfma16v(v4i &acc, const v4i &a, const v4i &b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// One wave's whole pass (ring prologue, chunk loop, epilogue) for a role fixed at compile
// time: the two roles keep disjoint accumulator live ranges, and both execute the same
// barrier sequence (one per chunk plus the prologue's).
template <int dbg, bool DIAGQ>
__device__ __forceinline__ void oz_diag_pass(int8_t *smem, const int8_t *baseA,
                                             const int8_t *baseB, size_t kstride, int c0,
                                             int nch, int cs, int wid, int slot, int8_t *out,
                                             int m, double im) {
    const int lane = threadIdx.x & 63;
    const int voff = wid * 4096 + lane * 16;
    // chunk of K step i: the pass starts at chunk cs of its split and wraps (exact integer
    // sums, so the order does not change a bit of the result)
    auto kat = [&](int i) {
        const int q = cs + i;
        return c0 + (q >= nch ? q - nch : q);
    };
    auto glds_one = [&](int kc, int stage, int g) {
        int8_t *sb = smem + stage * kOzStageBytes + (g >> 2) * kOzOpBytes;
        const int8_t *src = ((g >> 2) ? baseB : baseA) + (size_t)kc * kstride + (g & 3) * 1024;
        oz_glds(src + voff, sb + (4 * wid + (g & 3)) * 1024);
    };
    auto issue = [&](int kc, int stage) {
#pragma unroll
        for (int g = 0; g < 8; ++g) glds_one(kc, stage, g);
    };
    // accv: D2's diagonal blocks 0..3 (DIAGQ waves) or 4..7 (the off-diagonal waves, which
    // read the same slot fragments): 68 MFMAs per chunk on every wave instead of 64 / 72, so
    // the pair's chunk step (one barrier per chunk) is 6 % rather than 12.5 % longer than an
    // off-diagonal tile's and the pair lags its unit's tiles half as much
    v4i acc[8][8], accv[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i < 4) accv[i] = (v4i){0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
    }
    // fragment blk of this wave's slot: blocks 8..15 -> fa (A side), 0..7 -> fb (K side)
    auto frag = [&](int chunk, int blk) {
        const int8_t *S_ = smem + (chunk % kOzStages) * kOzStageBytes + slot * kOzOpBytes;
        return *(const v4i *)&S_[blk * 1024 + lane * 16];
    };
    auto step = [&](int it, v4i (&fa_c)[8], v4i (&fb_c)[8], v4i (&fa_n)[8], v4i (&fb_n)[8]) {
        if (!(dbg & 4)) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            oz_wait_vm<16>();
            __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        const int kc_next = kat(min(it + kOzStages, nch - 1));
        const int st_next = (it + kOzStages) % kOzStages;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            if constexpr (!DIAGQ) {
                // off-diagonal quadrant: rows 128 + 16 g (fa), cols 16 j (fb)
                oz_mfma16(acc[g][0], fb_c[0], fa_c[g]);
                if (!(dbg & 1)) glds_one(kc_next, st_next, g);
                oz_mfma16(acc[g][1], fb_c[1], fa_c[g]);
                if (!(dbg & 2)) fa_n[g] = frag(it + 1, 8 + g);
                oz_mfma16(acc[g][2], fb_c[2], fa_c[g]);
                if (!(dbg & 2)) fb_n[g] = frag(it + 1, g);
#pragma unroll
                for (int j = 3; j < 8; ++j) oz_mfma16(acc[g][j], fb_c[j], fa_c[g]);
                if (g >= 4) oz_mfma16v(accv[g - 4], fa_c[g], fa_c[g]);
            } else {
                // D1 (fb x fb) block (g, j <= g); D2 (fa x fa) block (g, j < g) in acc[j][g]
                // and its diagonal block in accv[g]
                oz_mfma16(acc[g][0], fb_c[0], fb_c[g]);
                if (!(dbg & 1)) glds_one(kc_next, st_next, g);
#pragma unroll
                for (int j = 1; j <= g; ++j) oz_mfma16(acc[g][j], fb_c[j], fb_c[g]);
                if (!(dbg & 2)) fa_n[g] = frag(it + 1, 8 + g);
#pragma unroll
                for (int j = 0; j < g; ++j) oz_mfma16(acc[j][g], fa_c[j], fa_c[g]);
                if (g < 4) oz_mfma16v(accv[g], fa_c[g], fa_c[g]);
                if (!(dbg & 2)) fb_n[g] = frag(it + 1, g);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    v4i fa0[8], fb0[8], fa1[8], fb1[8];
    if (nch > 0) {
#pragma unroll
        for (int st = 0; st < kOzStages - 1; ++st) issue(kat(min(st, nch - 1)), st);
        oz_wait_vm<16>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(kat(min(kOzStages - 1, nch - 1)), kOzStages - 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            fa0[i] = frag(0, 8 + i);
            fb0[i] = frag(0, i);
        }
    }
    int it = 0;
    for (; it + 1 < nch; it += 2) {
        step(it, fa0, fb0, fa1, fb1);
        step(it + 1, fa1, fb1, fa0, fb0);
    }
    if (it < nch) step(it, fa0, fb0, fa1, fb1);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const int hi = m / 2, lo = hi - m + 1;
    auto store = [&](int rowl, int col, const v4i &v) {
        unsigned int wv = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cval = v[r];
            int rr = cval - (int)rint((double)cval * im) * m;
            rr = rr > hi ? rr - m : (rr < lo ? rr + m : rr);
            wv |= ((unsigned int)rr & 0xffu) << (8 * r);
        }
        *(unsigned int *)(out + rowl * kOzT + col) = wv;
    };
    // (lane l, reg r of block (i, j) = row 16 i + (l & 15), column 16 j + 4 (l >> 4) + r)
    const int rl = lane & 15, cl = 4 * (lane >> 4);
    if constexpr (!DIAGQ) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) store(128 + 16 * i + rl, 16 * j + cl, acc[i][j]);
#pragma unroll
        for (int i = 4; i < 8; ++i) store(128 + 16 * i + rl, 128 + 16 * i + cl, accv[i - 4]);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j <= i; ++j) store(16 * i + rl, 16 * j + cl, acc[i][j]);
#pragma unroll
            for (int j = 0; j < i; ++j) store(128 + 16 * i + rl, 128 + 16 * j + cl, acc[j][i]);
            if (i < 4) store(128 + 16 * i + rl, 128 + 16 * i + cl, accv[i]);
        }
    }
}

// A full 256 x 256 off-diagonal tile on 4 waves (2 x 2, 128 x 128 each, 8 x 8 blocks of
// 16 x 16 per wave, 256 AGPR accumulators), a device pass of the unified launch below.
template <int dbg>
__device__ __forceinline__ void oz_full_pass(int8_t *smem, const int8_t *baseA,
                                             const int8_t *baseB, size_t kstride, int c0,
                                             int nch, int cs, int wid, int8_t *out, int m,
                                             double im) {
    const int lane = threadIdx.x & 63;
    const int wr = wid >> 1, wc = wid & 1;
    const int voff = wid * 4096 + lane * 16;
    auto kat = [&](int i) {  // as in oz_diag_pass
        const int q = cs + i;
        return c0 + (q >= nch ? q - nch : q);
    };
    auto glds_one = [&](int kc, int stage, int g) {
        int8_t *sb = smem + stage * kOzStageBytes + (g >> 2) * kOzOpBytes;
        const int8_t *src = ((g >> 2) ? baseB : baseA) + (size_t)kc * kstride + (g & 3) * 1024;
        oz_glds(src + voff, sb + (4 * wid + (g & 3)) * 1024);
    };
    auto issue = [&](int kc, int stage) {
#pragma unroll
        for (int g = 0; g < 8; ++g) glds_one(kc, stage, g);
    };
    v4i acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
    auto frag_a = [&](int chunk, int i) {
        const int8_t *A_ = smem + (chunk % kOzStages) * kOzStageBytes;
        return *(const v4i *)&A_[(wr * 8 + i) * 1024 + lane * 16];
    };
    auto frag_b = [&](int chunk, int j) {
        const int8_t *B_ = smem + (chunk % kOzStages) * kOzStageBytes + kOzOpBytes;
        return *(const v4i *)&B_[(wc * 8 + j) * 1024 + lane * 16];
    };
    auto step = [&](int it, v4i (&fa_c)[8], v4i (&fb_c)[8], v4i (&fa_n)[8], v4i (&fb_n)[8]) {
        if (!(dbg & 4)) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            oz_wait_vm<16>();
            __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        const int kc_next = kat(min(it + kOzStages, nch - 1));
        const int st_next = (it + kOzStages) % kOzStages;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            oz_mfma16(acc[g][0], fb_c[0], fa_c[g]);
            if (!(dbg & 1)) glds_one(kc_next, st_next, g);
            oz_mfma16(acc[g][1], fb_c[1], fa_c[g]);
            if (!(dbg & 2)) fa_n[g] = frag_a(it + 1, g);
            oz_mfma16(acc[g][2], fb_c[2], fa_c[g]);
            if (!(dbg & 2)) fb_n[g] = frag_b(it + 1, g);
#pragma unroll
            for (int j = 3; j < 8; ++j) oz_mfma16(acc[g][j], fb_c[j], fa_c[g]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    v4i fa0[8], fb0[8], fa1[8], fb1[8];
    if (nch > 0) {
#pragma unroll
        for (int st = 0; st < kOzStages - 1; ++st) issue(kat(min(st, nch - 1)), st);
        oz_wait_vm<16>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(kat(min(kOzStages - 1, nch - 1)), kOzStages - 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            fa0[i] = frag_a(0, i);
            fb0[i] = frag_b(0, i);
        }
    }
    int it = 0;
    for (; it + 1 < nch; it += 2) {
        step(it, fa0, fb0, fa1, fb1);
        step(it + 1, fa1, fb1, fa0, fb0);
    }
    if (it < nch) step(it, fa0, fb0, fa1, fb1);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const int hi = m / 2, lo = hi - m + 1;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int rowl = wr * 128 + i * 16 + (lane & 15);
            const int col = wc * 128 + j * 16 + 4 * (lane >> 4);
            unsigned int wv = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int cval = acc[i][j][r];
                int rr = cval - (int)rint((double)cval * im) * m;
                rr = rr > hi ? rr - m : (rr < lo ? rr + m : rr);
                wv |= ((unsigned int)rr & 0xffu) << (8 * r);
            }
            *(unsigned int *)(out + rowl * kOzT + col) = wv;
        }
}

// Unified launch: per (modulus, split) unit, nt (nt-1)/2 off-diagonal tiles and
// ceil(nt/2) diagonal pairs, all of one unit on one XCD (block b -> XCD b % 8) so that the
// pairs share their row blocks in L2 with the unit's off-diagonal tiles running beside them
// (launched alone, the pairs stream their rows from HBM).
// K rotation (round 3): a unit's row blocks are shared through the XCD's 4 MB L2, which
// spans ~32 chunk steps of the unit (8 row blocks x 16 KB per step), so a workgroup that runs
// more than ~32 chunks behind the rest reads from HBM.  The diagonal pairs do 68 MFMAs per
// wave per chunk against 64 and used to fall ~47 chunks behind over a C3 tile, and the
// workgroups that ran a pair in one round start the next round that much late: the pairs
// alone missed L2 for 1.2 GB per launch (profiles/r03_ozaki_pairs_l2.json).  Each pass now
// starts at the chunk its unit is expected to be at and wraps around the split: a workgroup
// that ran pairs in earlier rounds starts 1/16 of a pass further per such round, and a
// diagonal pair starts a further `lead` ahead, half its expected lag, so it is ahead of the
// unit for the first half of the pass and behind it for the second.  (A progress word
// published from the chunk loop measured 3.5x slower: the store in the loop makes the
// compiler wait out every LDS-DMA piece.)  The integer sums are exact: any order gives the
// same bits.  lead < 0: every pass starts at chunk 0 (the round-2 order, for A/B).
template <int dbg>
__global__ __launch_bounds__(256, 1) void k_oz_gemm16u(const int8_t *__restrict__ R, int n_oz,
                                                       int nkc, int nsplit,
                                                       int8_t *__restrict__ P, int lead_pm,
                                                       int late_pm, OzConsts C, const int *gate) {
    if (gated(gate)) return;
    __shared__ __attribute__((aligned(1024))) int8_t smem[kOzStages * kOzStageBytes];
    const int nt = n_oz / kOzT;
    const int ntiles = nt * (nt + 1) / 2;
    const int noff = nt * (nt - 1) / 2, npair = (nt + 1) / 2;
    const int nper = noff + npair;
    // persistent: workgroup b (one per CU, b -> XCD b % 8) takes virtual blocks b, b + grid,
    // ... so every round of a unit's tiles runs on the XCD whose L2 holds its row blocks
    const int xcd = blockIdx.x & 7, q0 = blockIdx.x >> 3, qs = gridDim.x >> 3;
    const int nunits = kOzMods * nsplit;
    for (int rnd = 0;; ++rnd) {
    const int q = q0 + rnd * qs;
    const int u = xcd + 8 * (q / nper);
    if (u >= nunits) break;
    // tile slot rotated per unit (a permutation of the unit's slots, so every tile is done
    // exactly once whatever nper and the grid are); when a round is one unit per XCD (C3)
    // each workgroup takes one diagonal pair in eight rounds
    const int local = (q % nper + 4 * (q / nper)) % nper;
    const int mod = u % kOzMods;
    const int split = u / kOzMods;
    const int per = (nkc + nsplit - 1) / nsplit;
    const int c0 = split * per;
    const int nch = max(0, min(nkc, c0 + per) - c0);
    if (rnd > 0) __syncthreads();  // the previous tile's LDS ring is drained
    const bool is_pair = local >= noff;
    // this workgroup's K start (see above): a pair pass takes ~68/64 of an off-diagonal
    // one, so every earlier round spent on a pair delays the start by late_pm / 1000 of a pass
    int cs = 0;
    if (nch > 0 && lead_pm >= 0) {
        int late = 0;  // earlier rounds of this workgroup that ran a diagonal pair
        for (int r0 = 0; r0 < rnd; ++r0) {
            const int q_ = q0 + r0 * qs;
            late += ((q_ % nper + 4 * (q_ / nper)) % nper) >= noff;
        }
        const long shift =
            ((long)nch * late * late_pm + (is_pair ? (long)nch * lead_pm : 0)) / 1000;
        cs = (int)(shift % nch);
    }
    const size_t kstride = (size_t)n_oz * kOzKC;
    const int8_t *plane = R + (size_t)mod * nkc * kstride;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int8_t *P0 = P + ((size_t)split * kOzMods + mod) * ntiles * (size_t)(kOzT * kOzT);
    if (local < noff) {
        // strictly lower tile te = I (I-1)/2 + K
        int I = (int)((sqrt(8.0 * local + 1.0) + 1.0) * 0.5);
        while ((I + 1) * I / 2 <= local) ++I;
        while (I * (I - 1) / 2 > local) --I;
        I = __builtin_amdgcn_readfirstlane(I);
        const int K = local - I * (I - 1) / 2;
        const int tile = I * (I + 1) / 2 + K;
        oz_full_pass<dbg>(smem, plane + (size_t)I * kOzT * kOzKC, plane + (size_t)K * kOzT * kOzKC,
                          kstride, c0, nch, cs, wid, P0 + (size_t)tile * (kOzT * kOzT),
                          C.m[mod], C.inv_m[mod]);
    } else {
        if (dbg & 16) continue;  // ablation: the diagonal pairs idle (traffic probe)
        const int pr = local - noff;
        const int I1 = 2 * pr, I2 = min(2 * pr + 1, nt - 1);  // odd nt: the last tile twice
        const int slot = wid & 1;
        const int Iw = slot ? I2 : I1;
        int8_t *out = P0 + (size_t)(Iw * (Iw + 1) / 2 + Iw) * (kOzT * kOzT);
        const int8_t *bA = plane + (size_t)I1 * kOzT * kOzKC;
        const int8_t *bB = plane + (size_t)I2 * kOzT * kOzKC;
        if (wid < 2)
            oz_diag_pass<dbg, false>(smem, bA, bB, kstride, c0, nch, cs, wid, slot, out,
                                     C.m[mod], C.inv_m[mod]);
        else
            oz_diag_pass<dbg, true>(smem, bA, bB, kstride, c0, nch, cs, wid, slot, out,
                                    C.m[mod], C.inv_m[mod]);
    }
    }
}

void launch_oz_gemm(hipStream_t s, const int8_t *R, int n_oz, int p_pad, int nsplit, int8_t *P,
                    int dbg, int lead_pm, int late_pm, const int *gate) {
    const int nt = n_oz / kOzT;
    const int nkc = p_pad / kOzKC;
    const OzConsts &C = oz_consts();
    if (lead_pm == kOzLeadDefault) lead_pm = 30;  // (68 - 64) / 68 / 2 of the pass
    if (late_pm < 0) late_pm = 62;                // (68 - 64) / 64 of the pass
    // per (modulus, split) unit -- kOzMods * nsplit units, a multiple of 8 (unit u -> XCD
    // u % 8) -- the off-diagonal tiles and the diagonal pairs in one launch
    const unsigned gu0 = (unsigned)(nt * (nt - 1) / 2 + (nt + 1) / 2) * kOzMods * nsplit;
    // one workgroup per CU (128 KB of LDS each), a multiple of 8 (the XCD count)
    static const unsigned cus8 = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v < 8)
            v = 256;
        return (unsigned)(v / 8 * 8);
    }();
    const unsigned gu = gu0 < cus8 ? gu0 : cus8;
    switch (dbg) {  // dbg != 0: timing ablations of bb_bench_ozaki only (results meaningless)
        case 1: k_oz_gemm16u<1><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        case 2: k_oz_gemm16u<2><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        case 3: k_oz_gemm16u<3><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        case 4: k_oz_gemm16u<4><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        case 7: k_oz_gemm16u<7><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        case 16: k_oz_gemm16u<16><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate); break;
        default:
            note_launch(KF_GRAM, (const void *)k_oz_gemm16u<0>);
            k_oz_gemm16u<0><<<gu, 256, 0, s>>>(R, n_oz, nkc, nsplit, P, lead_pm, late_pm, C, gate);
    }
}

// ---------------------------------------------------------------------------
// CRT: per lower-triangle element, sum the split residues, Garner (balanced digits) ->
// exact 128-bit C -> fp64 -> scale; written to red2 as the packed upper triangle
// (tri_index, the layout k_form_m reads).  Extra threads sum the X u partials.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int oz_smod(int v, int m, float imf) {
    int r = v - (int)rintf((float)v * imf) * m;
    const int hi = m / 2, lo = hi - m + 1;
    r = r > hi ? r - m : r;
    r = r < lo ? r + m : r;
    return r;
}

template <int NS>
__global__ __launch_bounds__(256) void k_oz_crt(const int8_t *__restrict__ P, int nsplit, int nt,
                                                int n_pad, const int *__restrict__ escale,
                                                const double *__restrict__ xu_part, int nxu,
                                                double *__restrict__ red2, OzConsts C, const int *gate) {
    if (gated(gate)) return;
    const int ntiles = nt * (nt + 1) / 2;
    // the first blocks sum the X.u partials (a long dependent-load chain per row: started
    // first, it overlaps the residue reconstruction instead of trailing it), 8 lanes per row
    const int nxb = (n_pad * 8 + 255) / 256;
    if ((int)blockIdx.x < nxb) {
        const int t = threadIdx.x & 7;
        const long r = ((long)blockIdx.x * 256 + threadIdx.x) >> 3;
        double v = 0.0;
        if (r < n_pad) {
            // eight loads in flight, summed in the same order as one at a time
            int q = t;
            for (; q + 56 < nxu; q += 64) {
                double x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = xu_part[(size_t)(q + 8 * u) * n_pad + r];
#pragma unroll
                for (int u = 0; u < 8; ++u) v += x[u];
            }
            for (; q < nxu; q += 8) v += xu_part[(size_t)q * n_pad + r];
        }
        // fixed-order combine of the 8 lane sums
        v += __shfl_xor(v, 4, 8);
        v += __shfl_xor(v, 2, 8);
        v += __shfl_xor(v, 1, 8);
        if (t == 0 && r < n_pad) red2[tri_count(n_pad) + r] = v;
        return;
    }
    const long gid = (long)(blockIdx.x - nxb) * 256 + threadIdx.x;
    const int tile = (int)(gid >> 14);
    const int e0 = (int)(gid & 16383) * 4;  // 4 consecutive columns of one tile row
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int K = tile - I * (I + 1) / 2;
    const int gi = I * kOzT + (e0 >> 8), gk0 = K * kOzT + (e0 & 255);
    if (gi < gk0 || gi >= n_pad) return;
    // residue sums of the 4 elements for every modulus: every word is loaded before any is
    // used (interleaved with the sums, the loads become 16 dependent round trips per wave)
    int rs[kOzMods][4];
    constexpr int NL = NS > 0 ? NS : 1;
    int w[kOzMods][NL];
#pragma unroll
    for (int k = 0; k < kOzMods; ++k)
#pragma unroll
        for (int sp = 0; sp < NL; ++sp)
            w[k][sp] = __builtin_nontemporal_load(
                (const int *)(P + (((size_t)sp * kOzMods + k) * ntiles + tile) *
                                      (size_t)(kOzT * kOzT) + e0));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < kOzMods; ++k) {
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int sp = 0; sp < NL; ++sp) {
            const int v = w[k][sp];
            s0 += (int)(int8_t)(v & 0xff);
            s1 += (int)(int8_t)((v >> 8) & 0xff);
            s2 += (int)(int8_t)((v >> 16) & 0xff);
            s3 += v >> 24;
        }
        for (int sp = NL; sp < (NS > 0 ? NS : nsplit); ++sp) {
            const int v = *(const int *)(P + (((size_t)sp * kOzMods + k) * ntiles + tile) *
                                                 (size_t)(kOzT * kOzT) + e0);
            s0 += (int)(int8_t)(v & 0xff);
            s1 += (int)(int8_t)((v >> 8) & 0xff);
            s2 += (int)(int8_t)((v >> 16) & 0xff);
            s3 += v >> 24;
        }
        rs[k][0] = s0;
        rs[k][1] = s1;
        rs[k][2] = s2;
        rs[k][3] = s3;
    }
    const int ei = escale[gi];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int gk = gk0 + q;
        if (gk > gi) break;
        // Garner digits a_k (balanced): a_k = ((r_k - sum_{j<k} a_j P_jk) invP_k) mod m_k.
        // The sums are pushed forward as each digit appears (independent 24-bit mads, |acc|
        // < 2^19), so the serial chain per digit is one subtraction, one multiply and one
        // fp64 reduction (|v| < 2^27: exact quotient within one, corrected).
        int a[kOzMods];
        int acc[kOzMods];
#pragma unroll
        for (int k = 0; k < kOzMods; ++k) acc[k] = 0;
#pragma unroll
        for (int k = 0; k < kOzMods; ++k) {
            const int m = kOzTab.m[k];
            int d;
            if (k == 0) {
                d = oz_smod(rs[0][q], m, kOzTab.inv_mf[0]);
            } else {
                const double v = (double)(rs[k][q] - acc[k]) * (double)kOzTab.invP[k];
                const double qd = rint(v * kOzTab.inv_md[k]);
                int t = (int)__builtin_fma(-qd, (double)m, v);
                const int hi = m / 2, lo = hi - m + 1;
                t = t > hi ? t - m : t;
                d = t < lo ? t + m : t;
            }
            a[k] = d;
#pragma unroll
            for (int j = k + 1; j < kOzMods; ++j) acc[j] += __mul24(d, kOzTab.Pmod[k][j]);
        }
        // C = sum_k a_k W_k with W_k = Wh_k + Wl_k (106 bits): every term as an exact
        // double-double (FMA split), then a pairwise tree of double-double additions (depth 4
        // instead of a 15-step Horner chain).  Balanced digits vanish above C's size, so the
        // sum is exact whenever C fits in ~106 bits and faithfully rounded beyond.
        double th[kOzMods], tl[kOzMods];
#pragma unroll
        for (int k = 0; k < kOzMods; ++k) {
            const double ad = (double)a[k];
            th[k] = ad * kOzTab.Wh[k];
            tl[k] = __builtin_fma(ad, kOzTab.Wh[k], -th[k]) + ad * kOzTab.Wl[k];
        }
#pragma unroll
        for (int w = 1; w < kOzMods; w *= 2) {
#pragma unroll
            for (int k = 0; k + w < kOzMods; k += 2 * w) {
                const double sh = th[k] + th[k + w];
                const double bv = sh - th[k];
                const double err = (th[k] - (sh - bv)) + (th[k + w] - bv);
                const double sl = err + (tl[k] + tl[k + w]);
                th[k] = sh + sl;
                tl[k] = sl - (th[k] - sh);
            }
        }
        const double hi = th[0], lo = tl[0];
        red2[tri_index(gk, gi)] = ldexp(hi + lo, ei + escale[gk]);
    }
}

void launch_oz_crt(hipStream_t s, const int8_t *P, int nsplit, int n_oz, int n_pad,
                   const int *escale, const double *xu_part, int nxu, double *red2, const int *gate) {
    const int nt = n_oz / kOzT;
    const long nquad = (long)(nt * (nt + 1) / 2) * kOzT * kOzT / 4;
    const unsigned g = (unsigned)((nquad + 255) / 256 + (n_pad * 8 + 255) / 256);
    const OzConsts &C = oz_consts();
    switch (nsplit) {
        case 1:
            note_launch(KF_REDUCE, (const void *)k_oz_crt<1>);
            k_oz_crt<1><<<g, 256, 0, s>>>(P, 1, nt, n_pad, escale, xu_part, nxu, red2, C, gate);
            break;
        case 2:
            note_launch(KF_REDUCE, (const void *)k_oz_crt<2>);
            k_oz_crt<2><<<g, 256, 0, s>>>(P, 2, nt, n_pad, escale, xu_part, nxu, red2, C, gate);
            break;
        case 4:
            note_launch(KF_REDUCE, (const void *)k_oz_crt<4>);
            k_oz_crt<4><<<g, 256, 0, s>>>(P, 4, nt, n_pad, escale, xu_part, nxu, red2, C, gate);
            break;
        default:
            note_launch(KF_REDUCE, (const void *)k_oz_crt<0>);
            k_oz_crt<0><<<g, 256, 0, s>>>(P, nsplit, nt, n_pad, escale, xu_part, nxu, red2, C, gate);
    }
}

}  // namespace bb
