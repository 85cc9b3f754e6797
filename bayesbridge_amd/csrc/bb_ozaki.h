// Ozaki-II (CRT) fp64-accurate Gram on int8 MFMA.
//
// G = X diag(D) X' = Y Y' with Y = X diag(sqrt(D)).  Each row i of Y is scaled by a power of
// two and rounded to an integer Yh_i with |Yh_ij| <= 2^b (b <= 53, so the rounding is the
// fp64 rounding of the scaled value, relative to the row's bound).  The exact integer Gram
// C = Yh Yh' (|C| <= K 2^2b < M/2) is recovered from its residues modulo kOzMods pairwise
// coprime moduli m_k <= 247:  C mod m_k = (Yh mod m_k)(Yh mod m_k)' mod m_k, each an int8
// GEMM with exact int32 accumulation on v_mfma_i32_16x16x64_i8 (k_oz_gemm16u).  Garner's mixed-radix
// reconstruction (balanced digits) gives C exactly as a 128-bit integer, which is rounded
// once to fp64 and scaled back: G_ik = C_ik 2^(e_i + e_k).
//
// Work: kOzMods symmetric int8 GEMMs (lower 256x256 tiles only) = kOzMods/2 full GEMM
// equivalents at 64x the per-clock rate of the fp64 MFMA Gram, plus one streaming pass over X
// (read 8 B, write kOzMods B per element).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

constexpr int kOzMods = 16;
constexpr int kOzT = 256;  // GEMM tile (rows of Y)
constexpr int kOzKC = 64;  // K bytes per residue chunk

struct OzConsts {
    int m[kOzMods];
    double inv_m[kOzMods];
    float inv_mf[kOzMods];
    int invP[kOzMods];             // (prod_{i<k} m_i)^-1 mod m_k  (k >= 1)
    int Pmod[kOzMods][kOzMods];    // Pmod[j][k] = (prod_{i<j} m_i) mod m_k  (j < k)
    double log2M;
};

// Host: moduli and Garner constants (computed once).
const OzConsts &oz_consts();
// Largest b with K 2^(2b+1) < M (capped at 53): the integer bits per scaled element.
int oz_bits_for(int K);
int oz_rows(int n_pad);                    // n_pad rounded up to kOzT
int oz_splits_for(int n_oz, int nkc);      // K splits of the int8 GEMM
size_t oz_residue_bytes(int n_oz, int p_pad);
size_t oz_partial_bytes(int n_oz, int nsplit);

// Setup: xmax[c * n_oz + i] = max_{j in chunk c} |X_ij| (c = 64-column chunk; rows >= n_pad 0).
void launch_oz_xmax(hipStream_t s, const double *X, int ldx, int n_pad, int n_oz, int p_pad,
                    double *xmax);
// Per sweep: row exponents from the bound max_c xmax[c][i] * max_{j in c} sqrt(D_j):
// rscale[i] = 2^(b - e_i), escale[i] = e_i - b.  part: scratch of
// oz_bound_groups(p_pad) * n_oz doubles (per chunk-group row maxima).
int oz_bound_groups(int p_pad);
void launch_oz_scale(hipStream_t s, const double *D, int p_pad, const double *xmax, int n_oz,
                     int b, double *part, double *rscale, int *escale, const int *gate = nullptr);
// Residues r = round(X_ij sqrt(D_j) rscale_i) mod m_k (int8), plane k, 64-column chunk c,
// stored as [16-row block][16-byte unit 0..3][row in block][16 B].  When u is
// given, the same pass writes the X.u partials xu_part[g * n_pad + i] (g = 256-column group,
// oz_xu_parts(p_pad) of them; rows < n_pad).
int oz_xu_parts(int p_pad, int n_oz);  // X.u partials of launch_oz_residues (<= p_pad / 64)
void launch_oz_residues(hipStream_t s, const double *X, int ldx, int n_pad, int n_oz, int p_pad,
                        const double *D, const double *rscale, int8_t *R,
                        const double *u = nullptr, double *xu_part = nullptr, const int *gate = nullptr);
// P[split][k][tile] = (R_k R_k')_tile mod m_k over the split's K chunks (int8, balanced).
extern int g_oz_res_nt;  // residue-plane stores non-temporal (bb_set_tuning key 1)
// lead_pm: the diagonal pairs' K lead in 1/1000 of the pass (kOzLeadDefault: the tuned
// value; < 0: no K rotation at all, every pass from chunk 0); late_pm: the start shift per
// earlier pair round in 1/1000 of the pass (< 0: the tuned value).  Results do not depend on
// either.
constexpr int kOzLeadDefault = -1000000;
void launch_oz_gemm(hipStream_t s, const int8_t *R, int n_oz, int p_pad, int nsplit, int8_t *P,
                    int dbg = 0, int lead_pm = kOzLeadDefault, int late_pm = -1, const int *gate = nullptr);
// red2[tri_index(r, c)] (r <= c < n_pad) = G(r, c); red2[tri_count(n_pad) + r] = sum_q
// xu_part[q][r].
void launch_oz_crt(hipStream_t s, const int8_t *P, int nsplit, int n_oz, int n_pad,
                   const int *escale, const double *xu_part, int nxu, double *red2, const int *gate = nullptr);

}  // namespace bb
