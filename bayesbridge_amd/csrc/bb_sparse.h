// bb_sparse.h -- host-side launch wrappers for the sparse-design (CSC/CSR) Woodbury sweep
// (BASELINE config C5: n = 5000, p = 200000, 1 % density, alpha = 0.3).
//
// The conditional drawn is the reference's beta | rest (Code/C/BridgeRegression.cpp:552-575)
// in its Woodbury form; with a sparse X the n x n Gram X diag(D) X' is an
// HBM-bound sparse product instead of a dense GEMM.
//
// Device layout (all indices int32, values fp64, the engine's p_local columns only):
//   CSC   colptr[p_loc + 1], rowidx[nnz], cval[nnz]   (rows sorted within a column)
//   CSR   rowptr[n_pad + 1], colidx[nnz], rval[nnz], cpos[nnz] = CSC position of entry k
//   pairs for every off-diagonal Gram entry (r, c), r < c, in packed upper-triangle order
//         e = tri_index(r, c): estart[e] .. estart[e + 1] index prod[] = X_rj X_cj over the
//         columns j where both are non-zero, j increasing, with either pidx[] = the
//         position of j in row c's CSR list (16 bit; rows of <= kSpColMaxRow non-zeros,
//         the by-column kernel) or pj[] = j (32 bit; the general kernel).  Diagonal
//         entries have empty segments (their sum comes from the row pass).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "bb_kernels.h"

namespace bb {

// Rows of X with more non-zeros than this (64 KB of LDS for D over the row) use the
// general pair-list kernel with 32-bit column indices.
constexpr int kSpColMaxRow = 8192;
int sp_col_max_row();

// cnt[c] = number of (r, j) pairs with r < c and X_rj X_cj != 0  (c < n_pad).
void launch_sp_count(hipStream_t s, const int *rowptr, const int *colidx, const int *cpos,
                     const int *colptr, int n_pad, unsigned long long *cnt);

// Fill estart / prod / pj given base[c] = sum_{c' < c} cnt[c'] (host exclusive scan).
// estart has tri_count(n_pad) + 1 words; the last one is written by the host.
void launch_sp_build(hipStream_t s, const int *rowptr, const int *colidx, const int *cpos,
                     const double *rval, const int *colptr, const int *rowidx,
                     const double *cval, int n_pad, const unsigned long long *base,
                     unsigned *estart, double *prod, int *pj, unsigned short *pidx);

// By-column Gram (rows of <= kSpColMaxRow non-zeros): the packed triangle of X diag(D) X'
// including its diagonal, and xu = X u (xu may be nullptr).  max_row = largest row nnz.
void launch_sp_gram_col(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                        const unsigned *estart, const double *prod, const unsigned short *pidx,
                        const double *D, const double *u, int n_pad, int max_row, double *tri,
                        double *xu, const int *gate = nullptr);

// out[e] = sum_k prod[k] D[pj[k]] over every packed entry e < tri_count(n_pad)
// (diagonal entries come out 0; k_sp_rows fills them).
void launch_sp_gram(hipStream_t s, const unsigned *estart, const double *prod, const int *pj,
                    const double *D, int n_pad, double *out, const int *gate = nullptr);

// Row pass over the CSR: xv[c] = sum_j X_cj v_j; with D != nullptr also
// tri[tri_index(c, c)] = sum_j X_cj^2 D_j (the Gram diagonal).
void launch_sp_rows(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                    int n_pad, const double *v, const double *D, double *xv, double *tri, const int *gate = nullptr);

// Woodbury beta update from the CSC: beta_j = u_j + D_j (X_j . w) / sig.
void launch_sp_beta(hipStream_t s, const int *colptr, const int *rowidx, const double *cval,
                    int p_loc, const double *w, const double *u, const double *D,
                    const DevScalars *sc, double *beta, double *beta_trace);

extern int g_sp_nt;  // sparse Gram variant (bb_set_tuning key 3, bb_sparse.hip)

}  // namespace bb
