// bb_logit.hip -- gfx950 kernels of the logistic bridge sweep (BASELINE config C4).
//
// The logistic model y_i ~ Bernoulli(1 / (1 + exp(-x_i'beta))) with the bridge prior is
// sampled by Polya-Gamma data augmentation (Polson, Scott & Windle 2013): given
// omega_i ~ PG(1, x_i'beta) the likelihood is Gaussian in beta, so
//   beta | omega, lambda, tau ~ N(A^-1 X'kappa, A^-1),  A = X'Omega X + diag(lambda / tau^2),
// kappa = y - 1/2 -- the reference's sample_beta_stable (Code/C/BridgeRegression.cpp:552-575)
// with sig2 = 1 and X'X replaced by X'Omega X; tau and lambda are the reference's
// conditionals unchanged (:453-465, :506-510).  There is no reference logistic model
// (BASELINE.md); the PG sampler restates the published algorithm (oracle/bb_oracle.c,
// bbo_pg1, same expressions in the same order).
#include <hip/hip_runtime.h>

#include "bb_kernels.h"
#include "bb_pg.h"
#include "bb_sampler.h"

namespace bb {

// omega_i ~ PG(1, psi_i) for i < n, 0 on the padding rows; psi = X beta (k_pre's sums).
__global__ __launch_bounds__(256) void k_pg(const double *__restrict__ psi, int n, int n_pad,
                                            Key key, uint64_t t, double *__restrict__ omega,
                                            uint32_t *err) {
    pg_draw_at(blockIdx.x * 256 + threadIdx.x, psi, n, n_pad, key, t, omega, err);
}

void launch_pg(hipStream_t s, const double *psi, int n, int n_pad, uint64_t k0, uint64_t k1,
               uint64_t t, double *omega, uint32_t *err) {
    k_pg<<<(n_pad + 255) / 256, 256, 0, s>>>(psi, n, n_pad, Key{k0, k1}, t, omega, err);
}

// kappa_i = y_i - 1/2 (0 on padding rows)
__global__ void k_kappa(const double *y, int n, int n_pad, double *kappa) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_pad) kappa[i] = i < n ? y[i] - 0.5 : 0.0;
}

void launch_kappa(hipStream_t s, const double *y, int n, int n_pad, double *kappa) {
    k_kappa<<<(n_pad + 255) / 256, 256, 0, s>>>(y, n, n_pad, kappa);
}

}  // namespace bb
