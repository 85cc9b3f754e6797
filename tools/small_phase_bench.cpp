// Phase timing of the fused small-p sweep kernel (bb_small.hip built with BB_SMALL_PHASES):
// one launch of `count` sweeps on a synthetic n x p Gaussian design; prints the kernel time
// per sweep and the split between S_alpha/rss, tau/sig2, lambda and beta.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DBB_SMALL_PHASES \
//         -I bayesbridge_amd/csrc tools/small_phase_bench.cpp bayesbridge_amd/csrc/bb_small.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "bb_kernels.h"

namespace bb {
void small_phase_ticks(unsigned long long out[4]);
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <class T>
T *up(const std::vector<T> &h) {
    T *d;
    CK(hipMalloc(&d, h.size() * sizeof(T) + 64));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 442, p = argc > 2 ? atoi(argv[2]) : 10;
    const int ortho = argc > 3 ? atoi(argv[3]) : 0, count = argc > 4 ? atoi(argv[4]) : 2000;
    if (p > bb::kSmallChainMaxP) return 2;  // the fused kernel's range
    std::mt19937_64 g(5);
    std::normal_distribution<double> N;
    std::vector<double> X((size_t)n * p), y(n), G((size_t)p * p), c(p), gd(p), b(p);
    for (auto &v : X) v = N(g);
    for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int j = 0; j < p; ++j) s += X[i + (size_t)j * n] * (j < 4 ? 1.0 + j : 0.0);
        y[i] = s + N(g);
    }
    for (int a = 0; a < p; ++a) {
        for (int bb_ = 0; bb_ < p; ++bb_) {
            double s = 0;
            for (int i = 0; i < n; ++i) s += X[i + (size_t)a * n] * X[i + (size_t)bb_ * n];
            G[a + (size_t)bb_ * p] = s;
        }
        double s = 0;
        for (int i = 0; i < n; ++i) s += X[i + (size_t)a * n] * y[i];
        c[a] = s;
        gd[a] = G[a + (size_t)a * p];
        b[a] = 0.1 * N(g);
    }
    std::vector<double> lam(p, 1.0);
    bb::DevScalars sc{};
    sc.tau = 1.0;
    sc.sig2 = 1.0;
    sc.alpha = 0.5;
    const int know = argc > 5 ? atoi(argv[5]) : 0;  // bit 0: tau known, bit 1: sig2 known
    bb::Hyper hy{0.0, 0.0, 2.0, 2.0, 1.0, 1.0, know & 1, (know >> 1) & 1, 1};
    double *dX = up(X), *dy = up(y), *dG = up(G), *dc = up(c), *dgd = up(gd), *db = up(b),
           *dl = up(lam);
    bb::DevScalars *dsc;
    CK(hipMalloc(&dsc, sizeof(sc)));
    CK(hipMemcpy(dsc, &sc, sizeof(sc), hipMemcpyHostToDevice));
    uint32_t *err;
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    std::vector<double> tz((size_t)count * p + 1);
    double *tb = up(tz), *tl = up(tz), *ts = up(tz), *tt = up(tz), *ta = up(tz);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        unsigned long long ph[4];
        bb::small_phase_ticks(ph);  // zero
        CK(hipEventRecord(e0));
        bb::launch_small_chain(nullptr, dX, n, n, p, dy, dG, p, dc, dgd, ortho, db, dl, dsc, hy,
                               11, 22, 1 + (uint64_t)rep * count, count, 0, 1, count, tb, tl, ts,
                               tt, ta, err);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        bb::small_phase_ticks(ph);
        uint32_t f = 0;
        CK(hipMemcpy(&f, err, 4, hipMemcpyDeviceToHost));
        // realtime clock: 100 MHz -> 10 ns per tick
        printf("n=%d p=%d ortho=%d: %.2f us/sweep (rss %.2f, tau/sig2 %.2f, lambda %.2f, beta "
               "%.2f us) flags %u\n",
               n, p, ortho, 1e3 * ms / count, 1e-2 * ph[0] / count, 1e-2 * ph[1] / count,
               1e-2 * ph[2] / count, 1e-2 * ph[3] / count, f);
    }
    return 0;
}
