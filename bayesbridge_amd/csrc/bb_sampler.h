// bb_sampler.h -- device-side variate generation for the stable Gibbs sweep (gfx950).
//
// Philox4x64-10 counter RNG held in registers, Box-Muller normals, Marsaglia-Tsang
// gamma, and the two attempt bodies of Devroye's (2009) double-rejection sampler for
// the exponentially tilted positive stable law, restating Code/C/retstable.cpp:94-271.
//
// Counter layout (DESIGN.md "RNG counter layout"): key = (seed, stream),
// ctr = (t, kind << 56 | j, a, b).  A variate depends only on its counter, so any
// lane may evaluate any attempt: the group sampler below evaluates G consecutive
// inner attempts of one coefficient in G lanes and keeps the first accepted one,
// which reproduces the sequential rejection loop exactly.
//
// All arithmetic is IEEE fp64; the library is compiled with -ffp-contract=off so
// that expression trees round like the CPU checker's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

enum Kind : unsigned {
    KIND_LAMBDA_INNER = 1,
    KIND_LAMBDA_OUTER = 2,
    KIND_TAU = 3,
    KIND_SIG2 = 4,
    KIND_BETA_Z = 5,
    KIND_DELTA = 6,
    KIND_ALPHA = 7,
};

struct Key {
    uint64_t k0, k1;
};

constexpr double kPi = 3.14159265358979323846;
constexpr double kSqrtPi = 1.772453850905516027298167483341;  // retstable.cpp:14-16
constexpr double kSqrt2 = 1.41421356237309504880;
constexpr double kPi2 = 1.57079632679489661923;

struct U4 {
    double r[4];
};

// 64 x 64 -> 128-bit product from four 32 x 32 -> 64 products, each later one with a 64-bit
// addend (v_mad_u64_u32): a c = (a1 c1 + Hu + Hv) 2^64 + Lv 2^32 + L(a0 c0) with
// u = a1 c0 + H(a0 c0) = Hu 2^32 + Lu and v = a0 c1 + Lu = Hv 2^32 + Lv.  No carry is lost:
// u, v < 2^64 and the high word is the true one.  231 instead of 300 VALU instructions per
// Philox block (no v_mul_lo_u32), the same bits.
__device__ __forceinline__ void mulhilo64(uint64_t a, uint64_t c, uint64_t &hi, uint64_t &lo) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t c0 = (uint32_t)c, c1 = (uint32_t)(c >> 32);
    const uint64_t p00 = (uint64_t)a0 * c0;
    const uint64_t u = (uint64_t)a1 * c0 + (p00 >> 32);
    const uint64_t v = (uint64_t)a0 * c1 + (uint32_t)u;
    hi = (uint64_t)a1 * c1 + (u >> 32) + (v >> 32);
    lo = (v << 32) | (uint32_t)p00;
}

__device__ __forceinline__ void philox4x64(uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3,
                                           uint64_t k0, uint64_t k1, uint64_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B97F4A7C15ULL;
            k1 += 0xBB67AE8584CAA73BULL;
        }
        uint64_t hi0, lo0, hi1, lo1;
        mulhilo64(0xD2E7470EE14C6C93ULL, c0, hi0, lo0);
        mulhilo64(0xCA5A826395121157ULL, c2, hi1, lo1);
        uint64_t n0 = hi1 ^ c1 ^ k0;
        uint64_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

// Four open-interval (0,1) uniforms with 53-bit resolution from one Philox block.
__device__ __forceinline__ U4 uniforms(Key key, uint64_t t, unsigned kind, uint64_t j, uint64_t a,
                                       uint64_t b) {
    uint64_t o[4];
    philox4x64(t, ((uint64_t)kind << 56) | j, a, b, key.k0, key.k1, o);
    U4 u;
#pragma unroll
    for (int i = 0; i < 4; ++i) u.r[i] = ((double)(o[i] >> 11) + 0.5) * 0x1.0p-53;
    return u;
}

__device__ __forceinline__ double bm_normal(double r0, double r1) {
    return sqrt(-2.0 * log(r0)) * cos(2.0 * kPi * r1);
}

// Standard normal variate with index j of stream `kind` at sweep t.
__device__ __forceinline__ double normal_at(Key key, uint64_t t, unsigned kind, uint64_t j) {
    U4 u = uniforms(key, t, kind, j, 0, 0);
    return bm_normal(u.r[0], u.r[1]);
}

// Attempt caps of the rejection loops (a debug build lowers them so that a bad input ends
// in an error flag within microseconds instead of seconds)
#ifndef BB_MAX_GAMMA_ATTEMPTS
#define BB_MAX_GAMMA_ATTEMPTS (1ull << 24)
#endif
#ifndef BB_MAX_STABLE_ROUNDS
#define BB_MAX_STABLE_ROUNDS (1 << 22)
#endif

// Ga(shape, rate 1): Marsaglia & Tsang (2000), one Philox block per attempt,
// boost u^(1/a) for shape < 1.  Stream (t, kind, j=0, attempt, 0).
__device__ inline double gamma1(double shape, Key key, uint64_t t, unsigned kind,
                                uint32_t *err) {
    double a = shape, boost = 1.0;
    if (a < 1.0) {
        U4 u = uniforms(key, t, kind, 0, 0, 1);
        boost = pow(u.r[0], 1.0 / a);
        a += 1.0;
    }
    double d = a - 1.0 / 3.0;
    double cc = 1.0 / sqrt(9.0 * d);
    for (uint64_t k = 0; k < BB_MAX_GAMMA_ATTEMPTS; ++k) {
        U4 u = uniforms(key, t, kind, 0, k, 0);
        double x = bm_normal(u.r[0], u.r[1]);
        double v = 1.0 + cc * x;
        if (v <= 0.0) continue;
        v = v * v * v;
        double uu = u.r[2];
        double x2 = x * x;
        if (uu < 1.0 - 0.0331 * x2 * x2) return d * v * boost;
        if (log(uu) < 0.5 * x2 + d * (1.0 - v + log(v))) return d * v * boost;
    }
    if (err) atomicOr(err, 1u);
    return __builtin_nan("");
}

// ---------------------------------------------------------------------------
// Tilted positive stable law, Code/C/retstable.cpp.
// ---------------------------------------------------------------------------
// The sampler's logarithms and sines, restricted to the arguments it produces, in straight-line
// code whose constants the compiler keeps in scalar registers or instruction literals (the ocml
// log and sin carry range reduction and special-case paths the sampler never takes: ~98 and
// ~80 VALU instructions; these are ~35 and ~20).  BB_SAMPLER_OCML=1 builds the ocml versions
// (A/B measurement; the draws then differ from these in the last bits only).
#ifndef BB_SAMPLER_OCML
#define BB_SAMPLER_OCML 0
#endif

// log x, x > 0 (also 0 -> -inf, +inf -> +inf, x < 0 or NaN -> NaN).  fdlibm's e_log.c method:
// x = 2^e (1 + f), 1 + f in [sqrt(1/2), sqrt(2)), s = f / (2 + f),
// log(1 + f) = f - hfsq + s (hfsq + R(s^2)), hfsq = f^2 / 2, R its degree-14 minimax polynomial
// (coefficients Lg1..Lg7), e ln 2 in two parts; within 1 ulp (tests/test_sampler_math_cpu.py
// checks this restatement against a 120-bit reference).
__device__ __forceinline__ double bb_log(double x) {
#if BB_SAMPLER_OCML
    return log(x);
#else
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                     Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                     Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    double m = __builtin_amdgcn_frexp_mant(x) * 2.0;  // [1, 2)
    int e = __builtin_amdgcn_frexp_exp(x) - 1;
    if (m > kSqrt2) {
        m *= 0.5;
        e += 1;
    }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)e;
    double r = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    if (!(x > 0.0 && x < __builtin_huge_val()))
        r = x == 0.0 ? -__builtin_huge_val() : (x > 0.0 ? x : __builtin_nan(""));
    return r;
#endif
}

// sin x for x in [0, pi] (the sampler's sinc arguments alpha U, (1 - alpha) U and U, with U in
// [0, pi) whenever the attempt can be accepted; other arguments return a finite value the
// rejected attempt discards).  y = x on [0, pi/2], else pi - x in two parts (the difference
// with the high part is exact, Sterbenz), then the Taylor polynomial of sin to degree 23 in
// Horner form; within 2 ulp (tests/test_sampler_math_cpu.py).
__device__ __forceinline__ double bb_sin_0pi(double x) {
#if BB_SAMPLER_OCML
    return sin(x);
#else
    constexpr double pi_hi = 3.141592653589793116, pi_lo = 1.2246467991473532e-16;
    constexpr double c3 = -1.6666666666666666e-01, c5 = 8.3333333333333333e-03,
                     c7 = -1.9841269841269841e-04, c9 = 2.7557319223985893e-06,
                     c11 = -2.5052108385441720e-08, c13 = 1.6059043836821613e-10,
                     c15 = -7.6471637318198164e-13, c17 = 2.8114572543455206e-15,
                     c19 = -8.2206352466243297e-18, c21 = 1.9572941063391263e-20,
                     c23 = -3.8681701706306835e-23;
    const double y = x > kPi2 ? (pi_hi - x) + pi_lo : x;
    const double z = y * y;
    double p = c23;
    p = p * z + c21;
    p = p * z + c19;
    p = p * z + c17;
    p = p * z + c15;
    p = p * z + c13;
    p = p * z + c11;
    p = p * z + c9;
    p = p * z + c7;
    p = p * z + c5;
    p = p * z + c3;
    return y + (y * z) * p;
#endif
}

__device__ __forceinline__ double sinc_mm(double x) {  // retstable.cpp:18-29
    double ax = fabs(x);
    if (ax < 0.006) {
        if (x == 0.) return 1;
        double x2 = x * x;
        if (ax < 2e-4) return 1. - x2 / 6.;
        return 1. - x2 / 6. * (1 - x2 / 20.);
    }
    return bb_sin_0pi(x) / x;
}

// x^y for x >= 0 as exp(y log x).  Every pow of retstable.cpp:94-271 has a non-negative
// base (sinc of |x| < pi, lambda^alpha, 1 + alpha zeta / sqrt(gamma), A, b/a, X, m), and
// exp(y log x) reproduces pow's special cases there (0^y, inf^-y, NaN for X < 0) at
// ~|y log x| * 2^-53 relative error -- far below the GPU/oracle tolerance -- for roughly
// half the instructions and registers of the correctly rounded ocml pow.
__device__ __forceinline__ double powp(double x, double y) { return exp(y * bb_log(x)); }

__device__ __forceinline__ double zolotarev_A_p(double x, double alpha, double ia) {
    return powp(ia * sinc_mm(ia * x), ia) * powp(alpha * sinc_mm(alpha * x), alpha) / sinc_mm(x);
}

// B(x) / B(0) = sinc(x) / (sinc(alpha x)^alpha sinc(ia x)^ia), the two powers as one exp:
// sinc(x) exp(-(alpha log sinc(alpha x) + ia log sinc(ia x))) (the same value to rounding).
// At stable index alpha = 1/2 (the bridge exponent 1, the lasso: the chain draws lambda at
// index alpha_bridge / 2) ia = alpha, so both sincs are one value s and alpha log s + ia log s
// = log s exactly (halving and doubling are exact): one sine, one division and one log fewer
// per inner attempt, the same bits.
__device__ __forceinline__ double b_over_b0_p(double x, double alpha, double ia) {
    const double la = bb_log(sinc_mm(alpha * x));
    const double l = (alpha == ia) ? la : alpha * la + ia * bb_log(sinc_mm(ia * x));
    return sinc_mm(x) * exp(-l);
}

// Per-coefficient constants (retstable.cpp:121-147), with the loop-invariant ratios of
// the inner loop hoisted (same expressions, so the same bits).
struct StableParams {
    double h, alpha, ia, V0, b, lambda_alpha, gamma, sgamma, xi, psi, c1;
    double c_alpha;  // ia^ia alpha^alpha = A(x) * B(x) / B(0) (the outer test's A from B / B0)
    double thr_w1, thr_w3;  // w1/(w1+w2), w3/(w2+w3)
    double neg_inv_alpha, inv_ia, inv_alpha;
};

// a wave-uniform double held in scalar registers (readfirstlane of both halves)
__device__ __forceinline__ double uniform_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)b);
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// UA: alpha and V0 are the same on every lane of the wave (the lambda launches and the small
// chain; not retstable_LD's batch, whose arguments are per draw), so the alpha-only
// constants are kept in scalar registers -- 16 VGPRs fewer across the sampler loop.
template <bool UA = false>
__device__ __forceinline__ StableParams stable_params(double h, double alpha, double V0) {
    StableParams s;
    if constexpr (UA) {
        alpha = uniform_d(alpha);
        V0 = uniform_d(V0);
    }
    auto un = [](double v) { return UA ? uniform_d(v) : v; };
    s.h = h;
    s.alpha = alpha;
    s.ia = un(1. - alpha);
    s.V0 = V0;
    s.c1 = sqrt(kPi2);
    const double c2 = 2. + s.c1;
    s.b = un((1. - alpha) / alpha);
    s.lambda_alpha = powp(h, alpha) * V0;
    s.gamma = s.lambda_alpha * alpha * (1. - alpha);
    s.sgamma = sqrt(s.gamma);
    double c3 = c2 * s.sgamma;
    s.xi = (1. + kSqrt2 * c3) / kPi;
    s.psi = c3 * exp(-s.gamma * kPi * kPi / 8.) / kSqrtPi;
    const double w1 = s.c1 * s.xi / s.sgamma;
    const double w2 = 2. * kSqrtPi * s.psi;
    const double w3 = s.xi * kPi;
    s.thr_w1 = w1 / (w1 + w2);
    s.thr_w3 = w3 / (w2 + w3);
    s.neg_inv_alpha = un(-1 / alpha);
    s.inv_ia = un(1. / (1. - alpha));
    s.inv_alpha = un(1 / alpha);
    s.c_alpha = un(powp(s.ia, s.ia) * powp(alpha, alpha));
    return s;
}

// Inner attempt i of outer attempt o (retstable.cpp:162-207), block (t, INNER|j, o, i).
// Returns whether (U, z, Z) is accepted by the inner test.
__device__ __forceinline__ bool stable_inner_body(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, uint64_t i, double &U,
                                             double &z, double &Z, double &B) {
    const double alpha = s.alpha, gamma = s.gamma, sgamma = s.sgamma;
    U4 r = uniforms(key, t, KIND_LAMBDA_INNER, j, o, i);
    double V = r.r[0];
    if (gamma >= 1) {
        if (V < s.thr_w1) U = fabs(bm_normal(r.r[2], r.r[3])) / sgamma;
        else {
            double W_ = r.r[2];
            U = kPi * (1. - W_ * W_);
        }
    } else {
        double W_ = r.r[2];
        if (V < s.thr_w3) U = kPi * W_;
        else U = kPi * (1. - W_ * W_);
    }
    double W = r.r[1];
    B = b_over_b0_p(U, alpha, s.ia);
    double zeta = sqrt(B);
    z = 1 / (1 - powp(1 + alpha * zeta / sgamma, s.neg_inv_alpha));
    double rho = kPi * exp(-s.lambda_alpha * (1. - 1. / (zeta * zeta))) /
                 ((1. + s.c1) * sgamma / zeta + z);
    double d = 0.;
    if (U >= 0 && gamma >= 1) d += s.xi * exp(-gamma * U * U / 2.);
    if (U > 0 && U < kPi) d += s.psi / sqrt(kPi - U);
    if (U >= 0 && U <= kPi && gamma < 1) d += s.xi;
    rho *= d;
    Z = W * rho;
    return (U < kPi && Z <= 1.);
}

// Outer test of outer attempt o (retstable.cpp:212-256) given the accepted inner triple and
// its B = B(U) / B(0).  The reference evaluates Zolotarev's A(U) afresh (retstable.cpp:213:
// three more sines and two more powers); A(U) B(U) / B(0) = (1 - alpha)^(1 - alpha) alpha^alpha
// identically (both are products of the same sinc powers), so A = c_alpha / B: the same value
// to rounding, and about a fifth of a sampler round's VALU instructions fewer.
__device__ __forceinline__ bool stable_outer_body(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, double U, double z,
                                             double Z, double B, double &X) {
    const double alpha = s.alpha;
    (void)U;
    double a = powp(s.c_alpha / B, s.inv_ia);
    double m = powp(s.b / a, alpha) * s.lambda_alpha;
    double delta = sqrt(m * alpha / a);
    double a1 = delta * s.c1;
    double a2 = delta;
    double a3 = z / a;
    double ssum = a1 + a2 + a3;
    U4 r = uniforms(key, t, KIND_LAMBDA_OUTER, j, o, 0);
    double V_ = r.r[0], N_ = 0., E_ = 0.;
    double Xc;
    if (V_ < a1 / ssum) {
        N_ = bm_normal(r.r[1], r.r[2]);
        Xc = m - delta * fabs(N_);
    } else {
        if (V_ < (a1 + a2) / ssum) Xc = m + delta * r.r[1];
        else {
            E_ = -bb_log(r.r[1]);
            Xc = m + delta + E_ * a3;
        }
    }
    double E = -bb_log(Z);
    double c = a * (Xc - m);
    c += (m != 0) ? s.h * (powp(Xc, -1. * s.b) - powp(m, -1. * s.b)) : 0.0;
    if (Xc < m) c -= N_ * N_ / 2.;
    else if (Xc > m + delta) c -= E_;
    X = Xc;
    return (Xc >= 0 && c <= E);
}

__device__ __noinline__ bool stable_inner_ni(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, uint64_t i, double &U,
                                             double &z, double &Z, double &B) {
    return stable_inner_body(s, key, t, j, o, i, U, z, Z, B);
}
__device__ __noinline__ bool stable_outer_ni(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, double U, double z,
                                             double Z, double B, double &X) {
    return stable_outer_body(s, key, t, j, o, U, z, Z, B, X);
}
template <bool NI>
__device__ __forceinline__ bool stable_inner(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, uint64_t i, double &U,
                                             double &z, double &Z, double &B) {
    if constexpr (NI) return stable_inner_ni(s, key, t, j, o, i, U, z, Z, B);
    else return stable_inner_body(s, key, t, j, o, i, U, z, Z, B);
}
template <bool NI>
__device__ __forceinline__ bool stable_outer(const StableParams &s, Key key, uint64_t t,
                                             uint64_t j, uint64_t o, double U, double z,
                                             double Z, double B, double &X) {
    if constexpr (NI) return stable_outer_ni(s, key, t, j, o, U, z, Z, B, X);
    else return stable_outer_body(s, key, t, j, o, U, z, Z, B, X);
}

#ifndef BB_STABLE_NOINLINE
#define BB_STABLE_NOINLINE 0
#endif

__device__ __forceinline__ double stable_finish(const StableParams &s, double X) {
    return exp(s.inv_alpha * bb_log(s.V0) - s.b * bb_log(X));  // :270
}

// Group sampler: the G lanes [gbase, gbase+G) of a wave cooperate on one coefficient by
// evaluating G consecutive INNER attempts of the current outer attempt in parallel; the
// lowest accepted inner attempt (counter order) feeds the outer test, which every lane of
// the group evaluates on identical inputs.  This reproduces the sequential double
// rejection loop exactly.  Every lane of the wave must call this (ballot/shuffle inside).
template <int G, bool NI = (BB_STABLE_NOINLINE != 0), bool UA = false>
__device__ inline double stable_group_draw(bool active, double h, double alpha, double V0,
                                           Key key, uint64_t t, uint64_t j, uint32_t *err) {
    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const uint64_t gmask = (G == 64) ? ~0ull : ((1ull << (G & 63)) - 1ull);
    if (active && alpha == 1.) active = false;  // :104-110 returns V0, no RNG used
    double result = V0;
    bool done = !active;
    StableParams s;
    if (active) {
        if (h < 0 || alpha < 0 || alpha > 1 || V0 < 0) atomicOr(err, 4u);  // :112-115
        s = stable_params<UA>(h, alpha, V0);
    }
    uint64_t o = 0, ib = 0;
    for (int iter = 0; iter < BB_MAX_STABLE_ROUNDS; ++iter) {
        bool acc = false;
        double U = 0.0, z = 0.0, Z = 0.0, B = 1.0;
        if (!done) acc = stable_inner<NI>(s, key, t, j, o, ib + (uint64_t)g, U, z, Z, B);
        const uint64_t m = (__ballot(acc) >> gbase) & gmask;
        const int win = m ? (__ffsll((unsigned long long)m) - 1) : 0;
        const double Uw = __shfl(U, gbase + win, 64);
        const double zw = __shfl(z, gbase + win, 64);
        const double Zw = __shfl(Z, gbase + win, 64);
        const double Bw = __shfl(B, gbase + win, 64);
        if (!done) {
            if (!m) {
                ib += G;
            } else {
                double X;
                if (stable_outer<NI>(s, key, t, j, o, Uw, zw, Zw, Bw, X)) {
                    result = stable_finish(s, X);
                    done = true;
                } else {
                    ++o;
                    ib = 0;
                }
            }
        }
        if (__all(done)) break;
    }
    if (!done) {
        atomicOr(err, 2u);
        result = __builtin_nan("");
    }
    return result;
}

// Latency-oriented variant for chains with few coefficients (bb_small.hip): the L lanes of a
// group are O = L / I segments of I lanes, and segment k evaluates I inner attempts of outer
// attempt o0 + k and then that attempt's outer test, so one round covers O outer attempts.
// Scanning the segments in counter order, the first one that either accepted no inner
// attempt (continue its inner loop next round) or passed its outer test (done) decides;
// outer attempts before it were rejected exactly as the sequential loop rejects them, so the
// draw is the same as stable_group_draw's.  About 1 in 8 draws needs a second round at
// I = 8, O = 4 (inner acceptance ~0.3, outer ~0.7 at alpha = 0.25).
template <int L, int I, bool UA = true>
__device__ __forceinline__ double stable_spec_draw(bool active, double h, double alpha, double V0, Key key,
                                          uint64_t t, uint64_t j, uint32_t *err) {
    static_assert(L <= 64 && (L & (L - 1)) == 0 && L % I == 0 && I < 64, "group shape");
    constexpr int O = L / I;
    const int lane = threadIdx.x & 63;
    const int g = lane & (L - 1), gbase = lane & ~(L - 1);
    const int seg = g / I, ii = g % I;
    const uint64_t imask = (1ull << I) - 1ull;
    if (active && alpha == 1.) active = false;  // retstable.cpp:104-110
    double result = V0;
    bool done = !active;
    StableParams s;
    if (active) {
        if (h < 0 || alpha < 0 || alpha > 1 || V0 < 0) atomicOr(err, 4u);  // :112-115
        s = stable_params<UA>(h, alpha, V0);
    }
    uint64_t o0 = 0, ib = 0;  // window's first outer attempt, its next inner attempt
    for (int iter = 0; iter < BB_MAX_STABLE_ROUNDS; ++iter) {
        const uint64_t o = o0 + (uint64_t)seg;
        double U = 0.0, z = 0.0, Z = 0.0, B = 1.0;
        bool acc = false;
        if (!done)
            acc = stable_inner<false>(s, key, t, j, o, (seg == 0 ? ib : 0) + (uint64_t)ii, U, z, Z,
                                      B);
        const uint64_t sb = ((__ballot(acc) >> gbase) >> (seg * I)) & imask;
        const int src = gbase + seg * I + (sb ? (__ffsll((unsigned long long)sb) - 1) : 0);
        const double Uw = __shfl(U, src, 64), zw = __shfl(z, src, 64), Zw = __shfl(Z, src, 64);
        const double Bw = __shfl(B, src, 64);
        double X = 0.0;
        bool oacc = false;
        if (!done && sb) oacc = stable_outer<false>(s, key, t, j, o, Uw, zw, Zw, Bw, X);
        const uint64_t hb = __ballot(ii == 0 && sb != 0) >> gbase;
        const uint64_t ab = __ballot(ii == 0 && oacc) >> gbase;
        unsigned H = 0, A = 0;
#pragma unroll
        for (int k = 0; k < O; ++k) {
            H |= (unsigned)((hb >> (k * I)) & 1ull) << k;
            A |= (unsigned)((ab >> (k * I)) & 1ull) << k;
        }
        const unsigned stop = (~H & ((1u << O) - 1u)) | A;
        const int k = stop ? (__ffs(stop) - 1) : O;
        const double Xk = __shfl(X, gbase + (k < O ? k : 0) * I, 64);
        if (!done) {
            if (k == O) {  // all O outer attempts rejected
                o0 += O;
                ib = 0;
            } else if ((A >> k) & 1u) {
                result = stable_finish(s, Xk);
                done = true;
            } else {  // outer attempt o0 + k needs more inner attempts
                ib = (k == 0) ? ib + I : (uint64_t)I;
                o0 += (uint64_t)k;
            }
        }
        if (__all(done)) break;
    }
    if (!done) {
        atomicOr(err, 2u);
        result = __builtin_nan("");
    }
    return result;
}

// Wave-adaptive form of stable_spec_draw<8, 8> (the fused lambda + X u launch): a wave holds 8
// coefficients on 8 "home" lanes each, and while more than 4 are unfinished each evaluates one
// outer attempt of 8 inner attempts per round on its home lanes, as stable_spec_draw<8, 8>.
// With a draw finishing in a round with probability ~0.66, a wave of 8 fixed groups runs the
// maximum of 8 geometric round counts (~3 rounds against a mean of ~1.5) with the finished
// groups' lanes idle.  Here, once m <= 4 coefficients are left, the wave's lanes are dealt to
// them: G = 16, 32 or 64 lanes each (m = 3-4, 2, 1), i.e. O = G / 8 outer attempts of 8 inner
// attempts per round, exactly the windows stable_spec_draw<G, 8> evaluates -- the same attempts
// on the same counters, accepted by the same tests in the same order, so the same draws.  A
// coefficient's per-draw constants and loop state move with it (shuffled from the group that
// served it the round before); its result is shuffled back to its home lanes.  Returns the
// draw of the home coefficient (every lane of its home group).  UA: alpha and V0 wave-uniform.
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const unsigned lo = (unsigned)__shfl((int)(unsigned)v, src, 64);
    const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
// lane of the group serving coefficient c in a round with unfinished set um and G lanes per
// coefficient (G == 8: its home lanes)
__device__ __forceinline__ int wave_group_base(int c, unsigned um, int G) {
    return G == 8 ? 8 * c : __popc(um & ((1u << c) - 1u)) * G;
}
__device__ __forceinline__ int nth_set_bit(unsigned x, int k) {
    for (int r = 0; r < k && x; ++r) x &= x - 1u;
    return x ? __ffs(x) - 1 : -1;
}
// The rounds of the wave-adaptive draw from a given state: um = the wave's unfinished home
// groups (bit c: lanes 8c..8c+7), and on every lane s / o0 / ib / jc = its home coefficient's
// constants, loop state and counter index (the wave-uniform fields of s valid on every lane).
// On return result holds, on the home lanes of every coefficient finished here, its draw; the
// return value is the set still unfinished (nonempty only at the round cap).  s, o0, ib and jc
// are overwritten (lanes serve other coefficients along the way).
__device__ __forceinline__ unsigned wave_draw_rounds(StableParams &s, uint64_t &o0, uint64_t &ib,
                                                     uint64_t &jc, unsigned um, double &result,
                                                     Key key, uint64_t t) {
    constexpr int I = 8;
    const int lane = threadIdx.x & 63;
    const int home = lane >> 3, ii = lane & 7;
    unsigned um_prev = um;
    int G_prev = 8;
    int c_cur = home;  // the coefficient this lane serves
    int iter = 0;
    for (; um && iter < BB_MAX_STABLE_ROUNDS; ++iter) {
        const int m = __popc(um);
        const int G = m > 4 ? 8 : m > 2 ? 16 : m > 1 ? 32 : 64;
        if (G > 8) {
            // deal the lanes: group `slot` serves the slot-th unfinished coefficient, whose
            // constants and state come from the lanes that served it the round before
            const int slot = lane / G;
            const int cn = nth_set_bit(um, slot);
            const int src = cn >= 0 ? wave_group_base(cn, um_prev, G_prev) : lane;
            s.h = __shfl(s.h, src, 64);
            s.lambda_alpha = __shfl(s.lambda_alpha, src, 64);
            s.gamma = __shfl(s.gamma, src, 64);
            s.sgamma = __shfl(s.sgamma, src, 64);
            s.xi = __shfl(s.xi, src, 64);
            s.psi = __shfl(s.psi, src, 64);
            s.thr_w1 = __shfl(s.thr_w1, src, 64);
            s.thr_w3 = __shfl(s.thr_w3, src, 64);
            o0 = shfl_u64(o0, src);
            ib = shfl_u64(ib, src);
            jc = shfl_u64(jc, src);
            c_cur = cn;
        }
        const bool serve = c_cur >= 0 && ((um >> c_cur) & 1u);
        const int base = G == 8 ? (lane & ~7) : (lane / G) * G;
        const int O = G / I, seg = (lane - base) >> 3;
        const uint64_t o = o0 + (uint64_t)seg;
        double U = 0.0, z = 0.0, Z = 0.0, B = 1.0;
        bool acc = false;
        if (serve)
            acc = stable_inner<false>(s, key, t, jc, o, (seg == 0 ? ib : 0) + (uint64_t)ii, U, z, Z,
                                      B);
        const unsigned sb = (unsigned)((__ballot(acc) >> (base + 8 * seg)) & 0xffull);
        const int wsrc = base + 8 * seg + (sb ? (__ffs(sb) - 1) : 0);
        const double Uw = __shfl(U, wsrc, 64), zw = __shfl(z, wsrc, 64), Zw = __shfl(Z, wsrc, 64);
        const double Bw = __shfl(B, wsrc, 64);
        double X = 0.0;
        bool oacc = false;
        if (serve && sb) oacc = stable_outer<false>(s, key, t, jc, o, Uw, zw, Zw, Bw, X);
        const unsigned long long hb = __ballot(ii == 0 && sb != 0) >> base;
        const unsigned long long ab = __ballot(ii == 0 && oacc) >> base;
        unsigned H = 0, A = 0;
        for (int k = 0; k < O; ++k) {
            H |= (unsigned)((hb >> (8 * k)) & 1ull) << k;
            A |= (unsigned)((ab >> (8 * k)) & 1ull) << k;
        }
        const unsigned stop = (~H & ((1u << O) - 1u)) | A;
        const int k = stop ? (__ffs(stop) - 1) : O;
        const double Xk = __shfl(X, base + 8 * (k < O ? k : 0), 64);
        bool fin = false;
        double res = 0.0;
        if (serve) {
            if (k == O) {  // all O outer attempts rejected
                o0 += (uint64_t)O;
                ib = 0;
            } else if ((A >> k) & 1u) {
                res = stable_finish(s, Xk);
                fin = true;
            } else {  // outer attempt o0 + k needs more inner attempts
                ib = (k == 0) ? ib + I : (uint64_t)I;
                o0 += (uint64_t)k;
            }
        }
        // the coefficients finished this round (wave-uniform), their results to the home lanes
        const unsigned long long fb = __ballot(fin && lane == base);
        unsigned fm = 0;
        for (unsigned long long x = fb; x; x &= x - 1ull) {
            const int b = __ffsll((unsigned long long)x) - 1;
            fm |= 1u << (G == 8 ? b / 8 : nth_set_bit(um, b / G));
        }
        const double hr = __shfl(res, wave_group_base(home, um, G), 64);
        if ((fm >> home) & 1u) result = hr;
        um_prev = um;
        G_prev = G;
        um &= ~fm;
    }
    return um;
}

__device__ __forceinline__ double stable_wave_draw(bool active, double h, double alpha, double V0,
                                                   Key key, uint64_t t, uint64_t j,
                                                   uint32_t *err) {
    const int lane = threadIdx.x & 63;
    const int home = lane >> 3, ii = lane & 7;
    if (active && alpha == 1.) active = false;  // retstable.cpp:104-110
    if (active && (h < 0 || alpha < 0 || alpha > 1 || V0 < 0)) atomicOr(err, 4u);  // :112-115
    // every lane forms constants (an inactive one from h = 1): the wave-uniform fields must be
    // valid on every lane that may serve another coefficient
    StableParams s = stable_params<true>(active ? h : 1.0, alpha, V0);
    double result = V0;
    uint64_t o0 = 0, ib = 0, jc = j;  // the served coefficient's loop state and index
    unsigned um = 0;                  // unfinished coefficients (wave-uniform)
    {
        const unsigned long long a = __ballot(active && ii == 0);
#pragma unroll
        for (int c = 0; c < 8; ++c) um |= (unsigned)((a >> (8 * c)) & 1ull) << c;
    }
    um = wave_draw_rounds(s, o0, ib, jc, um, result, key, t);
    if (um) {
        atomicOr(err, 2u);
        if ((um >> home) & 1u) result = __builtin_nan("");
    }
    return result;
}

}  // namespace bb
