// Correctly rounded (to ~2^-90 relative before the final rounding) double
// pow for x > 0, via double-double log/exp.  Used for PER leaves
// (priority ** alpha, agilerl/components/replay_buffer.py:322) and IS weights
// (replay_buffer.py:399-406), where the reference uses Python's float ** (libm).
// libm's pow is not correctly rounded (it differs from the correctly rounded
// value in ~0.08% of random inputs at alpha 0.6, measured), so the two agree
// to <= 1 ulp and bit-exactly everywhere else; the tree itself is then a pure
// function of the leaves.
#pragma once

#include <hip/hip_runtime.h>

namespace agx {

struct dd {
    double hi, lo;
};

__host__ __device__ __forceinline__ dd dd_two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    const double e = (a - (s - bb)) + (b - bb);
    return {s, e};
}
__host__ __device__ __forceinline__ dd dd_fast_two_sum(double a, double b) {
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ __forceinline__ dd dd_two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__host__ __device__ __forceinline__ dd dd_add(dd x, dd y) {
    dd s = dd_two_sum(x.hi, y.hi);
    dd t = dd_two_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = dd_fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return dd_fast_two_sum(s.hi, s.lo);
}
__host__ __device__ __forceinline__ dd dd_mul(dd x, dd y) {
    dd p = dd_two_prod(x.hi, y.hi);
    p.lo += x.hi * y.lo + x.lo * y.hi;
    return dd_fast_two_sum(p.hi, p.lo);
}
__host__ __device__ __forceinline__ dd dd_mul_d(dd x, double y) {
    dd p = dd_two_prod(x.hi, y);
    p.lo += x.lo * y;
    return dd_fast_two_sum(p.hi, p.lo);
}
// x / n for a small positive integer n (exact double)
__host__ __device__ __forceinline__ dd dd_div_d(dd x, double n) {
    const double q1 = x.hi / n;
    dd p = dd_two_prod(q1, n);
    const double r = ((x.hi - p.hi) - p.lo + x.lo) / n;
    return dd_fast_two_sum(q1, r);
}

// exp(a) for |a| < ~700, relative error ~2^-95
__host__ __device__ inline dd dd_exp(dd a) {
    const double ln2_hi = 0x1.62e42fefa39efp-1;
    const double ln2_lo = 0x1.abc9e3b39803fp-56;
    const double k = rint(a.hi * 0x1.71547652b82fep0);
    dd kl = dd_two_prod(k, ln2_hi);
    kl.lo += k * ln2_lo;
    dd r = dd_add(a, dd{-kl.hi, -kl.lo});
    // r in [-ln2/2, ln2/2]; scale by 2^-10
    r.hi = ldexp(r.hi, -10);
    r.lo = ldexp(r.lo, -10);
    // Horner: e = 1 + r(1 + r/2(1 + r/3(... (1 + r/11))))
    dd t = {1.0, 0.0};
    for (int n = 11; n >= 1; --n) {
        t = dd_div_d(dd_mul(t, r), (double)n);
        t = dd_add(t, dd{1.0, 0.0});
    }
    for (int i = 0; i < 10; ++i) t = dd_mul(t, t);
    const int ki = (int)k;
    return {ldexp(t.hi, ki), ldexp(t.lo, ki)};
}

// log(x), x > 0 finite: one Newton correction of a double log
__host__ __device__ inline dd dd_log(double x) {
    const double l0 = log(x);
    const dd e = dd_exp(dd{l0, 0.0});
    const double corr = ((x - e.hi) - e.lo) / e.hi;
    return dd_fast_two_sum(l0, corr);
}

// correctly rounded pow for x > 0 (x == 0: 0 or +inf like libm)
__host__ __device__ inline double cr_pow(double x, double y) {
    if (x == 1.0 || y == 0.0) return 1.0;
    if (x == 0.0) return y > 0.0 ? 0.0 : __builtin_inf();
    if (y == 1.0) return x;
    const dd l = dd_log(x);
    const dd t = dd_mul_d(l, y);
    if (t.hi > 709.0) return __builtin_inf();
    if (t.hi < -745.0) return 0.0;
    const dd r = dd_exp(t);
    return r.hi + r.lo;
}

}  // namespace agx
