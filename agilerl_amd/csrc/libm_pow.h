// pow(x, y) bit-identical to the host's libm (glibc >= 2.28) for the
// prioritized-replay domain, on the device.
//
// The reference computes PER leaves as ``priority ** alpha``
// (agilerl/components/replay_buffer.py:311-329) and IS weights as
// ``(p * size) ** (-beta)`` (:383-409) with Python floats, i.e. glibc's pow.
// That routine (sysdeps/ieee754/dbl-64/e_pow.c, from ARM optimized-routines)
// is not correctly rounded (<= 0.52 ulp), so matching it bit for bit means
// running ITS algorithm: log(x) = k ln2 + log(c) + log1p(z/c - 1) from a
// 128-entry table and a degree-8 polynomial, giving hi + lo; then
// exp(y * (hi + lo)) as 2^(k/128) * exp(r) from a 128-entry table and a
// degree-5 polynomial.  This is the FMA variant glibc's x86-64 ifunc runs on
// an FMA host (__pow_fma), and glibc builds it with GCC's default
// floating-point contraction: besides the source's explicit fma() calls, GCC
// fuses t1, lo1, the polynomial Horner steps, ar3 * poly into the lo sum,
// z + Shift, both r reduction steps and scale + scale * tmp (read off the
// GCC 11 -O2 -mfma code).  Each of those is an explicit __builtin_fma here,
// everything else rounds as written (-ffp-contract=off).
// The tables are regenerated from the published recipe by
// tools/gen_pow_tables.py; tests pin the result to libm bit for bit.
//
// Domain: x > 0 finite (normal), |y * log(x)| < 512 — every PER leaf and
// weight (priorities >= 1e-5, weights <= size^beta).  Outside it the
// device libm pow is returned (never reached on the PER path).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "libm_pow_tables.h"

namespace agx {

__device__ __forceinline__ double pw_asd(uint64_t u) { return __builtin_bit_cast(double, u); }
__device__ __forceinline__ uint64_t pw_asu(double x) { return __builtin_bit_cast(uint64_t, x); }

// log_inline of e_pow.c: returns hi, *tail = lo with hi + lo = log(x) (~2^-68 rel)
__device__ __forceinline__ double pw_log(uint64_t ix, double *tail) {
    constexpr uint64_t kOff = 0x3fe6955500000000ull;
    constexpr double kLn2hi = 0x1.62e42fefa3800p-1, kLn2lo = 0x1.ef35793c76730p-45;
    constexpr double A0 = -0x1p-1, A1 = 0x1.555555555556p-2 * -2, A2 = -0x1.0000000000006p-2 * -2;
    constexpr double A3 = 0x1.999999959554ep-3 * 4, A4 = -0x1.555555529a47ap-3 * 4;
    constexpr double A5 = 0x1.2495b9b4845e9p-3 * -8, A6 = -0x1.0002b8b263fc3p-3 * -8;
    const uint64_t tmp = ix - kOff;
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const double z = pw_asd(ix - (tmp & (0xfffull << 52)));
    const double kd = (double)k;
    const double invc = kPowLogTab[i][0], logc = kPowLogTab[i][1], logctail = kPowLogTab[i][2];
    const double r = __builtin_fma(z, invc, -1.0);  // exact: 1/c has few bits
    const double t1 = __builtin_fma(kd, kLn2hi, logc);
    const double t2 = t1 + r;
    const double lo1 = __builtin_fma(kd, kLn2lo, logctail);
    const double lo2 = t1 - t2 + r;
    const double ar = A0 * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = __builtin_fma(ar, r, -ar2);
    const double lo4 = t2 - hi + ar2;
    // A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6)), then lo1 + lo2 + lo3 + lo4 + ar3 * that
    const double q = __builtin_fma(__builtin_fma(__builtin_fma(r, A6, A5), ar2, __builtin_fma(r, A4, A3)), ar2,
                                   __builtin_fma(r, A2, A1));
    const double lo = __builtin_fma(ar3, q, lo1 + lo2 + lo3 + lo4);
    const double y = hi + lo;
    *tail = hi - y + lo;
    return y;
}

// exp_inline of e_pow.c (no sign bias; |x| < 512 so no special scaling)
__device__ __forceinline__ double pw_exp(double x, double xtail) {
    constexpr double kInvLn2N = 0x1.71547652b82fep0 * 128, kShift = 0x1.8p52;
    constexpr double kNegLn2hiN = -0x1.62e42fefa0000p-8, kNegLn2loN = -0x1.cf79abc9e3b3ap-47;
    constexpr double C2 = 0x1.ffffffffffdbdp-2, C3 = 0x1.555555555543cp-3;
    constexpr double C4 = 0x1.55555cf172b91p-5, C5 = 0x1.1111167a4d017p-7;
    double kd = __builtin_fma(kInvLn2N, x, kShift);  // InvLn2N * x + Shift
    const uint64_t ki = pw_asu(kd);
    kd -= kShift;
    double r = __builtin_fma(kd, kNegLn2loN, __builtin_fma(kd, kNegLn2hiN, x));
    r += xtail;
    const uint64_t idx = 2 * (ki % 128);
    const uint64_t top = ki << 45;
    const double tail = pw_asd(kPowExpTab[idx]);
    const uint64_t sbits = kPowExpTab[idx + 1] + top;
    const double r2 = r * r;
    // tail + r + r2 (C2 + r C3) + r2^2 (C4 + r C5)
    const double tmp = __builtin_fma(r2 * r2, __builtin_fma(r, C5, C4),
                                     __builtin_fma(__builtin_fma(r, C3, C2), r2, tail + r));
    const double scale = pw_asd(sbits);
    return __builtin_fma(scale, tmp, scale);
}

__device__ __forceinline__ double libm_pow(double x, double y) {
    const uint64_t ix = pw_asu(x);
    // x normal and positive (top 12 bits in [0x001, 0x7fe])
    if ((ix >> 52) - 1 >= 0x7fe - 1) return pow(x, y);
    double lo;
    const double hi = pw_log(ix, &lo);
    const double ehi = y * hi;
    const double elo = __builtin_fma(y, lo, __builtin_fma(y, hi, -ehi));
    if (!(fabs(ehi) < 512.0)) return pow(x, y);
    return pw_exp(ehi, elo);
}

}  // namespace agx
