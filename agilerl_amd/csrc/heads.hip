// Rainbow's dueling distributional head combine (DuelingDistributionalMLP.forward,
// agilerl/networks/custom_modules.py:127-162) after its value / advantage
// streams:
//   x[b,a,z] = (v[b,z] + adv[b,a,z]) - mean_a adv[b,a,z]
//   mode 2 (log=True):  logp = log_softmax_z(x)
//   mode 1 (q=False):   p = clamp(softmax_z(x), min=1e-3)          (not renormalised)
//   mode 0 (q=True):    q[b,a] = sum_z clamp(softmax_z(x), 1e-3) * support[z]
// and the gradient of each mode back to (v, adv).  One wave per batch row,
// lane z (Z <= 64 atoms): the action mean, every softmax max / sum and the
// support dot product are wave reductions — one launch instead of the eight
// tensor ops of the reference's form.  Softmax as torch computes it:
// exp(x - max) / sum, log form x - max - log(sum).
#include "agx_common.h"

namespace agx {

namespace heads {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

constexpr float kClampMin = 1e-3f;

__global__ __launch_bounds__(64) void dueling_fwd_kernel(const float *__restrict__ v, const float *__restrict__ adv,
                                                         const float *__restrict__ support, int A, int Z, int mode,
                                                         float *__restrict__ out) {
    const int64_t b = blockIdx.x;
    const int z = threadIdx.x;
    const bool live = z < Z;
    const float *ab = adv + b * (int64_t)A * Z;
    float s = 0.f;
    for (int a = 0; a < A; ++a) s += live ? ab[a * Z + z] : 0.f;
    const float mean = s / (float)A;
    const float vz = live ? v[b * Z + z] : 0.f;
    const float sup = (live && mode == 0) ? support[z] : 0.f;
    for (int a = 0; a < A; ++a) {
        const float x = live ? (vz + ab[a * Z + z]) - mean : -__builtin_inff();
        const float mx = wave_max(x);
        const float e = live ? expf(x - mx) : 0.f;
        const float sum = wave_sum(e);
        if (mode == 2) {
            if (live) out[(b * A + a) * Z + z] = (x - mx) - logf(sum);
        } else {
            const float p = fmaxf(e / sum, kClampMin);
            if (mode == 1) {
                if (live) out[(b * A + a) * Z + z] = p;
            } else {
                const float q = wave_sum(live ? p * sup : 0.f);
                if (z == 0) out[b * A + a] = q;
            }
        }
    }
}

// g: dL/d(out) ([B][A][Z], or [B][A] for mode 0) -> dv [B][Z], dadv [B][A][Z]
__global__ __launch_bounds__(64) void dueling_bwd_kernel(const float *__restrict__ v, const float *__restrict__ adv,
                                                         const float *__restrict__ support, const float *__restrict__ g,
                                                         int A, int Z, int mode, float *__restrict__ dv,
                                                         float *__restrict__ dadv) {
    const int64_t b = blockIdx.x;
    const int z = threadIdx.x;
    const bool live = z < Z;
    const float *ab = adv + b * (int64_t)A * Z;
    float *db = dadv + b * (int64_t)A * Z;
    float s = 0.f;
    for (int a = 0; a < A; ++a) s += live ? ab[a * Z + z] : 0.f;
    const float mean = s / (float)A;
    const float vz = live ? v[b * Z + z] : 0.f;
    const float sup = (live && mode == 0) ? support[z] : 0.f;
    float dsum = 0.f;  // sum_a dx[a, z]
    for (int a = 0; a < A; ++a) {
        const float x = live ? (vz + ab[a * Z + z]) - mean : -__builtin_inff();
        const float mx = wave_max(x);
        const float e = live ? expf(x - mx) : 0.f;
        const float sum = wave_sum(e);
        const float p = e / sum;
        float dx;
        if (mode == 2) {  // d log_softmax: g - p * sum_z g
            const float gz = live ? g[(b * A + a) * Z + z] : 0.f;
            dx = gz - p * wave_sum(gz);
        } else {  // through clamp(min) (gradient where p >= min, as torch) and softmax
            float gp = mode == 1 ? (live ? g[(b * A + a) * Z + z] : 0.f) : g[b * A + a] * sup;
            gp = (live && p >= kClampMin) ? gp : 0.f;
            dx = p * (gp - wave_sum(gp * p));
        }
        dx = live ? dx : 0.f;
        if (live) db[a * Z + z] = dx;  // d(adv) before the mean term
        dsum += dx;
    }
    if (live) dv[b * Z + z] = dsum;
    // d(adv)[a] = dx[a] - (1/A) sum_a' dx[a'] (the subtracted mean)
    const float corr = dsum / (float)A;
    for (int a = 0; a < A; ++a)
        if (live) db[a * Z + z] -= corr;
}

// Selected rows: only action sel[b] of each batch row is emitted ([B][Z]), the
// value the full form writes at out[b][sel[b]] bit for bit (same mean, same
// per-row softmax).  This is the reference's target_dist[range(B), a*] and
// log_p[range(B), a] (dqn_rainbow.py:313-367) fused into the producer, so the
// C51 step reads two contiguous [B][Z] arrays.
__global__ __launch_bounds__(64) void dueling_fwd_rows_kernel(const float *__restrict__ v,
                                                              const float *__restrict__ adv,
                                                              const int64_t *__restrict__ sel, int A, int Z, int mode,
                                                              float *__restrict__ out) {
    const int64_t b = blockIdx.x;
    const int z = threadIdx.x;
    const bool live = z < Z;
    const float *ab = adv + b * (int64_t)A * Z;
    float s = 0.f;
    for (int a = 0; a < A; ++a) s += live ? ab[a * Z + z] : 0.f;
    const float mean = s / (float)A;
    const float vz = live ? v[b * Z + z] : 0.f;
    const int a = (int)sel[b];
    const float x = live ? (vz + ab[a * Z + z]) - mean : -__builtin_inff();
    const float mx = wave_max(x);
    const float e = live ? expf(x - mx) : 0.f;
    const float sum = wave_sum(e);
    if (live) out[b * Z + z] = mode == 2 ? (x - mx) - logf(sum) : fmaxf(e / sum, kClampMin);
}

// log mode: g [B][Z] = dL/d(out[b][sel[b]]) (zero for every other action) ->
// dv [B][Z], dadv [B][A][Z]; the full form's arithmetic with those zeros
__global__ __launch_bounds__(64) void dueling_bwd_rows_kernel(const float *__restrict__ v,
                                                              const float *__restrict__ adv,
                                                              const int64_t *__restrict__ sel,
                                                              const float *__restrict__ g, int A, int Z,
                                                              float *__restrict__ dv, float *__restrict__ dadv) {
    const int64_t b = blockIdx.x;
    const int z = threadIdx.x;
    const bool live = z < Z;
    const float *ab = adv + b * (int64_t)A * Z;
    float *db = dadv + b * (int64_t)A * Z;
    float s = 0.f;
    for (int a = 0; a < A; ++a) s += live ? ab[a * Z + z] : 0.f;
    const float mean = s / (float)A;
    const float vz = live ? v[b * Z + z] : 0.f;
    const int a = (int)sel[b];
    const float x = live ? (vz + ab[a * Z + z]) - mean : -__builtin_inff();
    const float mx = wave_max(x);
    const float e = live ? expf(x - mx) : 0.f;
    const float sum = wave_sum(e);
    const float p = e / sum;
    const float gz = live ? g[b * Z + z] : 0.f;
    float dx = gz - p * wave_sum(gz);
    dx = live ? dx : 0.f;
    const float dsum = dx;
    if (live) dv[b * Z + z] = dsum;
    const float corr = dsum / (float)A;
    for (int k = 0; k < A; ++k)
        if (live) db[k * Z + z] = (k == a ? dx : 0.f) - corr;
}

}  // namespace heads

}  // namespace agx

using namespace agx;

extern "C" int agx_dueling_head_forward(const float *value, const float *advantage, const float *support, int64_t B,
                                        int64_t A, int64_t Z, int mode, float *out, void *stream) {
    AGX_REQUIRE(value && advantage && out && B >= 0 && A > 0 && Z >= 1 && Z <= 64 && mode >= 0 && mode <= 2,
                "agx_dueling_head_forward: bad arguments (need 1 <= Z <= 64, mode 0..2)");
    AGX_REQUIRE(mode != 0 || support, "agx_dueling_head_forward: mode 0 (q) needs the support");
    if (B == 0) return AGX_OK;
    AGX_REQUIRE(B < (1ll << 31), "agx_dueling_head_forward: batch too large");
    heads::dueling_fwd_kernel<<<(unsigned)B, 64, 0, as_stream(stream)>>>(value, advantage, support, (int)A, (int)Z,
                                                                        mode, out);
    return check_launch("agx_dueling_head_forward");
}

extern "C" int agx_dueling_head_backward(const float *value, const float *advantage, const float *support,
                                         const float *grad_out, int64_t B, int64_t A, int64_t Z, int mode,
                                         float *grad_value, float *grad_advantage, void *stream) {
    AGX_REQUIRE(value && advantage && grad_out && grad_value && grad_advantage && B >= 0 && A > 0 && Z >= 1 &&
                    Z <= 64 && mode >= 0 && mode <= 2,
                "agx_dueling_head_backward: bad arguments (need 1 <= Z <= 64, mode 0..2)");
    AGX_REQUIRE(mode != 0 || support, "agx_dueling_head_backward: mode 0 (q) needs the support");
    if (B == 0) return AGX_OK;
    AGX_REQUIRE(B < (1ll << 31), "agx_dueling_head_backward: batch too large");
    heads::dueling_bwd_kernel<<<(unsigned)B, 64, 0, as_stream(stream)>>>(value, advantage, support, grad_out, (int)A,
                                                                        (int)Z, mode, grad_value, grad_advantage);
    return check_launch("agx_dueling_head_backward");
}

extern "C" int agx_dueling_head_forward_rows(const float *value, const float *advantage, const int64_t *sel, int64_t B,
                                             int64_t A, int64_t Z, int mode, float *out, void *stream) {
    AGX_REQUIRE(value && advantage && sel && out && B >= 0 && A > 0 && Z >= 1 && Z <= 64 && (mode == 1 || mode == 2),
                "agx_dueling_head_forward_rows: bad arguments (need 1 <= Z <= 64, mode 1 or 2)");
    if (B == 0) return AGX_OK;
    AGX_REQUIRE(B < (1ll << 31), "agx_dueling_head_forward_rows: batch too large");
    heads::dueling_fwd_rows_kernel<<<(unsigned)B, 64, 0, as_stream(stream)>>>(value, advantage, sel, (int)A, (int)Z,
                                                                             mode, out);
    return check_launch("agx_dueling_head_forward_rows");
}

extern "C" int agx_dueling_head_backward_rows(const float *value, const float *advantage, const int64_t *sel,
                                              const float *grad_rows, int64_t B, int64_t A, int64_t Z,
                                              float *grad_value, float *grad_advantage, void *stream) {
    AGX_REQUIRE(value && advantage && sel && grad_rows && grad_value && grad_advantage && B >= 0 && A > 0 && Z >= 1 &&
                    Z <= 64,
                "agx_dueling_head_backward_rows: bad arguments (need 1 <= Z <= 64)");
    if (B == 0) return AGX_OK;
    AGX_REQUIRE(B < (1ll << 31), "agx_dueling_head_backward_rows: batch too large");
    heads::dueling_bwd_rows_kernel<<<(unsigned)B, 64, 0, as_stream(stream)>>>(value, advantage, sel, grad_rows,
                                                                             (int)A, (int)Z, grad_value,
                                                                             grad_advantage);
    return check_launch("agx_dueling_head_backward_rows");
}
