// Population optimiser step: per-agent, per-group gradient-norm clipping fused
// with Adam, over flat parameter buffers [P][n]; and Polyak averaging.
//
// Reference: clip_grad_norm_(actor.parameters(), max_grad_norm) then
// clip_grad_norm_(critic.parameters(), ...) (agilerl/algorithms/ppo.py:910-911;
// dqn_rainbow.py:479 with 10.0), then OptimizerWrapper.step
// (agilerl/algorithms/core/optimizer_wrapper.py:444-452) -> torch.optim.Adam:
//   m = lerp(m, g, 1-b1); v = b2*v + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// clip: coef = max_norm / (||g||_2 + 1e-6), g *= min(coef, 1).
// Polyak: agilerl/algorithms/dqn.py:349-358 — t = tau*o + (1-tau)*t.
//
// Two launches: (1) per-(agent, chunk) partial sums of squares per group into
// the workspace, (2) every block re-reduces its agent's partials in a fixed
// order (deterministic), derives the clip coefficients and updates its chunk.
// Traffic: 4 arrays read + 3 written = 28 B per parameter (+4 B norm pass).
#include "agx_common.h"

namespace agx {

constexpr int kOptBlock = 256;
constexpr int kOptPer = 4;  // params per thread per block
constexpr int kOptChunk = kOptBlock * kOptPer;
constexpr int kMaxGroups = 8;

struct Groups {
    int64_t off[kMaxGroups + 1];
    int G;
};

__device__ __forceinline__ int group_of(const Groups &g, int64_t j) {
    int k = 0;
    while (k + 1 < g.G && j >= g.off[k + 1]) ++k;
    return k;
}

__global__ __launch_bounds__(kOptBlock) void sumsq_kernel(const float *__restrict__ grads, int64_t n,
                                                          Groups gr, double *__restrict__ part) {
    const int p = blockIdx.y;
    const float *g = grads + (size_t)p * n;
    double acc[kMaxGroups];
#pragma unroll
    for (int k = 0; k < kMaxGroups; ++k) acc[k] = 0.0;
    const int64_t j0 = (int64_t)blockIdx.x * kOptChunk;
    for (int r = 0; r < kOptPer; ++r) {
        const int64_t j = j0 + r * kOptBlock + threadIdx.x;
        if (j < n) {
            const double x = (double)g[j];
            const int k = group_of(gr, j);
#pragma unroll
            for (int q = 0; q < kMaxGroups; ++q)
                if (q == k) acc[q] += x * x;
        }
    }
    __shared__ double red[kMaxGroups][kOptBlock / kWave];
#pragma unroll
    for (int k = 0; k < kMaxGroups; ++k) {
        const double s = wave_sum(acc[k]);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x / 64] = s;
    }
    __syncthreads();
    if (threadIdx.x < kMaxGroups) {
        double s = 0.0;
        for (int w = 0; w < kOptBlock / kWave; ++w) s += red[threadIdx.x][w];
        part[((size_t)p * gridDim.x + blockIdx.x) * kMaxGroups + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(kOptBlock) void adam_kernel(float *__restrict__ params,
                                                         float *__restrict__ grads,
                                                         float *__restrict__ m, float *__restrict__ v,
                                                         int64_t n, Groups gr, float max_norm,
                                                         const double *__restrict__ part,
                                                         const float *__restrict__ lr_dev,
                                                         float b1, float b2, float eps, float bc1,
                                                         float bc2_sqrt, int clip) {
    const int p = blockIdx.y;
    __shared__ float coef[kMaxGroups];
    if (threadIdx.x < kMaxGroups) {
        float c = 1.0f;
        if (clip && (int)threadIdx.x < gr.G) {
            double s = 0.0;
            for (int b = 0; b < (int)gridDim.x; ++b) s += part[((size_t)p * gridDim.x + b) * kMaxGroups + threadIdx.x];
            const float norm = (float)sqrt(s);
            const float cc = max_norm / (norm + 1e-6f);
            c = cc < 1.0f ? cc : 1.0f;
        }
        coef[threadIdx.x] = c;
    }
    __syncthreads();
    const float lr = lr_dev[p];
    const float step_size = lr / bc1;
    const size_t base = (size_t)p * n;
    const int64_t j0 = (int64_t)blockIdx.x * kOptChunk;
    for (int r = 0; r < kOptPer; ++r) {
        const int64_t j = j0 + r * kOptBlock + threadIdx.x;
        if (j >= n) break;
        float g = grads[base + j];
        if (clip) {
            g = g * coef[group_of(gr, j)];
            grads[base + j] = g;
        }
        float mm = m[base + j];
        mm = mm + (1.0f - b1) * (g - mm);  // lerp_(g, 1-b1)
        float vv = v[base + j];
        vv = vv * b2 + (1.0f - b2) * g * g;
        m[base + j] = mm;
        v[base + j] = vv;
        const float denom = sqrtf(vv) / bc2_sqrt + eps;
        params[base + j] = params[base + j] - step_size * (mm / denom);
    }
}

__global__ void polyak_kernel(float *__restrict__ t, const float *__restrict__ o, int64_t n, float tau) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        t[i] = tau * o[i] + (1.0f - tau) * t[i];
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_adam_workspace_bytes(int64_t P, int64_t n) {
    return (size_t)P * (size_t)ceil_div(n, kOptChunk) * kMaxGroups * sizeof(double);
}

extern "C" int agx_clip_adam(float *params, float *grads, float *exp_avg, float *exp_avg_sq, int64_t P,
                             int64_t n, const int64_t *group_offsets, int G, float max_norm,
                             const float *lr, float beta1, float beta2, float eps, int64_t step,
                             void *workspace, void *stream) {
    AGX_REQUIRE(params && grads && exp_avg && exp_avg_sq && lr && workspace, "agx_clip_adam: null pointer");
    AGX_REQUIRE(P > 0 && P <= 65535 && n > 0 && G >= 1 && G <= kMaxGroups && step >= 1,
                "agx_clip_adam: bad shape P=%lld n=%lld G=%d", (long long)P, (long long)n, G);
    Groups gr;
    gr.G = G;
    for (int k = 0; k <= kMaxGroups; ++k) gr.off[k] = k <= G ? group_offsets[k] : n;
    AGX_REQUIRE(gr.off[0] == 0 && gr.off[G] == n, "agx_clip_adam: group offsets must span [0, n)");
    hipStream_t s = as_stream(stream);
    const int64_t nblk = ceil_div(n, kOptChunk);
    double *part = static_cast<double *>(workspace);
    dim3 grid((unsigned)nblk, (unsigned)P);
    const int clip = max_norm > 0.0f;
    if (clip) sumsq_kernel<<<grid, kOptBlock, 0, s>>>(grads, n, gr, part);
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    adam_kernel<<<grid, kOptBlock, 0, s>>>(params, grads, exp_avg, exp_avg_sq, n, gr, max_norm, part, lr,
                                           beta1, beta2, eps, (float)bc1, (float)sqrt(bc2), clip);
    return check_launch("agx_clip_adam");
}

extern "C" int agx_polyak(float *target, const float *online, int64_t n, float tau, void *stream) {
    AGX_REQUIRE(target && online && n >= 0, "agx_polyak: bad arguments");
    if (n == 0) return AGX_OK;
    const int64_t blocks = ceil_div(n, 256);
    polyak_kernel<<<(unsigned)(blocks > 4096 ? 4096 : blocks), 256, 0, as_stream(stream)>>>(target, online, n, tau);
    return check_launch("agx_polyak");
}
