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
// Noise reset: NoisyLinear.reset_noise (agilerl/modules/custom_components.py:
// 116-131) for every noisy layer of a network in one launch.
//
// Two launches: (1) per-(agent, 8192-element chunk) partial sums of squares
// per group into the workspace, (2) every 1024-element block re-reduces its
// agent's partials in a fixed order (deterministic), derives the clip
// coefficients and updates its chunk.  Rows of more than 16 partials add a
// per-agent pre-reduction (1b) so the re-reduction does not grow with the
// square of the row length.
// Traffic: 4 arrays read + 3 written = 28 B per parameter (+4 B norm pass).
#include "agx_common.h"

namespace agx {

constexpr int kOptBlock = 256;
constexpr int kOptPer = 4;  // params per thread per block
constexpr int kOptChunk = kOptBlock * kOptPer;
constexpr int kSumChunk = kOptBlock * 4 * 8;  // sum-of-squares block: 8 float4 per thread
constexpr int kMaxGroups = 8;
typedef float f4 __attribute__((ext_vector_type(4)));

struct Groups {
    int64_t off[kMaxGroups + 1];
    int G;
};

__device__ __forceinline__ int group_of(const Groups &g, int64_t j) {
    int k = 0;
    while (k + 1 < g.G && j >= g.off[k + 1]) ++k;
    return k;
}

// (1) per-(agent, chunk) partial sums of squares per group.  V4: one float4
// per thread (n % 4 == 0, 16-byte aligned rows), else kOptPer strided floats.
template <bool V4>
__global__ __launch_bounds__(kOptBlock) void sumsq_kernel(const float *__restrict__ grads, int64_t n,
                                                          Groups gr, double *__restrict__ part) {
    const int p = blockIdx.y;
    const float *g = grads + (size_t)p * n;
    double acc[kMaxGroups];
#pragma unroll
    for (int k = 0; k < kMaxGroups; ++k) acc[k] = 0.0;
    const int64_t j0 = (int64_t)blockIdx.x * kSumChunk;
    auto add = [&](int64_t j, float xf) {
        const double x = (double)xf;
        const int k = group_of(gr, j);
#pragma unroll
        for (int q = 0; q < kMaxGroups; ++q)
            if (q == k) acc[q] += x * x;
    };
    if constexpr (V4) {
        f4 x[8];  // all loads in flight before the f64 accumulation
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int64_t j = j0 + 4 * (r * kOptBlock + threadIdx.x);
            x[r] = j < n ? *reinterpret_cast<const f4 *>(g + j) : f4{0.f, 0.f, 0.f, 0.f};
        }
        const int64_t jl = (j0 + kSumChunk < n ? j0 + kSumChunk : n) - 1;
        const int kb = group_of(gr, j0);
        if (kb == group_of(gr, jl)) {
            // the whole chunk in one group (all but the chunks a group boundary
            // cuts): one accumulator, no per-element group lookup — the same
            // additions in the same order as the general form, so the same bits
            double a = 0.0;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int64_t j = j0 + 4 * (r * kOptBlock + threadIdx.x);
                if (j < n) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const double xd = (double)x[r][e];
                        a += xd * xd;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < kMaxGroups; ++q)
                if (q == kb) acc[q] = a;
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int64_t j = j0 + 4 * (r * kOptBlock + threadIdx.x);
                if (j < n) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) add(j + e, x[r][e]);
                }
            }
        }
    } else {
        for (int r = 0; r < kSumChunk / kOptBlock; ++r) {
            const int64_t j = j0 + r * kOptBlock + threadIdx.x;
            if (j < n) add(j, g[j]);
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

__device__ __forceinline__ float clip_coef(double sumsq, float max_norm) {
    const float norm = (float)sqrt(sumsq);
    const float cc = max_norm / (norm + 1e-6f);
    return cc < 1.0f ? cc : 1.0f;
}

// (1b) many chunks: one block per agent reduces its partials in a fixed order
// (strided per-thread sums, then a fixed LDS tree) -> coef[p][group]
__global__ __launch_bounds__(kOptBlock) void clip_coef_kernel(const double *__restrict__ part, int nblk, int G,
                                                              float max_norm, float *__restrict__ coef) {
    const int p = blockIdx.x;
    __shared__ double red[kOptBlock];
    for (int k = 0; k < G; ++k) {
        double s = 0.0;
        for (int b = threadIdx.x; b < nblk; b += kOptBlock) s += part[((size_t)p * nblk + b) * kMaxGroups + k];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int h = kOptBlock / 2; h > 0; h >>= 1) {
            if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
            __syncthreads();
        }
        if (threadIdx.x == 0) coef[(size_t)p * kMaxGroups + k] = clip_coef(red[0], max_norm);
        __syncthreads();
    }
}

// (2) clip + Adam over one chunk.  Clip coefficients: from coef_dev when the
// partials were pre-reduced (many chunks), else every block re-reduces its
// agent's few partials in a fixed order.
// Per-agent Adam bias corrections for this update (torch.optim.Adam,
// single-tensor path: step_size = lr / (1 - b1^t), denom = sqrt(v) /
// sqrt(1 - b2^t) + eps) from each agent's own step count; active agents'
// counts advance by one.
__global__ void adam_prep_kernel(long long *__restrict__ steps, const unsigned char *__restrict__ active, int P,
                                 float b1, float b2, float *__restrict__ bc) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const bool on = !active || active[p];
    const long long t = steps[p] + 1;
    bc[2 * p] = (float)(1.0 - pow((double)b1, (double)t));
    bc[2 * p + 1] = (float)sqrt(1.0 - pow((double)b2, (double)t));
    if (on) steps[p] = t;
}

template <bool V4>
__global__ __launch_bounds__(kOptBlock) void adam_kernel(float *__restrict__ params,
                                                         float *__restrict__ grads,
                                                         float *__restrict__ m, float *__restrict__ v,
                                                         int64_t n, Groups gr, float max_norm,
                                                         const double *__restrict__ part, int nsum,
                                                         const float *__restrict__ coef_dev,
                                                         const float *__restrict__ lr_dev,
                                                         float b1, float b2, float eps,
                                                         const float *__restrict__ bc,
                                                         const unsigned char *__restrict__ active, int clip) {
    const int p = blockIdx.y;
    if (active && !active[p]) return;  // this agent stopped (target_kl): untouched
    const float bc1 = bc[2 * p], bc2_sqrt = bc[2 * p + 1];
    __shared__ float coef[kMaxGroups];
    if (threadIdx.x < kMaxGroups) {
        float c = 1.0f;
        if (clip && (int)threadIdx.x < gr.G) {
            if (coef_dev) {
                c = coef_dev[(size_t)p * kMaxGroups + threadIdx.x];
            } else {
                double s = 0.0;
                for (int b = 0; b < nsum; ++b) s += part[((size_t)p * nsum + b) * kMaxGroups + threadIdx.x];
                c = clip_coef(s, max_norm);
            }
        }
        coef[threadIdx.x] = c;
    }
    __syncthreads();
    const float lr = lr_dev[p];
    const float step_size = lr / bc1;
    const size_t base = (size_t)p * n;
    const int64_t j0 = (int64_t)blockIdx.x * kOptChunk;
    auto upd = [&](int64_t j, float g, float &pp, float &mm, float &vv, int k = -1) {
        if (clip) g = g * coef[k >= 0 ? k : group_of(gr, j)];
        mm = mm + (1.0f - b1) * (g - mm);  // lerp_(g, 1-b1)
        vv = vv * b2 + (1.0f - b2) * g * g;
        const float denom = sqrtf(vv) / bc2_sqrt + eps;
        pp = pp - step_size * (mm / denom);
        return g;
    };
    if constexpr (V4) {
        const int64_t j = j0 + 4 * threadIdx.x;
        if (j >= n) return;
        f4 g = *reinterpret_cast<const f4 *>(grads + base + j);
        f4 pp = *reinterpret_cast<const f4 *>(params + base + j);
        f4 mm = *reinterpret_cast<const f4 *>(m + base + j);
        f4 vv = *reinterpret_cast<const f4 *>(v + base + j);
        // one group lookup per float4 unless a group boundary falls inside it
        int k4 = -1;
        if (clip) {
            const int ka = group_of(gr, j);
            if (ka == group_of(gr, j + 3)) k4 = ka;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pe = pp[e], me = mm[e], ve = vv[e];
            g[e] = upd(j + e, g[e], pe, me, ve, k4);
            pp[e] = pe;
            mm[e] = me;
            vv[e] = ve;
        }
        if (clip) *reinterpret_cast<f4 *>(grads + base + j) = g;
        *reinterpret_cast<f4 *>(m + base + j) = mm;
        *reinterpret_cast<f4 *>(v + base + j) = vv;
        *reinterpret_cast<f4 *>(params + base + j) = pp;
    } else {
        for (int r = 0; r < kOptPer; ++r) {
            const int64_t j = j0 + r * kOptBlock + threadIdx.x;
            if (j >= n) break;
            float pe = params[base + j], me = m[base + j], ve = v[base + j];
            const float g = upd(j, grads[base + j], pe, me, ve);
            if (clip) grads[base + j] = g;
            m[base + j] = me;
            v[base + j] = ve;
            params[base + j] = pe;
        }
    }
}

__global__ void polyak_kernel(float *__restrict__ t, const float *__restrict__ o, int64_t n, float tau) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        t[i] = tau * o[i] + (1.0f - tau) * t[i];
}

// NoisyLinear.reset_noise over up to kMaxNoisy layers (custom_components.py:
// 116-131): from the layer's two N(0,1) draws, f(x) = sign(x) * sqrt(|x|)
// (torch's sign: (0 < x) - (x < 0); correctly rounded sqrt, as torch's),
// weight_epsilon[o][i] = f(out_o) * f(in_i) (eps_out.ger(eps_in)),
// bias_epsilon[o] = f(out_o).  blockIdx.y = layer; grid-stride over the
// layer's out*in + out outputs.
constexpr int kMaxNoisy = 16;
struct NoisySet {
    agx_noisy_layer l[kMaxNoisy];
};

__device__ __forceinline__ float scale_noise(float x) {
    const float s = (float)((0.0f < x) - (x < 0.0f));
    return s * sqrtf(fabsf(x));  // llvm.sqrt.f32: correctly rounded (__fsqrt_rn is the native approximation here)
}

__global__ __launch_bounds__(256) void noisy_reset_kernel(NoisySet set) {
    const agx_noisy_layer &L = set.l[blockIdx.y];
    const int64_t nin = L.in_features, nout = L.out_features, nw = nin * nout;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nw + nout;
         e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nw) {
            const int64_t o = e / nin, i = e - o * nin;
            L.weight_epsilon[e] = scale_noise(L.eps_out[o]) * scale_noise(L.eps_in[i]);
        } else {
            L.bias_epsilon[e - nw] = scale_noise(L.eps_out[e - nw]);
        }
    }
}

}  // namespace agx

using namespace agx;

extern "C" int agx_noisy_reset(const agx_noisy_layer *layers, int n_layers, void *stream) {
    AGX_REQUIRE(layers && n_layers >= 0 && n_layers <= kMaxNoisy, "agx_noisy_reset: bad layer list (n=%d, max %d)",
                n_layers, kMaxNoisy);
    if (n_layers == 0) return AGX_OK;
    NoisySet set;
    int64_t most = 0;
    for (int k = 0; k < n_layers; ++k) {
        const agx_noisy_layer &L = layers[k];
        AGX_REQUIRE(L.eps_in && L.eps_out && L.weight_epsilon && L.bias_epsilon && L.in_features > 0 &&
                        L.out_features > 0,
                    "agx_noisy_reset: layer %d: bad arguments", k);
        set.l[k] = L;
        const int64_t n = L.in_features * L.out_features + L.out_features;
        most = n > most ? n : most;
    }
    const int64_t blocks = ceil_div(most, 256);
    noisy_reset_kernel<<<dim3((unsigned)(blocks > 1024 ? 1024 : blocks), (unsigned)n_layers), 256, 0,
                         as_stream(stream)>>>(set);
    return check_launch("agx_noisy_reset");
}

extern "C" size_t agx_adam_workspace_bytes(int64_t P, int64_t n) {
    // partials [P][nblk][8] f64, then clip coefficients [P][8] f32, then bias corrections [P][2] f32
    return (size_t)P * (size_t)ceil_div(n, kSumChunk) * kMaxGroups * sizeof(double) +
           (size_t)P * kMaxGroups * sizeof(float) + (size_t)P * 2 * sizeof(float);
}

extern "C" int agx_clip_adam(float *params, float *grads, float *exp_avg, float *exp_avg_sq, int64_t P,
                             int64_t n, const int64_t *group_offsets, int G, float max_norm,
                             const float *lr, float beta1, float beta2, float eps, int64_t *steps,
                             const uint8_t *active, void *workspace, void *stream) {
    AGX_REQUIRE(params && grads && exp_avg && exp_avg_sq && lr && steps && workspace,
                "agx_clip_adam: null pointer");
    AGX_REQUIRE(P > 0 && P <= 65535 && n > 0 && G >= 1 && G <= kMaxGroups,
                "agx_clip_adam: bad shape P=%lld n=%lld G=%d", (long long)P, (long long)n, G);
    Groups gr;
    gr.G = G;
    for (int k = 0; k <= kMaxGroups; ++k) gr.off[k] = k <= G ? group_offsets[k] : n;
    AGX_REQUIRE(gr.off[0] == 0 && gr.off[G] == n, "agx_clip_adam: group offsets must span [0, n)");
    hipStream_t s = as_stream(stream);
    const int64_t nblk = ceil_div(n, kOptChunk), nsum = ceil_div(n, kSumChunk);
    double *part = static_cast<double *>(workspace);
    dim3 grid((unsigned)nblk, (unsigned)P);
    const int clip = max_norm > 0.0f;
    const bool v4 = n % 4 == 0 && ((uintptr_t)params | (uintptr_t)grads | (uintptr_t)exp_avg |
                                   (uintptr_t)exp_avg_sq) % 16 == 0;
    float *coef = nullptr;
    float *bc = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) +
                                          (size_t)P * nsum * kMaxGroups * sizeof(double) +
                                          (size_t)P * kMaxGroups * sizeof(float));
    adam_prep_kernel<<<(unsigned)ceil_div(P, 256), 256, 0, s>>>(reinterpret_cast<long long *>(steps), active, (int)P,
                                                               beta1, beta2, bc);
    if (clip) {
        const dim3 sgrid((unsigned)nsum, (unsigned)P);
        if (v4) sumsq_kernel<true><<<sgrid, kOptBlock, 0, s>>>(grads, n, gr, part);
        else sumsq_kernel<false><<<sgrid, kOptBlock, 0, s>>>(grads, n, gr, part);
        if (nsum > 16) {  // pre-reduce once per agent instead of once per block
            coef = reinterpret_cast<float *>(part + (size_t)P * nsum * kMaxGroups);
            clip_coef_kernel<<<(unsigned)P, kOptBlock, 0, s>>>(part, (int)nsum, G, max_norm, coef);
        }
    }
    if (v4)
        adam_kernel<true><<<grid, kOptBlock, 0, s>>>(params, grads, exp_avg, exp_avg_sq, n, gr, max_norm, part,
                                                     (int)nsum, coef, lr, beta1, beta2, eps, bc, active, clip);
    else
        adam_kernel<false><<<grid, kOptBlock, 0, s>>>(params, grads, exp_avg, exp_avg_sq, n, gr, max_norm, part,
                                                      (int)nsum, coef, lr, beta1, beta2, eps, bc, active, clip);
    return check_launch("agx_clip_adam");
}

extern "C" int agx_polyak(float *target, const float *online, int64_t n, float tau, void *stream) {
    AGX_REQUIRE(target && online && n >= 0, "agx_polyak: bad arguments");
    if (n == 0) return AGX_OK;
    const int64_t blocks = ceil_div(n, 256);
    polyak_kernel<<<(unsigned)(blocks > 4096 ? 4096 : blocks), 256, 0, as_stream(stream)>>>(target, online, n, tau);
    return check_launch("agx_polyak");
}
