// GAE / Monte-Carlo reverse scan over a population's time-major rollout SoA.
//
// Reference: agilerl/components/rollout_buffer.py:413-481
// (RolloutBuffer.compute_returns_and_advantages), NumPy>=2 dtype flow:
//   t == T-1 : gv = gamma(f64) * f64(last_value)            nnt = 1 - last_done
//   t <  T-1 : gv = f64(f32(gamma) * values[t+1])  (f32 mul) nnt = 1 - done[t+1]
//   delta = (f64(r_t) + gv*nnt) - f64(v_t);  c = delta + ((gamma*lam)*nnt)*c   (f64 carry)
//   adv_t = f32(c);  ret_t = adv_t + v_t (f32)
// MC (use_gae = 0, :468-477): c = f64(lv)*(1-ld); c = f64(r_t) + (gamma*c)*(1-done_t);
//   ret_t = f32(c); adv_t = ret_t - v_t.
// The library is compiled with -ffp-contract=off: every product and sum rounds
// separately, as in NumPy — the results are bit-exact to the reference.
//
// Layout & mapping: x[p][t][n]; one lane owns one (p, n) column and walks t
// downward; lanes of a wave are consecutive n, so every load/store is a
// coalesced row segment.  Loads are issued U steps ahead in registers (two
// register sets) so each lane keeps ~3U loads in flight: with P*N columns
// = 65536 at the §8d shape there are only 4 waves per CU, and latency is
// hidden by this per-lane ILP rather than by occupancy.
// Algorithmic bytes: 4 (r) + 1 (done) + 4 (v) in, 4 (adv) + 4 (ret) out = 17 B
// per transition.
#include <cstdlib>

#include "agx_common.h"

namespace agx {

constexpr int kGaeBlock = 256;
template <int kGaeU, bool kGae, bool kStats>
__global__ __launch_bounds__(kGaeBlock) void gae_kernel(
    const float *__restrict__ rewards, const uint8_t *__restrict__ dones,
    const float *__restrict__ values, const float *__restrict__ last_value,
    const uint8_t *__restrict__ last_done, int T, int N, double gamma, double gl,
    float *__restrict__ adv, float *__restrict__ ret, double *__restrict__ partials) {
    const int p = blockIdx.y;
    const int n = blockIdx.x * kGaeBlock + threadIdx.x;
    const bool live = n < N;
    const int nn = live ? n : N - 1;  // dead lanes shadow a live column, store nothing
    const size_t base = (size_t)p * T * N + nn;
    const size_t sN = (size_t)N;
    const float g32 = (float)gamma;

    double c;
    float v_next;      // values[t+1]
    double nnt_next;   // 1 - done[t+1] of the step above
    const double lv = (double)last_value[(size_t)p * N + nn];
    const double ld = (double)last_done[(size_t)p * N + nn];
    double s1 = 0.0, s2 = 0.0;

    // ---- one step ---------------------------------------------------------
    auto step = [&](int t, float r, float v, uint8_t d, bool top) {
        if (kGae) {
            double nnt, gv;
            if (top) {
                nnt = 1.0 - ld;
                gv = gamma * lv;
            } else {
                nnt = nnt_next;
                gv = (double)(g32 * v_next);
            }
            const double delta = ((double)r + gv * nnt) - (double)v;
            c = delta + (gl * nnt) * c;
            const float a = (float)c;
            if (live) {
                adv[base + (size_t)t * sN] = a;
                ret[base + (size_t)t * sN] = a + v;
            }
            if (kStats && live) {
                s1 += (double)a;
                s2 += (double)a * (double)a;
            }
            v_next = v;
            nnt_next = 1.0 - (double)d;
        } else {
            c = (double)r + (gamma * c) * (1.0 - (double)d);
            const float rt = (float)c;
            const float a = rt - v;
            if (live) {
                ret[base + (size_t)t * sN] = rt;
                adv[base + (size_t)t * sN] = a;
            }
            if (kStats && live) {
                s1 += (double)a;
                s2 += (double)a * (double)a;
            }
        }
    };

    c = kGae ? 0.0 : lv * (1.0 - ld);
    v_next = 0.0f;
    nnt_next = 1.0;

    // partial head chunk so the rest is whole chunks of U
    int t = T - 1;
    const int head = T % kGaeU;
    for (int i = 0; i < head; ++i, --t) {
        const size_t o = base + (size_t)t * sN;
        step(t, rewards[o], values[o], dones[o], t == T - 1);
    }
    if (t < 0) goto reduce;
    {
        float ra[kGaeU], va[kGaeU];
        uint8_t da[kGaeU];
#pragma unroll
        for (int i = 0; i < kGaeU; ++i) {
            const size_t o = base + (size_t)(t - i) * sN;
            ra[i] = rewards[o];
            va[i] = values[o];
            da[i] = dones[o];
        }
        while (true) {
            const int tn = t - kGaeU;  // top of the next chunk
            float rb[kGaeU], vb[kGaeU];
            uint8_t db[kGaeU];
            if (tn >= 0) {
#pragma unroll
                for (int i = 0; i < kGaeU; ++i) {
                    const size_t o = base + (size_t)(tn - i) * sN;
                    rb[i] = rewards[o];
                    vb[i] = values[o];
                    db[i] = dones[o];
                }
            }
#pragma unroll
            for (int i = 0; i < kGaeU; ++i) step(t - i, ra[i], va[i], da[i], (t - i) == T - 1);
            if (tn < 0) break;
            t = tn;
#pragma unroll
            for (int i = 0; i < kGaeU; ++i) {
                ra[i] = rb[i];
                va[i] = vb[i];
                da[i] = db[i];
            }
        }
    }
reduce:
    if (kStats) {
        __shared__ double red[2][kGaeBlock / kWave];
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        const int w = threadIdx.x / kWave;
        if ((threadIdx.x & (kWave - 1)) == 0) {
            red[0][w] = s1;
            red[1][w] = s2;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = 0.0, b = 0.0;
            for (int i = 0; i < kGaeBlock / kWave; ++i) {
                a += red[0][i];
                b += red[1][i];
            }
            double *dst = partials + ((size_t)p * gridDim.x + blockIdx.x) * 2;
            dst[0] = a;
            dst[1] = b;
        }
    }
}

// Fixed-order reduction of the per-block partials -> [mean, unbiased std].
__global__ void gae_stats_finalize(const double *__restrict__ partials, int nblk, int64_t count,
                                   double *__restrict__ stats) {
    const int p = blockIdx.x;
    __shared__ double red[2][256 / kWave];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
        a += partials[((size_t)p * nblk + i) * 2];
        b += partials[((size_t)p * nblk + i) * 2 + 1];
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x / 64] = a;
        red[1][threadIdx.x / 64] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s1 = 0.0, s2 = 0.0;
        for (int i = 0; i < (int)(blockDim.x / 64); ++i) {
            s1 += red[0][i];
            s2 += red[1][i];
        }
        const double n = (double)count;
        const double mean = s1 / n;
        double var = (s2 - s1 * mean) / (n > 1.0 ? n - 1.0 : 1.0);
        if (var < 0.0) var = 0.0;
        stats[2 * p] = mean;
        stats[2 * p + 1] = sqrt(var);
    }
}

__global__ void adv_normalize_kernel(float *__restrict__ adv, const double *__restrict__ stats,
                                     int64_t count) {
    const int p = blockIdx.y;
    const double mean = stats[2 * p];
    const double inv = 1.0 / (stats[2 * p + 1] + 1e-8);
    float *a = adv + (size_t)p * count;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x)
        a[i] = (float)(((double)a[i] - mean) * inv);
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_gae_workspace_bytes(int64_t P, int64_t T, int64_t N) {
    (void)T;
    return (size_t)P * (size_t)ceil_div(N, kGaeBlock) * 2 * sizeof(double);
}

extern "C" int agx_gae(const float *rewards, const uint8_t *dones, const float *values,
                       const float *last_value, const uint8_t *last_done, int64_t P, int64_t T,
                       int64_t N, double gamma, double gae_lambda, int use_gae, float *advantages,
                       float *returns, double *adv_stats, void *workspace, void *stream) {
    AGX_REQUIRE(P > 0 && T > 0 && N > 0, "agx_gae: empty shape P=%lld T=%lld N=%lld",
                (long long)P, (long long)T, (long long)N);
    AGX_REQUIRE(P <= 65535 && T * N < (int64_t)1 << 40 && N < (int64_t)1 << 31,
                "agx_gae: shape too large");
    AGX_REQUIRE(rewards && dones && values && last_value && last_done && advantages && returns,
                "agx_gae: null pointer");
    AGX_REQUIRE(!adv_stats || workspace, "agx_gae: adv_stats needs a workspace");
    hipStream_t s = as_stream(stream);
    const int nblk = (int)ceil_div(N, kGaeBlock);
    dim3 grid(nblk, (unsigned)P);
    const double gl = gamma * gae_lambda;
    double *part = static_cast<double *>(workspace);
    // prefetch depth: deeper register pipelines for long scans (per-lane ILP is
    // what hides HBM latency at 1-4 waves per SIMD); AGX_GAE_UNROLL overrides.
    int U = T >= 32 ? 16 : 8;  // measured on MI355X at P8 T1024 N8192: U8 3.75, U16 4.78, U32 4.51 TB/s
    if (const char *e = getenv("AGX_GAE_UNROLL")) U = atoi(e);
#define AGX_GAE_LAUNCH(UU, G, S)                                                                    \
    gae_kernel<UU, G, S><<<grid, kGaeBlock, 0, s>>>(rewards, dones, values, last_value, last_done, \
                                                    (int)T, (int)N, gamma, gl, advantages,         \
                                                    returns, part)
#define AGX_GAE_U(UU)                                          \
    if (use_gae) {                                             \
        if (adv_stats) AGX_GAE_LAUNCH(UU, true, true);         \
        else AGX_GAE_LAUNCH(UU, true, false);                  \
    } else {                                                   \
        if (adv_stats) AGX_GAE_LAUNCH(UU, false, true);        \
        else AGX_GAE_LAUNCH(UU, false, false);                 \
    }
    if (U >= 32) {
        AGX_GAE_U(32)
    } else if (U >= 16) {
        AGX_GAE_U(16)
    } else {
        AGX_GAE_U(8)
    }
#undef AGX_GAE_U
#undef AGX_GAE_LAUNCH
    int rc = check_launch("agx_gae");
    if (rc || !adv_stats) return rc;
    gae_stats_finalize<<<(unsigned)P, 256, 0, s>>>(part, nblk, T * N, adv_stats);
    return check_launch("agx_gae stats");
}

extern "C" int agx_adv_normalize(float *adv, const double *adv_stats, int64_t P, int64_t count,
                                 void *stream) {
    AGX_REQUIRE(adv && adv_stats && P > 0 && count >= 0 && P <= 65535,
                "agx_adv_normalize: bad arguments");
    if (count == 0) return AGX_OK;
    const int64_t blocks = ceil_div(count, 256);
    dim3 grid((unsigned)(blocks > 1024 ? 1024 : blocks), (unsigned)P);
    adv_normalize_kernel<<<grid, 256, 0, as_stream(stream)>>>(adv, adv_stats, count);
    return check_launch("agx_adv_normalize");
}
