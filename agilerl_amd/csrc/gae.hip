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
// hidden by this per-lane ILP rather than by occupancy (U = 32 at T >= 64).
// All memory ops are buffer ops on per-agent descriptors: the row offset
// t*N*4 is wave-uniform (SGPR soffset), the column offset one VGPR, so the
// 3U in-flight loads need no 64-bit address registers each.
// Algorithmic bytes: 4 (r) + 1 (done) + 4 (v) in, 4 (adv) + 4 (ret) out = 17 B
// per transition.
#include <cstdlib>

#include "agx_common.h"

namespace agx {

constexpr int kGaeBlock = 256;

// C adjacent columns per lane (C = 2: 8-byte r/v loads, 2-byte done loads,
// 8-byte stores — half the memory instructions of C = 1).
template <int C>
struct alignas(4 * C) FV {
    float v[C];
};
template <int C>
struct alignas(C) BV {
    uint8_t v[C];
};

template <int kGaeU, int C, bool kGae, bool kStats>
__global__ __launch_bounds__(kGaeBlock) void gae_kernel(
    const float *__restrict__ rewards, const uint8_t *__restrict__ dones,
    const float *__restrict__ values, const float *__restrict__ last_value,
    const uint8_t *__restrict__ last_done, int T, int N, double gamma, double gl,
    float *__restrict__ adv, float *__restrict__ ret, double *__restrict__ partials) {
    const int p = blockIdx.y;
    const int n = (blockIdx.x * kGaeBlock + threadIdx.x) * C;
    const bool live = n < N;
    const int nn = live ? n : N - C;  // dead lanes shadow a live column group, store nothing
    const float g32 = (float)gamma;
    // Buffer descriptors over this agent's [T][N] planes: the row offset t*N is
    // wave-uniform and goes in soffset (an SGPR), the lane's column offset in
    // one voffset VGPR — no 64-bit address per in-flight load (the flat form
    // needed ~190 VGPRs of addresses at U = 16).  Requires T*N*4 < 2^32.
    const size_t plane = (size_t)T * N;
    const auto rs_r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(rewards) + (size_t)p * plane, 0,
                                                        (int)(plane * 4), 0x00020000);
    const auto rs_v = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(values) + (size_t)p * plane, 0,
                                                        (int)(plane * 4), 0x00020000);
    const auto rs_d = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(dones) + (size_t)p * plane, 0,
                                                        (int)plane, 0x00020000);
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(adv + (size_t)p * plane, 0, (int)(plane * 4), 0x00020000);
    const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(ret + (size_t)p * plane, 0, (int)(plane * 4), 0x00020000);
    const int vo4 = nn * 4, vo1 = nn;
    auto ldf = [&](const decltype(rs_r) &rs, int t) {
        FV<C> x;
        if constexpr (C == 1) {
            x.v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo4, t * N * 4, 0));
        } else {
            // two dword loads: this toolchain drops the second element of the
            // 2-vector raw_buffer_load_b64 result (loads one dword, reuses it)
            x.v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo4, t * N * 4, 0));
            x.v[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo4 + 4, t * N * 4, 0));
        }
        return x;
    };
    auto ldb = [&](int t) {
        BV<C> x;
        if constexpr (C == 1) {
            x.v[0] = __builtin_amdgcn_raw_buffer_load_b8(rs_d, vo1, t * N, 0);
        } else {
            // two byte loads (this toolchain's raw_buffer_load_b16 result was
            // unpacked from the wrong half: the high byte came out as 0)
            x.v[0] = __builtin_amdgcn_raw_buffer_load_b8(rs_d, vo1, t * N, 0);
            x.v[1] = __builtin_amdgcn_raw_buffer_load_b8(rs_d, vo1 + 1, t * N, 0);
        }
        return x;
    };
    auto stf = [&](const decltype(rs_r) &rs, int t, const FV<C> &x) {
        if constexpr (C == 1) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x.v[0]), rs, vo4, t * N * 4, 0);
        } else {
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
            const u2 u = {__builtin_bit_cast(unsigned, x.v[0]), __builtin_bit_cast(unsigned, x.v[1])};
            __builtin_amdgcn_raw_buffer_store_b64(u, rs, vo4, t * N * 4, 0);  // (stores are fine)
        }
    };

    double c[C];
    float v_next[C];     // values[t+1]
    double nnt_next[C];  // 1 - done[t+1] of the step above
    double lv[C], ld[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        lv[k] = (double)last_value[(size_t)p * N + nn + k];
        ld[k] = (double)last_done[(size_t)p * N + nn + k];
    }
    double s1 = 0.0, s2 = 0.0;

    // ---- one step ---------------------------------------------------------
    auto step = [&](int t, const FV<C> &r, const FV<C> &v, const BV<C> &d, bool top) {
        FV<C> av, rv;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            if (kGae) {
                double nnt, gv;
                if (top) {
                    nnt = 1.0 - ld[k];
                    gv = gamma * lv[k];
                } else {
                    nnt = nnt_next[k];
                    gv = (double)(g32 * v_next[k]);
                }
                const double delta = ((double)r.v[k] + gv * nnt) - (double)v.v[k];
                c[k] = delta + (gl * nnt) * c[k];
                const float a = (float)c[k];
                av.v[k] = a;
                rv.v[k] = a + v.v[k];
                v_next[k] = v.v[k];
                nnt_next[k] = 1.0 - (double)d.v[k];
            } else {
                c[k] = (double)r.v[k] + (gamma * c[k]) * (1.0 - (double)d.v[k]);
                const float rt = (float)c[k];
                rv.v[k] = rt;
                av.v[k] = rt - v.v[k];
            }
            if (kStats && live) {
                s1 += (double)av.v[k];
                s2 += (double)av.v[k] * (double)av.v[k];
            }
        }
        if (live) {
            stf(rs_a, t, av);
            stf(rs_t, t, rv);
        }
    };

#pragma unroll
    for (int k = 0; k < C; ++k) {
        c[k] = kGae ? 0.0 : lv[k] * (1.0 - ld[k]);
        v_next[k] = 0.0f;
        nnt_next[k] = 1.0;
    }

    // partial head chunk so the rest is whole chunks of U
    int t = T - 1;
    const int head = T % kGaeU;
    for (int i = 0; i < head; ++i, --t) step(t, ldf(rs_r, t), ldf(rs_v, t), ldb(t), t == T - 1);
    if (t < 0) goto reduce;
    {
        FV<C> ra[kGaeU], va[kGaeU];
        BV<C> da[kGaeU];
#pragma unroll
        for (int i = 0; i < kGaeU; ++i) {
            ra[i] = ldf(rs_r, t - i);
            va[i] = ldf(rs_v, t - i);
            da[i] = ldb(t - i);
        }
        while (true) {
            const int tn = t - kGaeU;  // top of the next chunk
            FV<C> rb[kGaeU], vb[kGaeU];
            BV<C> db[kGaeU];
            if (tn >= 0) {
#pragma unroll
                for (int i = 0; i < kGaeU; ++i) {
                    rb[i] = ldf(rs_r, tn - i);
                    vb[i] = ldf(rs_v, tn - i);
                    db[i] = ldb(tn - i);
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

static int gae_cols(int64_t N) {
    // measured on MI355X at P8 T1024 N8192 (tools/gae_sweep.py): 1 column per
    // lane 4.78 TB/s vs 2.67 for 2 (half the waves) at U = 32
    int c = 1;
    if (const char *e = getenv("AGX_GAE_COLS")) c = atoi(e);
    return (c == 2 && N % 2 == 0) ? 2 : 1;
}

extern "C" size_t agx_gae_workspace_bytes(int64_t P, int64_t T, int64_t N) {
    (void)T;
    // sized for the 1-column layout (the most blocks)
    return (size_t)P * (size_t)ceil_div(N, kGaeBlock) * 2 * sizeof(double);
}

extern "C" int agx_gae(const float *rewards, const uint8_t *dones, const float *values,
                       const float *last_value, const uint8_t *last_done, int64_t P, int64_t T,
                       int64_t N, double gamma, double gae_lambda, int use_gae, float *advantages,
                       float *returns, double *adv_stats, void *workspace, void *stream) {
    AGX_REQUIRE(P > 0 && T > 0 && N > 0, "agx_gae: empty shape P=%lld T=%lld N=%lld",
                (long long)P, (long long)T, (long long)N);
    AGX_REQUIRE(P <= 65535 && T * N < (int64_t)1 << 30, "agx_gae: shape too large (T*N must be < 2^30)");
    AGX_REQUIRE(rewards && dones && values && last_value && last_done && advantages && returns,
                "agx_gae: null pointer");
    AGX_REQUIRE(!adv_stats || workspace, "agx_gae: adv_stats needs a workspace");
    hipStream_t s = as_stream(stream);
    const int C = gae_cols(N);
    const int nblk = (int)ceil_div(ceil_div(N, C), kGaeBlock);
    dim3 grid(nblk, (unsigned)P);
    const double gl = gamma * gae_lambda;
    double *part = static_cast<double *>(workspace);
    // prefetch depth: deeper register pipelines for long scans (per-lane ILP is
    // what hides HBM latency at 1-4 waves per SIMD); AGX_GAE_UNROLL overrides.
    // measured (buffer-load form, 1 column): U8 3.67, U16 4.29, U32 4.78 TB/s
    int U = T >= 64 ? 32 : (T >= 32 ? 16 : 8);
    if (const char *e = getenv("AGX_GAE_UNROLL")) U = atoi(e);
#define AGX_GAE_LAUNCH(UU, CC, G, S)                                                                    \
    gae_kernel<UU, CC, G, S><<<grid, kGaeBlock, 0, s>>>(rewards, dones, values, last_value, last_done, \
                                                        (int)T, (int)N, gamma, gl, advantages, returns, \
                                                        part)
#define AGX_GAE_U(UU, CC)                                      \
    if (use_gae) {                                             \
        if (adv_stats) AGX_GAE_LAUNCH(UU, CC, true, true);     \
        else AGX_GAE_LAUNCH(UU, CC, true, false);              \
    } else {                                                   \
        if (adv_stats) AGX_GAE_LAUNCH(UU, CC, false, true);    \
        else AGX_GAE_LAUNCH(UU, CC, false, false);             \
    }
#define AGX_GAE_C(UU)          \
    if (C == 2) {              \
        AGX_GAE_U(UU, 2)       \
    } else {                   \
        AGX_GAE_U(UU, 1)       \
    }
    if (U >= 32) {
        AGX_GAE_C(32)
    } else if (U >= 16) {
        AGX_GAE_C(16)
    } else {
        AGX_GAE_C(8)
    }
#undef AGX_GAE_C
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
