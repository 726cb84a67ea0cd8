// Microbenchmark (diagnostic): shader-clock cycles of the building blocks of
// the few-row forward on gfx950 -- dependent LDS reads, a batch of
// independent LDS reads, a 4-wave barrier, a dependent chain of 16 f32 MFMAs,
// a 16-lane DPP sum, a correctly rounded 1/sqrt.  One workgroup of 4 waves;
// wave 0 lane 0 reports.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_latency tools/lds_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

__global__ __launch_bounds__(256) void bench(long long *out, float *sink, int n, const int *__restrict__ chase) {
    __shared__ float lds[16384];
    const int tid = threadIdx.x;
    for (int i = tid; i < 16384; i += 256) lds[i] = (float)(i & 7) * 0.f + (i & 1 ? 1.f : 0.f);
    __syncthreads();
    long long t[16];
    float acc = 0.f;
    int idx = tid & 63;
    // 1: 32 dependent LDS reads (pointer chase through integer indices)
    t[0] = __builtin_readcyclecounter();
    for (int i = 0; i < 32; ++i) idx = (int)lds[idx] + ((idx + 64) & 4095);
    acc += idx;
    t[1] = __builtin_readcyclecounter() + (acc == -1.f);
    // 2: 24 independent LDS reads then their sum
    float v[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) v[i] = lds[(tid * 17 + i * 68) & 16383];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 24; ++i) s += v[i];
    acc += s;
    t[2] = __builtin_readcyclecounter() + (acc == -1.f);
    // 3: a barrier
    __syncthreads();
    t[3] = __builtin_readcyclecounter();
    // 4: 16 dependent MFMAs 16x16x4 f32
    f4 c = {0.f, 0.f, 0.f, 0.f};
    const float a = lds[tid], b = lds[tid + 1];
#pragma unroll
    for (int i = 0; i < 16; ++i) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    acc += c[0] + c[1] + c[2] + c[3];
    t[4] = __builtin_readcyclecounter() + (acc == -1.f);
    // 5: 16-lane DPP sum
    float r = acc;
    r += dpp<0xb1>(r);
    r += dpp<0x4e>(r);
    r += dpp<0x141>(r);
    r += dpp<0x140>(r);
    acc += r;
    t[5] = __builtin_readcyclecounter() + (acc == -1.f);
    // 6: correctly rounded 1 / sqrtf
    acc = 1.f / sqrtf(acc * acc / 64.f + 1e-5f);
    t[6] = __builtin_readcyclecounter() + (acc == -1.f);
    // 7: 8 LDS writes + barrier
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[(tid * 8 + i) & 16383] = acc + i;
    __syncthreads();
    t[7] = __builtin_readcyclecounter();
    // 8: a global store then a read of the clock
    sink[tid] = acc;
    t[8] = __builtin_readcyclecounter();
    // 9: one LDS read -> use
    float w = lds[(tid * 3) & 16383];
    acc += w;
    t[9] = __builtin_readcyclecounter() + (acc == -1.f);
    // 10: 16 independent MFMAs on 4 accumulators (4 chains of 4)
    f4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    acc += c0[0] + c1[1] + c2[2] + c3[3];
    t[10] = __builtin_readcyclecounter() + (acc == -1.f);
    // 11: 4 ds_read_b128 then use
    const f4 *l4 = reinterpret_cast<const f4 *>(lds);
    f4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = l4[(tid * 17 + i * 16) & 4095];
    acc += q[0][0] + q[1][1] + q[2][2] + q[3][3];
    t[11] = __builtin_readcyclecounter() + (acc == -1.f);
    // 12: 16 dependent scalar loads (uniform pointer chase, read-only buffer)
    int u = n;
    for (int i = 0; i < 16; ++i) u = chase[u];
    acc += u;
    t[12] = __builtin_readcyclecounter() + (acc == -1.f);
    // 13: 16 dependent vector loads (per-lane chase, L2 / L1 hits after the first pass)
    int vv = chase[(tid & 7) + n];
    for (int i = 0; i < 16; ++i) vv = chase[vv + (tid & 1)];
    acc += vv;
    t[13] = __builtin_readcyclecounter() + (acc == -1.f);
    sink[256 + tid] = acc;
    if (tid == 0)
        for (int i = 0; i < 13; ++i) out[i] = t[i + 1] - t[i];
}


__device__ __forceinline__ float rsum16(float v) {
    v += dpp<0xb1>(v);
    v += dpp<0x4e>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}

// the few-row forward's LayerNorm + affine + ReLU row pass (F = 64, 16 rows of
// stride 68), 8 registers per lane; 4 repetitions, each stamped
__global__ __launch_bounds__(256) void rowpass(long long *out, float *sink, const int *__restrict__ cfg) {
    __shared__ float S[4096];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, rq = lane >> 4, row = 4 * wave + rq;
    for (int i = tid; i < 4096; i += 256) S[i] = (float)((i * 37) % 101) * 0.01f;
    __syncthreads();
    const int F = cfg[0], ld = cfg[1], ln = cfg[2], relu = cfg[3];
    const int af = cfg[4];
    long long t[9];
    for (int rep = 0; rep < 4; ++rep) {
        t[2 * rep] = __builtin_readcyclecounter();
        float *y = S + row * ld;
        constexpr int M = 4;
        const int mp = (F + 15) >> 4;
        float v[M], ga[M], be[M];
        bool ok[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int j = sub + 16 * i;
            ok[i] = j < F;
            v[i] = ga[i] = be[i] = 0.f;
            if (i < mp) {
                v[i] = y[j];
                if (ln == 2) {
                    ga[i] = S[af + j];
                    be[i] = S[af + F + j];
                }
            }
        }
        long long ta = __builtin_readcyclecounter();
        float mean = 0.f, rstd = 1.f;
        if (ln) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < M; ++i) s = ok[i] ? s + v[i] : s;
            mean = rsum16(s) * (1.f / (float)F);
            float vs = 0.f;
#pragma unroll
            for (int i = 0; i < M; ++i) {
                const float d = v[i] - mean;
                vs = ok[i] ? vs + d * d : vs;
            }
            rstd = 1.f / sqrtf(rsum16(vs) / (float)F + 1e-5f);
        }
        long long tb = __builtin_readcyclecounter() + (rstd == 7.f);
#pragma unroll
        for (int i = 0; i < M; ++i) {
            if (i >= mp) break;
            const int j = sub + 16 * i;
            float x = v[i];
            if (ln) {
                const float xh = (x - mean) * rstd;
                x = ln == 2 ? xh * ga[i] + be[i] : xh;
            }
            if (relu) x = fmaxf(x, 0.f);
            y[j] = ok[i] ? x * 0.5f : 0.f;
        }
        if (rep == 3 && tid == 0) { out[20] = ta - t[2 * rep]; out[21] = tb - ta; }
        t[2 * rep + 1] = __builtin_readcyclecounter();
        __syncthreads();
    }
    t[8] = __builtin_readcyclecounter();
    if (tid == 0)
        for (int i = 0; i < 8; ++i) out[i] = t[i + 1] - t[i];
    sink[tid] = S[tid];
}

int main() {
    long long *out;
    float *sink;
    if (hipMalloc(&out, 64 * sizeof(long long)) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    int *chase;
    if (hipMalloc(&chase, 4096 * sizeof(int)) != hipSuccess) return 1;
    int hc[4096];
    for (int i = 0; i < 4096; ++i) hc[i] = (i * 97 + 64) & 1023;
    if (hipMemcpy(chase, hc, sizeof(hc), hipMemcpyHostToDevice) != hipSuccess) return 1;
    long long h[13];
    const char *names[13] = {"32 dependent LDS reads", "24 independent LDS reads + sum", "barrier (4 waves)",
                             "16 dependent MFMA 16x16x4 f32", "16-lane DPP sum", "1/sqrtf (correctly rounded)",
                             "8 LDS writes + barrier", "global store", "one LDS read -> use",
                             "16 MFMA on 4 accumulators", "4 ds_read_b128 -> use",
                             "16 dependent scalar loads", "16 dependent vector loads"};
    for (int rep = 0; rep < 3; ++rep) {
        bench<<<1, 256>>>(out, sink, 0, chase);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
        printf("rep %d\n", rep);
        for (int i = 0; i < 13; ++i) printf("  %-34s %6lld cycles\n", names[i], h[i]);
    }
    int hcfg[5] = {64, 68, 2, 1, 2048};
    if (hipMemcpy(chase, hcfg, sizeof(hcfg), hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        rowpass<<<1, 256>>>(out, sink, chase);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        long long h2[22];
        if (hipMemcpy(h2, out, sizeof(h2), hipMemcpyDeviceToHost) != hipSuccess) return 3;
        printf("row pass (F 64, LN + affine + ReLU): row pass / barrier cycles:");
        for (int i = 0; i < 8; ++i) printf(" %lld", h2[i]);
        printf("; last rep: loads %lld, stats %lld", h2[20], h2[21]);
        printf("\n");
    }
    return 0;
}
