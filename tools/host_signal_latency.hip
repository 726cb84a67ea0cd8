// Host <-> device hand-off latency of a resident workgroup (the persistent
// rollout / evaluation step's signalling): the host writes a
// payload (the env step's observations) and a release word, the workgroup
// polls the release word, reads the payload and stores a done word into
// coherent host memory that the host polls.  Mean round trip per step.
//
//   mode host: release + payload in coherent host memory (hipHostMalloc), the
//              form the rollout kernels use today (each device poll and the
//              payload read cross PCIe)
//   mode vram: release + payload in fine-grained device memory written by the
//              host through the BAR (device polls and reads stay local)
//
// hipcc --offload-arch=gfx950 -O2 tools/host_signal_latency.hip -o /tmp/hsl && /tmp/hsl host 4096 && /tmp/hsl vram 4096
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void pong(unsigned *rel, const float *payload, int pay_n, unsigned *done, int iters, float *sink,
                     unsigned long long timeout_ticks) {
    __shared__ int s_go;
    float acc = 0.f;
    for (int i = 1; i <= iters; ++i) {
        if (threadIdx.x == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int go = 1;
            while (__hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < (unsigned)i) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                    go = 0;
                    break;
                }
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) {
            if (threadIdx.x == 0) __hip_atomic_store(done, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        // the payload of step i is (float)(i + j): count reads that are not (stale data)
        for (int j = threadIdx.x; j < pay_n; j += blockDim.x) {
            const float v = __hip_atomic_load(payload + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            acc += v != (float)(i + j) ? 1.f : 0.f;
        }
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(done, (unsigned)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    sink[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const bool vram = argc > 1 && strcmp(argv[1], "vram") == 0;
    const int pay_bytes = argc > 2 ? atoi(argv[2]) : 4096;
    const int iters = argc > 3 ? atoi(argv[3]) : 2000;
    const int pay_n = pay_bytes / 4;
    unsigned *done_h = nullptr, *rel = nullptr;
    float *payload = nullptr, *sink = nullptr;
    CK(hipHostMalloc((void **)&done_h, 256, hipHostMallocCoherent | hipHostMallocMapped));
    if (vram) {
        CK(hipExtMallocWithFlags((void **)&rel, 256 + (size_t)pay_bytes, hipDeviceMallocFinegrained));
    } else {
        CK(hipHostMalloc((void **)&rel, 256 + (size_t)pay_bytes, hipHostMallocCoherent | hipHostMallocMapped));
    }
    payload = reinterpret_cast<float *>(reinterpret_cast<char *>(rel) + 256);
    CK(hipMalloc((void **)&sink, 1024 * 4));
    // the host writes through the pointer (a segfault here: not host-visible)
    std::atomic_ref<unsigned>(*rel).store(0, std::memory_order_release);
    memset(payload, 0, pay_bytes);
    *done_h = 0;
    printf("mode %s: host write through the pointer ok\n", vram ? "vram" : "host");
    fflush(stdout);
    float *stage = (float *)malloc(pay_bytes);
    for (int j = 0; j < pay_n; ++j) stage[j] = (float)j;
    hipLaunchKernelGGL(pong, dim3(1), dim3(256), 0, 0, rel, payload, pay_n, done_h, iters, sink,
                       (unsigned long long)(5.0 * 1e8));
    auto t0 = std::chrono::steady_clock::now();
    bool ok = true;
    for (int i = 1; i <= iters && ok; ++i) {
        if (i == 101) t0 = std::chrono::steady_clock::now();  // 100 warm-up steps
        for (int j = 0; j < pay_n; ++j) stage[j] = (float)(i + j);
        memcpy(payload, stage, pay_bytes);
        if (vram) _mm_sfence();  // write-combined BAR: the payload lands before the release word
        std::atomic_ref<unsigned>(*rel).store((unsigned)i, std::memory_order_release);
        if (vram) _mm_sfence();  // ... and the release word leaves the write-combining buffer now
        const auto w0 = std::chrono::steady_clock::now();
        for (;;) {
            const unsigned d = std::atomic_ref<unsigned>(*done_h).load(std::memory_order_acquire);
            if (d == 0xFFFFFFFFu) {
                ok = false;
                break;
            }
            if (d >= (unsigned)i) break;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() > 5.0) {
                ok = false;
                break;
            }
        }
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!ok) std::atomic_ref<unsigned>(*rel).store(0x7FFFFFFFu, std::memory_order_release);  // let the kernel finish
    CK(hipDeviceSynchronize());
    float hs[256];
    CK(hipMemcpy(hs, sink, sizeof(hs), hipMemcpyDeviceToHost));
    double stale = 0;
    for (int t = 0; t < 256; ++t) stale += hs[t];
    printf("mode %s payload %d B: %s, %.2f us per round trip over %d steps (host step includes writing the payload); "
           "stale payload words read: %.0f\n", vram ? "vram" : "host", pay_bytes, ok ? "ok" : "TIMEOUT",
           1e6 * dt / (iters - 100), iters - 100, stale);
    return ok ? 0 : 1;
}
