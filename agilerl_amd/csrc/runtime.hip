// Library-level entry points: error reporting, version, device info.
#include <chrono>
#include <cstring>

#include "agx_common.h"

namespace agx {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace agx

extern "C" const char *agx_last_error(void) { return agx::g_err; }

extern "C" int agx_version(void) { return 100; /* 0.1.0 */ }

extern "C" int agx_device_info(int *out3) {
    if (!out3) {
        agx::set_error("agx_device_info: null output");
        return AGX_EINVAL;
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        agx::set_error("agx_device_info: %s", hipGetErrorString(e));
        return AGX_EHIP;
    }
    out3[0] = prop.multiProcessorCount;
    int arch = 0;  // "gfx950:sramecc+:xnack-" -> 950
    for (const char *c = prop.gcnArchName + 3; *c >= '0' && *c <= '9'; ++c) arch = arch * 10 + (*c - '0');
    out3[1] = arch;
    out3[2] = prop.warpSize;
    return AGX_OK;
}

// STREAM-style kernels used by bench.py to measure the box's achievable HBM
// bandwidth (the roofline's "measured peak"): 16 B per lane, each block moves
// one contiguous 16 KiB tile per pass (4 loads in flight per lane).
//   mode 0: copy (read + write), nontemporal stores
//   mode 1: read-only (sum into one float per block, written once)
namespace agx {
typedef float v4f __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(256) void stream_kernel(const v4f *__restrict__ src, v4f *__restrict__ dst, int64_t n4) {
    constexpr int U = 4;
    const int64_t tile = (int64_t)blockDim.x * U;
    v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
    for (int64_t base = (int64_t)blockIdx.x * tile; base < n4; base += (int64_t)gridDim.x * tile) {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * blockDim.x + threadIdx.x;
            v[u] = i < n4 ? src[i] : v4f{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * blockDim.x + threadIdx.x;
            if (MODE == 0) {
                if (i < n4) __builtin_nontemporal_store(v[u], dst + i);
            } else {
                acc += v[u];
            }
        }
    }
    if (MODE == 1) {
        const float t = acc.x + acc.y + acc.z + acc.w;
        if (t == 12345.678f) dst[blockIdx.x] = acc;  // keeps the loads live; practically never stores
    }
}
}  // namespace agx

extern "C" int agx_debug_stream(const void *src, void *dst, int64_t bytes, int mode, int64_t grid, void *stream) {
    AGX_REQUIRE(src && dst && bytes > 0 && bytes % 16 == 0 && (mode == 0 || mode == 1) && grid >= 0,
                "agx_debug_stream: bad arguments");
    const int64_t n4 = bytes / 16;
    const int64_t tiles = agx::ceil_div(n4, 1024);
    const unsigned g = (unsigned)(grid > 0 && grid < tiles ? grid : tiles);
    if (mode == 0)
        agx::stream_kernel<0><<<g, 256, 0, agx::as_stream(stream)>>>(static_cast<const agx::v4f *>(src),
                                                                    static_cast<agx::v4f *>(dst), n4);
    else
        agx::stream_kernel<1><<<g, 256, 0, agx::as_stream(stream)>>>(static_cast<const agx::v4f *>(src),
                                                                    static_cast<agx::v4f *>(dst), n4);
    return agx::check_launch("agx_debug_stream");
}

// ---- coherent host memory and the persistent-rollout handshake (host side) ----
extern "C" void *agx_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        agx::set_error("agx_host_alloc: hipHostMalloc(%zu, coherent) failed", bytes);
        return nullptr;
    }
    std::memset(p, 0, bytes);
    return p;
}

extern "C" int agx_host_free(void *ptr) {
    if (!ptr) return AGX_OK;
    if (hipHostFree(ptr) != hipSuccess) {
        (void)hipGetLastError();
        agx::set_error("agx_host_free: hipHostFree failed");
        return AGX_EHIP;
    }
    return AGX_OK;
}

extern "C" void *agx_stream_create(void) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        agx::set_error("agx_stream_create: hipStreamCreateWithFlags failed");
        return nullptr;
    }
    return s;
}

extern "C" int agx_host_signal(agx_rollout_ctl *ctl, uint32_t seq) {
    AGX_REQUIRE(ctl, "agx_host_signal: null ctl");
    const unsigned nwg = __atomic_load_n(&ctl->nwg, __ATOMIC_RELAXED);
    for (unsigned w = 0; w < nwg; ++w) __atomic_store_n(agx::rollout_release_word(ctl, nwg, w), seq, __ATOMIC_RELEASE);
    __atomic_store_n(&ctl->seq, seq, __ATOMIC_RELEASE);
    return AGX_OK;
}

extern "C" int agx_host_signal_range(agx_rollout_ctl *ctl, int64_t w0, int64_t w1, uint32_t seq) {
    AGX_REQUIRE(ctl, "agx_host_signal_range: null ctl");
    const unsigned nwg = __atomic_load_n(&ctl->nwg, __ATOMIC_RELAXED);
    AGX_REQUIRE(w0 >= 0 && w0 <= w1 && w1 <= (int64_t)nwg, "agx_host_signal_range: [%lld, %lld) outside %u",
                (long long)w0, (long long)w1, nwg);
    for (int64_t w = w0; w < w1; ++w)
        __atomic_store_n(agx::rollout_release_word(ctl, nwg, (unsigned)w), seq, __ATOMIC_RELEASE);
    return AGX_OK;
}

extern "C" int agx_host_wait_range(const agx_rollout_ctl *ctl, int64_t w0, int64_t w1, uint32_t target,
                                   double timeout_s) {
    AGX_REQUIRE(ctl && w0 >= 0 && w0 < w1, "agx_host_wait_range: bad arguments");
    const uint32_t *done = agx::rollout_done_words(const_cast<agx_rollout_ctl *>(ctl));
    const auto t0 = std::chrono::steady_clock::now();
    int64_t i = w0;
    for (unsigned spin = 0;; ++spin) {
        while (i < w1 && __atomic_load_n(done + i, __ATOMIC_ACQUIRE) >= target) ++i;
        if (i == w1) return AGX_OK;
        if (__atomic_load_n(&ctl->timeout, __ATOMIC_RELAXED)) {
            agx::set_error("agx_host_wait_range: a workgroup timed out waiting for the host");
            return AGX_EHIP;
        }
        if ((spin & 1023) == 1023 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            agx::set_error("agx_host_wait_range: %lld of [%lld, %lld) not done after %.1f s", (long long)(w1 - i),
                           (long long)w0, (long long)w1, timeout_s);
            return AGX_EHIP;
        }
        __builtin_ia32_pause();
    }
}

// release [s0, s1) to seq, then wait until [w0, w1) reach target: one call
// for the pipelined pass's hand-over from one part to the next
extern "C" int agx_host_signal_wait_range(agx_rollout_ctl *ctl, int64_t s0, int64_t s1, uint32_t seq, int64_t w0,
                                          int64_t w1, uint32_t target, double timeout_s) {
    const int rc = agx_host_signal_range(ctl, s0, s1, seq);
    return rc != AGX_OK ? rc : agx_host_wait_range(ctl, w0, w1, target, timeout_s);
}

extern "C" int agx_host_wait(const agx_rollout_ctl *ctl, int64_t nwg, uint32_t target, double timeout_s) {
    AGX_REQUIRE(ctl && nwg > 0, "agx_host_wait: bad arguments");
    const uint32_t *done = agx::rollout_done_words(const_cast<agx_rollout_ctl *>(ctl));
    const auto t0 = std::chrono::steady_clock::now();
    int64_t i = 0;
    for (unsigned spin = 0;; ++spin) {
        while (i < nwg && __atomic_load_n(done + i, __ATOMIC_ACQUIRE) >= target) ++i;
        if (i == nwg) return AGX_OK;
        if (__atomic_load_n(&ctl->timeout, __ATOMIC_RELAXED)) {
            agx::set_error("agx_host_wait: a rollout workgroup timed out waiting for the host");
            return AGX_EHIP;
        }
        if ((spin & 1023) == 1023 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            agx::set_error("agx_host_wait: %lld of %lld workgroups not done after %.1f s", (long long)(nwg - i),
                           (long long)nwg, timeout_s);
            return AGX_EHIP;
        }
        __builtin_ia32_pause();
    }
}
