// Internal helpers shared by the libagx.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/agx.h"

namespace agx {

// persistent-rollout control block (agx.h agx_rollout_ctl): header, nwg done
// words, then one 64-byte release line per workgroup
__host__ __device__ inline unsigned *rollout_done_words(void *ctl) { return static_cast<unsigned *>(ctl) + 4; }
__host__ __device__ inline unsigned rollout_release_offset(unsigned nwg, unsigned w) {  // in words
    return ((4 + nwg + 15) / 16 + w) * 16;
}
__host__ __device__ inline unsigned *rollout_release_word(void *ctl, unsigned nwg, unsigned w) {
    return static_cast<unsigned *>(ctl) + rollout_release_offset(nwg, w);
}

// thread-local last error (agx_last_error)
void set_error(const char *fmt, ...);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch that was just queued; never synchronises.
inline int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return AGX_EHIP;
    }
    return AGX_OK;
}

#define AGX_REQUIRE(cond, ...)          \
    do {                                \
        if (!(cond)) {                  \
            ::agx::set_error(__VA_ARGS__); \
            return AGX_EINVAL;          \
        }                               \
    } while (0)

constexpr int kWave = 64;

// ---- wave-level reductions (64 lanes, xor butterflies) ------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// reduce within aligned groups of G lanes (G power of two <= 64)
template <int G, typename T>
__device__ __forceinline__ T group_sum(T v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace agx
