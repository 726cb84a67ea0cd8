// Host-side reference RNG streams the device path consumes as inputs.
//
// PPO's minibatch order comes from numpy's global legacy RandomState:
// PPO._learn_from_rollout_buffer_flat (agilerl/algorithms/ppo.py:836-842)
// does `indices = np.arange(num_samples)` once per learn() and then
// `np.random.shuffle(indices)` at the start of every epoch (cumulative: epoch
// e shuffles epoch e-1's order).  numpy 2.x implements that shuffle as
// Fisher-Yates from the top (`_shuffle_raw`: for i = n-1 .. 1, swap i with
// random_interval(i)), where random_interval(max) draws 32-bit MT19937
// outputs masked to the smallest all-ones mask >= max and rejects values >
// max.  This restates that published algorithm natively so the whole
// population's permutations ([E][P][S]) cost microseconds of host time
// instead of P*E Python-level shuffles; the caller passes the generator state
// it took from np.random.get_state() and writes the advanced state back, so
// the global numpy stream moves exactly as the reference's would.
#include <cstdint>
#include <cstring>

#include "agx_common.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

struct MT {
    uint32_t *key;
    int pos;

    void refill() {
        int i = 0;
        uint32_t y;
        for (; i < kN - kM; ++i) {
            y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        for (; i < kN - 1; ++i) {
            y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        y = (key[kN - 1] & kUpper) | (key[0] & kLower);
        key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        pos = 0;
    }
    uint32_t next32() {
        if (pos >= kN) refill();
        uint32_t y = key[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    uint64_t next64() {  // numpy mt19937_next64: high word first
        const uint64_t hi = next32();
        return (hi << 32) | next32();
    }
    // numpy random_interval(bitgen, max): uniform on [0, max] by masked rejection
    uint64_t interval(uint64_t max) {
        if (max == 0) return 0;
        uint64_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        mask |= mask >> 32;
        uint64_t v;
        if (max <= 0xffffffffull) {
            while ((v = (next32() & mask)) > max) {
            }
        } else {
            while ((v = (next64() & mask)) > max) {
            }
        }
        return v;
    }
};

}  // namespace

extern "C" int agx_host_shuffle_perms(uint32_t *mt_key, int32_t *mt_pos, int64_t P, int64_t epochs, int64_t S,
                                      const int64_t *epochs_per_agent, int64_t *perms) {
    AGX_REQUIRE(mt_key && mt_pos && perms, "agx_host_shuffle_perms: null pointer");
    AGX_REQUIRE(P > 0 && epochs > 0 && S > 0 && *mt_pos >= 0 && *mt_pos <= kN,
                "agx_host_shuffle_perms: bad arguments P=%lld epochs=%lld S=%lld pos=%d", (long long)P,
                (long long)epochs, (long long)S, (int)*mt_pos);
    if (epochs_per_agent)  // validate everything before the generator moves
        for (int64_t p = 0; p < P; ++p)
            AGX_REQUIRE(epochs_per_agent[p] >= 1 && epochs_per_agent[p] <= epochs,
                        "agx_host_shuffle_perms: agent %lld epochs %lld outside [1, %lld]", (long long)p,
                        (long long)epochs_per_agent[p], (long long)epochs);
    MT mt{mt_key, *mt_pos};
    for (int64_t p = 0; p < P; ++p) {
        int64_t *first = perms + (size_t)p * S;  // epoch 0 row of agent p
        for (int64_t i = 0; i < S; ++i) first[i] = i;
        const int64_t ep = epochs_per_agent ? epochs_per_agent[p] : epochs;
        for (int64_t e = 0; e < ep; ++e) {
            int64_t *x = perms + ((size_t)e * P + p) * S;
            if (e > 0) std::memcpy(x, perms + ((size_t)(e - 1) * P + p) * S, (size_t)S * sizeof(int64_t));
            for (int64_t i = S - 1; i >= 1; --i) {
                const int64_t j = (int64_t)mt.interval((uint64_t)i);
                const int64_t t = x[j];
                x[j] = x[i];
                x[i] = t;
            }
        }
    }
    *mt_pos = mt.pos;
    return AGX_OK;
}
