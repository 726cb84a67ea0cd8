// Rollout policy-step plumbing shared by the compiled (learner.hip) and the
// runtime-shape (graph_learner.hip) policy steps: the per-step argument block
// the persistent launches read from host memory, the Philox4x32-10 stream of
// the Gumbel-max sample, the host-staging loads, and the host side that
// fills an argument block from an agx_rollout_io.
#pragma once

#include "agx_common.h"

namespace agx {

__device__ __forceinline__ unsigned mulhilo(unsigned a, unsigned b, unsigned &hi) {
    const unsigned long long prod = (unsigned long long)a * b;
    hi = (unsigned)(prod >> 32);
    return (unsigned)prod;
}
// Philox4x32-10 (Salmon et al., SC'11)
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        unsigned h0, h1;
        const unsigned l0 = mulhilo(0xD2511F53u, c.x, h0);
        const unsigned l1 = mulhilo(0xCD9E8D57u, c.z, h1);
        c = make_uint4(h1 ^ c.y ^ k.x, l1, h0 ^ c.w ^ k.y, l0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

struct ActArgs {
    const float *params;
    const float *obs;  // agent p, env n at obs + p*obs_pstride + n*D
    long long obs_pstride;
    int N, P, sample;
    unsigned long long seed, counter;
    long long *act_out;  // agent p, env n at + p*out_pstride + n (each may be null)
    float *logp_out, *value_out, *ent_out;
    long long out_pstride;
    long long *act_flat;  // [P*N] contiguous copy (host staging) or null
    int act;              // 0: scatter only (the step after the last action)
    // rollout bookkeeping fused into the policy step (agx_ppo_rollout_step)
    float *obs_copy;      // obs also written here (rollout slot t), agent stride obs_copy_pstride
    long long obs_copy_pstride;
    const float *st_rew;  // [P*N] reward / done of the previous vector step, or null
    const unsigned char *st_done;
    float *rew_prev;      // rollout slot t-1, agent stride prev_pstride
    unsigned char *done_prev;
    long long prev_pstride;
    float *scores;        // [P*N] running episode score (on_policy.py:147-172), or null
    double *ret_sum;      // [P*N] sum of finished-episode returns
    long long *episodes;  // [P*N] finished-episode count
    // legal-action masks (1 = legal): agent p, env n at mask + p*mask_pstride + n*A, or null;
    // copied to mask_copy (rollout slot t, agent stride mask_copy_pstride) when set
    const unsigned char *mask;
    long long mask_pstride;
    unsigned char *mask_copy;
    long long mask_copy_pstride;
    const long long *env_base;  // [P] global index of each agent's env 0 (Philox stream), or null: p * N
};

// The env staging may be host memory that the host rewrites between the
// steps of one persistent launch: read it with system-scope loads, which
// bypass the vector L1 and the L2 (both may hold the previous step's lines).
__device__ __forceinline__ float ld_sys(const float *p) {
    return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned char ld_sys_u8(const unsigned char *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const unsigned w = __hip_atomic_load(reinterpret_cast<unsigned *>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
    return (unsigned char)(w >> (8 * (a & 3)));
}


// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
inline void fill_rollout_args(ActArgs &a, int D, int A, int64_t P, int64_t N, const float *params,
                              const agx_rollout_io *io, int act, int sample, uint64_t seed, uint64_t counter) {
    a.params = params;
    a.obs = io->stage_obs;
    a.obs_pstride = N * (int64_t)D;
    a.N = (int)N;
    a.P = (int)P;
    a.sample = sample;
    a.seed = seed;
    a.counter = counter;
    a.act_out = reinterpret_cast<long long *>(io->actions);
    a.logp_out = io->log_probs;
    a.value_out = io->values;
    a.ent_out = nullptr;
    a.out_pstride = io->slot_agent_stride;
    a.act_flat = reinterpret_cast<long long *>(io->actions_flat);
    a.act = act;
    a.obs_copy = io->obs_slot;
    a.obs_copy_pstride = io->obs_agent_stride;
    a.st_rew = io->stage_rew;
    a.st_done = io->stage_done;
    a.rew_prev = io->rewards_prev;
    a.done_prev = io->dones_prev;
    a.prev_pstride = io->prev_agent_stride;
    a.scores = io->scores;
    a.ret_sum = io->return_sum;
    a.episodes = reinterpret_cast<long long *>(io->episodes);
    a.mask = io->stage_mask;
    a.mask_pstride = N * (int64_t)A;
    a.mask_copy = io->mask_slot;
    a.mask_copy_pstride = io->mask_agent_stride;
    a.env_base = reinterpret_cast<const long long *>(io->agent_env_base);
}

inline int check_rollout_io(const agx_rollout_io *io, int act, const float *params, const char *who) {
    AGX_REQUIRE(io && io->stage_obs, "%s: null io / stage_obs", who);
    AGX_REQUIRE(!act || params, "%s: act needs params", who);
    AGX_REQUIRE(!io->stage_rew || (io->stage_done && io->rewards_prev && io->dones_prev),
                "%s: previous-step scatter needs rewards/dones slots", who);
    AGX_REQUIRE(!io->scores || (io->stage_rew && io->return_sum && io->episodes),
                "%s: episode accounting needs return_sum, episodes and stage rewards", who);
    return AGX_OK;
}


}  // namespace agx
