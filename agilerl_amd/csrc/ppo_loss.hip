// PPO clipped-surrogate loss: forward reductions + elementwise backward.
//
// Reference: agilerl/algorithms/ppo.py:868-902 (PPO._learn_from_rollout_buffer_flat)
//   ratio = exp(logp - old_logp)
//   pg    = mean(max(-A*ratio, -A*clamp(ratio, 1-e, 1+e)))
//   vclip = old_v + clamp(v - old_v, -e, e)
//   vl    = 0.5 * mean(max((v-R)^2, (vclip-R)^2))
//   loss  = pg + vf*vl - ent*mean(H);  approx_kl = mean((ratio-1) - log_ratio)
// and torch autograd's backward of it: maximum() splits ties 1/2:1/2, clamp()
// passes the gradient on the closed interval.  The per-sample gradients need
// only per-sample values and 1/b, so the backward is elementwise; the
// per-minibatch means are reported (loss.item(), KL early stop).
//
// Mapping: a group of G lanes owns one minibatch; each lane walks it in
// strides of 4*G samples with 16-byte vector loads (vector path: b % 4 == 0,
// 16-B aligned, no gather) or G samples with scalar loads (gather path, used
// when the shuffled minibatch index is applied here).  Group reductions are
// xor butterflies inside the wave — no LDS, no atomics, deterministic.
// Algorithmic bytes: 7 x 4 B in + 3 x 4 B out = 40 B per sample·epoch.
#include "agx_common.h"

namespace agx {

struct LossCoef {
    float lo, hi, clip, vf_half_inv_b, inv_b, g_h, vf, ent;
};

struct Acc {
    float pg = 0.f, vl = 0.f, h = 0.f, kl = 0.f, cf = 0.f;
};

__device__ __forceinline__ void loss_sample(float lp, float olp, float A, float R, float ov,
                                            float v, float H, const LossCoef &k, float &g_lp,
                                            float &g_v, Acc &acc) {
    const float lr = lp - olp;
    const float ratio = expf(lr);
    const float rc = fminf(fmaxf(ratio, k.lo), k.hi);
    const float p1 = -A * ratio;
    const float p2 = -A * rc;
    const float g1 = p1 > p2 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
    const float g2 = p2 > p1 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
    const float inr = (ratio >= k.lo && ratio <= k.hi) ? 1.f : 0.f;
    g_lp = ((g1 * -A + g2 * -A * inr) * k.inv_b) * ratio;
    const float dv = v - ov;
    const float dvc = fminf(fmaxf(dv, -k.clip), k.clip);
    const float vc = ov + dvc;
    const float eu = v - R;
    const float ec = vc - R;
    const float lu = eu * eu;
    const float lc = ec * ec;
    const float gu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
    const float gc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
    const float inv = (dv >= -k.clip && dv <= k.clip) ? 1.f : 0.f;
    g_v = k.vf_half_inv_b * (gu * 2.f * eu + gc * 2.f * ec * inv);
    acc.pg += fmaxf(p1, p2);
    acc.vl += fmaxf(lu, lc);
    acc.h += H;
    acc.kl += (ratio - 1.f) - lr;
    acc.cf += fabsf(ratio - 1.f) > k.clip ? 1.f : 0.f;
}

template <int G>
__device__ __forceinline__ void finish_group(Acc acc, const LossCoef &k, int64_t m, int lane_g,
                                             float *__restrict__ stats) {
    acc.pg = group_sum<G>(acc.pg);
    acc.vl = group_sum<G>(acc.vl);
    acc.h = group_sum<G>(acc.h);
    acc.kl = group_sum<G>(acc.kl);
    acc.cf = group_sum<G>(acc.cf);
    if (lane_g == 0 && stats) {
        const float pg = acc.pg * k.inv_b;
        const float vl = 0.5f * acc.vl * k.inv_b;
        const float el = -acc.h * k.inv_b;
        float *s = stats + m * 8;
        s[0] = pg + k.vf * vl + k.ent * el;
        s[1] = pg;
        s[2] = vl;
        s[3] = el;
        s[4] = acc.kl * k.inv_b;
        s[5] = acc.cf * k.inv_b;
        s[6] = 0.f;
        s[7] = 0.f;
    }
}

template <int G>
__global__ __launch_bounds__(256) void ppo_loss_vec(
    const float *__restrict__ logp, const float *__restrict__ old_logp,
    const float *__restrict__ adv, const float *__restrict__ ret,
    const float *__restrict__ old_v, const float *__restrict__ value,
    const float *__restrict__ ent, int64_t b, int64_t nmb, LossCoef k,
    float *__restrict__ g_logp, float *__restrict__ g_v, float *__restrict__ g_h,
    float *__restrict__ stats) {
    const int64_t m = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
    const int lg = threadIdx.x % G;
    if (m >= nmb) return;  // whole groups exit together
    Acc acc;
    const int64_t base = m * b;
    const float4 gh4 = make_float4(k.g_h, k.g_h, k.g_h, k.g_h);
    for (int64_t j = 4 * lg; j < b; j += 4 * G) {
        const int64_t o = (base + j) >> 2;
        const float4 lp = reinterpret_cast<const float4 *>(logp)[o];
        const float4 ol = reinterpret_cast<const float4 *>(old_logp)[o];
        const float4 A = reinterpret_cast<const float4 *>(adv)[o];
        const float4 R = reinterpret_cast<const float4 *>(ret)[o];
        const float4 ov = reinterpret_cast<const float4 *>(old_v)[o];
        const float4 v = reinterpret_cast<const float4 *>(value)[o];
        const float4 H = reinterpret_cast<const float4 *>(ent)[o];
        float4 gl, gv;
        loss_sample(lp.x, ol.x, A.x, R.x, ov.x, v.x, H.x, k, gl.x, gv.x, acc);
        loss_sample(lp.y, ol.y, A.y, R.y, ov.y, v.y, H.y, k, gl.y, gv.y, acc);
        loss_sample(lp.z, ol.z, A.z, R.z, ov.z, v.z, H.z, k, gl.z, gv.z, acc);
        loss_sample(lp.w, ol.w, A.w, R.w, ov.w, v.w, H.w, k, gl.w, gv.w, acc);
        reinterpret_cast<float4 *>(g_logp)[o] = gl;
        reinterpret_cast<float4 *>(g_v)[o] = gv;
        reinterpret_cast<float4 *>(g_h)[o] = gh4;
    }
    finish_group<G>(acc, k, m, lg, stats);
}

template <int G>
__global__ __launch_bounds__(256) void ppo_loss_gather(
    const float *__restrict__ logp, const float *__restrict__ old_logp,
    const float *__restrict__ adv, const float *__restrict__ ret,
    const float *__restrict__ old_v, const float *__restrict__ value,
    const float *__restrict__ ent, const int64_t *__restrict__ index, int64_t b, int64_t nmb,
    LossCoef k, float *__restrict__ g_logp, float *__restrict__ g_v, float *__restrict__ g_h,
    float *__restrict__ stats) {
    const int64_t m = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
    const int lg = threadIdx.x % G;
    if (m >= nmb) return;
    Acc acc;
    const int64_t base = m * b;
    for (int64_t j = lg; j < b; j += G) {
        const int64_t o = base + j;
        const int64_t src = index ? index[o] : o;
        float gl, gv;
        loss_sample(logp[o], old_logp[src], adv[src], ret[src], old_v[src], value[o], ent[o], k,
                    gl, gv, acc);
        g_logp[o] = gl;
        g_v[o] = gv;
        g_h[o] = k.g_h;
    }
    finish_group<G>(acc, k, m, lg, stats);
}

}  // namespace agx

using namespace agx;

static inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

extern "C" int agx_ppo_loss_fwd_bwd(const float *logp, const float *old_logp, const float *adv,
                                    const float *ret, const float *old_value, const float *value,
                                    const float *entropy, const int64_t *index, int64_t batch,
                                    int64_t num_minibatches, float clip_coef, float vf_coef,
                                    float ent_coef, float *g_logp, float *g_value,
                                    float *g_entropy, float *stats, void *stream) {
    AGX_REQUIRE(batch > 0 && num_minibatches >= 0, "agx_ppo_loss_fwd_bwd: bad batch %lld x %lld",
                (long long)batch, (long long)num_minibatches);
    AGX_REQUIRE(logp && old_logp && adv && ret && old_value && value && entropy && g_logp &&
                    g_value && g_entropy,
                "agx_ppo_loss_fwd_bwd: null pointer");
    if (num_minibatches == 0) return AGX_OK;
    LossCoef k;
    k.clip = clip_coef;
    k.lo = 1.f - clip_coef;
    k.hi = 1.f + clip_coef;
    k.inv_b = 1.f / (float)batch;
    k.vf = vf_coef;
    k.ent = ent_coef;
    k.vf_half_inv_b = vf_coef * 0.5f * k.inv_b;
    k.g_h = -ent_coef * k.inv_b;
    hipStream_t s = as_stream(stream);
    const bool vec = !index && batch % 4 == 0 && aligned16(logp) && aligned16(old_logp) &&
                     aligned16(adv) && aligned16(ret) && aligned16(old_value) &&
                     aligned16(value) && aligned16(entropy) && aligned16(g_logp) &&
                     aligned16(g_value) && aligned16(g_entropy);
    const int64_t per = vec ? batch / 4 : batch;  // lane-iterations per minibatch at G=1
    int G = 64;
    if (per < 64) G = 32;
    if (per < 32) G = 16;
    if (per < 16) G = 8;
    const int64_t blocks = ceil_div(num_minibatches, 256 / G);
    AGX_REQUIRE(blocks < ((int64_t)1 << 31), "agx_ppo_loss_fwd_bwd: too many minibatches");
#define AGX_LOSS(GG)                                                                           \
    case GG:                                                                                   \
        if (vec)                                                                               \
            ppo_loss_vec<GG><<<(unsigned)blocks, 256, 0, s>>>(                                 \
                logp, old_logp, adv, ret, old_value, value, entropy, batch, num_minibatches, k, \
                g_logp, g_value, g_entropy, stats);                                            \
        else                                                                                   \
            ppo_loss_gather<GG><<<(unsigned)blocks, 256, 0, s>>>(                              \
                logp, old_logp, adv, ret, old_value, value, entropy, index, batch,            \
                num_minibatches, k, g_logp, g_value, g_entropy, stats);                        \
        break;
    switch (G) {
        AGX_LOSS(64)
        AGX_LOSS(32)
        AGX_LOSS(16)
        AGX_LOSS(8)
    }
#undef AGX_LOSS
    return check_launch("agx_ppo_loss_fwd_bwd");
}
