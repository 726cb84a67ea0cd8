// Fused PPO learner: ONE persistent workgroup per agent runs every
// epoch x minibatch update of PPO._learn_from_rollout_buffer_flat
// (agilerl/algorithms/ppo.py:836-915) — gather, MLP forward, categorical
// log-prob / entropy, clipped-surrogate + clipped-value loss, backward through
// the shared-encoder actor-critic, two-group gradient-norm clip
// (ppo.py:910-911) and Adam (optimizer_wrapper.py:444-452) — without leaving
// the chip.
//
// Network (the reference's config-2 PPO nets, agilerl/utils/
// evolvable_networks.py:527-644, agilerl/networks/base.py:541-561):
//   encoder: ne-1 x [Linear -> LayerNorm(affine) -> ReLU], Linear(->lat) ->
//            LayerNorm(plain) -> ReLU
//   heads  : actor  Linear(lat->ha) -> LN(affine) -> ReLU -> Linear(->A)
//            critic Linear(lat->hc) -> LN(affine) -> ReLU -> Linear(->1)
//   The two head hidden layers run as ONE merged [ha+hc] layer (same input,
//   per-half LayerNorm), and d(latent) = [dz_a | dz_c] . [Wa; Wc] is one GEMM.
//
// Work split (512 threads = 8 waves, sub-batches of SB = 32 rows):
//   * all parameters live in LDS for the whole learn() (padded rows);
//   * GEMMs (forward Z = X W^T, backward dX = dZ W, dW += dZ^T X) are
//     f32 MFMA v_mfma_f32_16x16x4_f32 tiles (exact f32 FMA chains);
//   * the dW of every Linear weight stays in MFMA accumulator registers
//     across the minibatch (each wave owns a fixed set of 16x16 tiles), and
//     the clip + Adam update is applied straight from those registers;
//   * LayerNorm fwd/bwd and the loss are row passes (a wave per row, lanes
//     across features); bias / LN-affine / output-layer gradients are
//     reduced per wave into LDS partials and summed by fixed owner threads
//     in a fixed order (deterministic).
// Global memory traffic per update: the 32-row gathers of the rollout SoA
// and the Adam moments; parameters are written back once at the end.
#include <cmath>

#include "agx_common.h"

namespace agx {

constexpr int kNT = 512;
constexpr int kNW = kNT / kWave;  // 8 waves
constexpr int kSB = 32;           // rows per sub-batch
constexpr int kMaxSlot = 8;       // dW tiles per wave
constexpr int kVecSlot = 4;       // owned vector-gradient entries per thread
constexpr int kMaxA = 16;

typedef float f4 __attribute__((ext_vector_type(4)));

struct LearnPlan {
    // network
    int D, A, ne, ein[3], eout[3], lat, ha, hc, H;
    // global flat offsets (per agent row)
    int ew[3], eb[3], eg[3], ebe[3];
    int aw, ab, ag, abe, aow, aob, cw, cb, cg, cbe, cow, cob;
    int n, split;
    // LDS plan (floats)
    int l_ew[3], l_eld[3], l_eb[3], l_eg[3], l_ebe[3];
    int l_hw, l_hld, l_hb, l_hg, l_hbe;
    int l_aow, l_aob, l_cow, l_cob;
    int l_x0, ld_x0;
    int l_xe[3], ld_xe[3], l_re[3];
    int l_xh, ld_xh, l_rh;
    int l_s1, l_s2, ld_s;
    int l_lg, l_dlg, l_val, l_dval, l_row, l_red, red_e[3], red_h, l_stat;
    int lds_floats;
    int nvec;  // vector-gradient entries (<= kNT * kVecSlot)
    int ntiles, tile_begin[4];  // dW tiles: enc layers 0..ne-1, then head
};

// vector-gradient entry descriptor (host-built table in global memory)
struct VecDesc {
    int flat;   // global flat offset
    int lds;    // LDS offset of the parameter
    int group;  // clip group
    int kind;   // 0: sum of per-wave partials, 1: actor out W, 2: critic out W,
                // 3: actor out bias, 4: critic out bias
    int p0, p1; // kind 0: red base, wave stride; kind 1: a, column; kind 2: column
};

struct LearnArgs {
    const LearnPlan *plan;  // device copy (workspace), read through scalar loads
    const VecDesc *vec;
    float *params, *m, *v;
    const float *lr;
    float b1, b2, eps;
    long long step0;
    const float *obs;
    const long long *act;
    const float *old_logp, *adv, *ret, *old_v;
    long long S;
    const long long *perms;
    int E, B, P;
    float clip, vf, ent, max_norm;
    float *loss_out;
};

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// C[16x16] += A[16 x K] B[K x 16]; A(m,k) / B(k,n) fetched by functors
template <class FA, class FB>
__device__ __forceinline__ f4 mfma_tile(f4 acc, int K, FA a, FB b) {
    const int lane = threadIdx.x & 63;
    const int r = lane & 15, q = lane >> 4;
    for (int k0 = 0; k0 < K; k0 += 4) {
        const float av = a(r, k0 + q);
        const float bv = b(k0 + q, r);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    return acc;
}

__global__ __launch_bounds__(kNT, 1) void ppo_learn_kernel(LearnArgs g) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const LearnPlan &pl = *g.plan;
    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr16 = lane & 15, lq = lane >> 4;
    float *gp = g.params + (size_t)p * pl.n;
    float *gm = g.m + (size_t)p * pl.n;
    float *gv = g.v + (size_t)p * pl.n;
    const long long S = g.S;

    // ---------------- load parameters into LDS (zero padding) -------------
    for (int i = tid; i < pl.lds_floats; i += kNT) sm[i] = 0.f;
    __syncthreads();
    for (int e = 0; e < pl.ne; ++e) {
        const int fin = pl.ein[e], fout = pl.eout[e];
        for (int i = tid; i < fin * fout; i += kNT) sm[pl.l_ew[e] + (i / fin) * pl.l_eld[e] + i % fin] = gp[pl.ew[e] + i];
        for (int i = tid; i < fout; i += kNT) {
            sm[pl.l_eb[e] + i] = gp[pl.eb[e] + i];
            if (pl.eg[e] >= 0) {
                sm[pl.l_eg[e] + i] = gp[pl.eg[e] + i];
                sm[pl.l_ebe[e] + i] = gp[pl.ebe[e] + i];
            }
        }
    }
    for (int i = tid; i < pl.lat * pl.H; i += kNT) {
        const int o = i / pl.lat, c = i % pl.lat;
        const float w = o < pl.ha ? gp[pl.aw + o * pl.lat + c] : gp[pl.cw + (o - pl.ha) * pl.lat + c];
        sm[pl.l_hw + o * pl.l_hld + c] = w;
    }
    for (int o = tid; o < pl.H; o += kNT) {
        const bool a = o < pl.ha;
        const int oo = a ? o : o - pl.ha;
        sm[pl.l_hb + o] = gp[(a ? pl.ab : pl.cb) + oo];
        sm[pl.l_hg + o] = gp[(a ? pl.ag : pl.cg) + oo];
        sm[pl.l_hbe + o] = gp[(a ? pl.abe : pl.cbe) + oo];
    }
    for (int i = tid; i < pl.A * pl.ha; i += kNT) sm[pl.l_aow + i] = gp[pl.aow + i];
    for (int i = tid; i < pl.A; i += kNT) sm[pl.l_aob + i] = gp[pl.aob + i];
    for (int i = tid; i < pl.hc; i += kNT) sm[pl.l_cow + i] = gp[pl.cow + i];
    if (tid == 0) sm[pl.l_cob] = gp[pl.cob];

    // ---------------- ownership: dW tiles (MFMA accumulators) --------------
    // tile (layer, o0, i0) packed as (L+1) << 16 | o0/16 << 8 | i0/16; 0 = none
    int tpk[kMaxSlot];
#pragma unroll
    for (int s = 0; s < kMaxSlot; ++s) {
        const int t = wave + kNW * s;
        tpk[s] = 0;
        if (t < pl.ntiles) {
            int L = 0;
            while (L < pl.ne && t >= pl.tile_begin[L + 1]) ++L;
            const int local = t - pl.tile_begin[L];
            const int fin = L < pl.ne ? pl.ein[L] : pl.lat;
            const int ncol = (fin + 15) / 16;
            tpk[s] = ((L + 1) << 16) | ((local / ncol) << 8) | (local % ncol);  // L == ne: merged head
        }
    }
#define T_LAYER(s) ((tpk[s] >> 16) - 1)
#define T_O0(s) (((tpk[s] >> 8) & 255) * 16)
#define T_I0(s) ((tpk[s] & 255) * 16)
    __syncthreads();

    const int nmb = (int)((S + g.B - 1) / g.B);
    float loss_total = 0.f;
    long long step = g.step0;
    float *rowf = sm + pl.l_row;  // [5][SB]: act (bits), old_logp, adv, ret, old_v
    int *rowi = reinterpret_cast<int *>(rowf);

    for (int e = 0; e < g.E; ++e) {
        const long long *perm = g.perms + ((size_t)e * g.P + p) * S;
        for (int mb = 0; mb < nmb; ++mb) {
            const long long s0 = (long long)mb * g.B;
            const int bsz = (int)((s0 + g.B <= S) ? g.B : S - s0);
            const float inv_b = 1.f / (float)bsz;
            f4 acc[kMaxSlot];
#pragma unroll
            for (int s = 0; s < kMaxSlot; ++s) acc[s] = f4{0.f, 0.f, 0.f, 0.f};
            float vacc[kVecSlot] = {0.f, 0.f, 0.f, 0.f};
            float lsum = 0.f;  // per-thread loss partial (row threads)

            for (int sb = 0; sb < bsz; sb += kSB) {
                const int nrow = bsz - sb < kSB ? bsz - sb : kSB;
                // ---- P0: gather rows ------------------------------------------
                for (int i = tid; i < kSB * pl.ld_x0; i += kNT) sm[pl.l_x0 + i] = 0.f;
                __syncthreads();
                for (int i = tid; i < kSB * pl.D; i += kNT) {
                    const int r = i / pl.D, d = i % pl.D;
                    if (r < nrow) {
                        const long long src = perm[s0 + sb + r];
                        sm[pl.l_x0 + r * pl.ld_x0 + d] = g.obs[((size_t)p * S + src) * pl.D + d];
                    }
                }
                if (tid < kSB) {
                    const int r = tid;
                    if (r < nrow) {
                        const long long src = (size_t)p * S + perm[s0 + sb + r];
                        rowi[r] = (int)g.act[src];
                        rowf[kSB + r] = g.old_logp[src];
                        rowf[2 * kSB + r] = g.adv[src];
                        rowf[3 * kSB + r] = g.ret[src];
                        rowf[4 * kSB + r] = g.old_v[src];
                    } else {
                        rowi[r] = 0;
                        rowf[kSB + r] = rowf[2 * kSB + r] = rowf[3 * kSB + r] = rowf[4 * kSB + r] = 0.f;
                    }
                }
                __syncthreads();

                // ---- P1: encoder forward ----------------------------------------
                for (int L = 0; L < pl.ne; ++L) {
                    const int fin = pl.ein[L], fout = pl.eout[L];
                    const int K = (fin + 3) & ~3;
                    const int xb = L == 0 ? pl.l_x0 : pl.l_s1;
                    const int ldx = L == 0 ? pl.ld_x0 : pl.ld_s;
                    const int wb = pl.l_ew[L], ldw = pl.l_eld[L];
                    const int nt = (kSB / 16) * (fout / 16);
                    for (int t = wave; t < nt; t += kNW) {
                        const int m0 = (t % (kSB / 16)) * 16, n0 = (t / (kSB / 16)) * 16;
                        f4 c = f4{0.f, 0.f, 0.f, 0.f};
                        c = mfma_tile(c, K, [&](int m, int k) { return sm[xb + (m0 + m) * ldx + k]; },
                                      [&](int k, int n) { return sm[wb + (n0 + n) * ldw + k]; });
                        const float bias = sm[pl.l_eb[L] + n0 + lr16];
#pragma unroll
                        for (int i = 0; i < 4; ++i) sm[pl.l_s2 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i] + bias;
                    }
                    __syncthreads();
                    // LayerNorm + ReLU row pass: wave handles rows wave*4 .. +3
                    const bool affine = pl.eg[L] >= 0;
                    for (int rr = 0; rr < kSB / kNW; ++rr) {
                        const int r = wave * (kSB / kNW) + rr;
                        float z0 = lane < fout ? sm[pl.l_s2 + r * pl.ld_s + lane] : 0.f;
                        float z1 = lane + 64 < fout ? sm[pl.l_s2 + r * pl.ld_s + lane + 64] : 0.f;
                        const float mean = wave_sum(z0 + z1) / (float)fout;
                        const float d0 = lane < fout ? z0 - mean : 0.f;
                        const float d1 = lane + 64 < fout ? z1 - mean : 0.f;
                        const float var = wave_sum(d0 * d0 + d1 * d1) / (float)fout;
                        const float rstd = 1.f / sqrtf(var + 1e-5f);
                        if (lane == 0) sm[pl.l_re[L] + r] = rstd;
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int j = lane + 64 * h;
                            if (j < fout) {
                                const float xh = (h ? d1 : d0) * rstd;
                                sm[pl.l_xe[L] + r * pl.ld_xe[L] + j] = xh;
                                const float y = affine ? relu(xh * sm[pl.l_eg[L] + j] + sm[pl.l_ebe[L] + j]) : relu(xh);
                                sm[pl.l_s1 + r * pl.ld_s + j] = y;
                            }
                        }
                    }
                    __syncthreads();
                }

                // ---- P2: merged head forward --------------------------------------
                {
                    const int nt = (kSB / 16) * (pl.H / 16);
                    for (int t = wave; t < nt; t += kNW) {
                        const int m0 = (t % (kSB / 16)) * 16, n0 = (t / (kSB / 16)) * 16;
                        f4 c = f4{0.f, 0.f, 0.f, 0.f};
                        c = mfma_tile(c, pl.lat, [&](int m, int k) { return sm[pl.l_s1 + (m0 + m) * pl.ld_s + k]; },
                                      [&](int k, int n) { return sm[pl.l_hw + (n0 + n) * pl.l_hld + k]; });
                        const float bias = sm[pl.l_hb + n0 + lr16];
#pragma unroll
                        for (int i = 0; i < 4; ++i) sm[pl.l_s2 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i] + bias;
                    }
                    __syncthreads();
                    for (int rr = 0; rr < kSB / kNW; ++rr) {
                        const int r = wave * (kSB / kNW) + rr;
                        float z[4], sa = 0.f, sc = 0.f;
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int j = lane + 64 * h;
                            z[h] = j < pl.H ? sm[pl.l_s2 + r * pl.ld_s + j] : 0.f;
                            if (j < pl.ha) sa += z[h];
                            else if (j < pl.H) sc += z[h];
                        }
                        const float ma = wave_sum(sa) / (float)pl.ha, mc = wave_sum(sc) / (float)pl.hc;
                        float va = 0.f, vc = 0.f;
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int j = lane + 64 * h;
                            if (j < pl.ha) va += (z[h] - ma) * (z[h] - ma);
                            else if (j < pl.H) vc += (z[h] - mc) * (z[h] - mc);
                        }
                        const float ra = 1.f / sqrtf(wave_sum(va) / (float)pl.ha + 1e-5f);
                        const float rc = 1.f / sqrtf(wave_sum(vc) / (float)pl.hc + 1e-5f);
                        if (lane == 0) {
                            sm[pl.l_rh + 2 * r] = ra;
                            sm[pl.l_rh + 2 * r + 1] = rc;
                        }
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int j = lane + 64 * h;
                            if (j < pl.H) {
                                const float xh = j < pl.ha ? (z[h] - ma) * ra : (z[h] - mc) * rc;
                                sm[pl.l_xh + r * pl.ld_xh + j] = xh;
                                sm[pl.l_s1 + r * pl.ld_s + j] = relu(xh * sm[pl.l_hg + j] + sm[pl.l_hbe + j]);
                            }
                        }
                    }
                    __syncthreads();
                }

                // ---- P3: output layers (VALU dots) ---------------------------------
                for (int idx = tid; idx < kSB * (pl.A + 1); idx += kNT) {
                    const int r = idx % kSB, j = idx / kSB;
                    const float *y = sm + pl.l_s1 + r * pl.ld_s;
                    float s;
                    if (j < pl.A) {
                        s = sm[pl.l_aob + j];
                        const float *w = sm + pl.l_aow + j * pl.ha;
                        for (int o = 0; o < pl.ha; ++o) s += y[o] * w[o];
                        sm[pl.l_lg + r * kMaxA + j] = s;
                    } else {
                        s = sm[pl.l_cob];
                        const float *w = sm + pl.l_cow;
                        for (int o = 0; o < pl.hc; ++o) s += y[pl.ha + o] * w[o];
                        sm[pl.l_val + r] = s;
                    }
                }
                __syncthreads();

                // ---- P4: loss + d(logits), d(value) per row ------------------------
                if (tid < kSB) {
                    const int r = tid;
                    float *dl = sm + pl.l_dlg + r * kMaxA;
                    if (r < nrow) {
                        const float *lg = sm + pl.l_lg + r * kMaxA;
                        float mx = lg[0];
                        for (int a = 1; a < pl.A; ++a) mx = fmaxf(mx, lg[a]);
                        float se = 0.f;
                        for (int a = 0; a < pl.A; ++a) se += expf(lg[a] - mx);
                        const float lse = mx + logf(se);
                        const int a_t = rowi[r];
                        const float logp = lg[a_t] - lse;
                        // entropy H = -sum p log(p + 1e-8)  (torch_utils.py:188-199)
                        float Hs = 0.f, pg_dot = 0.f;
                        for (int a = 0; a < pl.A; ++a) {
                            const float pa = expf(lg[a] - lse);
                            const float lpe = logf(pa + 1e-8f);
                            Hs -= pa * lpe;
                            pg_dot += pa * -(lpe + pa / (pa + 1e-8f));  // sum_a p_a dH/dp_a
                        }
                        const float olp = rowf[kSB + r], A = rowf[2 * kSB + r], R = rowf[3 * kSB + r];
                        const float ov = rowf[4 * kSB + r], v = sm[pl.l_val + r];
                        const float lo = 1.f - g.clip, hi = 1.f + g.clip;
                        const float lrt = logp - olp;
                        const float ratio = expf(lrt);
                        const float rcl = fminf(fmaxf(ratio, lo), hi);
                        const float p1 = -A * ratio, p2 = -A * rcl;
                        const float g1 = p1 > p2 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
                        const float g2 = p2 > p1 ? 1.f : (p1 == p2 ? 0.5f : 0.f);
                        const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
                        const float g_logp = ((g1 * -A + g2 * -A * inr) * inv_b) * ratio;
                        const float dv = v - ov;
                        const float vcl = ov + fminf(fmaxf(dv, -g.clip), g.clip);
                        const float eu = v - R, ec = vcl - R;
                        const float lu = eu * eu, lc = ec * ec;
                        const float gu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
                        const float gc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
                        const float inv = (dv >= -g.clip && dv <= g.clip) ? 1.f : 0.f;
                        sm[pl.l_dval + r] = g.vf * 0.5f * inv_b * (gu * 2.f * eu + gc * 2.f * ec * inv);
                        const float g_H = -g.ent * inv_b;
                        for (int a = 0; a < pl.A; ++a) {
                            const float pa = expf(lg[a] - lse);
                            const float gh = -(logf(pa + 1e-8f) + pa / (pa + 1e-8f));  // dH/dp_a
                            dl[a] = g_logp * ((a == a_t ? 1.f : 0.f) - pa) + g_H * pa * (gh - pg_dot);
                        }
                        lsum += (fmaxf(p1, p2) + g.vf * 0.5f * fmaxf(lu, lc) - g.ent * Hs) * inv_b;
                    } else {
                        for (int a = 0; a < pl.A; ++a) dl[a] = 0.f;
                        sm[pl.l_dval + r] = 0.f;
                    }
                }
                __syncthreads();

                // ---- P5: head hidden backward row pass -----------------------------
                {
                    float pb[4] = {0.f, 0.f, 0.f, 0.f}, pgm[4] = {0.f, 0.f, 0.f, 0.f}, pbe[4] = {0.f, 0.f, 0.f, 0.f};
                    for (int rr = 0; rr < kSB / kNW; ++rr) {
                        const int r = wave * (kSB / kNW) + rr;
                        const float ra = sm[pl.l_rh + 2 * r], rc = sm[pl.l_rh + 2 * r + 1];
                        float xh[4], dxh[4], dyp[4];
                        float sa1 = 0.f, sa2 = 0.f, sc1 = 0.f, sc2 = 0.f;
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int j = lane + 64 * h;
                            xh[h] = dxh[h] = dyp[h] = 0.f;
                            if (j < pl.H) {
                                float dy;
                                if (j < pl.ha) {
                                    dy = 0.f;
                                    for (int a = 0; a < pl.A; ++a) dy += sm[pl.l_dlg + r * kMaxA + a] * sm[pl.l_aow + a * pl.ha + j];
                                } else {
                                    dy = sm[pl.l_dval + r] * sm[pl.l_cow + j - pl.ha];
                                }
                                xh[h] = sm[pl.l_xh + r * pl.ld_xh + j];
                                const float gam = sm[pl.l_hg + j];
                                const float y = xh[h] * gam + sm[pl.l_hbe + j];
                                dyp[h] = y > 0.f ? dy : 0.f;
                                dxh[h] = dyp[h] * gam;
                                if (j < pl.ha) {
                                    sa1 += dxh[h];
                                    sa2 += dxh[h] * xh[h];
                                } else {
                                    sc1 += dxh[h];
                                    sc2 += dxh[h] * xh[h];
                                }
                            }
                        }
                        const float ma1 = wave_sum(sa1) / (float)pl.ha, ma2 = wave_sum(sa2) / (float)pl.ha;
                        const float mc1 = wave_sum(sc1) / (float)pl.hc, mc2 = wave_sum(sc2) / (float)pl.hc;
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int j = lane + 64 * h;
                            if (j < pl.H) {
                                const bool isa = j < pl.ha;
                                const float dz = (isa ? ra : rc) * (dxh[h] - (isa ? ma1 : mc1) - xh[h] * (isa ? ma2 : mc2));
                                sm[pl.l_s2 + r * pl.ld_s + j] = dz;
                                pb[h] += dz;
                                pgm[h] += dyp[h] * xh[h];
                                pbe[h] += dyp[h];
                            }
                        }
                    }
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        const int j = lane + 64 * h;
                        if (j < pl.H) {
                            float *red = sm + pl.l_red + pl.red_h;
                            red[(0 * kNW + wave) * pl.H + j] = pb[h];
                            red[(1 * kNW + wave) * pl.H + j] = pgm[h];
                            red[(2 * kNW + wave) * pl.H + j] = pbe[h];
                        }
                    }
                }
                __syncthreads();

                // ---- P6: head dW (MFMA acc) and d(latent) = dZ . W_h -> S1 --------
                {
                    const int Le = pl.ne - 1;  // latent = relu(xhat of the last encoder layer)
                    const int xeb = pl.l_xe[Le], ldxe = pl.ld_xe[Le];
#pragma unroll
                    for (int s = 0; s < kMaxSlot; ++s) {
                        if (T_LAYER(s) == pl.ne) {
                            const int o0 = T_O0(s), i0 = T_I0(s);
                            acc[s] = mfma_tile(acc[s], kSB,
                                               [&](int m, int k) { return sm[pl.l_s2 + k * pl.ld_s + o0 + m]; },
                                               [&](int k, int n) { return relu(sm[xeb + k * ldxe + i0 + n]); });
                        }
                    }
                    const int nt = (kSB / 16) * (pl.lat / 16);
                    for (int t = wave; t < nt; t += kNW) {
                        const int m0 = (t % (kSB / 16)) * 16, n0 = (t / (kSB / 16)) * 16;
                        f4 c = f4{0.f, 0.f, 0.f, 0.f};
                        c = mfma_tile(c, pl.H, [&](int m, int k) { return sm[pl.l_s2 + (m0 + m) * pl.ld_s + k]; },
                                      [&](int k, int n) { return sm[pl.l_hw + k * pl.l_hld + n0 + n]; });
#pragma unroll
                        for (int i = 0; i < 4; ++i) sm[pl.l_s1 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i];
                    }
                }
                __syncthreads();

                // ---- P7: encoder backward, last layer first --------------------------
                for (int L = pl.ne - 1; L >= 0; --L) {
                    const int fin = pl.ein[L], fout = pl.eout[L];
                    const bool affine = pl.eg[L] >= 0;
                    {
                        float pb[2] = {0.f, 0.f}, pgm[2] = {0.f, 0.f}, pbe[2] = {0.f, 0.f};
                        for (int rr = 0; rr < kSB / kNW; ++rr) {
                            const int r = wave * (kSB / kNW) + rr;
                            const float rstd = sm[pl.l_re[L] + r];
                            float xh[2], dxh[2], dyp[2], s1 = 0.f, s2 = 0.f;
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const int j = lane + 64 * h;
                                xh[h] = dxh[h] = dyp[h] = 0.f;
                                if (j < fout) {
                                    const float dy = sm[pl.l_s1 + r * pl.ld_s + j];
                                    xh[h] = sm[pl.l_xe[L] + r * pl.ld_xe[L] + j];
                                    const float gam = affine ? sm[pl.l_eg[L] + j] : 1.f;
                                    const float y = affine ? xh[h] * gam + sm[pl.l_ebe[L] + j] : xh[h];
                                    dyp[h] = y > 0.f ? dy : 0.f;
                                    dxh[h] = dyp[h] * gam;
                                    s1 += dxh[h];
                                    s2 += dxh[h] * xh[h];
                                }
                            }
                            const float m1 = wave_sum(s1) / (float)fout, m2 = wave_sum(s2) / (float)fout;
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const int j = lane + 64 * h;
                                if (j < fout) {
                                    const float dz = rstd * (dxh[h] - m1 - xh[h] * m2);
                                    sm[pl.l_s2 + r * pl.ld_s + j] = dz;
                                    pb[h] += dz;
                                    pgm[h] += dyp[h] * xh[h];
                                    pbe[h] += dyp[h];
                                }
                            }
                        }
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int j = lane + 64 * h;
                            if (j < fout) {
                                float *red = sm + pl.l_red + pl.red_e[L];
                                red[(0 * kNW + wave) * fout + j] = pb[h];
                                if (affine) {
                                    red[(1 * kNW + wave) * fout + j] = pgm[h];
                                    red[(2 * kNW + wave) * fout + j] = pbe[h];
                                }
                            }
                        }
                    }
                    __syncthreads();
                    // dW_L += dZ^T X_in ; X_in = obs (L == 0) or y of layer L-1 (recomputed)
                    {
                        const bool in_aff = L > 0 && pl.eg[L - 1] >= 0;
                        const int xb = L == 0 ? pl.l_x0 : pl.l_xe[L - 1];
                        const int ldx = L == 0 ? pl.ld_x0 : pl.ld_xe[L - 1];
#pragma unroll
                        for (int s = 0; s < kMaxSlot; ++s) {
                            if (T_LAYER(s) == L) {
                                const int o0 = T_O0(s), i0 = T_I0(s);
                                const int col = i0 + lr16;
                                const bool cv = col < fin;
                                const float gam = (L > 0 && cv && in_aff) ? sm[pl.l_eg[L - 1] + col] : 1.f;
                                const float bet = (L > 0 && cv && in_aff) ? sm[pl.l_ebe[L - 1] + col] : 0.f;
                                acc[s] = mfma_tile(
                                    acc[s], kSB, [&](int m, int k) { return sm[pl.l_s2 + k * pl.ld_s + o0 + m]; },
                                    [&](int k, int n) {
                                        const float x = sm[xb + k * ldx + i0 + n];
                                        return L == 0 ? x : (cv ? relu(x * gam + bet) : 0.f);
                                    });
                            }
                        }
                        if (L > 0) {  // dX = dZ . W_L -> S1 (d of layer L-1's output)
                            const int nt = (kSB / 16) * (fin / 16);
                            for (int t = wave; t < nt; t += kNW) {
                                const int m0 = (t % (kSB / 16)) * 16, n0 = (t / (kSB / 16)) * 16;
                                f4 c = f4{0.f, 0.f, 0.f, 0.f};
                                c = mfma_tile(c, fout, [&](int m, int k) { return sm[pl.l_s2 + (m0 + m) * pl.ld_s + k]; },
                                              [&](int k, int n) { return sm[pl.l_ew[L] + k * pl.l_eld[L] + n0 + n]; });
#pragma unroll
                                for (int i = 0; i < 4; ++i) sm[pl.l_s1 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i];
                            }
                        }
                    }
                    __syncthreads();
                }

                // ---- P8: owners accumulate vector gradients (fixed order) ---------
#pragma unroll
                for (int s = 0; s < kVecSlot; ++s) {
                    const int vi = tid + kNT * s;
                    if (vi >= pl.nvec) continue;
                    const VecDesc d = g.vec[vi];
                    float x = 0.f;
                    if (d.kind == 0) {
                        for (int w = 0; w < kNW; ++w) x += sm[pl.l_red + d.p0 + w * d.p1];
                    } else if (d.kind == 1 || d.kind == 2) {  // out weight: sum_r dZout[r] * y_h[r][col]
                        const int col = d.p1;
                        const float gam = sm[pl.l_hg + col], bet = sm[pl.l_hbe + col];
                        for (int r = 0; r < kSB; ++r) {
                            const float dz = d.kind == 1 ? sm[pl.l_dlg + r * kMaxA + d.p0] : sm[pl.l_dval + r];
                            x += dz * relu(sm[pl.l_xh + r * pl.ld_xh + col] * gam + bet);
                        }
                    } else if (d.kind == 3) {
                        for (int r = 0; r < kSB; ++r) x += sm[pl.l_dlg + r * kMaxA + d.p0];
                    } else if (d.kind == 4) {
                        for (int r = 0; r < kSB; ++r) x += sm[pl.l_dval + r];
                    }
                    vacc[s] += x;
                }
                __syncthreads();
            }  // sub-batches

            // ---- P9: two-group gradient norms ---------------------------------
            float n0 = 0.f, n1 = 0.f;
#pragma unroll
            for (int s = 0; s < kMaxSlot; ++s) {
                const int L = T_LAYER(s);
                if (L >= 0) {
                    const int fin = L < pl.ne ? pl.ein[L] : pl.lat;
                    const int fout = L < pl.ne ? pl.eout[L] : pl.H;
                    const int col = T_I0(s) + lr16;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int o = T_O0(s) + lq * 4 + i;
                        if (col < fin && o < fout) {
                            const float x = acc[s][i];
                            if (L == pl.ne && o >= pl.ha) n1 += x * x;
                            else n0 += x * x;
                        }
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < kVecSlot; ++s) {
                const int vi = tid + kNT * s;
                if (vi < pl.nvec) {
                    if (g.vec[vi].group) n1 += vacc[s] * vacc[s];
                    else n0 += vacc[s] * vacc[s];
                }
            }
            n0 = wave_sum(n0);
            n1 = wave_sum(n1);
            // minibatch loss from the row threads (wave 0)
            const float lmb = wave_sum(lsum);
            float *stat = sm + pl.l_stat;
            if (lane == 0) {
                stat[2 * wave] = n0;
                stat[2 * wave + 1] = n1;
            }
            __syncthreads();
            float t0 = 0.f, t1 = 0.f;
            for (int w = 0; w < kNW; ++w) {
                t0 += stat[2 * w];
                t1 += stat[2 * w + 1];
            }
            if (tid == 0) loss_total += lmb;
            const float c0 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t0) + 1e-6f), 1.f) : 1.f;
            const float c1 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t1) + 1e-6f), 1.f) : 1.f;

            // ---- P10: Adam on owned entries --------------------------------------
            ++step;
            const float bc1 = (float)(1.0 - pow((double)g.b1, (double)step));
            const float bc2s = (float)sqrt(1.0 - pow((double)g.b2, (double)step));
            const float step_size = g.lr[p] / bc1;
            auto adam = [&](int flat, int lds, float gr) {
                float mm = gm[flat], vv = gv[flat];
                mm = mm + (1.f - g.b1) * (gr - mm);
                vv = vv * g.b2 + (1.f - g.b2) * gr * gr;
                gm[flat] = mm;
                gv[flat] = vv;
                const float denom = sqrtf(vv) / bc2s + g.eps;
                sm[lds] = sm[lds] - step_size * (mm / denom);
            };
#pragma unroll
            for (int s = 0; s < kMaxSlot; ++s) {
                const int L = T_LAYER(s);
                if (L >= 0) {
                    const int col = T_I0(s) + lr16;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int o = T_O0(s) + lq * 4 + i;
                        if (L < pl.ne) {
                            if (col < pl.ein[L] && o < pl.eout[L])
                                adam(pl.ew[L] + o * pl.ein[L] + col, pl.l_ew[L] + o * pl.l_eld[L] + col, acc[s][i] * c0);
                        } else if (col < pl.lat && o < pl.H) {
                            const bool isa = o < pl.ha;
                            const int flat = isa ? pl.aw + o * pl.lat + col : pl.cw + (o - pl.ha) * pl.lat + col;
                            adam(flat, pl.l_hw + o * pl.l_hld + col, acc[s][i] * (isa ? c0 : c1));
                        }
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < kVecSlot; ++s) {
                const int vi = tid + kNT * s;
                if (vi < pl.nvec) {
                    const VecDesc d = g.vec[vi];
                    adam(d.flat, d.lds, vacc[s] * (d.group ? c1 : c0));
                }
            }
            __syncthreads();
        }  // minibatches
    }      // epochs

    // ---------------- write parameters back ---------------------------------
    for (int e = 0; e < pl.ne; ++e) {
        const int fin = pl.ein[e], fout = pl.eout[e];
        for (int i = tid; i < fin * fout; i += kNT) gp[pl.ew[e] + i] = sm[pl.l_ew[e] + (i / fin) * pl.l_eld[e] + i % fin];
        for (int i = tid; i < fout; i += kNT) {
            gp[pl.eb[e] + i] = sm[pl.l_eb[e] + i];
            if (pl.eg[e] >= 0) {
                gp[pl.eg[e] + i] = sm[pl.l_eg[e] + i];
                gp[pl.ebe[e] + i] = sm[pl.l_ebe[e] + i];
            }
        }
    }
    for (int i = tid; i < pl.lat * pl.H; i += kNT) {
        const int o = i / pl.lat, c = i % pl.lat;
        const float w = sm[pl.l_hw + o * pl.l_hld + c];
        if (o < pl.ha) gp[pl.aw + o * pl.lat + c] = w;
        else gp[pl.cw + (o - pl.ha) * pl.lat + c] = w;
    }
    for (int o = tid; o < pl.H; o += kNT) {
        const bool a = o < pl.ha;
        const int oo = a ? o : o - pl.ha;
        gp[(a ? pl.ab : pl.cb) + oo] = sm[pl.l_hb + o];
        gp[(a ? pl.ag : pl.cg) + oo] = sm[pl.l_hg + o];
        gp[(a ? pl.abe : pl.cbe) + oo] = sm[pl.l_hbe + o];
    }
    for (int i = tid; i < pl.A * pl.ha; i += kNT) gp[pl.aow + i] = sm[pl.l_aow + i];
    for (int i = tid; i < pl.A; i += kNT) gp[pl.aob + i] = sm[pl.l_aob + i];
    for (int i = tid; i < pl.hc; i += kNT) gp[pl.cow + i] = sm[pl.l_cow + i];
    if (tid == 0) {
        gp[pl.cob] = sm[pl.l_cob];
        if (g.loss_out) g.loss_out[p] = loss_total / ((float)S * (float)g.E);
    }
}

// ---------------------------------------------------------------------------
// host-side planning
// ---------------------------------------------------------------------------
static int plan_learner(const agx_ppo_net *net, LearnPlan &pl, VecDesc *vec, int vec_cap) {
    pl = LearnPlan{};
    pl.D = net->obs_dim;
    pl.A = net->n_actions;
    pl.ne = net->n_enc;
    if (pl.ne < 2 || pl.ne > 3 || pl.A < 1 || pl.A > kMaxA || pl.D < 1 || pl.D > 128) return -1;
    int prev = pl.D;
    for (int e = 0; e < pl.ne; ++e) {
        pl.ein[e] = prev;
        pl.eout[e] = net->enc_dim[e + 1];
        if (pl.eout[e] % 16 || pl.eout[e] > 128 || pl.eout[e] < 16) return -1;
        if (e > 0 && pl.ein[e] % 16) return -1;
        pl.ew[e] = net->enc_w[e];
        pl.eb[e] = net->enc_b[e];
        pl.eg[e] = e < pl.ne - 1 ? net->enc_ln_w[e] : -1;
        pl.ebe[e] = e < pl.ne - 1 ? net->enc_ln_b[e] : -1;
        prev = pl.eout[e];
    }
    pl.lat = prev;
    pl.ha = net->head_actor;
    pl.hc = net->head_critic;
    pl.H = pl.ha + pl.hc;
    if (pl.ha % 16 || pl.hc % 16 || pl.ha < 16 || pl.hc < 16 || pl.H > 256) return -1;
    pl.aw = net->actor_w; pl.ab = net->actor_b; pl.ag = net->actor_ln_w; pl.abe = net->actor_ln_b;
    pl.aow = net->actor_out_w; pl.aob = net->actor_out_b;
    pl.cw = net->critic_w; pl.cb = net->critic_b; pl.cg = net->critic_ln_w; pl.cbe = net->critic_ln_b;
    pl.cow = net->critic_out_w; pl.cob = net->critic_out_b;
    pl.n = net->n_params;
    pl.split = net->critic_start;
    // ---- LDS plan
    int off = 0;
    auto take = [&](int n) { const int o = off; off += (n + 3) & ~3; return o; };
    for (int e = 0; e < pl.ne; ++e) {
        pl.l_eld[e] = ((pl.ein[e] + 3) & ~3) + 2;
        pl.l_ew[e] = take(pl.eout[e] * pl.l_eld[e]);
        pl.l_eb[e] = take(pl.eout[e]);
        pl.l_eg[e] = pl.eg[e] >= 0 ? take(pl.eout[e]) : -1;
        pl.l_ebe[e] = pl.eg[e] >= 0 ? take(pl.eout[e]) : -1;
    }
    pl.l_hld = pl.lat + 2;
    pl.l_hw = take(pl.H * pl.l_hld);
    pl.l_hb = take(pl.H);
    pl.l_hg = take(pl.H);
    pl.l_hbe = take(pl.H);
    pl.l_aow = take(pl.A * pl.ha);
    pl.l_aob = take(pl.A);
    pl.l_cow = take(pl.hc);
    pl.l_cob = take(1);
    pl.ld_x0 = ((pl.D + 15) & ~15) + 2;
    pl.l_x0 = take(kSB * pl.ld_x0);
    for (int e = 0; e < pl.ne; ++e) {
        pl.ld_xe[e] = pl.eout[e] + 2;
        pl.l_xe[e] = take(kSB * pl.ld_xe[e]);
        pl.l_re[e] = take(kSB);
    }
    pl.ld_xh = pl.H + 2;
    pl.l_xh = take(kSB * pl.ld_xh);
    pl.l_rh = take(2 * kSB);
    int wmax = pl.H;
    for (int e = 0; e < pl.ne; ++e) wmax = wmax > pl.eout[e] ? wmax : pl.eout[e];
    pl.ld_s = wmax + 2;
    pl.l_s1 = take(kSB * pl.ld_s);
    pl.l_s2 = take(kSB * pl.ld_s);
    pl.l_lg = take(kSB * kMaxA);
    pl.l_dlg = take(kSB * kMaxA);
    pl.l_val = take(kSB);
    pl.l_dval = take(kSB);
    pl.l_row = take(5 * kSB);
    pl.l_stat = take(4 * kNW);
    // partial buffers: [3][NW][width] per layer (plain LN layer: bias only)
    int red = 0;
    for (int e = 0; e < pl.ne; ++e) {
        pl.red_e[e] = red;
        red += (pl.eg[e] >= 0 ? 3 : 1) * kNW * pl.eout[e];
    }
    pl.red_h = red;
    red += 3 * kNW * pl.H;
    pl.l_red = take(red);
    pl.lds_floats = off;
    // ---- dW tiles
    pl.tile_begin[0] = 0;
    for (int e = 0; e < pl.ne; ++e) pl.tile_begin[e + 1] = pl.tile_begin[e] + (pl.eout[e] / 16) * ((pl.ein[e] + 15) / 16);
    pl.ntiles = pl.tile_begin[pl.ne] + (pl.H / 16) * (pl.lat / 16);
    if (pl.ntiles > kNW * kMaxSlot) return -2;
    // ---- vector gradients
    int nv = 0;
    auto add = [&](int flat, int lds, int group, int kind, int p0, int p1) {
        if (nv < vec_cap) vec[nv] = VecDesc{flat, lds, group, kind, p0, p1};
        ++nv;
    };
    for (int e = 0; e < pl.ne; ++e) {
        const int F = pl.eout[e];
        for (int j = 0; j < F; ++j) add(pl.eb[e] + j, pl.l_eb[e] + j, 0, 0, pl.red_e[e] + j, F);
        if (pl.eg[e] >= 0) {
            for (int j = 0; j < F; ++j) add(pl.eg[e] + j, pl.l_eg[e] + j, 0, 0, pl.red_e[e] + kNW * F + j, F);
            for (int j = 0; j < F; ++j) add(pl.ebe[e] + j, pl.l_ebe[e] + j, 0, 0, pl.red_e[e] + 2 * kNW * F + j, F);
        }
    }
    for (int j = 0; j < pl.H; ++j) {
        const bool a = j < pl.ha;
        const int jj = a ? j : j - pl.ha;
        const int grp = a ? 0 : 1;
        add((a ? pl.ab : pl.cb) + jj, pl.l_hb + j, grp, 0, pl.red_h + j, pl.H);
        add((a ? pl.ag : pl.cg) + jj, pl.l_hg + j, grp, 0, pl.red_h + kNW * pl.H + j, pl.H);
        add((a ? pl.abe : pl.cbe) + jj, pl.l_hbe + j, grp, 0, pl.red_h + 2 * kNW * pl.H + j, pl.H);
    }
    for (int a = 0; a < pl.A; ++a)
        for (int o = 0; o < pl.ha; ++o) add(pl.aow + a * pl.ha + o, pl.l_aow + a * pl.ha + o, 0, 1, a, o);
    for (int o = 0; o < pl.hc; ++o) add(pl.cow + o, pl.l_cow + o, 1, 2, 0, pl.ha + o);
    for (int a = 0; a < pl.A; ++a) add(pl.aob + a, pl.l_aob + a, 0, 3, a, 0);
    add(pl.cob, pl.l_cob, 1, 4, 0, 0);
    pl.nvec = nv;
    if (nv > kNT * kVecSlot) return -3;
    return 0;
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_ppo_learn_lds_bytes(const agx_ppo_net *net) {
    LearnPlan pl;
    if (!net || plan_learner(net, pl, nullptr, 0) != 0) return 0;
    return (size_t)pl.lds_floats * sizeof(float);
}

constexpr size_t kPlanBytes = (sizeof(LearnPlan) + 255) & ~(size_t)255;

extern "C" size_t agx_ppo_learn_workspace_bytes(const agx_ppo_net *net) {
    LearnPlan pl;
    if (!net || plan_learner(net, pl, nullptr, 0) != 0) return 0;
    return kPlanBytes + (size_t)pl.nvec * sizeof(VecDesc);
}

extern "C" int agx_ppo_learn_prepare(const agx_ppo_net *net, void *workspace, void *stream) {
    AGX_REQUIRE(net && workspace, "agx_ppo_learn_prepare: null pointer");
    LearnPlan pl;
    static thread_local VecDesc vec[kNT * kVecSlot];
    const int rc = plan_learner(net, pl, vec, kNT * kVecSlot);
    if (rc != 0) {
        set_error("agx_ppo_learn_prepare: network not supported by the fused learner (code %d)", rc);
        return AGX_EUNSUPPORTED;
    }
    // one-time upload of the plan + ownership table; synchronous so the host
    // copies may be reused immediately
    static thread_local LearnPlan plan_copy;
    plan_copy = pl;
    hipError_t e = hipMemcpyAsync(workspace, &plan_copy, sizeof(LearnPlan), hipMemcpyHostToDevice, as_stream(stream));
    if (e == hipSuccess)
        e = hipMemcpyAsync(static_cast<char *>(workspace) + kPlanBytes, vec, (size_t)pl.nvec * sizeof(VecDesc),
                           hipMemcpyHostToDevice, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    if (e != hipSuccess) {
        set_error("agx_ppo_learn_prepare: %s", hipGetErrorString(e));
        return AGX_EHIP;
    }
    return AGX_OK;
}

extern "C" int agx_ppo_learn(const agx_ppo_net *net, int64_t P, float *params, float *exp_avg,
                             float *exp_avg_sq, const float *lr, float beta1, float beta2, float eps,
                             int64_t adam_step0, const float *obs, const int64_t *actions,
                             const float *old_logp, const float *adv, const float *ret,
                             const float *old_value, int64_t S, const int64_t *perms, int64_t epochs,
                             int64_t batch, float clip_coef, float vf_coef, float ent_coef,
                             float max_grad_norm, float *loss_out, void *workspace, void *stream) {
    AGX_REQUIRE(net && params && exp_avg && exp_avg_sq && lr && obs && actions && old_logp && adv && ret &&
                    old_value && perms && workspace,
                "agx_ppo_learn: null pointer");
    AGX_REQUIRE(P > 0 && P <= 65535 && S > 0 && epochs > 0 && batch > 0, "agx_ppo_learn: bad sizes");
    LearnPlan pl;
    const int rc = plan_learner(net, pl, nullptr, 0);
    if (rc != 0) {
        set_error("agx_ppo_learn: network not supported by the fused learner (code %d)", rc);
        return AGX_EUNSUPPORTED;
    }
    const size_t lds = (size_t)pl.lds_floats * sizeof(float);
    AGX_REQUIRE(lds <= 160 * 1024, "agx_ppo_learn: network needs %zu B of LDS (> 160 KiB)", lds);
    AGX_REQUIRE(pl.n == net->n_params, "agx_ppo_learn: inconsistent parameter count");
    hipStream_t s = as_stream(stream);
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void *)ppo_learn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    LearnArgs a;
    a.plan = static_cast<const LearnPlan *>(workspace);
    a.vec = reinterpret_cast<const VecDesc *>(static_cast<const char *>(workspace) + kPlanBytes);
    a.params = params;
    a.m = exp_avg;
    a.v = exp_avg_sq;
    a.lr = lr;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.step0 = adam_step0;
    a.obs = obs;
    a.act = reinterpret_cast<const long long *>(actions);
    a.old_logp = old_logp;
    a.adv = adv;
    a.ret = ret;
    a.old_v = old_value;
    a.S = S;
    a.perms = reinterpret_cast<const long long *>(perms);
    a.E = (int)epochs;
    a.B = (int)batch;
    a.P = (int)P;
    a.clip = clip_coef;
    a.vf = vf_coef;
    a.ent = ent_coef;
    a.max_norm = max_grad_norm;
    a.loss_out = loss_out;
    ppo_learn_kernel<<<(unsigned)P, kNT, lds, s>>>(a);
    return check_launch("agx_ppo_learn");
}
