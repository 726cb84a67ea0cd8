// Runtime-shape fused PPO learner (include/agx_graph.h): the learner for the
// network shapes architecture mutations produce.
//
// agx_ppo_learn (learner.hip) compiles one plan per network shape: parameters
// in LDS, Adam moments in registers, every offset a constant.  An
// architecture mutation (hpo/mutation.py:829-885) moves an agent to one of
// thousands of shapes — any depth of encoder / head, any width, a latent of
// any size — so this kernel interprets a runtime LAYER LIST instead:
//
//   * one 256-thread workgroup per agent runs every epoch x minibatch update
//     of PPO.learn (ppo.py:836-920) in one launch, like agx_ppo_learn;
//   * a minibatch is processed layer by layer over all its rows: every Linear
//     (forward, dW, dX) is ONE operand form, C = A . B^T with both operands
//     contiguous along the contraction, on f32 MFMA 16x16x4 tiles whose
//     operand panels are staged through LDS from the agent's L2-resident
//     scratch.  The layouts that make that true are written where the data is
//     produced: activations row-major (the next layer's forward) AND
//     feature-major (the next layer's dW contracts over rows), and Adam writes
//     every weight both as nn.Linear [out][in] (forward) and transposed (dX);
//   * LayerNorm / ReLU forward runs in the forward GEMM's epilogue for layers
//     up to 64 wide (each wave owns whole rows), its backward in the
//     consumer's dX epilogue for single-consumer layers; wider / shared layers
//     and the PPO loss are row passes, 16 lanes per row (DPP row reductions);
//     bias and LN-affine gradients are per-wave partials summed in one fixed
//     order (an agent's update does not depend on its population);
//   * two-group gradient-norm clip (ppo.py:910-911) and Adam
//     (optimizer_wrapper.py:444-452) over the flat gradient row.
#include <cmath>
#include <cstdlib>

#include "agx_common.h"
#include "rollout.h"
#include "../../include/agx_graph.h"

namespace agx {

// the gather prologue of agx_ppo_learn (learner.hip): permuted, advantage-
// normalised, minibatch-ordered copy of the rollout
__global__ void ppo_gather_kernel(const float *__restrict__ obs, const long long *__restrict__ act,
                                  const float *__restrict__ old_logp, const float *__restrict__ adv,
                                  const float *__restrict__ ret, const float *__restrict__ old_v,
                                  const double *__restrict__ adv_stats, const long long *__restrict__ perms,
                                  const unsigned char *__restrict__ masks, int A, long long S, int D, int P,
                                  float *__restrict__ gobs, int *__restrict__ gact, unsigned *__restrict__ gmask,
                                  float *__restrict__ grow, unsigned *__restrict__ counters, int ncounters,
                                  const int *__restrict__ epochs_p, unsigned *__restrict__ err);

namespace {

constexpr int kGT = 256;  // 4 waves, one per SIMD: the whole 512-VGPR file per wave
constexpr int kGW = kGT / kWave;
constexpr int kGL = AGX_PPO_GRAPH_MAX_LAYERS;

typedef float f4 __attribute__((ext_vector_type(4)));

struct GLay {
    int fin, fout, w, b, g, be, ln, relu, src;
    int acc;  // dX goes to the source's second dY buffer (a consumer processed earlier wrote the first)
    // per-agent scratch offsets (floats; -1: not kept): output row-major,
    // output feature-major, xhat, rstd, d(output), d(output) from a second
    // consumer (the latent feeding both heads: the row pass adds the two),
    // transposed weight
    long long yr, yc, xh, rs, dy, dy2, wt;
    long long dyc;  // output layers: d(output) feature-major, written by the loss pass (-1 otherwise)
    int fuse;       // this layer's dX GEMM runs its source's LayerNorm / ReLU backward in the epilogue
    int fused;      // this layer's dZ (and column partials) come from its consumer's dX epilogue
    int ld;         // few-row form: the row stride of the layer's LDS tiles
    long long af;   // few-row form: the LN affine (gamma then beta) copied to LDS, -1: none
};

struct GArgs {
    GLay L[kGL];
    int nl, aout, cout, A, D, n, cstart, bp;
    long long oc, dzr, dzc, dzr1, dzc1, t1, t2, gr, ws_agent;  // dZ buffers by layer parity
    // partnered learner (ppo_learn_graph_part_kernel): K workgroups per agent,
    // R rows of each minibatch per partner; agent stride Q of the block index
    long long ws_part, wt0, wt_agent;  // a partner's scratch, the transposed weights' plan offset / size
    int K, R, Q;
    long long nslab;       // floats per exchange slab: gradient row, loss chunk, partial norms
    float *slabs, *sums;   // [P][2][K][nslab] partial gradients, [P][2][nslab] summed gradients
    float *wtb;            // [P][wt_agent] transposed weights shared by an agent's partners
    unsigned *cnt;         // barrier counters, timeout word, XCC ids (zeroed by the gather)
    unsigned *err;         // caller's sticky error word
    int write_through;     // test hook: the cross-XCD (release-fence) publish form always
    int ld0;               // few-row form: the observation tile's row stride (its offset: oc)
    long long lds_floats;  // few-row form: the LDS tiles' size (dynamic LDS)
    long long *stamps;     // diagnostic phase stamps of the partnered learner (agx_debug_graph_stamps), or null
    float *ws;
    float *params, *m, *v;
    const float *lr;
    float b1, b2, eps;
    long long *step;
    const float *gobs;
    const int *gact;
    const unsigned *gmask;
    const float *grow;
    long long S;
    int E, B, P;
    float clip, vf, ent, max_norm;
    double target_kl;
    const int *batch_p, *epochs_p;
    const float *ent_p;
    float *loss_out, *kl_out;
    int *epochs_out;
    const unsigned *skip;
    int dbg;  // diagnostic phase skips (AGX_GRAPH_DEBUG; timing attribution only, results wrong)
};

template <int C>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), C, 0xf, 0xf, true));
}
// sum / max over the 16 lanes of a DPP row
__device__ __forceinline__ float rsum16(float v) {
    v += dpp<0xb1>(v);
    v += dpp<0x4e>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}
__device__ __forceinline__ float rmax16(float v) {
    v = fmaxf(v, dpp<0xb1>(v));
    v = fmaxf(v, dpp<0x4e>(v));
    v = fmaxf(v, dpp<0x141>(v));
    v = fmaxf(v, dpp<0x140>(v));
    return v;
}
__device__ __forceinline__ float bperm(int lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(lane << 2, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// C[M x N] = A[M x K] . B[N x K]^T, both operands contiguous along k (the
// only operand form the learner needs, see the layouts above), in blocks of
// up to 128 x 128.  The block's A and B panels go through LDS 32 k at a time,
// double-buffered: every global load is a dword load of 64 consecutive lanes
// over 2 rows x 32 contiguous k (two full 128-byte lines), and the next
// chunk's loads fly under the current chunk's MFMAs.  Each wave owns up to 8
// of the block's 16x16 f32 MFMA tiles; MFMA kk takes k = 4kk + q from lane
// group q (LDS rows padded to 36 floats: the 64 lanes' reads hit 64 banks).
// lds: kGemmLds floats.  epi(m, n, c) per element.
constexpr int kBM = 128, kBN = 64, kKC = 32, kLdS = kKC + 4;
constexpr int kRS = kGT / kKC;                           // staging row stride
constexpr int kTPW = (kBM / 16) * (kBN / 16) / kGW;      // tiles per wave
constexpr int kPanel = (kBM + kBN) * kLdS;  // A rows then B rows
constexpr int kGemmLds = 2 * kPanel;        // double-buffered

// LNE: the forward of a layer at most kBN = 64 wide with its LayerNorm(+affine)
// / ReLU in the epilogue.  Each wave then owns WHOLE rows (m-tiles wave and
// wave + kGW, all four n-tile slots), so a row's statistics are register sums
// over the wave's tiles plus one DPP row reduction over the 16 column lanes:
// no separate row pass, no re-read of the pre-activations.  L / base / pr / bp
// describe the layer's outputs (as fwd_rows).
// MODE 2: the dX GEMM of a layer whose source S = L (passed as L) is at most
// kBN wide: the epilogue runs S's ReLU / LayerNorm(+affine) backward on the
// whole rows of dY it holds and writes S's dZ (dzr_s / dzc_s) and per-wave
// bias / LN-affine column partials (colp_s): S needs no row pass of its own.
template <int MODE = 0, class FE>
__device__ __forceinline__ void gemm_nt(const float *A, int lda, const float *B, int ldb, int M, int N, int K,
                                        float *lds, const float *bias, FE epi, const GLay &L,
                                        float *base = nullptr, const float *pr = nullptr, int bp = 0,
                                        float *dzr_s = nullptr, float *dzc_s = nullptr, float *colp_s = nullptr) {
    constexpr bool LNE = MODE == 1, ROWS = MODE != 0;  // ROWS: each wave owns whole rows
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int lr = tid / kKC, lk = tid % kKC;  // staging: rows lr + kRS i, column lk
    float cb[4] = {0.f, 0.f, 0.f, 0.f}, cg[4] = {0.f, 0.f, 0.f, 0.f}, cbe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int mb = 0; mb < M; mb += kBM)
        for (int nb = 0; nb < N; nb += kBN) {
            const int BM = M - mb < kBM ? M - mb : kBM, BN = N - nb < kBN ? N - nb : kBN;
            const int mtn = (BM + 15) >> 4, ntn = (BN + 15) >> 4, T = mtn * ntn;
            // slot j of this wave -> tile (m0, n0), valid (wave-uniform)
            auto tile = [&](int j, int &m0, int &n0) -> bool {
                if constexpr (ROWS) {
                    const int mt = wave + kGW * (j >> 2), nt = j & 3;
                    m0 = mt << 4;
                    n0 = nt << 4;
                    return mt < mtn && nt < ntn;
                } else {
                    const int t = wave + kGW * j;
                    m0 = (t % mtn) << 4;
                    n0 = (t / mtn) << 4;
                    return t < T;
                }
            };
            const float *Ab = A + (size_t)mb * lda, *Bb = B + (size_t)nb * ldb;
            float ra[kBM / kRS], rb[kBN / kRS];
            auto fetch = [&](int kc) {
                const int k = kc + lk;
                const bool kin = k < K;
                const int kk = kin ? k : 0;
                // unconditional loads from clamped (valid) addresses, then the predicate
#pragma unroll
                for (int i = 0; i < kBM / kRS; ++i) {
                    const int row = lr + kRS * i;
                    const float va = Ab[(size_t)(row < BM ? row : 0) * lda + kk];
                    ra[i] = (row < BM && kin) ? va : 0.f;
                }
#pragma unroll
                for (int i = 0; i < kBN / kRS; ++i) {
                    const int row = lr + kRS * i;
                    const float vb = Bb[(size_t)(row < BN ? row : 0) * ldb + kk];
                    rb[i] = (row < BN && kin) ? vb : 0.f;
                }
            };
            auto commit = [&](int buf) {
                float *As = lds + buf * kPanel, *Bs = As + kBM * kLdS;
#pragma unroll
                for (int i = 0; i < kBM / kRS; ++i) As[(lr + kRS * i) * kLdS + lk] = ra[i];
#pragma unroll
                for (int i = 0; i < kBN / kRS; ++i) Bs[(lr + kRS * i) * kLdS + lk] = rb[i];
            };
            f4 acc[kTPW];
            // per slot: the bias of column n0 + r (and with LNE the LN affine),
            // loaded with the first chunk: the latency hides under the panel fetch
            float bv_[kTPW];
#pragma unroll
            for (int j = 0; j < kTPW; ++j) {
                acc[j] = f4{0.f, 0.f, 0.f, 0.f};
                int m0, n0;
                const bool ok = tile(j, m0, n0) && n0 + r < BN;
                const float v = bias ? bias[nb + (ok ? n0 + r : 0)] : 0.f;
                bv_[j] = v;
            }
            fetch(0);
            if (mb | nb) __syncthreads();  // the previous block's last panels may still be read
            commit(0);
            __syncthreads();
            int buf = 0;
            for (int kc = 0; kc < K; kc += kKC) {
                const bool more = kc + kKC < K;
                if (more) fetch(kc + kKC);
                const float *As = lds + buf * kPanel, *Bs = As + kBM * kLdS;
#pragma unroll
                for (int j = 0; j < kTPW; ++j) {
                    int m0, n0;
                    if (tile(j, m0, n0)) {  // wave-uniform
                        float av[8], bv[8];
#pragma unroll
                        for (int kk = 0; kk < 8; ++kk) {
                            av[kk] = As[(m0 + r) * kLdS + 4 * kk + q];
                            bv[kk] = Bs[(n0 + r) * kLdS + 4 * kk + q];
                        }
#pragma unroll
                        for (int kk = 0; kk < 8; ++kk)
                            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bv[kk], acc[j], 0, 0, 0);
                    }
                }
                // the last chunk needs no barrier: the epilogue touches no panel, and
                // every caller separates two GEMMs by a workgroup barrier
                if (more) {
                    commit(buf ^ 1);
                    __syncthreads();
                }
                buf ^= 1;
            }
            if constexpr (LNE) {
                const float invF = 1.f / (float)N;
                // the LN affine of the lane's four columns, loaded before any store
                float ga_[4], be_[4];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const int n = (nt < ntn && (nt << 4) + r < BN) ? (nt << 4) + r : 0;
                    const float gv = pr[L.ln == 2 ? L.g + n : 0], bb = pr[L.ln == 2 ? L.be + n : 0];
                    ga_[nt] = L.ln == 2 ? gv : 1.f;
                    be_[nt] = L.ln == 2 ? bb : 0.f;
                }
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    if (wave + kGW * a >= mtn) break;  // wave-uniform
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = mb + ((wave + kGW * a) << 4) + 4 * q + i;
                        float v[4], s = 0.f;
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) {
                            const bool on = nt < ntn && (nt << 4) + r < BN;
                            v[nt] = on ? acc[4 * a + nt][i] + bv_[4 * a + nt] : 0.f;
                            s += v[nt];
                        }
                        float mean = 0.f, rstd = 1.f;
                        if (L.ln) {
                            mean = rsum16(s) * invF;
                            float vs = 0.f;
#pragma unroll
                            for (int nt = 0; nt < 4; ++nt) {
                                const float d = v[nt] - mean;
                                vs += (nt < ntn && (nt << 4) + r < BN) ? d * d : 0.f;
                            }
                            rstd = 1.f / sqrtf(rsum16(vs) / (float)N + 1e-5f);
                            if (r == 0 && row < M && L.rs >= 0) base[L.rs + row] = rstd;
                        }
                        if (row < M) {
#pragma unroll
                            for (int nt = 0; nt < 4; ++nt) {
                                const int n = (nt << 4) + r;
                                if (nt < ntn && n < BN) {
                                    float y = v[nt];
                                    if (L.ln) {
                                        const float xh = (y - mean) * rstd;
                                        if (L.xh >= 0) base[L.xh + (size_t)row * N + n] = xh;
                                        y = L.ln == 2 ? xh * ga_[nt] + be_[nt] : xh;
                                    }
                                    if (L.relu) y = relu(y);
                                    epi(row, n, y);
                                    if (L.yc >= 0) base[L.yc + (size_t)n * bp + row] = y;
                                }
                            }
                        }
                    }
                }
            } else if constexpr (MODE == 2) {
                const float invF = 1.f / (float)N;
                // every load of the epilogue before its first store: the LN affine of
                // the lane's columns, each row's rstd and the lane's xhat (or y)
                float ga_[4], be_[4];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const int n = (nt < ntn && (nt << 4) + r < BN) ? (nt << 4) + r : 0;
                    const float gv = pr[L.ln == 2 ? L.g + n : 0], bb = pr[L.ln == 2 ? L.be + n : 0];
                    ga_[nt] = L.ln == 2 ? gv : 1.f;
                    be_[nt] = L.ln == 2 ? bb : 0.f;
                }
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    if (wave + kGW * a >= mtn) break;  // wave-uniform
                    // the m-tile's loads (16 rows of xhat or y, their rstd) ahead of its stores
                    float xv[4][4], rsv[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = mb + ((wave + kGW * a) << 4) + 4 * q + i;
                        const bool rok = row < M;
                        const float rv = base[L.ln && rok ? L.rs + row : 0];
                        rsv[i] = L.ln ? rv : 1.f;
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) {
                            const int n = (nt << 4) + r;
                            const bool on = rok && nt < ntn && n < BN;
                            const size_t o = on ? (size_t)row * N + n : 0;
                            const float x = base[L.ln ? L.xh + o : (L.relu ? L.yr + o : 0)];
                            xv[i][nt] = on ? x : 0.f;
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = mb + ((wave + kGW * a) << 4) + 4 * q + i;
                        float dp[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) {
                            const bool on = nt < ntn && (nt << 4) + r < BN && row < M;
                            const float x = xv[i][nt];
                            const float pre = L.ln == 2 ? x * ga_[nt] + be_[nt] : x;
                            dp[nt] = (on && (!L.relu || pre > 0.f)) ? acc[4 * a + nt][i] : 0.f;
                            const float dx = dp[nt] * ga_[nt];
                            s1 += dx;
                            s2 += dx * x;
                        }
                        float m1 = 0.f, m2 = 0.f;
                        if (L.ln) {
                            m1 = rsum16(s1) * invF;
                            m2 = rsum16(s2) * invF;
                        }
                        if (row < M) {
#pragma unroll
                            for (int nt = 0; nt < 4; ++nt) {
                                const int n = (nt << 4) + r;
                                if (nt < ntn && n < BN) {
                                    const float x = xv[i][nt];
                                    const float dz = L.ln ? rsv[i] * (dp[nt] * ga_[nt] - m1 - x * m2) : dp[nt];
                                    dzr_s[(size_t)row * N + n] = dz;
                                    dzc_s[(size_t)n * bp + row] = dz;
                                    cb[nt] += dz;
                                    cg[nt] += dp[nt] * x;
                                    cbe[nt] += dp[nt];
                                }
                            }
                        }
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < kTPW; ++j) {
                    int m0, n0;
                    if (tile(j, m0, n0)) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int m = m0 + 4 * q + i, n = n0 + r;
                            if (m < BM && n < BN) epi(mb + m, nb + n, acc[j][i] + bv_[j]);
                        }
                    }
                }
            }
        }
    if constexpr (MODE == 2) {
        // the wave's four row groups (lanes l, l ^ 16, l ^ 32, l ^ 48), then per
        // wave into colp_s (the caller sums the waves in order)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            cb[nt] += __shfl_xor(cb[nt], 16, 64);
            cb[nt] += __shfl_xor(cb[nt], 32, 64);
            cg[nt] += __shfl_xor(cg[nt], 16, 64);
            cg[nt] += __shfl_xor(cg[nt], 32, 64);
            cbe[nt] += __shfl_xor(cbe[nt], 16, 64);
            cbe[nt] += __shfl_xor(cbe[nt], 32, 64);
        }
        if (q == 0) {
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const int n = (nt << 4) + r;
                if (n < N) {
                    colp_s[wave * N + n] = cb[nt];
                    colp_s[(kGW + wave) * N + n] = cg[nt];
                    colp_s[(2 * kGW + wave) * N + n] = cbe[nt];
                }
            }
        }
    }
}

// fixed-order workgroup sum of two per-thread values
__device__ __forceinline__ void block_sum2(float &a, float &b, float *red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    a = wave_sum(a);
    b = wave_sum(b);
    __syncthreads();  // red may still be read by the previous call
    if (lane == 0) {
        red[wave] = a;
        red[kGW + wave] = b;
    }
    __syncthreads();
    float ta = 0.f, tb = 0.f;
    for (int i = 0; i < kGW; ++i) {
        ta += red[i];
        tb += red[kGW + i];
    }
    a = ta;
    b = tb;
}

// LayerNorm(+affine) / ReLU forward of one layer's rows, 16 lanes per row;
// rows r, r + 32, r + 64, r + 96 of a 128-row block are processed together
// with C columns per lane cached in registers (F <= 16 C): all loads of the
// block are issued before the first reduction (one round trip, not three per
// row).  C = 0: any width, three passes over the row per 32 rows.
template <int C>
__device__ __forceinline__ void fwd_rows(const GLay &L, float *base, const float *pr, int bsz, int bp) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    float *yr = base + L.yr;
    const int F = L.fout;
    const float invF = 1.f / (float)F;
    auto out = [&](int row, int j, float y, float mean, float rstd, float ga, float be) {
        if (L.ln) {
            const float xh = (y - mean) * rstd;
            if (L.xh >= 0) base[L.xh + (size_t)row * F + j] = xh;
            y = L.ln == 2 ? xh * ga + be : xh;
        }
        if (L.relu) y = relu(y);
        yr[(size_t)row * F + j] = y;
        if (L.yc >= 0) base[L.yc + (size_t)j * bp + row] = y;
    };
    if constexpr (C > 0) {
        constexpr int R = 4;
        // the LN affine of the lane's columns, loaded before any store
        float ga[C], be[C];
#pragma unroll
        for (int i = 0; i < C; ++i) {
            const int j = sub + 16 * i < F ? sub + 16 * i : 0;
            const float a = pr[L.ln == 2 ? L.g + j : 0], b = pr[L.ln == 2 ? L.be + j : 0];
            ga[i] = a;
            be[i] = b;
        }
        for (int r0 = 0; r0 < bsz; r0 += R * 4 * kGW) {
            float z[R][C];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int row = r0 + 4 * wave + rq + 4 * kGW * u;
#pragma unroll
                for (int i = 0; i < C; ++i) {
                    const int j = sub + 16 * i;
                    const bool on = row < bsz && j < F;
                    const float v = yr[on ? (size_t)row * F + j : 0];
                    z[u][i] = on ? v : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int row = r0 + 4 * wave + rq + 4 * kGW * u;
                float mean = 0.f, rstd = 1.f;
                if (L.ln) {
                    float s = 0.f;
#pragma unroll
                    for (int i = 0; i < C; ++i) s += z[u][i];
                    mean = rsum16(s) * invF;
                    float vs = 0.f;
#pragma unroll
                    for (int i = 0; i < C; ++i) {
                        const float d = z[u][i] - mean;
                        vs += (sub + 16 * i < F) ? d * d : 0.f;
                    }
                    rstd = 1.f / sqrtf(rsum16(vs) / (float)F + 1e-5f);
                    if (row < bsz && sub == 0 && L.rs >= 0) base[L.rs + row] = rstd;
                }
                if (row < bsz) {
#pragma unroll
                    for (int i = 0; i < C; ++i) {
                        const int j = sub + 16 * i;
                        if (j < F) out(row, j, z[u][i], mean, rstd, ga[i], be[i]);
                    }
                }
            }
        }
    } else {
        for (int r0 = 0; r0 < bsz; r0 += 4 * kGW) {
            const int row = r0 + 4 * wave + rq;
            const bool live = row < bsz;
            float s = 0.f;
            if (live)
                for (int j = sub; j < F; j += 16) s += yr[(size_t)row * F + j];
            float mean = 0.f, rstd = 1.f;
            if (L.ln) {
                mean = rsum16(s) * invF;
                float vs = 0.f;
                if (live)
                    for (int j = sub; j < F; j += 16) {
                        const float dz = yr[(size_t)row * F + j] - mean;
                        vs += dz * dz;
                    }
                rstd = 1.f / sqrtf(rsum16(vs) / (float)F + 1e-5f);
                if (live && sub == 0 && L.rs >= 0) base[L.rs + row] = rstd;
            }
            if (!live) continue;
            for (int j = sub; j < F; j += 16)
                out(row, j, yr[(size_t)row * F + j], mean, rstd, L.ln == 2 ? pr[L.g + j] : 1.f,
                    L.ln == 2 ? pr[L.be + j] : 0.f);
        }
    }
}

// LayerNorm(+affine) / ReLU backward of one layer's rows: dY -> dZ (row-major
// dzr and feature-major dzc), plus dY' xhat and dY' feature-major (t1c, t2c)
// for the LN-affine gradients.  As fwd_rows: C columns per lane cached for
// 16 / C rows at once (F <= 16 C); C = 0: any width, re-reading the row.
// C > 0 also takes the bias / LN-affine column sums: per lane over its rows,
// across the wave's four row groups, then per wave into colp (LDS, [3][kGW][F]);
// the caller adds the waves in order.  No t1c / t2c round trip through memory.
template <int C>
__device__ __forceinline__ void bwd_rows(const GLay &L, float *base, const float *pr, int bsz, int bp, float *dzr,
                                         float *dzc, float *t1c, float *t2c, float *colp = nullptr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    const int F = L.fout;
    const float invF = 1.f / (float)F;
    const float *dy = base + L.dy;
    auto put = [&](int row, int j, float d, float xh, float dz) {
        if (L.ln == 2) {
            t1c[(size_t)j * bp + row] = d * xh;
            t2c[(size_t)j * bp + row] = d;
        }
        dzr[(size_t)row * F + j] = dz;
        dzc[(size_t)j * bp + row] = dz;
    };
    if constexpr (C > 0) {
        constexpr int R = 16 / C;  // 16 cached columns per lane: three loads each in flight
        // LN affine of the lane's columns (the ReLU mask of an LN layer is
        // recomputed from xhat: the same float ops as the forward, no y load)
        float gam[C], bet[C];
#pragma unroll
        for (int i = 0; i < C; ++i) {
            const int j = sub + 16 * i;
            const float v = pr[L.ln == 2 ? L.g + (j < F ? j : 0) : 0];
            const float b = pr[L.ln == 2 ? L.be + (j < F ? j : 0) : 0];
            gam[i] = L.ln == 2 ? v : 1.f;
            bet[i] = L.ln == 2 ? b : 0.f;
        }
        float cb[C], cg[C], cbe[C];  // the lane's column partial sums (dz, dy' xhat, dy')
#pragma unroll
        for (int i = 0; i < C; ++i) cb[i] = cg[i] = cbe[i] = 0.f;
        for (int r0 = 0; r0 < bsz; r0 += R * 4 * kGW) {
            float dp[R][C], xh[R][C], rs[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int row = r0 + 4 * wave + rq + 4 * kGW * u;
                const int rr = row < bsz ? row : 0;
                const float rv = base[L.ln ? L.rs + rr : 0];
                rs[u] = L.ln ? rv : 1.f;
#pragma unroll
                for (int i = 0; i < C; ++i) {
                    const int j = sub + 16 * i;
                    const bool on = row < bsz && j < F;
                    const size_t o = on ? (size_t)row * F + j : 0;
                    const float d = dy[o], d2 = base[L.dy2 >= 0 ? L.dy2 + o : 0];
                    const float y = base[(L.relu && !L.ln) ? L.yr + o : 0];
                    const float x = base[L.ln ? L.xh + o : 0];
                    const float pre = L.ln == 2 ? x * gam[i] + bet[i] : (L.ln ? x : y);
                    dp[u][i] = (on && (!L.relu || pre > 0.f)) ? (L.dy2 >= 0 ? d + d2 : d) : 0.f;
                    xh[u][i] = (on && L.ln) ? x : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int row = r0 + 4 * wave + rq + 4 * kGW * u;
                float m1 = 0.f, m2 = 0.f;
                if (L.ln) {
                    float s1 = 0.f, s2 = 0.f;
#pragma unroll
                    for (int i = 0; i < C; ++i) {
                        const float dx = dp[u][i] * gam[i];
                        s1 += dx;
                        s2 += dx * xh[u][i];
                    }
                    m1 = rsum16(s1) * invF;
                    m2 = rsum16(s2) * invF;
                }
                if (row < bsz) {
#pragma unroll
                    for (int i = 0; i < C; ++i) {
                        const int j = sub + 16 * i;
                        if (j < F) {
                            const float dz = L.ln ? rs[u] * (dp[u][i] * gam[i] - m1 - xh[u][i] * m2) : dp[u][i];
                            dzr[(size_t)row * F + j] = dz;
                            dzc[(size_t)j * bp + row] = dz;
                            cb[i] += dz;
                            cg[i] += dp[u][i] * xh[u][i];
                            cbe[i] += dp[u][i];
                        }
                    }
                }
            }
        }
        // the four row groups of the wave (lanes l, l ^ 16, l ^ 32, l ^ 48), one fixed order
#pragma unroll
        for (int i = 0; i < C; ++i) {
            cb[i] += __shfl_xor(cb[i], 16, 64);
            cb[i] += __shfl_xor(cb[i], 32, 64);
            if (L.ln == 2) {
                cg[i] += __shfl_xor(cg[i], 16, 64);
                cg[i] += __shfl_xor(cg[i], 32, 64);
                cbe[i] += __shfl_xor(cbe[i], 16, 64);
                cbe[i] += __shfl_xor(cbe[i], 32, 64);
            }
        }
        if (rq == 0) {
#pragma unroll
            for (int i = 0; i < C; ++i) {
                const int j = sub + 16 * i;
                if (j < F) {
                    colp[wave * F + j] = cb[i];
                    colp[(kGW + wave) * F + j] = cg[i];
                    colp[(2 * kGW + wave) * F + j] = cbe[i];
                }
            }
        }
    } else {
        for (int r0 = 0; r0 < bsz; r0 += 4 * kGW) {
            const int row = r0 + 4 * wave + rq;
            const bool live = row < bsz;
            // d(pre-activation) of column j: dY masked by the ReLU
            auto dpre = [&](int j) {
                const float d = dy[(size_t)row * F + j] + (L.dy2 >= 0 ? base[L.dy2 + (size_t)row * F + j] : 0.f);
                return (!L.relu || base[L.yr + (size_t)row * F + j] > 0.f) ? d : 0.f;
            };
            float m1 = 0.f, m2 = 0.f, rstd = 1.f;
            if (L.ln) {
                float s1 = 0.f, s2 = 0.f;
                if (live)
                    for (int j = sub; j < F; j += 16) {
                        const float dx = L.ln == 2 ? dpre(j) * pr[L.g + j] : dpre(j);
                        s1 += dx;
                        s2 += dx * base[L.xh + (size_t)row * F + j];
                    }
                m1 = rsum16(s1) * invF;
                m2 = rsum16(s2) * invF;
                rstd = live ? base[L.rs + row] : 0.f;
            }
            if (!live) continue;
            for (int j = sub; j < F; j += 16) {
                const float d = dpre(j);
                float dz = d, xh = 0.f;
                if (L.ln) {
                    xh = base[L.xh + (size_t)row * F + j];
                    const float dx = L.ln == 2 ? d * pr[L.g + j] : d;
                    dz = rstd * (dx - m1 - xh * m2);
                }
                put(row, j, d, xh, dz);
            }
        }
    }
}

// Forward of a minibatch (or a block of env rows) through the layer list:
// GEMM + bias -> Ls[l].yr, then LayerNorm(+affine) / ReLU as a row pass,
// keeping xhat / rstd / the feature-major copy where the plan has room for
// them (the learner; the policy step keeps outputs only).  xobs: the
// observation rows (stride = the first layer's fin).
__device__ __forceinline__ void forward_layers(const GLay *Ls, int nl, const float *xobs, int bsz, float *base, const float *pr,
                               int bp, float *lds, int dbg = 0, long long *st = nullptr) {
    for (int l = 0; l < nl; ++l) {
        const GLay &L = Ls[l];
        const float *x = L.src < 0 ? xobs : base + Ls[L.src].yr;
        float *yr = base + L.yr;
        const int F = L.fout;
        const float *bias = pr + L.b;
        const bool lne = F <= kBN && (L.ln || L.relu);  // LayerNorm / ReLU in the GEMM epilogue
        if (!(dbg & 1)) {
            if (lne)
                gemm_nt<1>(x, L.fin, pr + L.w, L.fin, bsz, F, L.fin, lds, bias,
                                   [&](int m, int n, float c) { yr[(size_t)m * F + n] = c; }, L, base, pr, bp);
            else
                gemm_nt<0>(x, L.fin, pr + L.w, L.fin, bsz, F, L.fin, lds, bias,
                                   [&](int m, int n, float c) { yr[(size_t)m * F + n] = c; }, L);
        }
        __syncthreads();
        if (lne || (L.ln == 0 && !L.relu && L.yc < 0) || (dbg & 8)) {
            if (st) st[1 + l] = (long long)__builtin_readcyclecounter();
            continue;
        }
        if (F <= 128) fwd_rows<8>(L, base, pr, bsz, bp);
        else fwd_rows<0>(L, base, pr, bsz, bp);
        __syncthreads();
        if (st) st[1 + l] = (long long)__builtin_readcyclecounter();
    }
}

// One minibatch's forward, PPO loss and backward over `bsz` rows (rows
// s0 .. s0 + bsz - 1 of the epoch's minibatch-ordered rollout, observations at
// xobs), accumulating the gradient row G (every entry written: dW by GEMM
// epilogues, bias / LN-affine sums by the column passes) and the loss / approx_kl
// partial sums.  inv_b = 1 / the whole minibatch's size (the loss is a mean over
// it).  base: this workgroup's activation scratch; wb: where the transposed
// weights live (wb + L.wt).  Shared by the one-workgroup-per-agent learner and
// the partnered one (each partner over its slice of the rows).
__device__ __forceinline__ void minibatch_grads(const GArgs &g, float *base, const float *wb, const float *pr, float *G,
                                                const float *xobs, const int *gact_e, const unsigned *gmask_e,
                                                const float *grow_e, long long s0, int bsz, float inv_b, float entp,
                                                float *lds, float *colp, float *colo, float &lsum, float &klsum,
                                                long long *st = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    const int bp = g.bp, A = g.A, D = g.D;
    const long long S = g.S;
    (void)wave;
    // observation, feature-major (the first layer's dW operand)
    for (int i = tid; i < bsz * D; i += kGT) {
        const int b = i / D, d = i - b * D;
        base[g.oc + (size_t)d * bp + b] = xobs[i];
    }

    // ---- forward, layer by layer ------------------------------------
    if (st) st[0] = (long long)__builtin_readcyclecounter();
    forward_layers(g.L, g.nl, xobs, bsz, base, pr, bp, lds, g.dbg, st);

    // ---- loss row pass: logits / value -> d(logits), d(value) (ppo.py:876-908)
    if (!(g.dbg & 8)) {
        const GLay &La = g.L[g.aout];
        const GLay &Lc = g.L[g.cout];
        const float *lgp = base + La.yr;
        const float *vp = base + Lc.yr;
        float *dla = base + La.dy;
        float *dlac = base + La.dyc;
        float *dlv = base + Lc.dy;
        const int a0 = sub, a1 = sub + 16;
        float cb0 = 0.f, cb1 = 0.f, cbv = 0.f;  // output-layer bias gradients (column partials)
        // four rows per 16-lane group at once: every input of the 128-row
        // block is loaded before the first reduction
        constexpr int R = 4;
        for (int rb = 0; rb < bsz; rb += R * 4 * kGW) {
            unsigned pbits[R];
            int pact[R];
            float plg0[R], plg1[R], polp[R], pad[R], pret[R], pov[R], pv[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int row0 = rb + 4 * wave + rq + 4 * kGW * u;
                const int row = row0 < bsz ? row0 : 0;
                pbits[u] = gmask_e ? gmask_e[s0 + row] : 0xffffffffu;
                plg0[u] = lgp[(size_t)row * A + (a0 < A ? a0 : 0)];
                plg1[u] = lgp[(size_t)row * A + (a1 < A ? a1 : 0)];
                pact[u] = gact_e[s0 + row];
                polp[u] = grow_e[s0 + row];
                pad[u] = grow_e[S + s0 + row];
                pret[u] = grow_e[2 * S + s0 + row];
                pov[u] = grow_e[3 * S + s0 + row];
                pv[u] = vp[row];
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
            const int row0 = rb + 4 * wave + rq + 4 * kGW * u;
            const bool live = row0 < bsz;
            const int row = live ? row0 : 0;
            const unsigned bits = pbits[u];
            const bool ok0 = (bits >> a0) & 1u, ok1 = (bits >> a1) & 1u;
            const float lg0 = a0 < A ? (ok0 ? plg0[u] : -1.0e8f) : -3.0e38f;
            const float lg1 = a1 < A ? (ok1 ? plg1[u] : -1.0e8f) : -3.0e38f;
            const float mx = rmax16(fmaxf(lg0, lg1));
            const float ex0 = a0 < A ? expf(lg0 - mx) : 0.f, ex1 = a1 < A ? expf(lg1 - mx) : 0.f;
            const float lse = mx + logf(rsum16(ex0 + ex1));
            const float p0 = a0 < A ? expf(lg0 - lse) : 0.f, p1 = a1 < A ? expf(lg1 - lse) : 0.f;
            const float lpe0 = logf(p0 + 1e-8f), lpe1 = logf(p1 + 1e-8f);
            const float Hs = -rsum16((a0 < A ? p0 * lpe0 : 0.f) + (a1 < A ? p1 * lpe1 : 0.f));
            const float gh0 = -(lpe0 + p0 / (p0 + 1e-8f)), gh1 = -(lpe1 + p1 / (p1 + 1e-8f));
            const float pg = rsum16((a0 < A ? p0 * gh0 : 0.f) + (a1 < A ? p1 * gh1 : 0.f));
            const int a_t = pact[u];
            const int srcl = (lane & ~15) + (a_t & 15);
            const float t0 = bperm(srcl, lg0), t1 = bperm(srcl, lg1);
            const float logp = (a_t < 16 ? t0 : t1) - lse;
            const float olp = polp[u], Ad = pad[u], Rt = pret[u], ov = pov[u];
            const float lo = 1.f - g.clip, hi = 1.f + g.clip;
            const float lrt = logp - olp;
            const float ratio = expf(lrt);
            const float rcl = fminf(fmaxf(ratio, lo), hi);
            const float q1 = -Ad * ratio, q2 = -Ad * rcl;
            const float g1 = q1 > q2 ? 1.f : (q1 == q2 ? 0.5f : 0.f);
            const float g2 = q2 > q1 ? 1.f : (q1 == q2 ? 0.5f : 0.f);
            const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
            const float g_logp = ((g1 * -Ad + g2 * -Ad * inr) * inv_b) * ratio;
            const float v = pv[u];
            const float dv = v - ov;
            const float vcl = ov + fminf(fmaxf(dv, -g.clip), g.clip);
            const float eu = v - Rt, ec = vcl - Rt;
            const float lu = eu * eu, lc = ec * ec;
            const float gu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
            const float gc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
            const float inv = (dv >= -g.clip && dv <= g.clip) ? 1.f : 0.f;
            const float g_H = -entp * inv_b;
            const float dl0 = g_logp * ((a0 == a_t ? 1.f : 0.f) - p0) + g_H * p0 * (gh0 - pg);
            const float dl1 = g_logp * ((a1 == a_t ? 1.f : 0.f) - p1) + g_H * p1 * (gh1 - pg);
            if (live) {
                const float d0 = ok0 ? dl0 : 0.f, d1 = ok1 ? dl1 : 0.f;
                if (a0 < A) {
                    dla[(size_t)row * A + a0] = d0;
                    dlac[(size_t)a0 * bp + row] = d0;
                    cb0 += d0;
                }
                if (a1 < A) {
                    dla[(size_t)row * A + a1] = d1;
                    dlac[(size_t)a1 * bp + row] = d1;
                    cb1 += d1;
                }
                if (sub == 0) {
                    const float dvv = g.vf * 0.5f * inv_b * (gu * 2.f * eu + gc * 2.f * ec * inv);
                    dlv[row] = dvv;
                    cbv += dvv;
                    lsum += (fmaxf(q1, q2) + g.vf * 0.5f * fmaxf(lu, lc) - entp * Hs) * inv_b;
                    klsum += ((ratio - 1.f) - lrt) * inv_b;  // approx_kl (ppo.py:899-902)
                }
            }
            }
        }
        // bias gradients of the output layers: the wave's four row groups,
        // then per wave into LDS (summed over the waves in order below)
        cb0 += __shfl_xor(cb0, 16, 64);
        cb0 += __shfl_xor(cb0, 32, 64);
        cb1 += __shfl_xor(cb1, 16, 64);
        cb1 += __shfl_xor(cb1, 32, 64);
        cbv += __shfl_xor(cbv, 16, 64);
        cbv += __shfl_xor(cbv, 32, 64);
        if (rq == 0) {
            colo[wave * 33 + a0] = cb0;
            colo[wave * 33 + a1] = cb1;
            if (sub == 0) colo[wave * 33 + 32] = cbv;
        }
    }
    __syncthreads();
    if (!(g.dbg & 8) && tid <= A) {
        float sb = 0.f;
        for (int w = 0; w < kGW; ++w) sb += colo[w * 33 + (tid < A ? tid : 32)];
        G[tid < A ? g.L[g.aout].b + tid : g.L[g.cout].b] = sb;
    }
    if (st) st[17] = (long long)__builtin_readcyclecounter();

    // ---- backward, layer by layer (reverse) ----------------------------
    float *t1c = base + g.t1, *t2c = base + g.t2;
    for (int l = g.nl - 1; l >= 0; --l) {
        const GLay &L = g.L[l];
        const int F = L.fout;
        float *dzr = base + ((l & 1) ? g.dzr1 : g.dzr), *dzc = base + ((l & 1) ? g.dzc1 : g.dzc);
        float *colp_l = colp + (l & 1) * 3 * kGW * 128;
        // output layers: the loss pass wrote dZ in both layouts and the bias gradient;
        // fused layers: the consumer's dX epilogue wrote dZ and the column partials
        const bool outl = L.dyc >= 0;
        // dY -> dZ through ReLU and LayerNorm(+affine)
        if (!(g.dbg & 8) && !outl && !L.fused) {
            if (F <= 128) bwd_rows<8>(L, base, pr, bsz, bp, dzr, dzc, t1c, t2c, colp_l);
            else bwd_rows<0>(L, base, pr, bsz, bp, dzr, dzc, t1c, t2c);
        }
        if (!outl && !L.fused) __syncthreads();
        if (st) st[18 + 3 * l] = (long long)__builtin_readcyclecounter();
        // bias / LN-affine gradients: column sums over the rows (fixed order);
        // up to 8 feature groups summed before the first store
        if (F <= 128 && !(g.dbg & 24) && !outl) {  // the row pass left per-wave partials in LDS
            for (int o = tid; o < F; o += kGT) {
                float sb = 0.f, sg = 0.f, sbe = 0.f;
                for (int w = 0; w < kGW; ++w) {
                    sb += colp_l[w * F + o];
                    sg += colp_l[(kGW + w) * F + o];
                    sbe += colp_l[(2 * kGW + w) * F + o];
                }
                G[L.b + o] = sb;
                if (L.ln == 2) {
                    G[L.g + o] = sg;
                    G[L.be + o] = sbe;
                }
            }
        }
        for (int ob = 0; ob < ((g.dbg & 16) || F <= 128 || outl ? 0 : F); ob += 8 * 4 * kGW) {
            float rb_[8], rg_[8], rbe_[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int o = ob + 4 * kGW * k + 4 * wave + rq;
                const bool on = o < F;
                float sb = 0.f, sg = 0.f, sbe = 0.f;
                if (ob + 4 * kGW * k < F) {  // wave-uniform
                    for (int b = sub; b < bsz; b += 16) {
                        const size_t x = (size_t)(on ? o : 0) * bp + b;
                        const float v0 = dzc[x];
                        sb += on ? v0 : 0.f;
                        if (L.ln == 2) {
                            const float v1 = t1c[x], v2 = t2c[x];
                            sg += on ? v1 : 0.f;
                            sbe += on ? v2 : 0.f;
                        }
                    }
                }
                rb_[k] = rsum16(sb);
                rg_[k] = L.ln == 2 ? rsum16(sg) : 0.f;
                rbe_[k] = L.ln == 2 ? rsum16(sbe) : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int o = ob + 4 * kGW * k + 4 * wave + rq;
                if (o < F && sub == 0) {
                    G[L.b + o] = rb_[k];
                    if (L.ln == 2) {
                        G[L.g + o] = rg_[k];
                        G[L.be + o] = rbe_[k];
                    }
                }
            }
        }
        // dW = dZ^T X (contraction over the rows), then dX = dZ W into the
        // source's dY (one GEMM call site for both: instruction-cache footprint)
        const float *xc = L.src < 0 ? base + g.oc : base + g.L[L.src].yc;
        const int fin = L.fin;
        for (int job = 0; job < (L.src >= 0 ? 2 : 1); ++job) {
            if (job) __syncthreads();  // the dW GEMM's last panels are still being read
            if (st && job) st[19 + 3 * l] = (long long)__builtin_readcyclecounter();
            if (g.dbg & (job ? 4 : 2)) continue;
            const float *ga = job ? (outl ? base + L.dy : dzr) : (outl ? base + L.dyc : dzc);
            const float *gb = job ? wb + L.wt : xc;
            const int lda = job ? F : bp, ldb = job ? F : bp;
            const int M = job ? bsz : F, K = job ? F : bsz;
            float *dst = job ? base + (L.acc ? g.L[L.src].dy2 : g.L[L.src].dy) : G + L.w;
            if (job && L.fuse) {  // the source's dZ (other parity) from the epilogue
                const int s_ = L.src;
                gemm_nt<2>(ga, lda, gb, ldb, M, fin, K, lds, nullptr, [](int, int, float) {}, g.L[s_], base, pr,
                           bp, base + ((s_ & 1) ? g.dzr1 : g.dzr), base + ((s_ & 1) ? g.dzc1 : g.dzc),
                           colp + (s_ & 1) * 3 * kGW * 128);
            } else {
                gemm_nt<0>(ga, lda, gb, ldb, M, fin, K, lds, nullptr,
                                   [&](int m, int n, float c) { dst[(size_t)m * fin + n] = c; }, L);
            }
        }
        __syncthreads();
        if (st) st[20 + 3 * l] = (long long)__builtin_readcyclecounter();
    }

}

__global__ __launch_bounds__(kGT) void ppo_learn_graph_kernel(const GArgs g) {
    __shared__ float red[2 * kGW];
    __shared__ __attribute__((aligned(16))) float lds[kGemmLds];
    __shared__ float colp[2 * 3 * kGW * 128];  // per-wave bias / LN-affine column partials (F <= 128), by layer parity
    __shared__ float colo[kGW * 33];       // per-wave output-layer bias partials (32 logits + the value)
    if (g.skip && __hip_atomic_load(g.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    const int p = blockIdx.x;
    const int tid = threadIdx.x;
    float *const pr = g.params + (size_t)p * g.n;
    float *const gm = g.m + (size_t)p * g.n;
    float *const gv = g.v + (size_t)p * g.n;
    float *const base = g.ws + (size_t)p * g.ws_agent;
    float *const G = base + g.gr;
    const int D = g.D;
    const long long S = g.S;

    // transposed weight copies (the dX operand)
    for (int l = 0; l < g.nl; ++l) {
        const GLay &L = g.L[l];
        if (L.wt < 0) continue;
        float *wt = base + L.wt;
        for (int i = tid; i < L.fout * L.fin; i += kGT) {
            const int o = i / L.fin, c = i - o * L.fin;
            wt[(size_t)c * L.fout + o] = pr[L.w + i];
        }
    }
    __syncthreads();

    int Bp = g.batch_p ? g.batch_p[p] : g.B;
    if (Bp > g.B) Bp = g.B;  // the scratch holds g.B rows (the caller's batch: the population's largest)
    const int Ep = g.epochs_p ? g.epochs_p[p] : g.E;
    const float entp = g.ent_p ? g.ent_p[p] : g.ent;
    const int nmb = (int)((S + Bp - 1) / Bp);
    float loss_total = 0.f;
    double kl_total = 0.0;
    int n_done = 0, epochs_done = 0;
    const long long step0 = g.step[p];
    double pb1 = pow((double)g.b1, (double)step0), pb2 = pow((double)g.b2, (double)step0);
    const float lr_p = g.lr[p];

    for (int e = 0; e < Ep; ++e) {
        const size_t ge = (size_t)e * g.P + p;
        const float *gobs_e = g.gobs + ge * S * D;
        const int *gact_e = g.gact + ge * S;
        const unsigned *gmask_e = g.gmask ? g.gmask + ge * S : nullptr;
        const float *grow_e = g.grow + ge * 4 * S;
        for (int mb = 0; mb < nmb; ++mb) {
            const long long s0 = (long long)mb * Bp;
            const int bsz = (int)((s0 + Bp <= S) ? Bp : S - s0);
            const float inv_b = 1.f / (float)bsz;
            const float *xobs = gobs_e + s0 * D;

            float lsum = 0.f, klsum = 0.f;
            minibatch_grads(g, base, base, pr, G, xobs, gact_e, gmask_e, grow_e, s0, bsz, inv_b, entp, lds, colp,
                            colo, lsum, klsum);
            // ---- loss / kl, clip, Adam ------------------------------------------
            block_sum2(lsum, klsum, red);
            if (tid == 0) loss_total += lsum;
            kl_total += (double)klsum;
            ++n_done;
            float q0 = 0.f, q1 = 0.f;
            for (int f = tid; f < g.n; f += kGT) {
                const float x = G[f];
                if (f < g.cstart) q0 += x * x;
                else q1 += x * x;
            }
            block_sum2(q0, q1, red);
            const float c0 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(q0) + 1e-6f), 1.f) : 1.f;
            const float c1 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(q1) + 1e-6f), 1.f) : 1.f;
            pb1 *= (double)g.b1;
            pb2 *= (double)g.b2;
            const float bc1 = (float)(1.0 - pb1);
            const float bc2s = (float)sqrt(1.0 - pb2);
            const float step_size = lr_p / bc1;
            const float ob1 = 1.f - g.b1, ob2 = 1.f - g.b2;
            // Adam over each parameter region, four elements per thread per round:
            // all loads of a round issued before its stores (the stores could
            // alias the loads as far as the compiler knows)
            auto adam_region = [&](int f0, int cnt, long long wt, int fin, int fout) {
                constexpr int U = 16;  // elements per thread per round: all loads, then all stores
                for (int i0 = tid; i0 < cnt; i0 += U * kGT) {
                    float gg[U], mm[U], vv[U], pp[U];
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        const int i = i0 + k * kGT;
                        const int f = f0 + (i < cnt ? i : 0);
                        gg[k] = G[f];
                        mm[k] = gm[f];
                        vv[k] = gv[f];
                        pp[k] = pr[f];
                    }
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        const int i = i0 + k * kGT;
                        if (i >= cnt) break;
                        const int f = f0 + i;
                        const float gc = gg[k] * (f < g.cstart ? c0 : c1);
                        const float m = mm[k] + ob1 * (gc - mm[k]);
                        const float v = vv[k] * g.b2 + ob2 * gc * gc;
                        const float np = pp[k] - step_size * (m / (sqrtf(v) / bc2s + g.eps));
                        gm[f] = m;
                        gv[f] = v;
                        pr[f] = np;
                        if (wt >= 0) {
                            const int o = i / fin, c = i - o * fin;
                            base[wt + (size_t)c * fout + o] = np;
                        }
                    }
                }
            };
            // regions: per layer W (with its transposed copy), b, LN weight, LN bias
            for (int rg = 0; rg < ((g.dbg & 32) ? 0 : 4 * g.nl); ++rg) {
                const GLay &L = g.L[rg >> 2];
                const int kind = rg & 3;
                if (kind >= 2 && L.ln != 2) continue;
                const int f0 = kind == 0 ? L.w : kind == 1 ? L.b : kind == 2 ? L.g : L.be;
                adam_region(f0, kind == 0 ? L.fout * L.fin : L.fout, kind == 0 ? L.wt : -1, kind == 0 ? L.fin : 1,
                            kind == 0 ? L.fout : 1);
            }
            __syncthreads();
        }  // minibatches
        ++epochs_done;
        if (g.target_kl > 0.0 && kl_total / (double)n_done > g.target_kl) break;  // ppo.py:917-918
    }  // epochs
    if (tid == 0) {
        if (g.loss_out) g.loss_out[p] = loss_total / ((float)S * (float)Ep);
        if (g.kl_out) g.kl_out[p] = n_done ? (float)(kl_total / (double)n_done) : 0.f;
        if (g.epochs_out) g.epochs_out[p] = epochs_done;
        g.step[p] = step0 + n_done;
    }
}


// ---------------------------------------------------------------------------
// Partnered runtime-shape learner: an agent's minibatch is split over K
// workgroups ("partners", R rows each) that exchange gradients through L2,
// the compiled learner's scheme (learner.hip) on a runtime layer list:
//   1. each partner runs minibatch_grads over its rows into its own slab of
//      the agent's exchange area (partial gradient row + loss / approx_kl);
//   2. barrier 1, then reduce-scatter: partner kk sums the float4 chunks it
//      owns ([kk cs, (kk + 1) cs)) over the K slabs in partner order, keeps the
//      sums in the agent's sum slab and publishes per-wave partial two-group
//      squared norms;
//   3. barrier 2: every partner sums the K x 4 partial norms in one fixed
//      order (identical clip coefficients everywhere) and runs Adam on its own
//      chunks, writing the parameters, both Adam moments and the transposed
//      weight copy (the dX operand, shared by the agent's partners);
//   4. barrier 3 and an agent-scope acquire: the next update's plain loads of
//      the parameters see every partner's chunks.
// The K partners of an agent are placed on one XCD (block b -> agent b % Q,
// partner b / Q, Q a multiple of 8); that is checked at run time from
// HW_REG_XCC_ID, and a split placement publishes with an agent release (the
// L2 write-back) before every ticket.  Barriers are tickets with bounded spins;
// a timeout sets the caller's error word (AGX_LEARN_ERR_TIMEOUT) and the
// partner exits.  An agent's result depends on K (the row split), never on
// which other agents share the launch.
// ---------------------------------------------------------------------------
constexpr int kMaxGK = 16;
constexpr size_t kLdsMax = 160 * 1024;  // LDS per CU (gfx950)
constexpr unsigned kGSpinMax = 1u << 23;

__device__ __forceinline__ bool gpart_sync(unsigned *ctr, unsigned target, bool release, unsigned *tmo,
                                           unsigned *err, int *s_ok) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's stores have left
    __syncthreads();
    if (threadIdx.x == 0) {
        if (release) {  // partners on other XCDs: write this L2's dirty lines back first
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned before = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        int ok = 1;
        while (before + 1u < target && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kGSpinMax) {
                __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (err) __hip_atomic_fetch_or(err, AGX_LEARN_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// this CU's L1 no longer holds lines other partners have rewritten (the
// parameters after an Adam step): one agent-scope acquire, waited for by the
// whole workgroup before its next plain loads
__device__ __forceinline__ void gpart_acquire() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// inner stamps of minibatch_grads: [0] forward start, [1 + l] layer l's forward
// done, [17] loss pass done, [18 + 3l] / [19 + 3l] / [20 + 3l] layer l's row pass,
// dW and dX done
constexpr int kGStampsIn = 18 + 3 * kGL;

__device__ __forceinline__ float ld_sc1(const float *p) {
    return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- the few-row form (ppo_learn_graph_part_kernel<true>) --------------------
// A partner's slice of at most kFR = 16 minibatch rows stays in LDS for the
// whole update: the observation tile, every layer's output Y, xhat and rstd,
// and dY, each a [16][ld] row-major tile (ld = the width rounded up to 16,
// + 4: float4 row reads spread over the banks).  The padding columns are zero
// from the kernel's start and never written, so every contraction runs over
// whole 16-wide chunks with no masks; rows past the slice carry finite values
// and a zero gradient.  One 16-row MFMA m-tile covers the slice, its n-tiles
// go round the four waves; LayerNorm / ReLU (forward and backward) are row
// passes, 16 lanes per row, one row per lane group; bias / LN-affine
// gradients are column sums over the 16 rows, one thread per column, in row
// order.  Weights come from L2 (buffer loads, the agent's partners share
// them): W [out][in] for the forward, the transposed copy for dX.
constexpr int kFR = 16;

__device__ __forceinline__ f4 bload4(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// C[16 x N] = X[16 x K] . W^T, W's row n at byte woff + 4 n K of the buffer
// wr: lane (r, q) feeds k = 16c + 4q + j to MFMA j of chunk c (float4 reads
// of X from LDS and of W from L2, four chunks' loads in flight).  epi(row, n,
// v) for the lane's outputs with n < N.  Rows of W past N read other finite
// parameters (or zeros past the buffer) and are never stored.
// TRANSB: W is [K][N] instead (row k at byte woff + 4 k N): MFMA j of chunk c
// takes W[16c + 4q + j][n0 + r], one dword per lane, 16 lanes on one 64-byte
// row segment (the dX of a layer straight from its nn.Linear weight).
template <bool TRANSB = false, class FE>
__device__ __forceinline__ void few_gemm(const float *X, int ldx, __amdgpu_buffer_rsrc_t wr, int woff, int K, int N,
                                         const float *bias, FE epi) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int nc = (K + 15) >> 4, ntile = (N + 15) >> 4;
    const float *xr = X + r * ldx + 4 * q;
    for (int t = wave; t < ntile; t += kGW) {
        const int n0 = t << 4;
        const int wrow = TRANSB ? woff + (4 * q * N + n0 + r) * 4 : woff + ((n0 + r) * K + 4 * q) * 4;
        const float bv = bias ? bias[n0 + r < N ? n0 + r : 0] : 0.f;  // in flight under the MFMAs
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int c0 = 0; c0 < nc; c0 += 4) {
            f4 wv[4], xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u < nc ? c0 + u : nc - 1;
                if constexpr (TRANSB) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        wv[u][j] = __builtin_bit_cast(
                            float, __builtin_amdgcn_raw_buffer_load_b32(wr, wrow + ((16 * c + j) * N) * 4, 0, 0));
                } else {
                    wv[u] = bload4(wr, wrow + c * 64);
                }
                xv[u] = *reinterpret_cast<const f4 *>(xr + 16 * c);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (c0 + u >= nc) break;  // uniform
#pragma unroll
                for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[u][j], wv[u][j], acc, 0, 0, 0);
            }
        }
        if (n0 + r < N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) epi(4 * q + j, n0 + r, acc[j] + bv);
        }
    }
}

// few_gemm with W [16-rounded N][ldw] and the bias in LDS, zero padded to
// whole 16 x 16 tiles (the evaluation pass's resident weights)
template <class FE>
__device__ __forceinline__ void few_gemm_l(const float *X, int ldx, const float *W, int ldw, int K, int N,
                                           const float *bias, FE epi) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int nc = (K + 15) >> 4, ntile = (N + 15) >> 4;
    const float *xr = X + r * ldx + 4 * q;
    for (int t = wave; t < ntile; t += kGW) {
        const int n0 = t << 4;
        const float *wr = W + (n0 + r) * ldw + 4 * q;
        const float bv = bias[n0 + r];
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int c0 = 0; c0 < nc; c0 += 4) {  // four chunks' reads in flight, then their MFMAs
            f4 xv[4], wv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u < nc ? c0 + u : nc - 1;
                xv[u] = *reinterpret_cast<const f4 *>(xr + 16 * c);
                wv[u] = *reinterpret_cast<const f4 *>(wr + 16 * c);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (c0 + u >= nc) break;  // uniform
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[u][j], wv[u][j], acc, 0, 0, 0);
            }
        }
        if (n0 + r < N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) epi(4 * q + j, n0 + r, acc[j] + bv);
        }
    }
}

// dW[o][i] = sum over the 16 rows of dZ[row][o] X[row][i] (o < F, i < fin)
// straight into the gradient row Gw ([F][fin]); tiles round the waves
__device__ __forceinline__ void few_dw(const float *dZ, int ldz, const float *X, int ldx, int F, int fin, float *Gw) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 15, q = lane >> 4;
    const int tm = (F + 15) >> 4, tn = (fin + 15) >> 4, nt = tm * tn;
    auto put = [&](int o0, int i0, const f4 &acc) {
        const int i = i0 + r;
        if (i < fin) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = o0 + 4 * q + j;
                if (o < F) Gw[o * fin + i] = acc[j];
            }
        }
    };
    // two tiles per pass (t and t + kGW): both tiles' LDS reads in flight,
    // then two independent MFMA chains; each tile's sum order unchanged
    for (int t = wave; t < nt; t += 2 * kGW) {
        const int t2 = t + kGW;
        const bool two = t2 < nt;  // uniform
        const int o0 = (t % tm) << 4, i0 = (t / tm) << 4;
        const int o1 = two ? (t2 % tm) << 4 : o0, i1 = two ? (t2 / tm) << 4 : i0;
        float a[4], b[4], a2[4], b2[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            a[kk] = dZ[(4 * kk + q) * ldz + o0 + r];
            b[kk] = X[(4 * kk + q) * ldx + i0 + r];
            a2[kk] = dZ[(4 * kk + q) * ldz + o1 + r];
            b2[kk] = X[(4 * kk + q) * ldx + i1 + r];
        }
        f4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], b[kk], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[kk], b2[kk], acc2, 0, 0, 0);
        }
        put(o0, i0, acc);
        if (two) put(o1, i1, acc2);
    }
}

// LayerNorm(+affine) / ReLU of one row in place (16 lanes per row, sub =
// the lane's column phase), the row's values held in M registers per lane
// (F <= 16 M): every LDS read issued before the first use, the same float
// operations in the same order as the column loops
constexpr int kRowRegs = 8;
// the fields a row pass reads, loaded with the layer's other fields before its
// GEMM (not re-read from the layer table after the barrier)
struct LayRow {
    int ln, relu;
    long long af, rs, xh;
};
template <int M>
__device__ __forceinline__ void few_row_pass(float *y, float *S, const LayRow &L, int F, int ld, int row, int sub) {
    // whole 16-column chunks up to the 16-rounded width (a uniform bound: no
    // per-lane branches); the padding columns read zero and are written zero,
    // columns >= F enter no sum
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
            if (L.ln == 2) {
                ga[i] = S[L.af + j];
                be[i] = S[L.af + F + j];
            }
        }
    }
    float mean = 0.f, rstd = 1.f;
    if (L.ln) {
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
        if (sub == 0 && L.rs >= 0) S[L.rs + row] = rstd;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
        if (i >= mp) break;  // uniform
        const int j = sub + 16 * i;
        float x = v[i];
        if (L.ln) {
            const float xh = (x - mean) * rstd;
            if (L.xh >= 0) S[L.xh + row * ld + j] = ok[i] ? xh : 0.f;
            x = L.ln == 2 ? xh * ga[i] + be[i] : xh;
        }
        if (L.relu) x = relu(x);
        y[j] = ok[i] ? x : 0.f;
    }
}

// The backward of few_row_pass for one row: dY -> dZ in place through the
// ReLU mask and the LayerNorm(+affine) backward, dY' (the affine's input
// gradient) to T for the gamma / beta sums; registers as in few_row_pass, the
// same float operations in the same order as the column loops.
template <int M>
__device__ __forceinline__ void few_row_back(float *dy, const float *xh, float *T, const float *S, const LayRow &L,
                                             int F, int row, int sub) {
    const int mp = (F + 15) >> 4;
    float d[M], x[M], ga[M], be[M];
    bool ok[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int j = sub + 16 * i;
        ok[i] = j < F;
        d[i] = x[i] = ga[i] = be[i] = 0.f;
        if (i < mp) {
            d[i] = dy[j];
            x[i] = xh[j];
            if (L.ln == 2) {
                ga[i] = S[L.af + j];
                be[i] = S[L.af + F + j];
            }
        }
    }
    const float rs = L.ln ? S[L.rs + row] : 1.f;
    float dp[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const float pre = L.ln == 2 ? x[i] * ga[i] + be[i] : x[i];
        dp[i] = (!L.relu || pre > 0.f) ? d[i] : 0.f;
    }
    float m1 = 0.f, m2 = 0.f;
    if (L.ln) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const float dx = dp[i] * (L.ln == 2 ? ga[i] : 1.f);
            s1 = ok[i] ? s1 + dx : s1;
            s2 = ok[i] ? s2 + dx * x[i] : s2;
        }
        const float invF = 1.f / (float)F;
        m1 = rsum16(s1) * invF;
        m2 = rsum16(s2) * invF;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
        if (i >= mp) break;  // uniform
        const int j = sub + 16 * i;
        if (L.ln == 2) T[j] = ok[i] ? dp[i] : 0.f;
        const float v = L.ln ? rs * (dp[i] * (L.ln == 2 ? ga[i] : 1.f) - m1 - x[i] * m2) : dp[i];
        dy[j] = ok[i] ? v : 0.f;
    }
}

// Forward of the 16-row LDS tiles through the layer list: the few-row GEMM
// (+ bias) into Y, then LayerNorm(+affine) / ReLU as a row pass in place,
// keeping xhat / rstd where the plan has them (the learner; the policy step
// keeps Y only).  The observation tile is at oc (row stride ld0).
// WLDS: the weights are LDS-resident (layer l's W [16-rounded fout][ldw[l]]
// at S + wl[l], zero padded, its bias after it; the evaluation pass copies
// them once per launch); run: the layers to compute (bit l), the others are
// skipped (the evaluation's forward needs the actor's path only).
template <bool WLDS = false>
__device__ __forceinline__ void few_forward(const GLay *Ls, int nl, float *S, const float *pr,
                                            __amdgpu_buffer_rsrc_t prs, long long oc, int ld0, long long *st,
                                            unsigned run = ~0u, const long long *wl = nullptr,
                                            const int *ldw = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    const int row = 4 * wave + rq;
    for (int l = 0; l < nl; ++l) {
        if (!((run >> l) & 1u)) continue;  // uniform
        const GLay &L = Ls[l];
        const int F = L.fout, ld = L.ld;
        const LayRow lr{L.ln, L.relu, L.af, L.rs, L.xh};
        const float *X = L.src < 0 ? S + oc : S + Ls[L.src].yr;
        const int ldx = L.src < 0 ? ld0 : Ls[L.src].ld;
        float *Y = S + L.yr;
        // the LN affine for this update's row passes (forward and backward) to
        // LDS, its loads in flight under the GEMM
        float ga[2] = {0.f, 0.f}, be[2] = {0.f, 0.f};
        if (!WLDS && L.ln == 2) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (tid + h * kGT < F) {
                    ga[h] = pr[L.g + tid + h * kGT];
                    be[h] = pr[L.be + tid + h * kGT];
                }
        }
        if constexpr (WLDS) {
            const float *W = S + wl[l];
            few_gemm_l(X, ldx, W, ldw[l], L.fin, F, W + (long long)((F + 15) & ~15) * ldw[l],
                       [&](int m, int n, float v) { Y[m * ld + n] = v; });
        } else {
            few_gemm(X, ldx, prs, L.w * 4, L.fin, F, pr + L.b, [&](int m, int n, float v) { Y[m * ld + n] = v; });
        }
        if (!WLDS && L.ln == 2) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (tid + h * kGT < F) {
                    S[L.af + tid + h * kGT] = ga[h];
                    S[L.af + F + tid + h * kGT] = be[h];
                }
        }
        __syncthreads();
        if (lr.ln || lr.relu) {
            float *y = Y + row * ld;
            if (F <= 64) {
                few_row_pass<4>(y, S, lr, F, ld, row, sub);
            } else if (F <= 16 * kRowRegs) {
                few_row_pass<kRowRegs>(y, S, lr, F, ld, row, sub);
            } else {
                const float invF = 1.f / (float)F;
                float mean = 0.f, rstd = 1.f;
                if (L.ln) {
                    float s = 0.f;
                    for (int j = sub; j < F; j += 16) s += y[j];
                    mean = rsum16(s) * invF;
                    float vs = 0.f;
                    for (int j = sub; j < F; j += 16) {
                        const float d = y[j] - mean;
                        vs += d * d;
                    }
                    rstd = 1.f / sqrtf(rsum16(vs) / (float)F + 1e-5f);
                    if (sub == 0 && L.rs >= 0) S[L.rs + row] = rstd;
                }
                for (int j = sub; j < F; j += 16) {
                    float v = y[j];
                    if (L.ln) {
                        const float xh = (v - mean) * rstd;
                        if (L.xh >= 0) S[L.xh + row * ld + j] = xh;
                        v = L.ln == 2 ? xh * S[L.af + j] + S[L.af + F + j] : xh;
                    }
                    if (L.relu) v = relu(v);
                    y[j] = v;
                }
            }
            __syncthreads();
        }
        if (st) st[1 + l] = (long long)__builtin_readcyclecounter();
    }

}

// One update's gradient of a partner's rows (rk <= 16 of them, observations
// at xobs, rollout rows s0 ..) into the gradient row G, plus the loss /
// approx_kl partial sums: the few-row counterpart of minibatch_grads, same
// float operations per element.  S: the LDS tiles (plan_few).
__device__ __forceinline__ void few_grads(const GArgs &g, float *S, const float *pr, const float *wb, float *G,
                                          const float *xobs, const int *gact_e, const unsigned *gmask_e,
                                          const float *grow_e, long long s0, int rk, float inv_b, float entp,
                                          float &lsum, float &klsum, long long *st) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    const int row = 4 * wave + rq;  // the lane group's row in the row passes
    const int A = g.A, D = g.D;
    const long long S_ = g.S;
    const auto prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(pr), 0, __builtin_amdgcn_readfirstlane(g.n * 4),
                                                       0x00020000);
    // observation rows (zero past the slice)
    {
        float *x0 = S + g.oc;
        for (int i = tid; i < kFR * D; i += kGT) {
            const int b = i / D, d = i - b * D;
            float v = 0.f;
            if (b < rk) v = xobs[i];
            x0[b * g.ld0 + d] = v;
        }
    }
    __syncthreads();
    if (st) st[0] = (long long)__builtin_readcyclecounter();

    // ---- forward -------------------------------------------------------
    few_forward(g.L, g.nl, S, pr, prs, g.oc, g.ld0, st);

    // ---- PPO loss row pass: logits / value -> d(logits), d(value) (ppo.py:876-908)
    {
        const GLay &La = g.L[g.aout];
        const GLay &Lc = g.L[g.cout];
        const float *lgp = S + La.yr + row * La.ld;
        float *dla = S + La.dy + row * La.ld;
        const bool live = row < rk;
        const int rr = live ? row : 0;
        const int a0 = sub, a1 = sub + 16;
        const unsigned bits = gmask_e ? gmask_e[s0 + rr] : 0xffffffffu;
        const float plg0 = lgp[a0 < A ? a0 : 0], plg1 = lgp[a1 < A ? a1 : 0];
        const int a_t = gact_e[s0 + rr];
        const float olp = grow_e[s0 + rr], Ad = grow_e[S_ + s0 + rr];
        const float Rt = grow_e[2 * S_ + s0 + rr], ov = grow_e[3 * S_ + s0 + rr];
        const float v = S[Lc.yr + row * Lc.ld];
        const bool ok0 = (bits >> a0) & 1u, ok1 = (bits >> a1) & 1u;
        const float lg0 = a0 < A ? (ok0 ? plg0 : -1.0e8f) : -3.0e38f;
        const float lg1 = a1 < A ? (ok1 ? plg1 : -1.0e8f) : -3.0e38f;
        const float mx = rmax16(fmaxf(lg0, lg1));
        const float ex0 = a0 < A ? expf(lg0 - mx) : 0.f, ex1 = a1 < A ? expf(lg1 - mx) : 0.f;
        const float lse = mx + logf(rsum16(ex0 + ex1));
        const float p0 = a0 < A ? expf(lg0 - lse) : 0.f, p1 = a1 < A ? expf(lg1 - lse) : 0.f;
        const float lpe0 = logf(p0 + 1e-8f), lpe1 = logf(p1 + 1e-8f);
        const float Hs = -rsum16((a0 < A ? p0 * lpe0 : 0.f) + (a1 < A ? p1 * lpe1 : 0.f));
        const float gh0 = -(lpe0 + p0 / (p0 + 1e-8f)), gh1 = -(lpe1 + p1 / (p1 + 1e-8f));
        const float pg = rsum16((a0 < A ? p0 * gh0 : 0.f) + (a1 < A ? p1 * gh1 : 0.f));
        const int srcl = (lane & ~15) + (a_t & 15);
        const float t0 = bperm(srcl, lg0), t1 = bperm(srcl, lg1);
        const float logp = (a_t < 16 ? t0 : t1) - lse;
        const float lo = 1.f - g.clip, hi = 1.f + g.clip;
        const float lrt = logp - olp;
        const float ratio = expf(lrt);
        const float rcl = fminf(fmaxf(ratio, lo), hi);
        const float q1 = -Ad * ratio, q2 = -Ad * rcl;
        const float g1 = q1 > q2 ? 1.f : (q1 == q2 ? 0.5f : 0.f);
        const float g2 = q2 > q1 ? 1.f : (q1 == q2 ? 0.5f : 0.f);
        const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        const float g_logp = ((g1 * -Ad + g2 * -Ad * inr) * inv_b) * ratio;
        const float dv = v - ov;
        const float vcl = ov + fminf(fmaxf(dv, -g.clip), g.clip);
        const float eu = v - Rt, ec = vcl - Rt;
        const float lu = eu * eu, lc = ec * ec;
        const float gu = lu > lc ? 1.f : (lu == lc ? 0.5f : 0.f);
        const float gc = lc > lu ? 1.f : (lu == lc ? 0.5f : 0.f);
        const float inv = (dv >= -g.clip && dv <= g.clip) ? 1.f : 0.f;
        const float g_H = -entp * inv_b;
        const float dl0 = g_logp * ((a0 == a_t ? 1.f : 0.f) - p0) + g_H * p0 * (gh0 - pg);
        const float dl1 = g_logp * ((a1 == a_t ? 1.f : 0.f) - p1) + g_H * p1 * (gh1 - pg);
        // rows past the slice: a zero gradient (their tiles hold the last minibatch's rows)
        if (a0 < A) dla[a0] = (live && ok0) ? dl0 : 0.f;
        if (a1 < A) dla[a1] = (live && ok1) ? dl1 : 0.f;
        if (sub == 0) {
            const float dvv = g.vf * 0.5f * inv_b * (gu * 2.f * eu + gc * 2.f * ec * inv);
            S[Lc.dy + row * Lc.ld] = live ? dvv : 0.f;
            if (live) {
                lsum += (fmaxf(q1, q2) + g.vf * 0.5f * fmaxf(lu, lc) - entp * Hs) * inv_b;
                klsum += ((ratio - 1.f) - lrt) * inv_b;  // approx_kl (ppo.py:899-902)
            }
        }
    }
    __syncthreads();
    if (st) st[17] = (long long)__builtin_readcyclecounter();

    // ---- backward, layer by layer (reverse) ------------------------------
    float *T = S + g.t1;  // dY' of the current LN-affine layer (its gamma / beta gradients)
    for (int l = g.nl - 1; l >= 0; --l) {
        const GLay &L = g.L[l];
        const int F = L.fout, ld = L.ld;
        float *dZ = S + L.dy;  // dY in, dZ out (in place)
        if (L.ln || L.relu) {
            float *dy = dZ + row * ld;
            const float *xh = S + (L.ln ? L.xh : L.yr) + row * ld;  // xhat, or Y for a plain ReLU
            const LayRow lr{L.ln, L.relu, L.af, L.rs, L.xh};
            if (F <= 64) {
                few_row_back<4>(dy, xh, T + row * ld, S, lr, F, row, sub);
            } else if (F <= 16 * kRowRegs) {
                few_row_back<kRowRegs>(dy, xh, T + row * ld, S, lr, F, row, sub);
            } else {
                const float invF = 1.f / (float)F;
                float m1 = 0.f, m2 = 0.f, rs = 1.f;
                auto dpre = [&](int j, float &x) {
                    const float d = dy[j];
                    x = xh[j];
                    const float pre = L.ln == 2 ? x * S[L.af + j] + S[L.af + F + j] : x;
                    return (!L.relu || pre > 0.f) ? d : 0.f;
                };
                if (L.ln) {
                    float s1 = 0.f, s2 = 0.f;
                    for (int j = sub; j < F; j += 16) {
                        float x;
                        const float dx = dpre(j, x) * (L.ln == 2 ? S[L.af + j] : 1.f);
                        s1 += dx;
                        s2 += dx * x;
                    }
                    m1 = rsum16(s1) * invF;
                    m2 = rsum16(s2) * invF;
                    rs = S[L.rs + row];
                }
                for (int j = sub; j < F; j += 16) {
                    float x;
                    const float dp = dpre(j, x);
                    if (L.ln == 2) T[row * ld + j] = dp;
                    dy[j] = L.ln ? rs * (dp * (L.ln == 2 ? S[L.af + j] : 1.f) - m1 - x * m2) : dp;
                }
            }
            __syncthreads();
        }
        if (st) st[18 + 3 * l] = (long long)__builtin_readcyclecounter();
        // bias / LN-affine gradients: column sums in row order, one sum per
        // wave (0: bias, 1: gamma, 2: beta), the 16 rows' terms loaded first
        if (wave < (L.ln == 2 ? 3 : 1)) {
            const float *src = wave == 0 ? dZ : T;
            const long long go = wave == 0 ? L.b : wave == 1 ? L.g : L.be;
            for (int j = lane; j < F; j += kWave) {
                float v[kFR];
#pragma unroll
                for (int b = 0; b < kFR; ++b) {
                    v[b] = src[b * ld + j];
                    if (wave == 1) v[b] = v[b] * S[L.xh + b * ld + j];
                }
                float sum = 0.f;
#pragma unroll
                for (int b = 0; b < kFR; ++b) sum += v[b];
                G[go + j] = sum;
            }
        }
        const float *X = L.src < 0 ? S + g.oc : S + g.L[L.src].yr;
        const int ldx = L.src < 0 ? g.ld0 : g.L[L.src].ld;
        few_dw(dZ, ld, X, ldx, F, L.fin, G + L.w);
        if (st) st[19 + 3 * l] = (long long)__builtin_readcyclecounter();
        if (L.src >= 0) {  // dX = dZ W into the source's dY (the second consumer adds)
            const GLay &Ls = g.L[L.src];
            float *dys = S + Ls.dy;
            const int lds_ = Ls.ld;
            if (L.acc)
                few_gemm<true>(dZ, ld, prs, L.w * 4, F, L.fin, nullptr,
                               [&](int m, int n, float v) { dys[m * lds_ + n] += v; });
            else
                few_gemm<true>(dZ, ld, prs, L.w * 4, F, L.fin, nullptr,
                               [&](int m, int n, float v) { dys[m * lds_ + n] = v; });
        }
        __syncthreads();
        if (st) st[20 + 3 * l] = (long long)__builtin_readcyclecounter();
    }
}

// FEW: the few-row form (few_grads, activations in dynamic LDS); else the
// general form (minibatch_grads over the partner's global scratch)
template <bool FEW>
__global__ __launch_bounds__(kGT) void ppo_learn_graph_part_kernel(const GArgs g) {
    __shared__ float red[2 * kGW];
    __shared__ __attribute__((aligned(16))) float lds[kGemmLds];
    __shared__ float colp[2 * 3 * kGW * 128];
    __shared__ float colo[kGW * 33];
    __shared__ int s_ok;
    __shared__ long long s_st[16 + kGStampsIn];  // phase stamps (agent 0, partner 0, update 1), then per layer
    if (g.skip && __hip_atomic_load(g.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    const int b = blockIdx.x;
    const int p = b % g.Q, kk = b / g.Q;
    if (p >= g.P) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int K = g.K, P = g.P, n = g.n, D = g.D;
    const long long S = g.S;
    float *const pr = g.params + (size_t)p * n;
    float *const gm = g.m + (size_t)p * n;
    float *const gv = g.v + (size_t)p * n;
    // the activation scratch: the few-row form's LDS tiles (zeroed once: their
    // padding columns stay zero), else this partner's block of the global scratch
    extern __shared__ __attribute__((aligned(16))) float gdyn[];
    float *const base = FEW ? gdyn : g.ws + ((size_t)p * K + kk) * g.ws_part;
    if constexpr (FEW) {
        for (int i = tid; i < (int)g.lds_floats; i += kGT) gdyn[i] = 0.f;
    }
    float *const wsh = g.wtb + (size_t)p * g.wt_agent;  // the agent's shared transposed weights
    float *const wb = wsh - g.wt0;                      // wb + L.wt lands in wsh
    unsigned *const c0 = g.cnt + p, *const c1 = g.cnt + P + p, *const c2 = g.cnt + 2 * P + p;
    unsigned *const c3 = g.cnt + 3 * P + p, *const tmo = g.cnt + 4 * P;
    unsigned *const xcc = g.cnt + 4 * P + 1 + (size_t)p * kMaxGK;
    // float4 ownership: chunks [own0, own1) of the n4s = n4 + 1 chunks (the
    // gradient row padded to n4 chunks, then the loss / approx_kl chunk)
    const int n4 = (n + 3) / 4, n4s = n4 + 1, nal = 4 * n4;
    const int cs = (n4s + K - 1) / K;
    const int own0 = kk * cs < n4s ? kk * cs : n4s, own1 = own0 + cs < n4s ? own0 + cs : n4s;
    const int f0 = 4 * own0, f1 = 4 * own1 < n ? 4 * own1 : n;  // owned parameter floats

    // placement id + the transposed copies of the owned weights, one setup barrier
    if (tid == 0) {
        int x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        __hip_atomic_store(xcc + kk, (unsigned)(x & 15) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int l = 0; l < (FEW ? 0 : g.nl); ++l) {
        const GLay &L = g.L[l];
        if (L.wt < 0) continue;
        const int cnt = L.fout * L.fin;
        const int i0 = f0 - L.w > 0 ? f0 - L.w : 0, i1 = f1 - L.w < cnt ? f1 - L.w : cnt;
        float *wt = wb + L.wt;
        for (int i = i0 + tid; i < i1; i += kGT) {
            const int o = i / L.fin, c = i - o * L.fin;
            wt[(size_t)c * L.fout + o] = pr[L.w + i];
        }
    }
    if (!gpart_sync(c0, (unsigned)K, true, tmo, g.err, &s_ok)) return;
    bool local;
    {
        const unsigned v = lane < K ? __hip_atomic_load(xcc + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned v0 = __builtin_amdgcn_readlane(v, 0);
        bool same = v0 != 0u;
        for (int q = 1; q < K; ++q) same = same && __builtin_amdgcn_readlane(v, q) == v0;
        local = same && !g.write_through;
    }
    gpart_acquire();

    int Bp = g.batch_p ? g.batch_p[p] : g.B;
    if (Bp > g.B) Bp = g.B;
    const int Ep = g.epochs_p ? g.epochs_p[p] : g.E;
    const float entp = g.ent_p ? g.ent_p[p] : g.ent;
    const int nmb = (int)((S + Bp - 1) / Bp);
    float loss_total = 0.f;
    double kl_total = 0.0;
    int n_done = 0, epochs_done = 0;
    const long long step0 = g.step[p];
    double pb1 = pow((double)g.b1, (double)step0), pb2 = pow((double)g.b2, (double)step0);
    const float lr_p = g.lr[p];

    for (int e = 0; e < Ep; ++e) {
        const size_t ge = (size_t)e * P + p;
        const float *gobs_e = g.gobs + ge * S * D;
        const int *gact_e = g.gact + ge * S;
        const unsigned *gmask_e = g.gmask ? g.gmask + ge * S : nullptr;
        const float *grow_e = g.grow + ge * 4 * S;
        for (int mb = 0; mb < nmb; ++mb) {
            const long long s0 = (long long)mb * Bp;
            const int bsz = (int)((s0 + Bp <= S) ? Bp : S - s0);
            const float inv_b = 1.f / (float)bsz;
            const int r0 = kk * g.R, rk = bsz - r0 < 0 ? 0 : (bsz - r0 < g.R ? bsz - r0 : g.R);
            const int upd = e * nmb + mb;
            float *const slab0 = g.slabs + ((size_t)p * 2 + (upd & 1)) * K * g.nslab;  // partner 0's slab
            float *const G = slab0 + (size_t)kk * g.nslab;
            float *const sum = g.sums + ((size_t)p * 2 + (upd & 1)) * g.nslab;

            const bool stamp = g.stamps && b == 0 && upd == 1 && tid == 0;
#define GST(i) \
    if (stamp) s_st[i] = (long long)__builtin_readcyclecounter()
            GST(0);
            // ---- 1. this partner's rows -> its partial gradient row ----------------
            float lsum = 0.f, klsum = 0.f;
            if (rk > 0) {
                if constexpr (FEW)
                    few_grads(g, base, pr, wb, G, gobs_e + (s0 + r0) * D, gact_e, gmask_e, grow_e, s0 + r0, rk, inv_b,
                              entp, lsum, klsum, stamp ? s_st + 16 : nullptr);
                else
                    minibatch_grads(g, base, wb, pr, G, gobs_e + (s0 + r0) * D, gact_e, gmask_e,
                                                      grow_e, s0 + r0, rk, inv_b, entp, lds, colp, colo, lsum, klsum,
                                                      stamp ? s_st + 16 : nullptr);
            } else {  // no rows this minibatch (a short last minibatch): publish zeros
                for (int i = tid; i < n; i += kGT) G[i] = 0.f;
            }
            GST(1);
            block_sum2(lsum, klsum, red);
            if (tid == 0) {
                G[nal] = lsum;
                G[nal + 1] = klsum;
            }
            GST(2);
            if (!gpart_sync(c1, (unsigned)(K * (upd + 1)), !local, tmo, g.err, &s_ok)) return;
            GST(3);

            // ---- 2. reduce-scatter of the owned chunks + partial norms ---------------
            // few-row form with at most four owned chunks per thread: the sums stay
            // in registers for Adam and the chunks' moments / parameters are loaded
            // before barrier 2 (they land while it waits)
            const bool regs = FEW && own1 - own0 <= 4 * kGT;
            f4 tg[2][2];
            float mg[2][2][4], vg[2][2][4], pg[2][2][4];
            float q0 = 0.f, q1 = 0.f;
            {
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab0, 0, __builtin_amdgcn_readfirstlane(
                                                                                 (int)(K * g.nslab * 4)), 0x00020000);
                // two chunks per thread per round, partner order, up to 16 loads in flight
                int rr = 0;
                for (int cb = own0 + tid; cb < own1; cb += 2 * kGT, ++rr) {
                    f4 t[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
                    for (int q0_ = 0; q0_ < K; q0_ += 8) {  // uniform
                        f4 x[2][8];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int c = cb + h * kGT, cl = c < own1 ? c : own0;
#pragma unroll
                            for (int q = 0; q < 8; ++q) {
                                const int qq = q0_ + q, qs = qq < K ? qq : K - 1;
                                const f4 v = __builtin_bit_cast(
                                    f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((qs * g.nslab + 4 * cl) * 4), 0, 16));
                                x[h][q] = qq < K ? v : f4{0.f, 0.f, 0.f, 0.f};
                            }
                        }
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            if (q0_ == 0) {
                                t[h] = x[h][0];
#pragma unroll
                                for (int q = 1; q < 8; ++q) t[h] += x[h][q];
                            } else {
#pragma unroll
                                for (int q = 0; q < 8; ++q) t[h] += x[h][q];
                            }
                        }
                    }
                    if (regs) {
                        if (rr == 0) {
                            tg[0][0] = t[0];
                            tg[0][1] = t[1];
                        } else {
                            tg[1][0] = t[0];
                            tg[1][1] = t[1];
                        }
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int c = cb + h * kGT;
                        if (c >= own1) break;
                        // (the loss / approx_kl chunk n4 always: every partner reads it after barrier 2)
                        if (!regs || c >= n4) *reinterpret_cast<f4 *>(sum + 4 * c) = t[h];
#pragma unroll
                        for (int cc = 0; cc < 4; ++cc) {
                            const int f = 4 * c + cc;
                            const float x2 = f < n ? t[h][cc] * t[h][cc] : 0.f;
                            if (f < g.cstart) q0 += x2;
                            else q1 += x2;
                        }
                    }
                }
                q0 = wave_sum(q0);
                q1 = wave_sum(q1);
                if (lane < 2) sum[nal + 4 + (kk * kGW + wave) * 2 + lane] = lane ? q1 : q0;
            }
            if (regs) {
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int cc = 0; cc < 4; ++cc) {
                            const int f = 4 * (own0 + tid + (2 * r + h) * kGT) + cc;
                            const int fs = f < f1 ? f : f0;
                            mg[r][h][cc] = gm[fs];
                            vg[r][h][cc] = gv[fs];
                            pg[r][h][cc] = pr[fs];
                        }
            }
            GST(4);
            if (!gpart_sync(c2, (unsigned)(K * (upd + 1)), !local, tmo, g.err, &s_ok)) return;
            GST(5);

            // ---- 3. norms (fixed order), loss words, Adam on the owned floats ---------
            float t0, t1, lmb, klmb;
            {
                const int np = 2 * kGW * K;  // <= 128 words: lanes l and l + 64
                float v = 0.f;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int w = lane + 64 * h;
                    const float x = ld_sc1(sum + nal + 4 + (w < np ? w : 0));
                    v += w < np ? x : 0.f;
                }
                const float lw = ld_sc1(sum + nal), kw = ld_sc1(sum + nal + 1);
                t0 = wave_sum((lane & 1) ? 0.f : v);
                t1 = wave_sum((lane & 1) ? v : 0.f);
                lmb = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, lw)));
                klmb = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, kw)));
            }
            GST(6);
            if (tid == 0) loss_total += lmb;
            kl_total += (double)klmb;
            ++n_done;
            const float cl0 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t0) + 1e-6f), 1.f) : 1.f;
            const float cl1 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t1) + 1e-6f), 1.f) : 1.f;
            pb1 *= (double)g.b1;
            pb2 *= (double)g.b2;
            const float bc1 = (float)(1.0 - pb1);
            const float bc2s = (float)sqrt(1.0 - pb2);
            const float step_size = lr_p / bc1;
            const float ob1 = 1.f - g.b1, ob2 = 1.f - g.b2;
            // the owned float range [f0, f1) in one pass, U elements per thread per
            // round (all loads of a round first); an element inside a layer's W
            // also goes to the transposed copy (the layer found by a short scan of
            // the layer list: contiguous W ranges, at most 16 layers)
            if (regs) {
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int cc = 0; cc < 4; ++cc) {
                            const int f = 4 * (own0 + tid + (2 * r + h) * kGT) + cc;
                            if (f >= f1) continue;
                            const float gc = tg[r][h][cc] * (f < g.cstart ? cl0 : cl1);
                            const float m = mg[r][h][cc] + ob1 * (gc - mg[r][h][cc]);
                            const float v = vg[r][h][cc] * g.b2 + ob2 * gc * gc;
                            gm[f] = m;
                            gv[f] = v;
                            pr[f] = pg[r][h][cc] - step_size * (m / (sqrtf(v) / bc2s + g.eps));
                        }
            } else {
                constexpr int U = 8;
                for (int i0 = f0 + tid; i0 < f1; i0 += U * kGT) {
                    float gg[U], mm[U], vv[U], pp[U];
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        const int i = i0 + k * kGT;
                        const int f = i < f1 ? i : f0;
                        gg[k] = sum[f];  // this partner's own reduce-scatter stores
                        mm[k] = gm[f];
                        vv[k] = gv[f];
                        pp[k] = pr[f];
                    }
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        const int f = i0 + k * kGT;
                        if (f >= f1) break;
                        const float gc = gg[k] * (f < g.cstart ? cl0 : cl1);
                        const float m = mm[k] + ob1 * (gc - mm[k]);
                        const float v = vv[k] * g.b2 + ob2 * gc * gc;
                        const float np_ = pp[k] - step_size * (m / (sqrtf(v) / bc2s + g.eps));
                        gm[f] = m;
                        gv[f] = v;
                        pr[f] = np_;
                        if constexpr (!FEW) {  // the few-row form's dX reads W itself
                            for (int l = 0; l < g.nl; ++l) {
                                const GLay &L = g.L[l];
                                const int i = f - L.w;
                                if (L.wt >= 0 && i >= 0 && i < L.fout * L.fin) {
                                    const int o = i / L.fin, c = i - o * L.fin;
                                    wb[L.wt + (size_t)c * L.fout + o] = np_;
                                    break;
                                }
                            }
                        }
                    }
                }
            }
            GST(7);
            // ---- 4. every partner's chunks visible to this one's next plain loads ---------
            if (!gpart_sync(c3, (unsigned)(K * (upd + 1)), !local, tmo, g.err, &s_ok)) return;
            GST(8);
            gpart_acquire();
            GST(9);
#undef GST
        }  // minibatches
        ++epochs_done;
        if (g.target_kl > 0.0 && kl_total / (double)n_done > g.target_kl) break;  // ppo.py:917-918
    }  // epochs
    if (tid == 0 && kk == 0) {
        if (g.loss_out) g.loss_out[p] = loss_total / ((float)S * (float)Ep);
        if (g.kl_out) g.kl_out[p] = n_done ? (float)(kl_total / (double)n_done) : 0.f;
        if (g.epochs_out) g.epochs_out[p] = epochs_done;
        g.step[p] = step0 + n_done;
    }
    if (g.stamps && b == 0 && tid < 16 + kGStampsIn) g.stamps[tid] = s_st[tid];
}


struct GActArgs {
    GLay L[kGL];
    int nl, aout, cout, A, D, n, rows;
    int ld0;                 // few-row form: the observation tile's row stride
    long long oc, lds_floats;  // few-row form: its offset, the LDS tiles' size
    long long ws_block;  // scratch floats per (agent, row block)
    long long obs_off;   // persistent rollout: the step's observation rows [rows][D] in the block scratch
    float *ws;
    const float *params;
    const float *obs;  // agent p, env n at obs + p*obs_pstride + n*D
    long long obs_pstride;
    int N, P, sample;
    unsigned long long seed, counter;
    long long *act_out;
    float *logp_out, *value_out, *ent_out;
    long long out_pstride;
    long long *act_flat;
    const unsigned char *mask;
    long long mask_pstride;
    const long long *env_base;
};

// The categorical step of rows [0, nrow) of agent p's row block n0 (logits at
// lgp [nrow][A], values at vp) — masked logits (illegal -> -1e8,
// distributions.py:16-28), Gumbel-max sample from the Philox stream of
// agx_ppo_act, log-prob, entropy, value; 16 lanes per row, actions a and a + 16
// per lane.  HOST_MASK: the mask is host staging (system-scope loads), copied to
// mask_copy when that is set.
struct GSample {
    int A, N, sample;
    int lda, ldv;  // row strides of the logits and the values
    unsigned long long seed, counter;
    const long long *env_base;
    const unsigned char *mask;
    long long mask_pstride;
    unsigned char *mask_copy;
    long long mask_copy_pstride;
    long long *act_out;
    float *logp_out, *value_out, *ent_out;
    long long out_pstride;
    long long *act_flat;
    long long env_off = -1;  // >= 0: the block's agent's first env (else env_base[p], or p N)
};
template <bool HOST_MASK>
__device__ __forceinline__ void graph_sample(const GSample &g, const float *lgp, const float *vp, int p, int n0,
                                             int nrow) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane & 15, rq = lane >> 4;
    const int A = g.A;
    const int a0 = sub, a1 = sub + 16;
    for (int r0 = 0; r0 < nrow; r0 += 4 * kGW) {
        const int r = r0 + 4 * wave + rq;
        const bool live = r < nrow;
        const int rr = live ? r : 0;
        float lg0 = a0 < A ? lgp[(size_t)rr * g.lda + a0] : -3.0e38f;
        float lg1 = a1 < A ? lgp[(size_t)rr * g.lda + a1] : -3.0e38f;
        if (g.mask && live) {
            const size_t mo = (size_t)p * g.mask_pstride + (size_t)(n0 + r) * A;
            unsigned char ok0 = 1, ok1 = 1;
            if (a0 < A) ok0 = HOST_MASK ? ld_sys_u8(g.mask + mo + a0) : g.mask[mo + a0];
            if (a1 < A) ok1 = HOST_MASK ? ld_sys_u8(g.mask + mo + a1) : g.mask[mo + a1];
            if (HOST_MASK && g.mask_copy) {
                const size_t co = (size_t)p * g.mask_copy_pstride + (size_t)(n0 + r) * A;
                if (a0 < A) g.mask_copy[co + a0] = ok0;
                if (a1 < A) g.mask_copy[co + a1] = ok1;
            }
            if (a0 < A && !ok0) lg0 = -1.0e8f;
            if (a1 < A && !ok1) lg1 = -1.0e8f;
        }
        const float mx = rmax16(fmaxf(lg0, lg1));
        const float lse = mx + logf(rsum16((a0 < A ? expf(lg0 - mx) : 0.f) + (a1 < A ? expf(lg1 - mx) : 0.f)));
        const float p0 = a0 < A ? expf(lg0 - lse) : 0.f, p1 = a1 < A ? expf(lg1 - lse) : 0.f;
        const float H = -rsum16((a0 < A ? p0 * logf(p0 + 1e-8f) : 0.f) + (a1 < A ? p1 * logf(p1 + 1e-8f) : 0.f));
        float sc0 = lg0, sc1 = lg1;
        if (g.sample) {
            const unsigned long long env = (g.env_off >= 0   ? (unsigned long long)g.env_off
                                            : g.env_base ? (unsigned long long)g.env_base[p]
                                                         : (unsigned long long)p * g.N) +
                                           n0 + rr;
            auto gumbel = [&](int a, float lg) {
                const uint4 rnd = philox(make_uint4((unsigned)env, (unsigned)(env >> 32), (unsigned)g.counter,
                                                    (unsigned)(g.counter >> 32) ^ ((unsigned)(a >> 2) << 24)),
                                         make_uint2((unsigned)g.seed, (unsigned)(g.seed >> 32)));
                const unsigned w = (a & 3) == 0 ? rnd.x : (a & 3) == 1 ? rnd.y : (a & 3) == 2 ? rnd.z : rnd.w;
                const float u = ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);
                return a < A ? lg - logf(-logf(u)) : -3.0e38f;
            };
            sc0 = gumbel(a0, lg0);
            sc1 = A > 16 ? gumbel(a1, lg1) : -3.0e38f;
        }
        // first maximum over the actions: lane-local (a0 < a1), then the lowest
        // index among the lanes holding the row maximum
        const float bl = fmaxf(sc0, sc1);
        const int il = sc0 >= sc1 ? a0 : a1;
        const float best = rmax16(bl);
        const int choice = (int)(-rmax16(bl == best ? -(float)il : -1.0e9f));
        const int srcl = (lane & ~15) + (choice & 15);
        const float c0 = bperm(srcl, lg0), c1 = bperm(srcl, lg1);
        if (live && sub == 0) {
            const size_t o = (size_t)p * g.out_pstride + n0 + r;
            if (g.act_out) g.act_out[o] = choice;
            if (g.logp_out) g.logp_out[o] = (choice < 16 ? c0 : c1) - lse;
            if (g.ent_out) g.ent_out[o] = H;
            if (g.value_out) g.value_out[o] = vp[(size_t)r * g.ldv];
            if (g.act_flat)  // host staging: system-scope (write-through) store
                __hip_atomic_store(g.act_flat + (size_t)p * g.N + n0 + r, (long long)choice, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Rollout policy step (PPO.get_action, ppo.py:567-633) of workgroup (p, row
// block): forward through the layer list, then graph_sample.
// FEW: the block's 16 rows through few_forward's LDS tiles (act_plan_few).
template <bool FEW>
__global__ __launch_bounds__(kGT) void ppo_act_graph_kernel(const GActArgs g) {
    __shared__ __attribute__((aligned(16))) float lds[kGemmLds];
    extern __shared__ __attribute__((aligned(16))) float gdyn[];
    const int p = blockIdx.y, n0 = blockIdx.x * g.rows;
    const int nrow = g.N - n0 < g.rows ? g.N - n0 : g.rows;
    const float *pr = g.params + (size_t)p * g.n;
    const float *obs = g.obs + (size_t)p * g.obs_pstride + (size_t)n0 * g.D;
    const GLay &La = g.L[g.aout], &Lc = g.L[g.cout];
    if constexpr (FEW) {
        const int tid = threadIdx.x;
        for (int i = tid; i < (int)g.lds_floats; i += kGT) gdyn[i] = 0.f;
        __syncthreads();
        for (int i = tid; i < nrow * g.D; i += kGT) {
            const int b = i / g.D, d = i - b * g.D;
            gdyn[g.oc + b * g.ld0 + d] = obs[i];
        }
        __syncthreads();
        const auto prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(pr), 0,
                                                           __builtin_amdgcn_readfirstlane(g.n * 4), 0x00020000);
        few_forward(g.L, g.nl, gdyn, pr, prs, g.oc, g.ld0, nullptr);
        GSample s{g.A, g.N, g.sample, La.ld, Lc.ld, g.seed, g.counter, g.env_base, g.mask, g.mask_pstride, nullptr, 0,
                  g.act_out, g.logp_out, g.value_out, g.ent_out, g.out_pstride, g.act_flat};
        graph_sample<false>(s, gdyn + La.yr, gdyn + Lc.yr, p, n0, nrow);
    } else {
        float *base = g.ws + ((size_t)p * gridDim.x + blockIdx.x) * g.ws_block;
        forward_layers(g.L, g.nl, obs, nrow, base, pr, g.rows, lds);
        GSample s{g.A, g.N, g.sample, g.A, 1, g.seed, g.counter, g.env_base, g.mask, g.mask_pstride, nullptr, 0,
                  g.act_out, g.logp_out, g.value_out, g.ent_out, g.out_pstride, g.act_flat};
        graph_sample<false>(s, base + La.yr, base + Lc.yr, p, n0, nrow);
    }
}

// Persistent rollout of a runtime-shape population (agx_ppo_rollout_graph_
// persistent / agx_ppo_eval_graph_persistent): agx_ppo_rollout_persistent's
// host-paced loop (learner.hip) around ppo_act_graph_kernel's step.  Step t:
// wait for the host's release, then the step's ActArgs (host memory): the
// observation rows from the host staging (system-scope loads) into this
// block's scratch and the rollout slot, the previous step's reward / done into
// slot t-1 with the episode accounting, and (act) the forward + sample; the
// actions go to the host staging; then this block's done word.
template <bool FEW>
__global__ __launch_bounds__(kGT) void ppo_rollout_graph_persistent_kernel(const GActArgs ga, const ActArgs *steps,
                                                                           int nsteps, agx_rollout_ctl *ctl,
                                                                           unsigned long long timeout_ticks,
                                                                           unsigned base_seq) {
    __shared__ __attribute__((aligned(16))) float lds[kGemmLds];
    extern __shared__ __attribute__((aligned(16))) float gdyn[];
    __shared__ ActArgs s_args;
    __shared__ int s_go;
    const int tid = threadIdx.x;
    const int p = blockIdx.y, n0 = blockIdx.x * ga.rows;
    const int blk = blockIdx.y * gridDim.x + blockIdx.x;
    const int D = ga.D;
    unsigned *rel = rollout_release_word(ctl, gridDim.x * gridDim.y, blk);
    float *base = ga.ws + ((size_t)p * gridDim.x + blockIdx.x) * ga.ws_block;
    float *obs_rows = base + ga.obs_off;  // [rows][D]: this step's observations
    constexpr int kArgWords = (int)(sizeof(ActArgs) / 4);
    if (tid == 0)  // this workgroup is resident (agx_rollout_ctl.started counts them)
        __hip_atomic_fetch_add(&ctl->started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (FEW) {  // the LDS tiles' padding (and the rows past the block) stay zero
        for (int i = tid; i < (int)ga.lds_floats; i += kGT) gdyn[i] = 0.f;
    }
    for (int t = 0; t < nsteps; ++t) {
        if (tid < kArgWords)
            reinterpret_cast<unsigned *>(&s_args)[tid] = reinterpret_cast<const unsigned *>(steps + t)[tid];
        if (tid == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int go = 1;
            for (;;) {
                const unsigned v = __hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v == AGX_ROLLOUT_ABORT) {
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                if (v == AGX_ROLLOUT_STOP) {
                    go = 0;
                    break;
                }
                if (v >= base_seq + (unsigned)(t + 1)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) return;
        const ActArgs g = s_args;
        const int nrow = g.N - n0 < ga.rows ? g.N - n0 : ga.rows;
        // the host staging of this block's rows (one round trip), then the
        // previous step's reward / done and the episode accounting
        const float *ob = g.obs + (size_t)p * g.obs_pstride + (size_t)n0 * D;
        for (int i = tid; i < nrow * D; i += kGT) {
            const float x = ld_sys(ob + i);
            if constexpr (FEW) {
                const int b = i / D, d = i - b * D;
                gdyn[ga.oc + b * ga.ld0 + d] = x;
            } else {
                obs_rows[i] = x;
            }
            if (g.obs_copy) g.obs_copy[(size_t)p * g.obs_copy_pstride + (size_t)n0 * D + i] = x;
        }
        if (g.st_rew && tid < nrow) {
            const size_t idx = (size_t)p * g.N + n0 + tid;
            const float rw = ld_sys(g.st_rew + idx);
            const unsigned char dn = ld_sys_u8(g.st_done + idx);
            const int env = n0 + tid;
            g.rew_prev[(size_t)p * g.prev_pstride + env] = rw;
            g.done_prev[(size_t)p * g.prev_pstride + env] = dn;
            if (g.scores) {
                float sc = g.scores[idx] + rw;
                if (dn) {
                    g.ret_sum[idx] += (double)sc;
                    g.episodes[idx] += 1;
                    sc = 0.f;
                }
                g.scores[idx] = sc;
            }
        }
        if (g.act) {
            __syncthreads();  // the observation rows are in the scratch
            const float *pr = g.params + (size_t)p * ga.n;
            const GLay &La = ga.L[ga.aout], &Lc = ga.L[ga.cout];
            if constexpr (FEW) {
                const auto prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(pr), 0,
                                                                   __builtin_amdgcn_readfirstlane(ga.n * 4), 0x00020000);
                few_forward(ga.L, ga.nl, gdyn, pr, prs, ga.oc, ga.ld0, nullptr);
                GSample sp{ga.A, g.N, g.sample, La.ld, Lc.ld, g.seed, g.counter, g.env_base, g.mask, g.mask_pstride,
                           g.mask_copy, g.mask_copy_pstride, g.act_out, g.logp_out, g.value_out, g.ent_out,
                           g.out_pstride, g.act_flat};
                graph_sample<true>(sp, gdyn + La.yr, gdyn + Lc.yr, p, n0, nrow);
            } else {
                forward_layers(ga.L, ga.nl, obs_rows, nrow, base, pr, ga.rows, lds);
                GSample sp{ga.A, g.N, g.sample, ga.A, 1, g.seed, g.counter, g.env_base, g.mask, g.mask_pstride,
                           g.mask_copy, g.mask_copy_pstride, g.act_out, g.logp_out, g.value_out, g.ent_out,
                           g.out_pstride, g.act_flat};
                graph_sample<true>(sp, base + La.yr, base + Lc.yr, p, n0, nrow);
            }
        }
        // the host-memory stores (actions) are system-scope write-through: wait
        // for their acknowledgements, then this block's done word
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store(rollout_done_words(ctl) + blk, base_seq + (unsigned)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// One evaluation pass of a WHOLE population in one persistent launch
// (agx_ppo_eval_multi_persistent): agent p runs ITS network (its own few-row
// policy-step plan, agents[p]) on its own parameter row over envs
// [p N, (p + 1) N) of the packed host staging, whatever group it trains in;
// the host paces the steps as for ppo_rollout_graph_persistent_kernel.  Step t
// samples with counter agents[p].counter0 + t from the agent's own Philox
// stream (seed, env base).
struct EvalAgent {
    GLay L[kGL];
    int nl, aout, cout, n, ld0;
    long long oc, lds_floats;
    unsigned run;       // the layers on the actor's path (the critic's are not computed)
    int ldw[kGL];       // LDS-resident weights (the WLDS kernel): row stride of layer l's W,
    long long wl[kGL];  // its offset in floats (W, then the bias), -1: layer not run
    long long lds_w;    // floats of LDS with the weights
    const float *params;
    long long env_base;
    unsigned long long seed, counter0;
};

// The episode tally of an evaluation pass on the device (agx_eval_tally):
// at each step the previous env step's reward / done from the host staging
// into the env's running score (f64, as the reference's numpy tally), its
// first finished episode's score, and each workgroup's count of finished envs
// for the host's end-of-pass test.
struct EvalTally {
    const float *rew;
    const unsigned char *done;
    double *scores, *completed;
    unsigned char *finished;
    unsigned *fin_words;
    int prev;  // the staging holds a reward / done when the launch starts
};

constexpr int kEvalStamps = 6 + kGL;  // agx_debug_eval_stamps: per step

template <bool WLDS>
__global__ __launch_bounds__(kGT) void ppo_eval_multi_persistent_kernel(const EvalAgent *__restrict__ agents, int N,
                                                                        int A, int D, const float *stage_obs,
                                                                        long long *act_flat, int nsteps,
                                                                        agx_rollout_ctl *ctl,
                                                                        unsigned long long timeout_ticks,
                                                                        unsigned base_seq, long long *stamps,
                                                                        const EvalTally tally) {
    extern __shared__ __attribute__((aligned(16))) float gdyn[];
    __shared__ int s_go;
    const int tid = threadIdx.x;
    const int p = blockIdx.y, n0 = blockIdx.x * kFR;
    const int blk = blockIdx.y * gridDim.x + blockIdx.x;
    const int nrow = N - n0 < kFR ? N - n0 : kFR;
    const EvalAgent &ag = agents[p];
    unsigned *rel = rollout_release_word(ctl, gridDim.x * gridDim.y, blk);
    const float *pr = ag.params;
    const auto prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(pr), 0,
                                                       __builtin_amdgcn_readfirstlane(ag.n * 4), 0x00020000);
    for (int i = tid; i < (int)ag.lds_floats; i += kGT) gdyn[i] = 0.f;  // padding and rows past the block
    if constexpr (WLDS) {  // the actor path's weights, once for the whole pass (zero padded)
        __syncthreads();   // the zeroing above before the LN affine copies below
        for (int l = 0; l < ag.nl; ++l) {
            if (!((ag.run >> l) & 1u)) continue;
            const GLay &L = ag.L[l];
            const int K = L.fin, F = L.fout, ldw = ag.ldw[l], Fp = (F + 15) & ~15;
            float *W = gdyn + ag.wl[l];
            for (int i = tid; i < Fp * ldw; i += kGT) {
                const int n = i / ldw, k = i - n * ldw;
                W[i] = (n < F && k < K) ? pr[L.w + n * K + k] : 0.f;
            }
            for (int i = tid; i < Fp; i += kGT) W[Fp * ldw + i] = i < F ? pr[L.b + i] : 0.f;
            if (L.ln == 2)  // the LN affine's LDS copy too (few_forward<true> does not reload it)
                for (int i = tid; i < F; i += kGT) {
                    gdyn[L.af + i] = pr[L.g + i];
                    gdyn[L.af + F + i] = pr[L.be + i];
                }
        }
    }
    const GLay &La = ag.L[ag.aout], &Lc = ag.L[ag.cout];
    for (int t = 0; t < nsteps; ++t) {
        if (tid == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int go = 1;
            for (;;) {
                const unsigned v = __hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v == AGX_ROLLOUT_ABORT) {
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                if (v == AGX_ROLLOUT_STOP) {
                    go = 0;
                    break;
                }
                if (v >= base_seq + (unsigned)(t + 1)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) return;
        const bool stamp = stamps && blk == 0 && tid == 0 && t >= 2 && t < 34;
        long long *stp = stamp ? stamps + kEvalStamps * (t - 2) : nullptr;
        if (stamp) stp[0] = (long long)__builtin_amdgcn_s_memrealtime();
        const float *ob = stage_obs + ((size_t)p * N + n0) * D;
        for (int i = tid; i < nrow * D; i += kGT) {
            const int b = i / D, d = i - b * D;
            gdyn[ag.oc + b * ag.ld0 + d] = ld_sys(ob + i);
        }
        if (tally.rew && (t > 0 || tally.prev) && tid < 64) {  // one wave: the block's <= 16 envs
            int fin = 0;
            if (tid < nrow) {
                const size_t idx = (size_t)p * N + n0 + tid;
                const float rw = ld_sys(tally.rew + idx);
                const unsigned char dn = ld_sys_u8(tally.done + idx);
                const double sc = tally.scores[idx] + (double)rw;
                tally.scores[idx] = sc;
                fin = tally.finished[idx];
                if (dn && !fin) {
                    tally.finished[idx] = 1;
                    tally.completed[idx] = sc;
                    fin = 1;
                }
            }
            const unsigned cnt = (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(fin != 0));
            if (tid == 0) __hip_atomic_store(tally.fin_words + blk, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        if (stamp) {
            stp[1] = (long long)__builtin_amdgcn_s_memrealtime();
            stp[4] = (long long)__builtin_readcyclecounter();
        }
        few_forward<WLDS>(ag.L, ag.nl, gdyn, pr, prs, ag.oc, ag.ld0, stp ? stp + 5 : nullptr, ag.run, ag.wl, ag.ldw);
        if (stamp) stp[2] = (long long)__builtin_amdgcn_s_memrealtime();
        GSample sp{A, N, 1, La.ld, Lc.ld, ag.seed, ag.counter0 + (unsigned long long)t, nullptr, nullptr, 0,
                   nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, act_flat, ag.env_base};
        graph_sample<true>(sp, gdyn + La.yr, gdyn + Lc.yr, p, n0, nrow);
        // the actions are system-scope (write-through) stores: their acknowledgements, then the done word
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store(rollout_done_words(ctl) + blk, base_seq + (unsigned)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        if (stamp) stp[3] = (long long)__builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
long long r4(long long x) { return (x + 3) & ~3ll; }

// validate the layer list; fill the layer table and the per-agent scratch plan
int plan_graph(const agx_ppo_graph *net, int64_t batch, GArgs &a) {
    AGX_REQUIRE(net, "agx_ppo_graph: null graph");
    const int nl = net->n_layers;
    AGX_REQUIRE(nl >= 2 && nl <= kGL, "agx_ppo_graph: %d layers (2..%d)", nl, kGL);
    AGX_REQUIRE(net->obs_dim >= 1 && net->n_params > 0 && net->critic_start > 0 && net->critic_start < net->n_params,
                "agx_ppo_graph: bad sizes");
    AGX_REQUIRE(net->n_actions >= 1 && net->n_actions <= AGX_PPO_GRAPH_MAX_ACTIONS,
                "agx_ppo_graph: %d actions (1..%d)", net->n_actions, AGX_PPO_GRAPH_MAX_ACTIONS);
    AGX_REQUIRE(net->actor_out >= 0 && net->actor_out < nl && net->critic_out >= 0 && net->critic_out < nl &&
                    net->actor_out != net->critic_out,
                "agx_ppo_graph: bad output layers");
    const int64_t bp = (batch + 15) / 16 * 16;
    AGX_REQUIRE(batch >= 1 && bp < (1 << 30), "agx_ppo_graph: bad batch %lld", (long long)batch);
    bool is_src[kGL] = {};
    int consumers[kGL] = {};
    int maxw = 0;
    long long nw = 0;
    for (int l = 0; l < nl; ++l) {
        const agx_ppo_layer &x = net->layers[l];
        AGX_REQUIRE(x.src >= -1 && x.src < l, "agx_ppo_graph: layer %d reads layer %d (not topological)", l, x.src);
        const int fin = x.src < 0 ? net->obs_dim : net->layers[x.src].fout;
        AGX_REQUIRE(x.fin == fin && x.fout >= 1, "agx_ppo_graph: layer %d width mismatch", l);
        AGX_REQUIRE(x.ln >= 0 && x.ln <= 2, "agx_ppo_graph: layer %d ln %d", l, x.ln);
        AGX_REQUIRE((x.ln == 0 && !x.relu) || x.fout <= AGX_PPO_GRAPH_MAX_WIDTH,
                    "agx_ppo_graph: layer %d width %d > %d", l, x.fout, AGX_PPO_GRAPH_MAX_WIDTH);
        auto in = [&](long long off, long long len) { return off >= 0 && off + len <= net->n_params; };
        AGX_REQUIRE(in(x.w, (long long)x.fin * x.fout) && in(x.b, x.fout) &&
                        (x.ln != 2 || (in(x.ln_w, x.fout) && in(x.ln_b, x.fout))),
                    "agx_ppo_graph: layer %d parameters outside the row", l);
        if (x.src >= 0) {
            is_src[x.src] = true;
            AGX_REQUIRE(++consumers[x.src] <= 2, "agx_ppo_graph: layer %d feeds more than two layers", x.src);
        }
        maxw = x.fout > maxw ? x.fout : maxw;
        nw += (long long)x.fin * x.fout + x.fout * (x.ln == 2 ? 3 : 1);
    }
    AGX_REQUIRE(nw == net->n_params, "agx_ppo_graph: layers cover %lld of %d parameters", nw, net->n_params);
    const agx_ppo_layer &la = net->layers[net->actor_out], &lc = net->layers[net->critic_out];
    AGX_REQUIRE(la.fout == net->n_actions && lc.fout == 1 && la.ln == 0 && lc.ln == 0 && !la.relu && !lc.relu &&
                    !is_src[net->actor_out] && !is_src[net->critic_out],
                "agx_ppo_graph: the output layers must be plain Linear(-> n_actions) / Linear(-> 1)");
    long long off = 0;
    bool seen[kGL] = {};
    for (int l = nl - 1; l >= 0; --l) {  // backward order: the first consumer writes dY, later ones add
        const int s = net->layers[l].src;
        a.L[l].acc = (s >= 0 && seen[s]) ? 1 : 0;
        if (s >= 0) seen[s] = true;
    }
    for (int l = 0; l < nl; ++l) {
        const agx_ppo_layer &x = net->layers[l];
        GLay &L = a.L[l];
        L.fin = x.fin;
        L.fout = x.fout;
        L.w = x.w;
        L.b = x.b;
        L.g = x.ln == 2 ? x.ln_w : -1;
        L.be = x.ln == 2 ? x.ln_b : -1;
        L.ln = x.ln;
        L.relu = x.relu ? 1 : 0;
        L.src = x.src;
        L.yr = off;
        off = r4(off + bp * x.fout);
        L.yc = -1;
        if (is_src[l]) {
            L.yc = off;
            off = r4(off + (long long)x.fout * bp);
        }
        L.xh = L.rs = -1;
        if (x.ln) {
            L.xh = off;
            off = r4(off + bp * x.fout);
            L.rs = off;
            off = r4(off + bp);
        }
        L.dy = off;
        off = r4(off + bp * x.fout);
        L.dy2 = -1;
        if (consumers[l] == 2) {
            L.dy2 = off;
            off = r4(off + bp * x.fout);
        }
        L.wt = -1;  // allocated after the gradient row (below)
        L.dyc = -1;
        if (l == net->actor_out) {  // the value layer's (width 1) row- and feature-major forms coincide
            L.dyc = off;
            off = r4(off + (long long)x.fout * bp);
        } else if (l == net->critic_out) {
            L.dyc = L.dy;
        }
    }
    a.oc = off;
    off = r4(off + (long long)net->obs_dim * bp);
    a.dzr = off;
    off = r4(off + bp * maxw);
    a.dzc = off;
    off = r4(off + bp * maxw);
    a.dzr1 = off;
    off = r4(off + bp * maxw);
    a.dzc1 = off;
    off = r4(off + bp * maxw);
    // backward fusion: a layer whose only consumer is the next layer, at most
    // kBN wide with a LayerNorm / ReLU, gets its dZ from that consumer's dX
    // epilogue (dZ buffers alternate by layer parity, so the consumer's own dZ
    // and its source's never share one)
    for (int l = 0; l < nl; ++l) {
        a.L[l].fuse = a.L[l].fused = 0;
    }
    for (int l = 1; l < nl; ++l) {
        const agx_ppo_layer &x = net->layers[l], &sx = net->layers[l - 1];
        if (x.src == l - 1 && consumers[l - 1] == 1 && sx.fout <= kBN && (sx.ln || sx.relu)) {
            a.L[l].fuse = 1;
            a.L[l - 1].fused = 1;
        }
    }
    a.t1 = off;
    off = r4(off + bp * maxw);
    a.t2 = off;
    off = r4(off + bp * maxw);
    a.gr = off;
    off = r4(off + net->n_params);
    // the transposed weights last: a partner's scratch is everything before the
    // gradient row (its gradient goes to the exchange slab, the transposed
    // weights are shared by the agent's partners)
    a.ws_part = (a.gr + 63) & ~63ll;
    a.wt0 = off;
    for (int l = 0; l < nl; ++l) {
        const agx_ppo_layer &x = net->layers[l];
        if (x.src >= 0) {
            a.L[l].wt = off;
            off = r4(off + (long long)x.fin * x.fout);
        }
    }
    a.wt_agent = ((off - a.wt0) + 63) & ~63ll;
    a.ws_agent = (off + 63) & ~63ll;  // 256-byte aligned agent blocks
    a.nl = nl;
    a.aout = net->actor_out;
    a.cout = net->critic_out;
    a.A = net->n_actions;
    a.D = net->obs_dim;
    a.n = net->n_params;
    a.cstart = net->critic_start;
    a.bp = (int)bp;
    return AGX_OK;
}


constexpr int kActRows = 4 * kGW;  // env rows per policy-step workgroup (one row pass)

// the policy step keeps each layer's output only
long long act_plan(const GArgs &full, GActArgs &a) {
    long long off = 0;
    for (int l = 0; l < full.nl; ++l) {
        a.L[l] = full.L[l];
        GLay &L = a.L[l];
        L.yr = off;
        off = r4(off + (long long)kActRows * L.fout);
        L.yc = L.xh = L.rs = L.dy = L.dy2 = L.wt = L.dyc = -1;
        L.fuse = L.fused = 0;
    }
    a.nl = full.nl;
    a.aout = full.aout;
    a.cout = full.cout;
    a.A = full.A;
    a.D = full.D;
    a.n = full.n;
    a.rows = kActRows;
    a.obs_off = off;
    off = r4(off + (long long)kActRows * full.D);
    a.ws_block = (off + 63) & ~63ll;
    return a.ws_block;
}

// The policy step's few-row form: act_plan's layer table with every output
// a [16][ld] LDS tile (+ the LN affine copy), and the observation tile.  ->
// dynamic LDS bytes, 0 when it does not fit beside the kernel's static LDS
// (or AGX_GRAPH_FEW=0).  The policy-step block is kActRows = 16 rows either way.
template <class KER>
size_t act_plan_few(KER kernel, GActArgs &a) {
    if (const char *e = getenv("AGX_GRAPH_FEW"))
        if (atoi(e) == 0) return 0;
    static_assert(kActRows == kFR, "the few-row policy step covers one row block");
    auto ldof = [](int w) { return (w + 15) / 16 * 16 + 4; };
    long long off = 0;
    for (int l = 0; l < a.nl; ++l) {
        GLay &L = a.L[l];
        L.ld = ldof(L.fout);
        L.yr = off;
        off += (long long)kFR * L.ld;
        L.af = -1;
        if (L.ln == 2) {
            L.af = off;
            off += 2 * ((L.fout + 3) / 4 * 4);
        }
        L.xh = L.rs = -1;
    }
    a.ld0 = ldof(a.D);
    a.oc = off;
    off += (long long)kFR * a.ld0;
    a.lds_floats = (off + 3) & ~3ll;
    hipFuncAttributes fa{};
    const size_t st = hipFuncGetAttributes(&fa, (const void *)kernel) == hipSuccess ? fa.sharedSizeBytes : 8 * 1024;
    const size_t bytes = (size_t)a.lds_floats * 4;
    if (st >= kLdsMax || bytes > kLdsMax - st) return 0;
    (void)hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsMax - st));
    return bytes;
}

struct GraphWs {
    size_t gobs, gact, gmask, grow, agents, total;
};
GraphWs graph_ws(const GArgs &a, int64_t P, int64_t S, int64_t epochs) {
    GraphWs w;
    const size_t per = (size_t)epochs * P * S;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    w.gobs = 0;
    w.gact = up(per * a.D * 4);
    w.gmask = w.gact + up(per * 4);
    w.grow = w.gmask + up(per * 4);
    w.agents = w.grow + up(per * 4 * 4);
    w.total = w.agents + (size_t)P * a.ws_agent * 4;
    return w;
}

// The partnered learner's split of a minibatch: K partners of R rows
// (AGX_GRAPH_ROWS, default 16) while the whole grid (Q x K workgroups, Q = P
// rounded up to the 8 XCDs) stays co-resident; K = 1: the one-workgroup-per-
// agent kernel.  AGX_GRAPH_SPLIT caps K (tests, diagnostics).
int cu_count_g() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        hipDeviceProp_t prop;
        n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                ? prop.multiProcessorCount
                : 256;
        if (n <= 0) n = 256;
    }
    return n;
}
template <bool FEW>
int part_occupancy(size_t dyn) {  // co-resident partner workgroups per CU with dyn bytes of dynamic LDS
    static size_t last = (size_t)-1;
    static int n = 1;
    if (dyn != last) {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, ppo_learn_graph_part_kernel<FEW>, kGT, dyn) != hipSuccess)
            v = 1;
        n = v < 1 ? 1 : v;
        last = dyn;
    }
    return n;
}
// dynamic LDS the few-row form may take: the CU's 160 KB less the kernel's
// static LDS (queried once)
size_t few_lds_budget() {
    static size_t b = 0;
    if (!b) {
        hipFuncAttributes fa{};
        const size_t st = hipFuncGetAttributes(&fa, (const void *)ppo_learn_graph_part_kernel<true>) == hipSuccess
                              ? fa.sharedSizeBytes
                              : 8 * 1024;
        b = st < kLdsMax ? kLdsMax - st : 1;
        (void)hipFuncSetAttribute((const void *)ppo_learn_graph_part_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)b);
    }
    return b;
}
// the few-row form's plan: the general plan (validation, parameter offsets,
// transposed weights, accumulation order) with every activation tile moved to
// LDS: per layer Y, xhat + rstd (LayerNorm), dY, each [16][ld]; the
// observation tile; one dY' tile for the LN-affine gradients.  -> LDS bytes
// (0: the plan does not fit, or the graph is invalid)
size_t plan_few(const agx_ppo_graph *net, GArgs &a) {
    if (plan_graph(net, kFR, a) != AGX_OK) return 0;
    auto ldof = [](int w) { return (w + 15) / 16 * 16 + 4; };
    long long off = 0;
    int ldmax = 0;
    bool affine = false;
    for (int l = 0; l < a.nl; ++l) {
        GLay &L = a.L[l];
        L.ld = ldof(L.fout);
        L.yr = off;
        off += (long long)kFR * L.ld;
        L.xh = L.rs = -1;
        if (L.ln) {
            L.xh = off;
            off += (long long)kFR * L.ld;
            L.rs = off;
            off += kFR;
        }
        L.dy = off;
        off += (long long)kFR * L.ld;
        L.af = -1;
        if (L.ln == 2) {
            L.af = off;
            off += 2 * ((L.fout + 3) / 4 * 4);
        }
        L.yc = L.dy2 = L.dyc = -1;
        L.fuse = L.fused = 0;
        ldmax = L.ld > ldmax ? L.ld : ldmax;
        affine = affine || L.ln == 2;
    }
    a.ld0 = ldof(a.D);
    a.oc = off;
    off += (long long)kFR * a.ld0;
    a.t1 = off;
    if (affine) off += (long long)kFR * ldmax;
    a.lds_floats = (off + 3) & ~3ll;
    a.ws_part = 0;  // no global activation scratch
    const size_t bytes = (size_t)a.lds_floats * 4;
    return bytes <= few_lds_budget() ? bytes : 0;
}
// How a learn() runs, chosen per call (the workspace query makes the same
// choice): the few-row partnered form when a minibatch splits into at most
// kMaxGK slices of at most 16 rows whose tiles fit in LDS (AGX_GRAPH_FEW=0
// turns it off); else the general partnered form, K partners of R rows
// (AGX_GRAPH_ROWS, default 16); K = 1: one workgroup per agent.  The whole
// grid (Q x K workgroups, Q = P rounded up to the 8 XCDs) must be co-resident.
// AGX_GRAPH_SPLIT caps K (tests, diagnostics).
struct Split {
    int K = 1, R = 1, Q = 1;
    bool few = false;
    size_t dyn = 0;  // dynamic LDS bytes (few-row form)
};
Split graph_split(const agx_ppo_graph *net, int64_t P, int64_t batch) {
    Split sp;
    int rows = 16;
    if (const char *e = getenv("AGX_GRAPH_ROWS")) rows = atoi(e) >= 1 ? atoi(e) : 16;
    int cap = kMaxGK;
    if (const char *e = getenv("AGX_GRAPH_SPLIT")) cap = atoi(e) >= 1 ? atoi(e) : 1;
    bool few_ok = true;
    if (const char *e = getenv("AGX_GRAPH_FEW")) few_ok = atoi(e) != 0;
    sp.Q = (int)((P + 7) / 8 * 8);
    const int64_t cus = cu_count_g();
    int k = (int)((batch + rows - 1) / rows);
    if (k > cap) k = cap;
    if (few_ok && k > 1 && (batch + k - 1) / k <= kFR) {
        GArgs a{};
        const size_t dyn = plan_few(net, a);
        if (dyn && (int64_t)sp.Q * k <= (int64_t)part_occupancy<true>(dyn) * cus) {
            sp.few = true;
            sp.dyn = dyn;
            sp.K = k;
            sp.R = (int)((batch + k - 1) / k);
            return sp;
        }
    }
    while (k > 1 && (int64_t)sp.Q * k > (int64_t)part_occupancy<false>(0) * cus) --k;
    if (k > 1 && (int64_t)P * k > (int64_t)part_occupancy<false>(0) * cus) k = 1;
    sp.K = k < 1 ? 1 : k;
    sp.R = (int)((batch + sp.K - 1) / sp.K);
    return sp;
}
struct PartWs {
    size_t cnt, gobs, gact, gmask, grow, scratch, wt, slabs, sums, total;
    long long nslab;
};
PartWs part_ws(const GArgs &a, int64_t P, int64_t S, int64_t epochs, int K) {
    PartWs w;
    const size_t per = (size_t)epochs * P * S;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    w.cnt = 0;
    w.gobs = up(((size_t)4 * P + 1 + (size_t)kMaxGK * P) * 4);
    w.gact = w.gobs + up(per * a.D * 4);
    w.gmask = w.gact + up(per * 4);
    w.grow = w.gmask + up(per * 4);
    w.scratch = w.grow + up(per * 4 * 4);
    w.wt = w.scratch + up((size_t)P * K * a.ws_part * 4);
    w.nslab = ((long long)(a.n + 3) / 4 * 4 + 4 + 2 * kGW * K + 63) / 64 * 64;
    w.slabs = w.wt + up((size_t)P * a.wt_agent * 4);
    w.sums = w.slabs + up((size_t)P * 2 * K * w.nslab * 4);
    w.total = w.sums + (size_t)P * 2 * w.nslab * 4;
    return w;
}

}  // namespace
}  // namespace agx

using namespace agx;

static long long *&g_graph_stamps() {
    static long long *p = nullptr;
    return p;
}
extern "C" int agx_debug_graph_stamps(int64_t *buf) {
    g_graph_stamps() = reinterpret_cast<long long *>(buf);
    return AGX_OK;
}

extern "C" int agx_ppo_graph_check(const agx_ppo_graph *net) {
    GArgs a{};
    return plan_graph(net, 1, a);
}

extern "C" size_t agx_ppo_learn_graph_workspace_bytes(const agx_ppo_graph *net, int64_t P, int64_t S,
                                                      int64_t epochs, int64_t batch) {
    GArgs a{};
    if (P <= 0 || S <= 0 || epochs <= 0 || batch <= 0) return 0;
    const int64_t bb = batch < S ? batch : S;
    if (plan_graph(net, bb, a) != AGX_OK) return 0;
    size_t total = graph_ws(a, P, S, epochs).total;
    const Split sp = graph_split(net, P, bb);
    if (sp.K > 1) {  // room for either kernel: the split may change with the call's batch
        GArgs ap{};
        if (sp.few ? !plan_few(net, ap) : plan_graph(net, sp.R, ap) != AGX_OK) return 0;
        const size_t t = part_ws(ap, P, S, epochs, sp.K).total;
        total = t > total ? t : total;
    }
    return total;
}

extern "C" int agx_ppo_learn_graph(const agx_ppo_graph *net, const agx_ppo_learn_args *x, void *workspace,
                                   void *stream) {
    AGX_REQUIRE(net && x && workspace, "agx_ppo_learn_graph: null net / args / workspace");
    AGX_REQUIRE(x->params && x->exp_avg && x->exp_avg_sq && x->adam_step && x->lr && x->obs && x->actions &&
                    x->old_logp && x->adv && x->ret && x->old_value && x->perms,
                "agx_ppo_learn_graph: null pointer");
    const int64_t P = x->P, S = x->S, epochs = x->epochs, batch = x->batch;
    AGX_REQUIRE(P > 0 && P <= 65535 && S > 0 && S < (1ll << 31) && epochs > 0 && batch > 0 && epochs * P <= 65535,
                "agx_ppo_learn_graph: bad sizes P=%lld S=%lld epochs=%lld batch=%lld", (long long)P, (long long)S,
                (long long)epochs, (long long)batch);
    const int64_t bb = batch < S ? batch : S;
    const Split sp = graph_split(net, P, bb);
    const int K = sp.K, R = sp.R, Q = sp.Q;
    GArgs a{};
    const int rc = plan_graph(net, K > 1 ? R : bb, a);
    if (rc != AGX_OK) return rc;
    if (sp.few) AGX_REQUIRE(plan_few(net, a) == sp.dyn, "agx_ppo_learn_graph: few-row plan changed");
    char *ws = static_cast<char *>(workspace);
    hipStream_t s = as_stream(stream);
    size_t o_gobs, o_gact, o_gmask, o_grow;
    unsigned *counters = nullptr;
    int ncounters = 0;
    PartWs pw{};
    GraphWs w{};
    if (K > 1) {
        pw = part_ws(a, P, S, epochs, K);
        o_gobs = pw.gobs, o_gact = pw.gact, o_gmask = pw.gmask, o_grow = pw.grow;
        counters = reinterpret_cast<unsigned *>(ws + pw.cnt);
        ncounters = (int)(pw.gobs / sizeof(unsigned));
    } else {
        w = graph_ws(a, P, S, epochs);
        o_gobs = w.gobs, o_gact = w.gact, o_gmask = w.gmask, o_grow = w.grow;
    }
    float *gobs = reinterpret_cast<float *>(ws + o_gobs);
    int *gact = reinterpret_cast<int *>(ws + o_gact);
    unsigned *gmask = x->action_masks ? reinterpret_cast<unsigned *>(ws + o_gmask) : nullptr;
    float *grow = reinterpret_cast<float *>(ws + o_grow);
    dim3 ggrid((unsigned)ceil_div(S, 256), (unsigned)(epochs * P));
    ppo_gather_kernel<<<ggrid, 256, 0, s>>>(x->obs, reinterpret_cast<const long long *>(x->actions), x->old_logp,
                                            x->adv, x->ret, x->old_value, x->adv_stats,
                                            reinterpret_cast<const long long *>(x->perms), x->action_masks, a.A, S,
                                            a.D, (int)P, gobs, gact, gmask, grow, counters, ncounters,
                                            x->epochs_per_agent, x->error_word);
    const int rc2 = check_launch("agx_ppo_learn_graph gather");
    if (rc2) return rc2;
    a.ws = reinterpret_cast<float *>(ws + (K > 1 ? pw.scratch : w.agents));
    a.params = x->params;
    a.m = x->exp_avg;
    a.v = x->exp_avg_sq;
    a.lr = x->lr;
    a.b1 = x->beta1;
    a.b2 = x->beta2;
    a.eps = x->eps;
    a.step = reinterpret_cast<long long *>(x->adam_step);
    a.gobs = gobs;
    a.gact = gact;
    a.gmask = gmask;
    a.grow = grow;
    a.S = S;
    a.E = (int)epochs;
    a.B = (int)(batch < S ? batch : S);
    a.P = (int)P;
    a.clip = x->clip_coef;
    a.vf = x->vf_coef;
    a.ent = x->ent_coef;
    a.max_norm = x->max_grad_norm;
    a.target_kl = x->target_kl;
    a.batch_p = x->batch_per_agent;
    a.epochs_p = x->epochs_per_agent;
    a.ent_p = x->ent_coef_per_agent;
    a.loss_out = x->loss_out;
    a.kl_out = x->kl_out;
    a.epochs_out = x->epochs_out;
    a.skip = x->skip_if_set;
    {
        const char *d = getenv("AGX_GRAPH_DEBUG");
        a.dbg = d ? atoi(d) : 0;
    }
    a.err = x->error_word;
    if (K > 1) {
        a.K = K;
        a.R = R;
        a.Q = Q;
        a.nslab = pw.nslab;
        a.wtb = reinterpret_cast<float *>(ws + pw.wt);
        a.slabs = reinterpret_cast<float *>(ws + pw.slabs);
        a.sums = reinterpret_cast<float *>(ws + pw.sums);
        a.cnt = counters;
        a.stamps = g_graph_stamps();
        {
            const char *wt = getenv("AGX_LEARN_WRITETHROUGH");
            a.write_through = wt && atoi(wt) != 0;
        }
        AGX_REQUIRE((int64_t)Q * K <= 65535, "agx_ppo_learn_graph: too many workgroups");
        if (sp.few)
            ppo_learn_graph_part_kernel<true><<<(unsigned)(Q * K), kGT, sp.dyn, s>>>(a);
        else
            ppo_learn_graph_part_kernel<false><<<(unsigned)(Q * K), kGT, 0, s>>>(a);
    } else {
        ppo_learn_graph_kernel<<<(unsigned)P, kGT, 0, s>>>(a);
    }
    return check_launch("agx_ppo_learn_graph");
}

extern "C" size_t agx_ppo_act_graph_workspace_bytes(const agx_ppo_graph *net, int64_t P, int64_t N) {
    GArgs full{};
    GActArgs a{};
    if (P <= 0 || N <= 0 || plan_graph(net, 1, full) != AGX_OK) return 0;
    return (size_t)P * ceil_div(N, kActRows) * act_plan(full, a) * sizeof(float);
}

extern "C" int agx_ppo_act_graph(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params,
                                 const float *obs, int64_t obs_agent_stride, const uint8_t *action_mask,
                                 int64_t mask_agent_stride, int sample, uint64_t seed, uint64_t counter,
                                 int64_t *actions, float *log_probs, float *values, float *entropy,
                                 int64_t out_agent_stride, int64_t *actions_flat, const int64_t *agent_env_base,
                                 void *workspace, void *stream) {
    AGX_REQUIRE(net && params && obs && workspace && P > 0 && N > 0 && P <= 65535, "agx_ppo_act_graph: bad arguments");
    GArgs full{};
    const int rc = plan_graph(net, 1, full);
    if (rc != AGX_OK) return rc;
    GActArgs a{};
    act_plan(full, a);
    a.ws = static_cast<float *>(workspace);
    a.params = params;
    a.obs = obs;
    a.obs_pstride = obs_agent_stride;
    a.N = (int)N;
    a.P = (int)P;
    a.sample = sample;
    a.seed = seed;
    a.counter = counter;
    a.act_out = reinterpret_cast<long long *>(actions);
    a.logp_out = log_probs;
    a.value_out = values;
    a.ent_out = entropy;
    a.out_pstride = out_agent_stride;
    a.act_flat = reinterpret_cast<long long *>(actions_flat);
    a.mask = action_mask;
    a.mask_pstride = mask_agent_stride;
    a.env_base = reinterpret_cast<const long long *>(agent_env_base);
    dim3 grid((unsigned)ceil_div(N, kActRows), (unsigned)P);
    if (const size_t dyn = act_plan_few(ppo_act_graph_kernel<true>, a))
        ppo_act_graph_kernel<true><<<grid, kGT, dyn, as_stream(stream)>>>(a);
    else
        ppo_act_graph_kernel<false><<<grid, kGT, 0, as_stream(stream)>>>(a);
    return check_launch("agx_ppo_act_graph");
}

// ---------------------------------------------------------------------------
// persistent rollout / evaluation of runtime-shape populations
// ---------------------------------------------------------------------------
extern "C" int64_t agx_ppo_rollout_graph_workgroups(int64_t P, int64_t N) { return P * ceil_div(N, kActRows); }

extern "C" int64_t agx_ppo_rollout_graph_max_workgroups(void) {
    static int occ = -1;
    if (occ < 0) {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, ppo_rollout_graph_persistent_kernel<false>, kGT, 0) !=
            hipSuccess)
            v = 0;
        occ = v;
    }
    return (int64_t)occ * cu_count_g();
}

extern "C" size_t agx_ppo_rollout_graph_ctl_bytes(int64_t P, int64_t N) {
    const unsigned nwg = (unsigned)agx_ppo_rollout_graph_workgroups(P, N);
    return (size_t)rollout_release_offset(nwg, nwg) * sizeof(unsigned);
}

namespace {
int launch_graph_persistent(const agx_ppo_graph *net, int64_t P, int64_t N, ActArgs *steps, int64_t nsteps,
                            uint32_t base, agx_rollout_ctl *ctl, double timeout_s, void *workspace, void *stream,
                            const char *who) {
    GArgs full{};
    const int rc = plan_graph(net, 1, full);
    if (rc != AGX_OK) return rc;
    const int64_t nwg = agx_ppo_rollout_graph_workgroups(P, N);
    if (nwg > agx_ppo_rollout_graph_max_workgroups()) {
        set_error("%s: %lld workgroups cannot all be resident; use per-step launches", who, (long long)nwg);
        return AGX_EUNSUPPORTED;
    }
    GActArgs a{};
    act_plan(full, a);
    a.ws = static_cast<float *>(workspace);
    a.N = (int)N;
    a.P = (int)P;
    const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    ctl->nwg = (uint32_t)nwg;
    dim3 grid((unsigned)ceil_div(N, kActRows), (unsigned)P);
    // the few-row form when its tiles fit and the grid stays co-resident with them
    size_t dyn = act_plan_few(ppo_rollout_graph_persistent_kernel<true>, a);
    if (dyn) {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, ppo_rollout_graph_persistent_kernel<true>, kGT, dyn) !=
                hipSuccess ||
            (int64_t)v * cu_count_g() < nwg)
            dyn = 0;
    }
    if (dyn)
        ppo_rollout_graph_persistent_kernel<true><<<grid, kGT, dyn, as_stream(stream)>>>(a, steps, (int)nsteps, ctl,
                                                                                         ticks, base);
    else
        ppo_rollout_graph_persistent_kernel<false><<<grid, kGT, 0, as_stream(stream)>>>(a, steps, (int)nsteps, ctl,
                                                                                         ticks, base);
    return check_launch(who);
}
}  // namespace

extern "C" int agx_ppo_rollout_graph_persistent(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params,
                                                const agx_rollout_io *ios, int64_t nsteps, uint32_t base,
                                                uint64_t seed, uint64_t counter0, void *args_host,
                                                agx_rollout_ctl *ctl, double timeout_s, void *workspace,
                                                void *stream) {
    AGX_REQUIRE(net && ios && params && args_host && ctl && workspace && P > 0 && N > 0 && P <= 65535 && nsteps >= 1,
                "agx_ppo_rollout_graph_persistent: bad arguments");
    AGX_REQUIRE((uint64_t)base + (uint64_t)nsteps < AGX_ROLLOUT_STOP, "agx_ppo_rollout_graph_persistent: base wraps");
    AGX_REQUIRE(timeout_s > 0 && timeout_s < 3600, "agx_ppo_rollout_graph_persistent: timeout_s out of range");
    AGX_REQUIRE(net->obs_dim >= 1, "agx_ppo_rollout_graph_persistent: bad graph");
    ActArgs *steps = static_cast<ActArgs *>(args_host);
    for (int64_t t = 0; t < nsteps; ++t) {
        const bool last = t + 1 == nsteps;
        if (int rc = check_rollout_io(ios + t, 1, params, "agx_ppo_rollout_graph_persistent")) return rc;
        fill_rollout_args(steps[t], net->obs_dim, net->n_actions, P, N, params, ios + t, 1, last ? 0 : 1, seed,
                          last ? 0 : counter0 + 1 + (uint64_t)t);
    }
    return launch_graph_persistent(net, P, N, steps, nsteps, base, ctl, timeout_s, workspace, stream,
                                   "agx_ppo_rollout_graph_persistent");
}

extern "C" int agx_ppo_eval_graph_persistent(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params,
                                             const float *stage_obs, const uint8_t *stage_mask,
                                             int64_t *actions_flat, const int64_t *agent_env_base, int64_t nsteps,
                                             uint32_t base, uint64_t seed, uint64_t counter0, void *args_host,
                                             agx_rollout_ctl *ctl, double timeout_s, void *workspace, void *stream) {
    AGX_REQUIRE(net && params && stage_obs && actions_flat && args_host && ctl && workspace && P > 0 && N > 0 &&
                    P <= 65535 && nsteps >= 1,
                "agx_ppo_eval_graph_persistent: bad arguments");
    AGX_REQUIRE((uint64_t)base + (uint64_t)nsteps < AGX_ROLLOUT_STOP, "agx_ppo_eval_graph_persistent: base wraps");
    AGX_REQUIRE(timeout_s > 0 && timeout_s < 3600, "agx_ppo_eval_graph_persistent: timeout_s out of range");
    ActArgs *steps = static_cast<ActArgs *>(args_host);
    for (int64_t t = 0; t < nsteps; ++t) {
        ActArgs a{};
        a.params = params;
        a.obs = stage_obs;
        a.obs_pstride = N * (int64_t)net->obs_dim;
        a.N = (int)N;
        a.P = (int)P;
        a.sample = 1;
        a.seed = seed;
        a.counter = counter0 + (uint64_t)t;
        a.act_flat = reinterpret_cast<long long *>(actions_flat);
        a.act = 1;
        a.mask = stage_mask;
        a.mask_pstride = N * (int64_t)net->n_actions;
        a.env_base = reinterpret_cast<const long long *>(agent_env_base);
        steps[t] = a;
    }
    return launch_graph_persistent(net, P, N, steps, nsteps, base, ctl, timeout_s, workspace, stream,
                                   "agx_ppo_eval_graph_persistent");
}

// ---------------------------------------------------------------------------
// evaluation of a whole population, every agent on its own network
// ---------------------------------------------------------------------------
static long long *&g_eval_stamps() {
    static long long *p = nullptr;
    return p;
}
// diagnostic: block 0's stamps of steps 2..33 of agx_ppo_eval_multi_persistent,
// kEvalStamps per step: release seen, observations staged, forward done, done
// word written (s_memrealtime, 100 MHz), then the shader clock at the forward's
// start and after each layer (0: not run); int64[32 * kEvalStamps], or null
// to stop
extern "C" int agx_debug_eval_stamps(int64_t *buf) {
    g_eval_stamps() = reinterpret_cast<long long *>(buf);
    return AGX_OK;
}

extern "C" size_t agx_ppo_eval_multi_bytes(int64_t P) { return P > 0 ? (size_t)P * sizeof(EvalAgent) : 0; }

namespace {
// agent p's policy-step plan (act_plan + act_plan_few) into x; -> its dynamic
// LDS bytes (0: the plan does not fit).  Only the layers on the actor's path
// run; wlds: their weights get LDS tiles after the activation tiles.
size_t eval_agent_plan(const agx_ppo_graph *net, EvalAgent &x, bool wlds) {
    GArgs full{};
    if (plan_graph(net, 1, full) != AGX_OK) return 0;
    GActArgs a{};
    act_plan(full, a);
    const size_t dyn = wlds ? act_plan_few(ppo_eval_multi_persistent_kernel<true>, a)
                            : act_plan_few(ppo_eval_multi_persistent_kernel<false>, a);
    if (!dyn) return 0;
    for (int l = 0; l < kGL; ++l) x.L[l] = a.L[l];
    x.nl = a.nl;
    x.aout = a.aout;
    x.cout = a.cout;
    x.n = a.n;
    x.ld0 = a.ld0;
    x.oc = a.oc;
    x.lds_floats = a.lds_floats;
    x.run = 0;
    for (int l = a.aout; l >= 0; l = a.L[l].src) x.run |= 1u << l;
    long long off = a.lds_floats;
    for (int l = 0; l < kGL; ++l) {
        x.wl[l] = -1;
        x.ldw[l] = 0;
        if (!wlds || l >= a.nl || !((x.run >> l) & 1u)) continue;
        const long long fp = (a.L[l].fout + 15) / 16 * 16;
        x.ldw[l] = (a.L[l].fin + 15) / 16 * 16 + 4;
        x.wl[l] = off;
        off += fp * x.ldw[l] + fp;
    }
    x.lds_w = (off + 3) & ~3ll;
    if (!wlds) return dyn;
    hipFuncAttributes fa{};
    const size_t st = hipFuncGetAttributes(&fa, (const void *)ppo_eval_multi_persistent_kernel<true>) == hipSuccess
                          ? fa.sharedSizeBytes
                          : 8 * 1024;
    const size_t bytes = (size_t)x.lds_w * 4;
    return bytes <= kLdsMax - st ? bytes : 0;
}

// the population's form: 1 LDS-resident weights, 0 weights from L2, -1 none
// (every workgroup co-resident either way); dyn: the launch's LDS bytes
int eval_form(const agx_ppo_graph *const *nets, int64_t P, int64_t N, size_t *dyn_out) {
    if (!nets || P <= 0 || N <= 0 || P > 65535) return -1;
    if (const char *e = getenv("AGX_GRAPH_FEW"))
        if (atoi(e) == 0) return -1;
    bool wl_ok = true;
    if (const char *e = getenv("AGX_EVAL_WLDS"))
        if (atoi(e) == 0) wl_ok = false;
    for (int w = wl_ok ? 1 : 0; w >= 0; --w) {
        size_t dyn = 0;
        bool ok = true;
        for (int64_t p = 0; p < P && ok; ++p) {
            EvalAgent x{};
            if (!nets[p] || nets[p]->obs_dim != nets[0]->obs_dim || nets[p]->n_actions != nets[0]->n_actions)
                return -1;
            const size_t d = eval_agent_plan(nets[p], x, w == 1);
            ok = d != 0;
            dyn = d > dyn ? d : dyn;
        }
        if (!ok) continue;
        int v = 0;
        const hipError_t e = w ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                     &v, ppo_eval_multi_persistent_kernel<true>, kGT, dyn)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                     &v, ppo_eval_multi_persistent_kernel<false>, kGT, dyn);
        if (e != hipSuccess || (int64_t)v * cu_count_g() < P * ceil_div(N, kFR)) continue;
        if (dyn_out) *dyn_out = dyn;
        return w;
    }
    return -1;
}
}  // namespace

extern "C" int agx_ppo_eval_multi_supported(const agx_ppo_graph *const *nets, int64_t P, int64_t N) {
    return eval_form(nets, P, N, nullptr) >= 0 ? 1 : 0;
}

extern "C" int agx_ppo_eval_multi_persistent(const agx_ppo_graph *const *nets, const float *const *params,
                                             const int64_t *env_base, const uint64_t *seeds,
                                             const uint64_t *counters, int64_t P, int64_t N, const float *stage_obs,
                                             int64_t *actions_flat, int64_t nsteps, uint32_t base, void *agents_host,
                                             void *agents_dev, agx_rollout_ctl *ctl, double timeout_s,
                                             const agx_eval_tally *tally, void *stream) {
    AGX_REQUIRE(nets && params && env_base && seeds && counters && stage_obs && actions_flat && agents_host &&
                    agents_dev && ctl && P > 0 && N > 0 && P <= 65535 && nsteps >= 1,
                "agx_ppo_eval_multi_persistent: bad arguments");
    AGX_REQUIRE((uint64_t)base + (uint64_t)nsteps < AGX_ROLLOUT_STOP, "agx_ppo_eval_multi_persistent: base wraps");
    AGX_REQUIRE(timeout_s > 0 && timeout_s < 3600, "agx_ppo_eval_multi_persistent: timeout_s out of range");
    size_t dyn = 0;
    const int form = eval_form(nets, P, N, &dyn);
    AGX_REQUIRE(form >= 0, "agx_ppo_eval_multi_persistent: unsupported population");
    EvalAgent *ag = static_cast<EvalAgent *>(agents_host);
    for (int64_t p = 0; p < P; ++p) {
        AGX_REQUIRE(params[p], "agx_ppo_eval_multi_persistent: agent %lld has no parameters", (long long)p);
        EvalAgent x{};
        eval_agent_plan(nets[p], x, form == 1);
        x.params = params[p];
        x.env_base = env_base[p];
        x.seed = seeds[p];
        x.counter0 = counters[p];
        ag[p] = x;
    }
    hipStream_t s = as_stream(stream);
    if (hipMemcpyAsync(agents_dev, agents_host, (size_t)P * sizeof(EvalAgent), hipMemcpyHostToDevice, s) !=
        hipSuccess) {
        set_error("agx_ppo_eval_multi_persistent: agent table copy failed");
        return AGX_EHIP;
    }
    const int64_t nwg = P * ceil_div(N, kFR);
    const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    ctl->nwg = (uint32_t)nwg;
    dim3 grid((unsigned)ceil_div(N, kFR), (unsigned)P);
    EvalTally et{};
    if (tally) {
        AGX_REQUIRE(tally->stage_rew && tally->stage_done && tally->scores && tally->completed && tally->finished &&
                        tally->fin_words,
                    "agx_ppo_eval_multi_persistent: incomplete tally");
        et = EvalTally{tally->stage_rew, tally->stage_done, tally->scores, tally->completed, tally->finished,
                       tally->fin_words, tally->prev ? 1 : 0};
    }
    auto *kern = form == 1 ? ppo_eval_multi_persistent_kernel<true> : ppo_eval_multi_persistent_kernel<false>;
    kern<<<grid, kGT, dyn, s>>>(static_cast<const EvalAgent *>(agents_dev), (int)N, nets[0]->n_actions,
                                nets[0]->obs_dim, stage_obs, reinterpret_cast<long long *>(actions_flat), (int)nsteps,
                                ctl, ticks, base, g_eval_stamps(), et);
    return check_launch("agx_ppo_eval_multi_persistent");
}
