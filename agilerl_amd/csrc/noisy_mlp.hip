// Rainbow's dueling head streams (include/agx_noisy.h): every stream's
// NoisyLinear -> LayerNorm -> ReLU ... -> NoisyLinear stack, one launch per
// layer depth forward and one per depth backward.
//
// Forward, one depth: out[b][n] = sum_k act(in)[b][k] * W[n][k] + bias[n],
//   W = w_mu + w_sigma * w_eps and bias likewise, each rounded as torch's
//   two elementwise ops round it (custom_components.py:124-131);
//   act(in) = in for depth 0 (the latent), relu(LN(in) * gamma + beta) for
//   deeper layers (the previous layer's LayerNorm + ReLU folded into this
//   layer's operand loads, mlp.py create_mlp order Linear -> LN -> ReLU).
//   A workgroup owns a 16-row x 16-column output tile; its four waves split
//   the K dimension (v_mfma_f32_16x16x4_f32 chains) and their partial tiles
//   are summed in wave order through LDS.
// Backward, one depth (two roles in one launch):
//   role W: dW[n][k] = sum_b dy[b][n] * act(in)[b][k] (16 n x 64 k per
//     workgroup, 16 k per wave, the whole batch reduced in each wave), the
//     bias gradient and, on hidden layers, the LayerNorm affine gradients;
//     d mu = dW, d sigma = dW * eps (the reference's autograd of mu + sigma * eps);
//   role X: d act(in)[b][k] = sum_n dy[b][n] * W[n][k] (16 b x 16 k per
//     workgroup, the waves split n), summed over both streams at depth 0.
//   dy = the incoming gradient on the output layer; on a hidden layer the
//   LayerNorm + ReLU backward of the gradient of its activation, recomputed
//   in the loads from per-row statistics (mean, rstd and the two row sums
//   of the LayerNorm backward).
// Row statistics never take a pass over a row: the workgroup that writes a
// 16-feature tile of a hidden output also writes that tile's mean and sum of
// squared deviations per row (ln_part), and the role-X workgroup that writes
// a tile of a hidden activation's gradient writes that tile's two
// LayerNorm-backward sums; a consumer combines a row's tiles in tile order
// (Chan's pairwise update for the moments).  Forward and backward read the
// same partials through the same code, and y = xhat * gamma + beta is
// rounded explicitly, so the ReLU mask the backward recomputes is the
// forward's.
#include <cstdint>

#include "agx_common.h"
#include "../../include/agx_noisy.h"

namespace agx {

namespace nmlp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = AGX_NOISY_MAX_ROWS;

struct Layer {
    const float *in, *in_g, *in_b;  // input [B][K]; in_g: the input is relu(LN(in) * in_g + in_b)
    const float *in_part;           // LN statistics tiles of in [B][ceil(K/16)][2] (with in_g)
    const float *w_mu, *w_sig, *w_eps, *b_mu, *b_sig, *b_eps;
    float *out;                     // [B][N]
    float *out_part;                // hidden layers: LN statistics tiles of out [B][ceil(N/16)][2]
    const float *dsrc;              // backward: d/d out (out_g == null) or d/d relu(LN(out)) [B][N]
    const float *out_g, *out_b;     // LayerNorm affine of this layer's output (hidden layers)
    const float *s_part;            // backward, hidden layers: LN-backward sum tiles of dsrc [B][ceil(N/16)][2]
    float *gw_mu, *gw_sig, *gb_mu, *gb_sig, *g_g, *g_b;
    float *din;                     // role X output [B][K] (null: none)
    float *din_part;                // role X, with in_g: LN-backward sum tiles of din [B][ceil(K/16)][2]
    int K, N, tiles_w, tiles_x;
};

struct Level {
    Layer s[AGX_NOISY_MAX_STREAMS];
    int S, B, sum_din;
    float eps;
};

__device__ __forceinline__ float wval(const Layer &L, int64_t i) {
    const float w = L.w_mu[i];
    return L.w_sig ? __fadd_rn(w, __fmul_rn(L.w_sig[i], L.w_eps[i])) : w;
}

__device__ __forceinline__ float bval(const Layer &L, int n) {
    const float b = L.b_mu[n];
    return L.b_sig ? __fadd_rn(b, __fmul_rn(L.b_sig[n], L.b_eps[n])) : b;
}

__device__ __forceinline__ float ln_xhat(float h, float mu, float rs) { return __fmul_rn(__fsub_rn(h, mu), rs); }
__device__ __forceinline__ float ln_y(float xhat, float g, float b) { return __fadd_rn(__fmul_rn(xhat, g), b); }

// a row's mean and rstd from its tiles' (mean, M2), combined in tile order
// (eight tiles' loads in flight at a time)
__device__ __forceinline__ void ln_stats(const float *part, int N, float eps, float &mu, float &rs) {
    const int T = (N + 15) >> 4;
    float na = 0.f, ma = 0.f, qa = 0.f;
    for (int t0 = 0; t0 < T; t0 += 8) {
        float mb[8], qb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = min(t0 + j, T - 1);
            mb[j] = part[2 * t];
            qb[j] = part[2 * t + 1];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = t0 + j;
            if (t >= T) break;
            const float nb = (float)min(16, N - 16 * t);
            if (t == 0) {
                na = nb;
                ma = mb[j];
                qa = qb[j];
            } else {
                const float n = na + nb, d = mb[j] - ma;
                ma = ma + d * (nb / n);
                qa = (qa + qb[j]) + (d * d) * (na * nb / n);
                na = n;
            }
        }
    }
    mu = ma;
    rs = __frsqrt_rn(qa / (float)N + eps);
}

// a row's LayerNorm-backward sums (s1 = sum g, s2 = sum g * xhat, g = da * [y > 0] * gamma) from its tiles
__device__ __forceinline__ void ln_sums(const float *part, int N, float &s1, float &s2) {
    const int T = (N + 15) >> 4;
    float a = 0.f, b = 0.f;
    for (int t0 = 0; t0 < T; t0 += 8) {
        float pa[8], pb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = min(t0 + j, T - 1);
            pa[j] = part[2 * t];
            pb[j] = part[2 * t + 1];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (t0 + j >= T) break;
            a += pa[j];
            b += pb[j];
        }
    }
    s1 = a;
    s2 = b;
}

__device__ __forceinline__ float ln_relu_g(float xh, float da, float gam, float bet) {
    return ln_y(xh, gam, bet) > 0.f ? __fmul_rn(da, gam) : 0.f;
}

// d/d out[b][n] of a hidden layer from the gradient of its activation
__device__ __forceinline__ float ln_relu_bwd(float h, float da, float gam, float bet, float mu, float rs, float s1,
                                             float s2, float invN) {
    const float xh = ln_xhat(h, mu, rs);
    const float gx = ln_relu_g(xh, da, gam, bet);
    return rs * ((gx - s1 * invN) - xh * (s2 * invN));
}

// one 16-lane group's tile partials of a row (lane group = lanes with equal lane >> 4), value v valid if ok
__device__ __forceinline__ void tile_moments(float v, bool ok, int cnt, int lane, float &m, float &q2) {
    const float s = group_sum<16>(ok ? v : 0.f);
    m = __shfl(s, lane & ~15, 64) / (float)cnt;
    const float d = ok ? v - m : 0.f;
    q2 = __shfl(group_sum<16>(d * d), lane & ~15, 64);
}


// ---------------------------------------------------------------------------
__device__ __forceinline__ void fwd_body(const Level &lv, const Layer &L, int blk) {
    __shared__ float st[2][16];
    __shared__ f32x4 red[3][64];
    const int B = lv.B, K = L.K, N = L.N;
    const int nrb = (B + 15) >> 4;
    const int n0 = (blk / nrb) * 16, b0 = (blk % nrb) * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool ln = L.in_g != nullptr;
    const int r = b0 + (lane & 15), n = n0 + (lane & 15), q = lane >> 4;
    const bool rok = r < B, nok = n < N;
    // every load is unconditional (indices clamped, pointers selected
    // uniformly), and the first K chunk's operands and the epilogue's bias are
    // requested before the LayerNorm statistics are combined: one memory
    // round trip ahead of the MFMAs instead of three in a row
    const float *xrow = L.in + (int64_t)(rok ? r : 0) * K;
    const int64_t wrow = (int64_t)(nok ? n : 0) * K;
    const bool noisy = L.w_sig != nullptr;
    const float *wsig = noisy ? L.w_sig : L.w_mu, *weps = noisy ? L.w_eps : L.w_mu;
    const float *ing = ln ? L.in_g : L.w_mu, *inb = ln ? L.in_b : L.w_mu;
    const float *bsig = noisy ? L.b_sig : L.b_mu, *beps = noisy ? L.b_eps : L.b_mu;
    const int nb_ = nok ? n : N - 1;
    const float bmu = L.b_mu[nb_], bs = bsig[nb_], be = beps[nb_];
    float xv[4][4], wm[4][4], ws[4][4], we[4][4], gg[4][4], gb[4][4];
#define NMLP_LOAD(KC)                                                   \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                     \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                 \
            const int kk = min((KC) + 64 * u + 4 * q + j, K - 1);       \
            xv[u][j] = xrow[kk];                                        \
            wm[u][j] = L.w_mu[wrow + kk];                               \
            ws[u][j] = wsig[wrow + kk];                                 \
            we[u][j] = weps[wrow + kk];                                 \
            gg[u][j] = ing[kk];                                         \
            gb[u][j] = inb[kk];                                         \
        }                                                               \
    }
    NMLP_LOAD(wave * 16)
    if (ln) {
        if (threadIdx.x < 16) {
            const int b = b0 + threadIdx.x;
            float mu = 0.f, rs = 0.f;
            if (b < B) ln_stats(L.in_part + (int64_t)b * (((K + 15) >> 4) * 2), K, lv.eps, mu, rs);
            st[0][threadIdx.x] = mu;
            st[1][threadIdx.x] = rs;
        }
        __syncthreads();
    }
    const float mu = ln ? st[0][lane & 15] : 0.f, rs = ln ? st[1][lane & 15] : 0.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int kc = wave * 16; kc < K; kc += 256) {  // four 16-deep k blocks of this wave per chunk
        float a[4][4], w[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool kok = kc + 64 * u + 4 * q + j < K;
                float x = xv[u][j];
                if (ln) x = fmaxf(ln_y(ln_xhat(x, mu, rs), gg[u][j], gb[u][j]), 0.f);
                a[u][j] = (rok && kok) ? x : 0.f;
                const float wf = noisy ? __fadd_rn(wm[u][j], __fmul_rn(ws[u][j], we[u][j])) : wm[u][j];
                w[u][j] = (nok && kok) ? wf : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][j], w[u][j], acc, 0, 0, 0);
        if (kc + 256 < K) {
            NMLP_LOAD(kc + 256)
        }
    }
#undef NMLP_LOAD
    if (wave) red[wave - 1][lane] = acc;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) acc += red[w][lane];
        const int col = n0 + (lane & 15);
        const bool cok = col < N;
        const float bias = noisy ? __fadd_rn(bmu, __fmul_rn(bs, be)) : bmu;
        const int T = (N + 15) >> 4, cnt = min(16, N - n0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = b0 + 4 * q + i;
            const float v = acc[i] + bias;
            if (row < B && cok) L.out[(int64_t)row * N + col] = v;
            if (L.out_part) {
                float m, q2;
                tile_moments(v, cok, cnt, lane, m, q2);
                if ((lane & 15) == 0 && row < B) {
                    float *p = L.out_part + ((int64_t)row * T + (n0 >> 4)) * 2;
                    p[0] = m;
                    p[1] = q2;
                }
            }
        }
    }
}

// stream dispatch with constant indices into the kernel argument (a
// runtime-indexed Level would be copied to scratch)
__global__ __launch_bounds__(256) void fwd_kernel(Level lv) {
    int blk = blockIdx.x;
#pragma unroll
    for (int s = 0; s < AGX_NOISY_MAX_STREAMS; ++s) {
        if (s < lv.S) {
            if (blk < lv.s[s].tiles_w || s + 1 == lv.S) {
                fwd_body(lv, lv.s[s], blk);
                return;
            }
            blk -= lv.s[s].tiles_w;
        }
    }
}

// ---------------------------------------------------------------------------
// role W: 16 output features x 64 input features of one stream's layer
__device__ __forceinline__ void bwd_weights(const Level &lv, const Layer &L, int blk) {
    __shared__ float tab[6][kRows];  // out-LN mean, rstd, s1, s2 | in-LN mean, rstd
    const int B = lv.B, K = L.K, N = L.N;
    const int nkt = (K + 63) >> 6;
    const int n0 = (blk / nkt) * 16, kt = blk % nkt;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool oln = L.out_g != nullptr, iln = L.in_g != nullptr;
    const int q = lane >> 4;
    const int n = n0 + (lane & 15), k = kt * 64 + wave * 16 + (lane & 15);
    const bool nok = n < N, kok = k < K;
    const int nc_ = nok ? n : N - 1, kc_ = kok ? k : K - 1;
    const float *og = oln ? L.out_g : L.dsrc, *ob = oln ? L.out_b : L.dsrc, *oh = oln ? L.out : L.dsrc;
    const float *ig = iln ? L.in_g : L.in, *ib = iln ? L.in_b : L.in;
    // the first 64 rows' operands are requested before the row statistics are
    // combined (unconditional loads, clamped indices)
    const float gn = og[nc_], bn = ob[nc_], gk = ig[kc_], bk = ib[kc_];
    float dv[4][4], hv[4][4], xv[4][4];
#define NMLP_LOADW(BC)                                                  \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                     \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                 \
            const int bb = min((BC) + 16 * u + 4 * q + j, B - 1);       \
            dv[u][j] = L.dsrc[(int64_t)bb * N + nc_];                   \
            hv[u][j] = oh[(int64_t)bb * N + nc_];                       \
            xv[u][j] = L.in[(int64_t)bb * K + kc_];                     \
        }                                                               \
    }
    NMLP_LOADW(0)
    if (oln || iln) {
        for (int b = threadIdx.x; b < B; b += 256) {
            if (oln) {
                const int64_t o = (int64_t)b * (((N + 15) >> 4) * 2);
                float mu, rs, s1, s2;
                ln_stats(L.out_part + o, N, lv.eps, mu, rs);
                ln_sums(L.s_part + o, N, s1, s2);
                tab[0][b] = mu;
                tab[1][b] = rs;
                tab[2][b] = s1;
                tab[3][b] = s2;
            }
            if (iln) {
                float mu, rs;
                ln_stats(L.in_part + (int64_t)b * (((K + 15) >> 4) * 2), K, lv.eps, mu, rs);
                tab[4][b] = mu;
                tab[5][b] = rs;
            }
        }
        __syncthreads();
    }
    const float invN = 1.f / (float)N;
    // every wave reduces the whole batch for its 16 features: the bias and
    // LayerNorm-affine sums ride along (reduced over the four lane groups after)
    float sb = 0.f, sg = 0.f, sbeta = 0.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int bc = 0; bc < B; bc += 64) {  // four 16-row blocks in flight
        float a[4][4], x[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int b = bc + 16 * u + 4 * q + j;
                const int bb = min(b, B - 1);
                const bool bok = b < B;
                float d = dv[u][j];
                if (oln) {
                    const float xh = ln_xhat(hv[u][j], tab[0][bb], tab[1][bb]);
                    const float gm = (bok && ln_y(xh, gn, bn) > 0.f) ? dv[u][j] : 0.f;
                    sbeta += gm;
                    sg = __fmaf_rn(gm, xh, sg);
                    d = ln_relu_bwd(hv[u][j], d, gn, bn, tab[0][bb], tab[1][bb], tab[2][bb], tab[3][bb], invN);
                }
                float xa = xv[u][j];
                if (iln) xa = fmaxf(ln_y(ln_xhat(xa, tab[4][bb], tab[5][bb]), gk, bk), 0.f);
                a[u][j] = (bok && nok) ? d : 0.f;
                x[u][j] = (bok && kok) ? xa : 0.f;
                sb += a[u][j];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][j], x[u][j], acc, 0, 0, 0);
        if (bc + 64 < B) {
            NMLP_LOADW(bc + 64)
        }
    }
#undef NMLP_LOADW
    // lane: dW[n0 + 4q + i][k]
    if (kok) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int nn = n0 + 4 * q + i;
            if (nn < N) {
                const int64_t o = (int64_t)nn * K + k;
                L.gw_mu[o] = acc[i];
                if (L.w_sig) L.gw_sig[o] = __fmul_rn(acc[i], L.w_eps[o]);
            }
        }
    }
    if (kt == 0 && wave == 0) {  // bias (and LayerNorm affine) gradients of the 16 features
        sb += __shfl_xor(sb, 16, 64);
        sb += __shfl_xor(sb, 32, 64);
        sg += __shfl_xor(sg, 16, 64);
        sg += __shfl_xor(sg, 32, 64);
        sbeta += __shfl_xor(sbeta, 16, 64);
        sbeta += __shfl_xor(sbeta, 32, 64);
        if (q == 0 && nok) {
            L.gb_mu[n] = sb;
            if (L.b_sig) L.gb_sig[n] = __fmul_rn(sb, L.b_eps[n]);
            if (oln) {
                L.g_g[n] = sg;
                L.g_b[n] = sbeta;
            }
        }
    }
}

// role X: d act(in) for 16 rows x 16 input features, over streams [s_lo, s_hi)
__device__ __forceinline__ void bwd_inputs(const Level &lv, const Layer &L0, int s_lo, int s_hi, int blk) {
    __shared__ float rt[6][16];  // out-LN mean, rstd, s1, s2 of the stream in hand | in-LN mean, rstd
    __shared__ f32x4 red[3][64];
    const int B = lv.B, K = L0.K;
    const int nrb = (B + 15) >> 4;
    const int k0 = (blk / nrb) * 16, b0 = (blk % nrb) * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = lane >> 4;
    const int r = b0 + (lane & 15), k = k0 + (lane & 15);
    const bool rok = r < B, kok = k < K;
    const bool dpart = L0.din_part != nullptr;
    // the epilogue's operands (din's LayerNorm inputs), requested up front
    const int kx = kok ? k : K - 1;
    const float *pin = dpart ? L0.in : L0.din, *pig = dpart ? L0.in_g : L0.din, *pib = dpart ? L0.in_b : L0.din;
    float hin[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) hin[i] = pin[(int64_t)min(b0 + 4 * q + i, B - 1) * K + kx];
    const float gin = pig[kx], bin = pib[kx];
    if (dpart && threadIdx.x < 16) {  // the input's LN statistics of the 16 rows (for din's backward sums)
        const int b = b0 + threadIdx.x;
        float mu = 0.f, rs = 0.f;
        if (b < B) ln_stats(L0.in_part + (int64_t)b * (((K + 15) >> 4) * 2), K, lv.eps, mu, rs);
        rt[4][threadIdx.x] = mu;
        rt[5][threadIdx.x] = rs;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < AGX_NOISY_MAX_STREAMS; ++s) {
        if (s < s_lo || s >= s_hi) continue;
        const Layer &L = lv.s[s];
        const int N = L.N;
        const bool oln = L.out_g != nullptr;
        const int64_t drow = (int64_t)(rok ? r : 0) * N;
        const int kc_ = kok ? k : K - 1;
        const bool noisy = L.w_sig != nullptr;
        const float *wsig = noisy ? L.w_sig : L.w_mu, *weps = noisy ? L.w_eps : L.w_mu;
        const float *oh = oln ? L.out : L.dsrc, *og = oln ? L.out_g : L.dsrc, *ob = oln ? L.out_b : L.dsrc;
        // the stream's first n chunk is requested before its row statistics are combined
        float dv[4][4], hv[4][4], gv[4][4], bv[4][4], wm[4][4], ws[4][4], we[4][4];
#define NMLP_LOADX(NC)                                                  \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) {                 \
            _Pragma("unroll") for (int j = 0; j < 4; ++j) {             \
                const int nn = min((NC) + 64 * u + 4 * q + j, N - 1);   \
                dv[u][j] = L.dsrc[drow + nn];                           \
                hv[u][j] = oh[drow + nn];                               \
                gv[u][j] = og[nn];                                      \
                bv[u][j] = ob[nn];                                      \
                const int64_t wi = (int64_t)nn * K + kc_;               \
                wm[u][j] = L.w_mu[wi];                                  \
                ws[u][j] = wsig[wi];                                    \
                we[u][j] = weps[wi];                                    \
            }                                                           \
        }
        NMLP_LOADX(wave * 16)
        float mu = 0.f, rs = 0.f, s1 = 0.f, s2 = 0.f;
        if (oln) {
            __syncthreads();  // rt of the previous stream consumed
            if (threadIdx.x < 16) {
                const int b = b0 + threadIdx.x;
                float m = 0.f, v = 0.f, a1 = 0.f, a2 = 0.f;
                if (b < B) {
                    const int64_t o = (int64_t)b * (((N + 15) >> 4) * 2);
                    ln_stats(L.out_part + o, N, lv.eps, m, v);
                    ln_sums(L.s_part + o, N, a1, a2);
                }
                rt[0][threadIdx.x] = m;
                rt[1][threadIdx.x] = v;
                rt[2][threadIdx.x] = a1;
                rt[3][threadIdx.x] = a2;
            }
            __syncthreads();
            mu = rt[0][lane & 15];
            rs = rt[1][lane & 15];
            s1 = rt[2][lane & 15];
            s2 = rt[3][lane & 15];
        }
        const float invN = 1.f / (float)N;
        for (int nc = wave * 16; nc < N; nc += 256) {  // four 16-deep n blocks in flight, loads unconditional
            float a[4][4], w[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool nok = nc + 64 * u + 4 * q + j < N;
                    float d = dv[u][j];
                    if (oln) d = ln_relu_bwd(hv[u][j], d, gv[u][j], bv[u][j], mu, rs, s1, s2, invN);
                    a[u][j] = (rok && nok) ? d : 0.f;
                    const float wf = noisy ? __fadd_rn(wm[u][j], __fmul_rn(ws[u][j], we[u][j])) : wm[u][j];
                    w[u][j] = (nok && kok) ? wf : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][j], w[u][j], acc, 0, 0, 0);
            if (nc + 256 < N) {
                NMLP_LOADX(nc + 256)
            }
        }
#undef NMLP_LOADX
    }
    if (wave) red[wave - 1][lane] = acc;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) acc += red[w][lane];
        const int Tk = (K + 15) >> 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ri = 4 * q + i, row = b0 + ri;
            if (row < B && kok) L0.din[(int64_t)row * K + k] = acc[i];
            if (dpart) {  // this tile's LayerNorm-backward sums of din (the level below reads them)
                float gx = 0.f, xh = 0.f;
                if (row < B && kok) {
                    xh = ln_xhat(hin[i], rt[4][ri], rt[5][ri]);
                    gx = ln_relu_g(xh, acc[i], gin, bin);
                }
                const float a1 = __shfl(group_sum<16>(gx), lane & ~15, 64);
                const float a2 = __shfl(group_sum<16>(__fmul_rn(gx, xh)), lane & ~15, 64);
                if ((lane & 15) == 0 && row < B) {
                    float *p = L0.din_part + ((int64_t)row * Tk + (k0 >> 4)) * 2;
                    p[0] = a1;
                    p[1] = a2;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void bwd_kernel(Level lv) {
    int blk = blockIdx.x;
#pragma unroll
    for (int s = 0; s < AGX_NOISY_MAX_STREAMS; ++s) {
        if (s < lv.S) {
            if (blk < lv.s[s].tiles_w) {
                bwd_weights(lv, lv.s[s], blk);
                return;
            }
            blk -= lv.s[s].tiles_w;
        }
    }
    if (lv.sum_din) {
        bwd_inputs(lv, lv.s[0], 0, lv.S, blk);
        return;
    }
#pragma unroll
    for (int s = 0; s < AGX_NOISY_MAX_STREAMS; ++s) {
        if (s < lv.S) {
            if (blk < lv.s[s].tiles_x) {
                bwd_inputs(lv, lv.s[s], s, s + 1, blk);
                return;
            }
            blk -= lv.s[s].tiles_x;
        }
    }
}

}  // namespace nmlp

// ---------------------------------------------------------------------------
static int check_layers(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, int64_t B, const char *who) {
    AGX_REQUIRE(layers && S >= 1 && S <= AGX_NOISY_MAX_STREAMS && NL >= 1 && NL <= AGX_NOISY_MAX_LAYERS,
                "%s: need 1..%d streams of 1..%d layers", who, AGX_NOISY_MAX_STREAMS, AGX_NOISY_MAX_LAYERS);
    AGX_REQUIRE(B >= 0 && B <= AGX_NOISY_MAX_ROWS, "%s: batch %lld outside [0, %d]", who, (long long)B,
                AGX_NOISY_MAX_ROWS);
    for (int s = 0; s < S; ++s) {
        for (int l = 0; l < NL; ++l) {
            const agx_noisy_stream_layer &L = layers[s * NL + l];
            AGX_REQUIRE(L.w_mu && L.b_mu && L.out && L.fin > 0 && L.fout > 0, "%s: stream %d layer %d incomplete", who,
                        s, l);
            AGX_REQUIRE((L.w_sigma == nullptr) == (L.w_eps == nullptr) &&
                            (L.b_sigma == nullptr) == (L.b_eps == nullptr) &&
                            (L.w_sigma == nullptr) == (L.b_sigma == nullptr),
                        "%s: stream %d layer %d: sigma and eps come together, for weight and bias", who, s, l);
            const bool hidden = l < NL - 1;
            AGX_REQUIRE(hidden == (L.ln_gamma != nullptr) && hidden == (L.ln_beta != nullptr) &&
                            hidden == (L.ln_part != nullptr),
                        "%s: stream %d layer %d: hidden layers (only) carry the LayerNorm affine and ln_part", who, s,
                        l);
            AGX_REQUIRE(l == 0 ? L.fin == layers[0].fin : L.fin == layers[s * NL + l - 1].fout,
                        "%s: stream %d layer %d: fin %d does not match its input", who, s, l, L.fin);
        }
    }
    return AGX_OK;
}

static nmlp::Layer make_layer(const agx_noisy_stream_layer *layers, int NL, int s, int l, const float *x) {
    const agx_noisy_stream_layer &L = layers[s * NL + l];
    nmlp::Layer d{};
    if (l == 0) {
        d.in = x;
    } else {
        const agx_noisy_stream_layer &P = layers[s * NL + l - 1];
        d.in = P.out;
        d.in_g = P.ln_gamma;
        d.in_b = P.ln_beta;
        d.in_part = P.ln_part;
    }
    d.w_mu = L.w_mu;
    d.w_sig = L.w_sigma;
    d.w_eps = L.w_eps;
    d.b_mu = L.b_mu;
    d.b_sig = L.b_sigma;
    d.b_eps = L.b_eps;
    d.out = L.out;
    d.out_part = L.ln_part;
    d.K = L.fin;
    d.N = L.fout;
    return d;
}

static int64_t part_floats(int64_t B, int32_t n) { return B * ceil_div(n, 16) * 2; }

static int forward_streams(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, const float *const *xs,
                           int64_t B, float ln_eps, void *stream) {
    const int nrb = (int)ceil_div(B, 16);
    for (int l = 0; l < NL; ++l) {
        nmlp::Level lv{};
        lv.S = S;
        lv.B = (int)B;
        lv.eps = ln_eps;
        int grid = 0;
        for (int s = 0; s < S; ++s) {
            lv.s[s] = make_layer(layers, NL, s, l, xs[s]);
            lv.s[s].tiles_w = (int)ceil_div(lv.s[s].N, 16) * nrb;
            grid += lv.s[s].tiles_w;
        }
        nmlp::fwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(lv);
        if (int rc = check_launch("agx_noisy_streams_forward")) return rc;
    }
    return AGX_OK;
}

extern "C" int agx_noisy_streams_forward(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, const float *x,
                                         int64_t B, float ln_eps, void *stream) {
    if (int rc = check_layers(layers, S, NL, B, "agx_noisy_streams_forward")) return rc;
    AGX_REQUIRE(x, "agx_noisy_streams_forward: x is NULL");
    if (B == 0) return AGX_OK;
    const float *xs[AGX_NOISY_MAX_STREAMS];
    for (int s = 0; s < AGX_NOISY_MAX_STREAMS; ++s) xs[s] = x;
    return forward_streams(layers, S, NL, xs, B, ln_eps, stream);
}

extern "C" int agx_noisy_streams_forward_each(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL,
                                              const float *const *xs, int64_t B, float ln_eps, void *stream) {
    if (int rc = check_layers(layers, S, NL, B, "agx_noisy_streams_forward_each")) return rc;
    AGX_REQUIRE(xs, "agx_noisy_streams_forward_each: xs is NULL");
    for (int s = 0; s < S; ++s) AGX_REQUIRE(xs[s], "agx_noisy_streams_forward_each: xs[%d] is NULL", s);
    if (B == 0) return AGX_OK;
    return forward_streams(layers, S, NL, xs, B, ln_eps, stream);
}

extern "C" size_t agx_noisy_streams_workspace_bytes(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL,
                                                    int64_t B) {
    if (!layers || S < 1 || S > AGX_NOISY_MAX_STREAMS || NL < 1 || NL > AGX_NOISY_MAX_LAYERS || B < 0) return 0;
    int64_t n = 0;
    for (int s = 0; s < S; ++s)
        for (int l = 0; l + 1 < NL; ++l) n += B * layers[s * NL + l].fout + part_floats(B, layers[s * NL + l].fout);
    return (size_t)n * sizeof(float);
}

extern "C" int agx_noisy_streams_backward(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, const float *x,
                                          int64_t B, float ln_eps, const float *const *grad_out, float *grad_x,
                                          void *workspace, void *stream) {
    if (int rc = check_layers(layers, S, NL, B, "agx_noisy_streams_backward")) return rc;
    AGX_REQUIRE(x && grad_out, "agx_noisy_streams_backward: x / grad_out is NULL");
    AGX_REQUIRE(NL == 1 || workspace, "agx_noisy_streams_backward: workspace is NULL");
    for (int s = 0; s < S; ++s) {
        AGX_REQUIRE(grad_out[s], "agx_noisy_streams_backward: grad_out[%d] is NULL", s);
        for (int l = 0; l < NL; ++l) {
            const agx_noisy_stream_layer &L = layers[s * NL + l];
            AGX_REQUIRE(L.grad_w_mu && L.grad_b_mu && (L.w_sigma == nullptr || (L.grad_w_sigma && L.grad_b_sigma)) &&
                            (l == NL - 1 || (L.grad_ln_gamma && L.grad_ln_beta)),
                        "agx_noisy_streams_backward: stream %d layer %d: gradient outputs missing", s, l);
        }
    }
    if (B == 0) return AGX_OK;
    // da[s][l]: d loss / d relu(LN(out of layer l)) of stream s, hidden layers l < NL - 1;
    // sp[s][l]: its tiles' LayerNorm-backward sums
    float *da[AGX_NOISY_MAX_STREAMS][AGX_NOISY_MAX_LAYERS] = {};
    float *sp[AGX_NOISY_MAX_STREAMS][AGX_NOISY_MAX_LAYERS] = {};
    float *p = static_cast<float *>(workspace);
    for (int s = 0; s < S; ++s)
        for (int l = 0; l + 1 < NL; ++l) {
            const int32_t f = layers[s * NL + l].fout;
            da[s][l] = p;
            p += B * f;
            sp[s][l] = p;
            p += part_floats(B, f);
        }
    const int nrb = (int)ceil_div(B, 16);
    for (int l = NL - 1; l >= 0; --l) {
        nmlp::Level lv{};
        lv.S = S;
        lv.B = (int)B;
        lv.eps = ln_eps;
        lv.sum_din = l == 0;
        int grid = 0;
        for (int s = 0; s < S; ++s) {
            const agx_noisy_stream_layer &L = layers[s * NL + l];
            nmlp::Layer &d = lv.s[s];
            d = make_layer(layers, NL, s, l, x);
            d.dsrc = l == NL - 1 ? grad_out[s] : da[s][l];
            d.out_g = L.ln_gamma;
            d.out_b = L.ln_beta;
            d.s_part = l == NL - 1 ? nullptr : sp[s][l];
            d.gw_mu = L.grad_w_mu;
            d.gw_sig = L.grad_w_sigma;
            d.gb_mu = L.grad_b_mu;
            d.gb_sig = L.grad_b_sigma;
            d.g_g = L.grad_ln_gamma;
            d.g_b = L.grad_ln_beta;
            d.din = l == 0 ? grad_x : da[s][l - 1];
            d.din_part = l == 0 ? nullptr : sp[s][l - 1];
            d.tiles_w = (int)ceil_div(d.N, 16) * (int)ceil_div(d.K, 64);
            d.tiles_x = d.din ? (int)ceil_div(d.K, 16) * nrb : 0;
            grid += d.tiles_w;
        }
        if (lv.sum_din) {
            grid += lv.s[0].tiles_x;  // one set of role-X tiles sums every stream (same K)
        } else {
            for (int s = 0; s < S; ++s) grid += lv.s[s].tiles_x;
        }
        nmlp::bwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(lv);
        if (int rc = check_launch("agx_noisy_streams_backward")) return rc;
    }
    return AGX_OK;
}

}  // namespace agx
