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
// Row statistics are always computed by one wave over the row in the same
// order (row_stats / row_bwd_sums), and y = xhat * gamma + beta is rounded
// explicitly, so the ReLU mask the backward recomputes is the forward's.
#include <cstdint>

#include "agx_common.h"
#include "../../include/agx_noisy.h"

namespace agx {

namespace nmlp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = AGX_NOISY_MAX_ROWS;

struct Layer {
    const float *in, *in_g, *in_b;  // input [B][K]; in_g: the input is relu(LN(in) * in_g + in_b)
    const float *w_mu, *w_sig, *w_eps, *b_mu, *b_sig, *b_eps;
    float *out;                     // [B][N]
    const float *dsrc;              // backward: d/d out (out_g == null) or d/d relu(LN(out)) [B][N]
    const float *out_g, *out_b;     // LayerNorm affine of this layer's output (hidden layers)
    float *gw_mu, *gw_sig, *gb_mu, *gb_sig, *g_g, *g_b;
    float *din;                     // role X output [B][K] (null: none)
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

// mean and rstd of one row of length K, by one wave (every lane returns lane 0's values)
__device__ __forceinline__ void row_stats(const float *row, int K, float eps, int lane, float &mu, float &rs) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += row[k];
    mu = __shfl(wave_sum(s), 0, 64) / (float)K;
    float v = 0.f;
    for (int k = lane; k < K; k += 64) {
        const float d = __fsub_rn(row[k], mu);
        v = __fmaf_rn(d, d, v);
    }
    v = __shfl(wave_sum(v), 0, 64) / (float)K;
    rs = __frsqrt_rn(__fadd_rn(v, eps));
}

// LayerNorm + ReLU backward of a row: with g = da * [y > 0] * gamma, s1 = sum g, s2 = sum g * xhat
__device__ __forceinline__ void row_bwd_sums(const float *h, const float *da, const float *gam, const float *bet, int N,
                                             float mu, float rs, int lane, float &s1, float &s2) {
    float a1 = 0.f, a2 = 0.f;
    for (int n = lane; n < N; n += 64) {
        const float xh = ln_xhat(h[n], mu, rs);
        const float gx = ln_y(xh, gam[n], bet[n]) > 0.f ? __fmul_rn(da[n], gam[n]) : 0.f;
        a1 += gx;
        a2 = __fmaf_rn(gx, xh, a2);
    }
    s1 = __shfl(wave_sum(a1), 0, 64);
    s2 = __shfl(wave_sum(a2), 0, 64);
}

// d/d out[b][n] of a hidden layer from the gradient of its activation
__device__ __forceinline__ float ln_relu_bwd(float h, float da, float gam, float bet, float mu, float rs, float s1,
                                             float s2, float invN) {
    const float xh = ln_xhat(h, mu, rs);
    const float gx = ln_y(xh, gam, bet) > 0.f ? __fmul_rn(da, gam) : 0.f;
    return rs * ((gx - s1 * invN) - xh * (s2 * invN));
}

__device__ __forceinline__ Layer pick(const Level &lv, int s) { return s == 0 ? lv.s[0] : lv.s[1]; }

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fwd_kernel(Level lv) {
    __shared__ float st_mu[16], st_rs[16];
    __shared__ f32x4 red[3][64];
    int blk = blockIdx.x, si = 0;
    if (blk >= lv.s[0].tiles_w) {
        blk -= lv.s[0].tiles_w;
        si = 1;
    }
    const Layer L = pick(lv, si);
    const int B = lv.B, K = L.K, N = L.N;
    const int nrb = (B + 15) >> 4;
    const int n0 = (blk / nrb) * 16, b0 = (blk % nrb) * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool ln = L.in_g != nullptr;
    if (ln) {
        for (int i = wave * 4; i < wave * 4 + 4; ++i) {
            float mu = 0.f, rs = 0.f;
            if (b0 + i < B) row_stats(L.in + (int64_t)(b0 + i) * K, K, lv.eps, lane, mu, rs);
            if (lane == 0) {
                st_mu[i] = mu;
                st_rs[i] = rs;
            }
        }
        __syncthreads();
    }
    const int r = b0 + (lane & 15), n = n0 + (lane & 15), q = lane >> 4;
    const bool rok = r < B, nok = n < N;
    const float mu = ln ? st_mu[lane & 15] : 0.f, rs = ln ? st_rs[lane & 15] : 0.f;
    const float *xrow = L.in + (int64_t)(rok ? r : 0) * K;
    const int64_t wrow = (int64_t)(nok ? n : 0) * K;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int kb = wave * 16; kb < K; kb += 64) {
        float a[4], w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = kb + 4 * q + j;
            const bool kok = k < K;
            float xv = (rok && kok) ? xrow[k] : 0.f;
            if (ln && rok && kok) xv = fmaxf(ln_y(ln_xhat(xv, mu, rs), L.in_g[k], L.in_b[k]), 0.f);
            a[j] = xv;
            w[j] = (nok && kok) ? wval(L, wrow + k) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], w[j], acc, 0, 0, 0);
    }
    if (wave) red[wave - 1][lane] = acc;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) acc += red[w][lane];
        const int col = n0 + (lane & 15);
        if (col < N) {
            const float bias = bval(L, col);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = b0 + 4 * q + i;
                if (row < B) L.out[(int64_t)row * N + col] = acc[i] + bias;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// role W: 16 output features x 64 input features of one stream's layer
__device__ void bwd_weights(const Level &lv, const Layer &L, int blk) {
    __shared__ float tab[6][kRows];  // out-LN mean, rstd, s1, s2 | in-LN mean, rstd
    const int B = lv.B, K = L.K, N = L.N;
    const int nkt = (K + 63) >> 6;
    const int n0 = (blk / nkt) * 16, kt = blk % nkt;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool oln = L.out_g != nullptr, iln = L.in_g != nullptr;
    if (oln || iln) {
        for (int b = wave; b < B; b += 4) {
            if (oln) {
                float mu, rs, s1, s2;
                row_stats(L.out + (int64_t)b * N, N, lv.eps, lane, mu, rs);
                row_bwd_sums(L.out + (int64_t)b * N, L.dsrc + (int64_t)b * N, L.out_g, L.out_b, N, mu, rs, lane, s1,
                             s2);
                if (lane == 0) {
                    tab[0][b] = mu;
                    tab[1][b] = rs;
                    tab[2][b] = s1;
                    tab[3][b] = s2;
                }
            }
            if (iln) {
                float mu, rs;
                row_stats(L.in + (int64_t)b * K, K, lv.eps, lane, mu, rs);
                if (lane == 0) {
                    tab[4][b] = mu;
                    tab[5][b] = rs;
                }
            }
        }
        __syncthreads();
    }
    const float invN = 1.f / (float)N;
    auto dy = [&](int b, int n) -> float {
        const int64_t i = (int64_t)b * N + n;
        if (!oln) return L.dsrc[i];
        return ln_relu_bwd(L.out[i], L.dsrc[i], L.out_g[n], L.out_b[n], tab[0][b], tab[1][b], tab[2][b], tab[3][b],
                           invN);
    };
    auto act = [&](int b, int k) -> float {
        const float v = L.in[(int64_t)b * K + k];
        return iln ? fmaxf(ln_y(ln_xhat(v, tab[4][b], tab[5][b]), L.in_g[k], L.in_b[k]), 0.f) : v;
    };
    const int q = lane >> 4;
    const int n = n0 + (lane & 15), k = kt * 64 + wave * 16 + (lane & 15);
    const bool nok = n < N, kok = k < K;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int bb = 0; bb < B; bb += 16) {
        float a[4], x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int b = bb + 4 * q + j;
            const bool bok = b < B;
            a[j] = (bok && nok) ? dy(b, n) : 0.f;
            x[j] = (bok && kok) ? act(b, k) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], x[j], acc, 0, 0, 0);
    }
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
        float sb = 0.f, sg = 0.f, sbeta = 0.f;
        if (nok) {
            for (int b = q; b < B; b += 4) {
                sb += dy(b, n);
                if (oln) {
                    const int64_t i = (int64_t)b * N + n;
                    const float xh = ln_xhat(L.out[i], tab[0][b], tab[1][b]);
                    const float g = ln_y(xh, L.out_g[n], L.out_b[n]) > 0.f ? L.dsrc[i] : 0.f;
                    sbeta += g;
                    sg = __fmaf_rn(g, xh, sg);
                }
            }
        }
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
__device__ void bwd_inputs(const Level &lv, int s_lo, int s_hi, int blk) {
    __shared__ float rt[4][16];
    __shared__ f32x4 red[3][64];
    const Layer L0 = pick(lv, s_lo);
    const int B = lv.B, K = L0.K;
    const int nrb = (B + 15) >> 4;
    const int k0 = (blk / nrb) * 16, b0 = (blk % nrb) * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = lane >> 4;
    const int r = b0 + (lane & 15), k = k0 + (lane & 15);
    const bool rok = r < B, kok = k < K;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = s_lo; s < s_hi; ++s) {
        const Layer L = pick(lv, s);
        const int N = L.N;
        const bool oln = L.out_g != nullptr;
        float mu = 0.f, rs = 0.f, s1 = 0.f, s2 = 0.f;
        if (oln) {
            __syncthreads();  // rt of the previous stream consumed
            for (int i = wave * 4; i < wave * 4 + 4; ++i) {
                float m = 0.f, v = 0.f, a1 = 0.f, a2 = 0.f;
                if (b0 + i < B) {
                    const int64_t o = (int64_t)(b0 + i) * N;
                    row_stats(L.out + o, N, lv.eps, lane, m, v);
                    row_bwd_sums(L.out + o, L.dsrc + o, L.out_g, L.out_b, N, m, v, lane, a1, a2);
                }
                if (lane == 0) {
                    rt[0][i] = m;
                    rt[1][i] = v;
                    rt[2][i] = a1;
                    rt[3][i] = a2;
                }
            }
            __syncthreads();
            mu = rt[0][lane & 15];
            rs = rt[1][lane & 15];
            s1 = rt[2][lane & 15];
            s2 = rt[3][lane & 15];
        }
        const float invN = 1.f / (float)N;
        const int64_t drow = (int64_t)(rok ? r : 0) * N;
        for (int nb = wave * 16; nb < N; nb += 64) {
            float a[4], w[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = nb + 4 * q + j;
                const bool nok = n < N;
                float d = (rok && nok) ? L.dsrc[drow + n] : 0.f;
                if (oln && rok && nok) d = ln_relu_bwd(L.out[drow + n], d, L.out_g[n], L.out_b[n], mu, rs, s1, s2, invN);
                a[j] = d;
                w[j] = (nok && kok) ? wval(L, (int64_t)n * K + k) : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], w[j], acc, 0, 0, 0);
        }
    }
    if (wave) red[wave - 1][lane] = acc;
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) acc += red[w][lane];
        if (kok) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = b0 + 4 * q + i;
                if (row < B) L0.din[(int64_t)row * K + k] = acc[i];
            }
        }
    }
}

__global__ __launch_bounds__(256) void bwd_kernel(Level lv) {
    int blk = blockIdx.x;
    for (int s = 0; s < lv.S; ++s) {
        const int t = s == 0 ? lv.s[0].tiles_w : lv.s[1].tiles_w;
        if (blk < t) {
            bwd_weights(lv, pick(lv, s), blk);
            return;
        }
        blk -= t;
    }
    if (lv.sum_din) {
        bwd_inputs(lv, 0, lv.S, blk);
        return;
    }
    for (int s = 0; s < lv.S; ++s) {
        const int t = s == 0 ? lv.s[0].tiles_x : lv.s[1].tiles_x;
        if (blk < t) {
            bwd_inputs(lv, s, s + 1, blk);
            return;
        }
        blk -= t;
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
            AGX_REQUIRE(hidden == (L.ln_gamma != nullptr) && hidden == (L.ln_beta != nullptr),
                        "%s: stream %d layer %d: hidden layers (only) carry the LayerNorm affine", who, s, l);
            AGX_REQUIRE(l == 0 ? L.fin == layers[l].fin : L.fin == layers[s * NL + l - 1].fout,
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
    }
    d.w_mu = L.w_mu;
    d.w_sig = L.w_sigma;
    d.w_eps = L.w_eps;
    d.b_mu = L.b_mu;
    d.b_sig = L.b_sigma;
    d.b_eps = L.b_eps;
    d.out = L.out;
    d.K = L.fin;
    d.N = L.fout;
    return d;
}

extern "C" int agx_noisy_streams_forward(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, const float *x,
                                         int64_t B, float ln_eps, void *stream) {
    if (int rc = check_layers(layers, S, NL, B, "agx_noisy_streams_forward")) return rc;
    AGX_REQUIRE(x, "agx_noisy_streams_forward: x is NULL");
    if (B == 0) return AGX_OK;
    const int nrb = (int)ceil_div(B, 16);
    for (int l = 0; l < NL; ++l) {
        nmlp::Level lv{};
        lv.S = S;
        lv.B = (int)B;
        lv.eps = ln_eps;
        int grid = 0;
        for (int s = 0; s < S; ++s) {
            lv.s[s] = make_layer(layers, NL, s, l, x);
            lv.s[s].tiles_w = (int)ceil_div(lv.s[s].N, 16) * nrb;
            grid += lv.s[s].tiles_w;
        }
        nmlp::fwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(lv);
        if (int rc = check_launch("agx_noisy_streams_forward")) return rc;
    }
    return AGX_OK;
}

extern "C" size_t agx_noisy_streams_workspace_bytes(const agx_noisy_stream_layer *layers, int32_t S, int32_t NL, int64_t B) {
    if (!layers || S < 1 || S > AGX_NOISY_MAX_STREAMS || NL < 1 || NL > AGX_NOISY_MAX_LAYERS || B < 0) return 0;
    size_t n = 0;
    for (int s = 0; s < S; ++s)
        for (int l = 0; l + 1 < NL; ++l) n += (size_t)B * (size_t)layers[s * NL + l].fout;
    return n * sizeof(float);
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
    // da[s][l]: d loss / d relu(LN(out of layer l)) of stream s, hidden layers l < NL - 1
    float *da[AGX_NOISY_MAX_STREAMS][AGX_NOISY_MAX_LAYERS] = {};
    float *p = static_cast<float *>(workspace);
    for (int s = 0; s < S; ++s)
        for (int l = 0; l + 1 < NL; ++l) {
            da[s][l] = p;
            p += B * layers[s * NL + l].fout;
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
            d.gw_mu = L.grad_w_mu;
            d.gw_sig = L.grad_w_sigma;
            d.gb_mu = L.grad_b_mu;
            d.gb_sig = L.grad_b_sigma;
            d.g_g = L.grad_ln_gamma;
            d.g_b = L.grad_ln_beta;
            d.din = l == 0 ? grad_x : da[s][l - 1];
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
