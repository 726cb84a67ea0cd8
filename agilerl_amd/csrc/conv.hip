// Convolution layers of EvolvableCNN (agilerl/modules/cnn.py:224-552,
// create_cnn utils/evolvable_networks.py:460-525: Conv2d -> activation per
// layer; the Atari encoders of configs 3 and 5 are 8x8/4, 4x4/2, 3x3/1 over
// 4x84x84 uint8 frames) as implicit GEMMs on the f32 matrix cores.
//
//   forward  Y[b,co,oh,ow] = act(bias[co] + sum_{ci,kh,kw} W[co,ci,kh,kw] X[b,ci,oh*s+kh,ow*s+kw])
//            GEMM  M = Cout, N = B*OH*OW, K = Cin*KH*KW; the first layer reads the
//            uint8 frames straight from the replay / rollout storage and applies the
//            reference's image normalisation on load ((x - low) / (high - low),
//            algo_utils.py:1134-1183): 4x fewer bytes than a separate f32 copy.
//   wgrad    dW[co,(ci,kh,kw)] = sum_p dZ[co,p] Xcol[(ci,kh,kw),p], dZ = dY * act'(Y);
//            M = Cout, N = Cin*KH*KW + 1 (the extra ones-column gives db), K = B*OH*OW,
//            split over workgroups (partials in a workspace, summed in a fixed order).
//   dgrad    dX[b,ci,ih,iw] = sum_{co,kh,kw} W[co,ci,kh,kw] dZ[b,co,(ih-kh)/s,(iw-kw)/s]
//            over the taps that land on the output grid; M = Cin, N = B*H*W, K = Cout*KH*KW.
//
// One kernel template serves the three: a 64x64 output tile per 256-thread
// workgroup (4 waves, each 32x32 = 2x2 v_mfma_f32_16x16x4_f32 tiles), K in
// steps of 16 staged through LDS (rows padded to 80 floats: the two 32-lane
// halves of a ds_read_b32 land in disjoint banks), the next step's operands
// gathered into registers while the current one multiplies.  The operand
// gathers and the epilogue are the only per-mode code (functors below).
#include "agx_common.h"

namespace agx {

namespace conv {

constexpr int BM = 64, BN = 64, BK = 16, NT = 256, LDP = 80;
typedef float f4 __attribute__((ext_vector_type(4)));

struct Shape {
    int B, Cin, H, W, Cout, KH, KW, S, OH, OW;
};

// ---- forward -------------------------------------------------------------
template <bool U8>
struct FwdOps {
    const float *w;      // [Cout][Cin*KH*KW]
    const void *x;       // [B][Cin][H][W], f32 or u8
    const float *bias;   // [Cout] or null
    float *y;            // [B][Cout][OH][OW]
    float lo, rng;  // u8 normalisation: (x - lo) / rng
    int relu;
    Shape s;
    int M, N, K;
    __device__ float a(int m, int k) const { return (m < M && k < K) ? w[(size_t)m * K + k] : 0.f; }
    __device__ float b(int k, int n) const {
        if (k >= K || n >= N) return 0.f;
        const int kw = k % s.KW, t = k / s.KW, kh = t % s.KH, ci = t / s.KH;
        const int ow = n % s.OW, t2 = n / s.OW, oh = t2 % s.OH, bb = t2 / s.OH;
        const size_t o = (((size_t)bb * s.Cin + ci) * s.H + (oh * s.S + kh)) * s.W + (ow * s.S + kw);
        if constexpr (U8) {
            const float v = (float)static_cast<const unsigned char *>(x)[o];
            return (v - lo) / rng;  // IEEE division, as the reference's tensor op
        } else {
            return static_cast<const float *>(x)[o];
        }
    }
    __device__ void store(int m, int n, float v, int) const {
        if (m >= M || n >= N) return;
        if (bias) v += bias[m];
        if (relu) v = v > 0.f ? v : 0.f;
        const int ow = n % s.OW, t2 = n / s.OW, oh = t2 % s.OH, bb = t2 / s.OH;
        y[(((size_t)bb * s.Cout + m) * s.OH + oh) * s.OW + ow] = v;
    }
};

// ---- weight gradient (split over the p = (b, oh, ow) reduction) ----------
template <bool U8>
struct WgradOps {
    const float *dy;     // [B][Cout][OH][OW] gradient of the layer output
    const float *yact;   // post-activation output (ReLU mask), or null
    const void *x;       // layer input
    float lo, rng;
    float *part;         // [splits][Cout][K+1]
    Shape s;
    int M, N, K;         // M = Cout, N = Cin*KH*KW + 1, K = B*OH*OW (split over blockIdx.z)
    __device__ float a(int m, int p) const {
        if (m >= M || p >= K) return 0.f;
        const int ow = p % s.OW, t = p / s.OW, oh = t % s.OH, bb = t / s.OH;
        const size_t o = (((size_t)bb * s.Cout + m) * s.OH + oh) * s.OW + ow;
        const float g = dy[o];
        return (yact && !(yact[o] > 0.f)) ? 0.f : g;
    }
    __device__ float b(int p, int n) const {
        if (p >= K || n >= N) return 0.f;
        if (n == N - 1) return 1.f;  // ones column -> bias gradient
        const int kw = n % s.KW, t = n / s.KW, kh = t % s.KH, ci = t / s.KH;
        const int ow = p % s.OW, t2 = p / s.OW, oh = t2 % s.OH, bb = t2 / s.OH;
        const size_t o = (((size_t)bb * s.Cin + ci) * s.H + (oh * s.S + kh)) * s.W + (ow * s.S + kw);
        if constexpr (U8) return ((float)static_cast<const unsigned char *>(x)[o] - lo) / rng;
        else return static_cast<const float *>(x)[o];
    }
    __device__ void store(int m, int n, float v, int z) const {
        if (m < M && n < N) part[((size_t)z * M + m) * N + n] = v;
    }
};

// ---- data gradient -------------------------------------------------------
struct DgradOps {
    const float *w;      // [Cout][Cin][KH][KW]
    const float *dy, *yact;
    float *dx;           // [B][Cin][H][W]
    Shape s;
    int M, N, K;         // M = Cin, N = B*H*W, K = Cout*KH*KW
    __device__ float a(int ci, int k) const {
        if (ci >= M || k >= K) return 0.f;
        const int kw = k % s.KW, t = k / s.KW, kh = t % s.KH, co = t / s.KH;
        return w[(((size_t)co * s.Cin + ci) * s.KH + kh) * s.KW + kw];
    }
    __device__ float b(int k, int n) const {
        if (k >= K || n >= N) return 0.f;
        const int kw = k % s.KW, t = k / s.KW, kh = t % s.KH, co = t / s.KH;
        const int iw = n % s.W, t2 = n / s.W, ih = t2 % s.H, bb = t2 / s.H;
        const int ph = ih - kh, pw = iw - kw;
        if (ph < 0 || pw < 0 || ph % s.S || pw % s.S) return 0.f;
        const int oh = ph / s.S, ow = pw / s.S;
        if (oh >= s.OH || ow >= s.OW) return 0.f;
        const size_t o = (((size_t)bb * s.Cout + co) * s.OH + oh) * s.OW + ow;
        const float g = dy[o];
        return (yact && !(yact[o] > 0.f)) ? 0.f : g;
    }
    __device__ void store(int ci, int n, float v, int) const {
        if (ci >= M || n >= N) return;
        const int iw = n % s.W, t2 = n / s.W, ih = t2 % s.H, bb = t2 / s.H;
        dx[(((size_t)bb * s.Cin + ci) * s.H + ih) * s.W + iw] = v;
    }
};

// K range [k0, k1); chunk > 0 splits it over blockIdx.z (split-K, partial tiles per z)
template <class Ops>
__global__ __launch_bounds__(NT) void igemm_kernel(Ops ops, int k0, int k1, int chunk) {
    if (chunk > 0) {
        k0 += (int)blockIdx.z * chunk;
        k1 = k0 + chunk < k1 ? k0 + chunk : k1;
    }
    if (k0 >= k1) k1 = k0;  // empty split: stores zeros
    __shared__ float As[2][BK][LDP];  // As[k][m]
    __shared__ float Bs[2][BK][LDP];  // Bs[k][n]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m_blk = blockIdx.y * BM, n_blk = blockIdx.x * BN;
    // staging: thread t gathers A(m = t / 4 ... ) and B for one K-step: 4 values each
    float ra[4], rb[4];
    auto gather = [&](int kb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + i * NT;       // 0 .. 1023
            const int am = e / BK, ak = e % BK;  // A: 64 rows x 16 k
            ra[i] = kb + ak < k1 ? ops.a(m_blk + am, kb + ak) : 0.f;  // never past this split's K range
            const int bk = e / BN, bn = e % BN;  // B: 16 k x 64 cols (consecutive n: coalesced)
            rb[i] = kb + bk < k1 ? ops.b(kb + bk, n_blk + bn) : 0.f;
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + i * NT;
            As[buf][e % BK][e / BK] = ra[i];
            Bs[buf][e / BN][e % BN] = rb[i];
        }
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;  // this wave's 32x32 sub-tile
    const int r = lane & 15, q = lane >> 4;
    int buf = 0;
    if (k0 < k1) {
        gather(k0);
        stash(0);
    }
    __syncthreads();
    for (int kb = k0; kb < k1; kb += BK) {
        const bool more = kb + BK < k1;
        if (more) gather(kb + BK);  // next step's operands in flight during the MFMAs
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const float a0 = As[buf][kk + q][wm + r], a1 = As[buf][kk + q][wm + 16 + r];
            const float b0 = Bs[buf][kk + q][wn + r], b1 = Bs[buf][kk + q][wn + 16 + r];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) {
            stash(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    }
    // C layout: lane holds rows 4q + i, column r of each 16x16 tile
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                ops.store(m_blk + wm + 16 * i + 4 * q + e, n_blk + wn + 16 * j + r, acc[i][j][e], (int)blockIdx.z);
}

// fixed-order sum of the wgrad split partials: dW (+)= sum_z part[z], db (+)= last column
__global__ void wgrad_reduce_kernel(const float *__restrict__ part, int splits, int M, int N, float *__restrict__ dw,
                                    float *__restrict__ db, int accumulate) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += part[(size_t)z * M * N + i];
    const int m = i / N, n = i % N;
    if (n < N - 1) {
        float *d = dw + (size_t)m * (N - 1) + n;
        *d = accumulate ? *d + v : v;
    } else if (db) {
        db[m] = accumulate ? db[m] + v : v;
    }
}

}  // namespace conv

}  // namespace agx

using namespace agx;
using namespace agx::conv;

static int check_shape(const agx_conv2d_shape *sh, Shape &s, const char *who) {
    AGX_REQUIRE(sh, "%s: null shape", who);
    s.B = (int)sh->batch;
    s.Cin = sh->in_channels;
    s.H = sh->height;
    s.W = sh->width;
    s.Cout = sh->out_channels;
    s.KH = sh->kernel_h;
    s.KW = sh->kernel_w;
    s.S = sh->stride;
    AGX_REQUIRE(s.B > 0 && s.Cin > 0 && s.H > 0 && s.W > 0 && s.Cout > 0 && s.KH > 0 && s.KW > 0 && s.S > 0 &&
                    s.KH <= s.H && s.KW <= s.W,
                "%s: bad shape", who);
    s.OH = (s.H - s.KH) / s.S + 1;
    s.OW = (s.W - s.KW) / s.S + 1;
    AGX_REQUIRE((int64_t)s.B * s.Cout * s.OH * s.OW < (1ll << 31) && (int64_t)s.B * s.Cin * s.H * s.W < (1ll << 31),
                "%s: tensor too large for 32-bit indexing", who);
    return AGX_OK;
}

extern "C" int agx_conv2d_forward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low,
                                  float x_high, const float *w, const float *bias, int relu, float *y, void *stream) {
    Shape s;
    if (int rc = check_shape(shape, s, "agx_conv2d_forward")) return rc;
    AGX_REQUIRE(x && w && y, "agx_conv2d_forward: null pointer");
    AGX_REQUIRE(!x_is_u8 || x_high > x_low, "agx_conv2d_forward: u8 input needs high > low");
    const int M = s.Cout, N = s.B * s.OH * s.OW, K = s.Cin * s.KH * s.KW;
    dim3 grid((unsigned)ceil_div(N, BN), (unsigned)ceil_div(M, BM));
    hipStream_t st = as_stream(stream);
    if (x_is_u8) {
        FwdOps<true> o{w, x, bias, y, x_low, x_high - x_low, relu, s, M, N, K};
        igemm_kernel<<<grid, NT, 0, st>>>(o, 0, K, 0);
    } else {
        FwdOps<false> o{w, x, bias, y, 0.f, 1.f, relu, s, M, N, K};
        igemm_kernel<<<grid, NT, 0, st>>>(o, 0, K, 0);
    }
    return check_launch("agx_conv2d_forward");
}

extern "C" size_t agx_conv2d_wgrad_workspace_bytes(const agx_conv2d_shape *shape) {
    Shape s;
    if (check_shape(shape, s, "agx_conv2d_wgrad_workspace_bytes")) return 0;
    const int64_t P = (int64_t)s.B * s.OH * s.OW;
    const int64_t splits = P / 4096 + 1;
    return (size_t)(splits < 128 ? splits : 128) * s.Cout * (s.Cin * s.KH * s.KW + 1) * sizeof(float);
}

extern "C" int agx_conv2d_backward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low,
                                   float x_high, const float *w, const float *y_act, const float *dy, float *dx,
                                   float *dw, float *db, int accumulate, void *workspace, void *stream) {
    Shape s;
    if (int rc = check_shape(shape, s, "agx_conv2d_backward")) return rc;
    AGX_REQUIRE(x && w && dy && dw && workspace, "agx_conv2d_backward: null pointer");
    hipStream_t st = as_stream(stream);
    const int K = s.Cin * s.KH * s.KW;
    const int P = s.B * s.OH * s.OW;
    int splits = P / 4096 + 1;
    if (splits > 128) splits = 128;
    const int chunk = (int)(ceil_div(ceil_div(P, splits), BK) * BK);
    float *part = static_cast<float *>(workspace);
    const int M = s.Cout, N = K + 1;
    dim3 grid((unsigned)ceil_div(N, BN), (unsigned)ceil_div(M, BM), (unsigned)splits);
    if (x_is_u8) {
        WgradOps<true> o{dy, y_act, x, x_low, x_high - x_low, part, s, M, N, P};
        igemm_kernel<<<grid, NT, 0, st>>>(o, 0, P, chunk);
    } else {
        WgradOps<false> o{dy, y_act, x, 0.f, 1.f, part, s, M, N, P};
        igemm_kernel<<<grid, NT, 0, st>>>(o, 0, P, chunk);
    }
    wgrad_reduce_kernel<<<(unsigned)ceil_div(M * N, 256), 256, 0, st>>>(part, splits, M, N, dw, db, accumulate);
    if (int rc = check_launch("agx_conv2d_backward wgrad")) return rc;
    if (dx) {
        AGX_REQUIRE(!x_is_u8, "agx_conv2d_backward: no data gradient for a u8 input layer");
        DgradOps o{w, dy, y_act, dx, s, s.Cin, s.B * s.H * s.W, s.Cout * s.KH * s.KW};
        dim3 g2((unsigned)ceil_div(o.N, BN), (unsigned)ceil_div(o.M, BM));
        igemm_kernel<<<g2, NT, 0, st>>>(o, 0, o.K, 0);
        if (int rc = check_launch("agx_conv2d_backward dgrad")) return rc;
    }
    return AGX_OK;
}
