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
//            split over enough workgroups to fill the chip (>= ~1024 tiles x splits;
//            partials in a workspace, summed in a fixed order).
//   dgrad    dX[b,ci,ih,iw] = sum_{co,kh,kw} W[co,ci,kh,kw] dZ[b,co,(ih-kh)/s,(iw-kw)/s]
//            over the taps that land on the output grid; M = Cin, N = B*H*W, K = Cout*KH*KW.
//
// One kernel template serves the three: a BM x BN output tile per 256-thread
// workgroup (4 waves, each 32x32 = 2x2 v_mfma_f32_16x16x4_f32 tiles; 64x64, or
// 32x128 when M <= 32 so a 32-channel layer wastes no MFMA rows), K in steps of
// 16 staged through LDS (rows padded by 16 floats), the next step's operands
// gathered into registers while the current one multiplies.
//
// Gathers are table driven: im2col index arithmetic (the div / mod chains
// that turn a GEMM index into a tensor offset) is done ONCE per workgroup into
// LDS tables over the K range it walks (in chunks of kTab entries), and once
// per thread for its fixed output column — every thread of a 256-thread tile
// keeps the same GEMM column for the whole K loop (bn = tid % BN).  A gathered
// element then costs one LDS table read and one global load; with the old
// per-element decode the kernels were VALU-bound several times over the MFMA
// time.
#include "agx_common.h"

namespace agx {

namespace conv {

#ifndef AGX_CONV_BK
#define AGX_CONV_BK 16
#endif
constexpr int BK = AGX_CONV_BK, NT = 256, kTab = 1024, kTapMax = 16;
typedef float f4 __attribute__((ext_vector_type(4)));

struct Shape {
    int B, Cin, H, W, Cout, KH, KW, S, OH, OW;
};

// per-workgroup LDS: operand double buffers + gather tables
template <int BM, int BN, bool COLS, bool LUT, int TAB>
struct Smem {
    static constexpr int LDA = BM + 16, LDB = BN + 16;
    float As[2][BK][LDA];  // As[k][m]
    float Bs[2][BK][LDB];  // Bs[k][n]
    int tabA[TAB], tabB[TAB];
    float lut[LUT ? 256 : 1];  // u8 inputs: the normalised value of each byte, (b - low) / (high - low)
    // dgrad: per output column, oh of tap kh / ow of tap kw (-1: no tap), int16;
    // rows padded to an odd word count: lanes read 64 different columns' entry a,
    // and an even row stride put them in few LDS banks (forward / wgrad
    // workgroups do not allocate it)
    short col[COLS ? BN : 1][2 * kTapMax + 2];
};

// u8 layers: the per-element IEEE division (a dozen VALU ops in every gather)
// becomes a read of the workgroup's 256-entry table of the same quotients
template <bool U8, class SM>
__device__ __forceinline__ float ld_xt(const void *x, int o, const SM &sm) {
    if constexpr (U8) return sm.lut[static_cast<const unsigned char *>(x)[o]];
    else return static_cast<const float *>(x)[o];
}
template <bool U8, class SM>
__device__ __forceinline__ void fill_lut(SM &sm, int tid, float lo, float rng) {
    // visible to the gathers after the barrier that opens the first K chunk
    if constexpr (U8)
        if (tid < 256) sm.lut[tid] = ((float)tid - lo) / rng;
}

// ---- forward -------------------------------------------------------------
template <bool U8>
struct FwdOps {
    const float *w;      // [Cout][Cin*KH*KW]
    const void *x;       // [B][Cin][H][W], f32 or u8
    const float *bias;   // [Cout] or null
    float *y;            // [B][Cout][OH][OW]
    float lo, rng;       // u8 normalisation: (x - lo) / rng
    int relu;
    Shape s;
    int M, N, K;
    long long gx, gw, gb, gy;  // per-group element strides (population-batched launch)
    // two-level group index (agx_conv2d_forward_grouped2): g = g1 + G1 * g2,
    // the g2 strides below; G1 <= 0: one level (g1 = g)
    long long gx2, gw2, gb2, gy2;
    int G1;
    __device__ FwdOps at(int g) const {
        const long long g1 = G1 > 0 ? g % G1 : g, g2 = G1 > 0 ? g / G1 : 0;
        FwdOps o = *this;
        o.x = static_cast<const char *>(x) + (g1 * gx + g2 * gx2) * (U8 ? 1 : 4);
        o.w = w + (g1 * gw + g2 * gw2);
        o.bias = bias ? bias + (g1 * gb + g2 * gb2) : nullptr;
        o.y = y + (g1 * gy + g2 * gy2);
        return o;
    }
    __device__ int kend(int k1) const { return k1; }
    static constexpr bool kRowSum = false, kCols = false, kLut = U8;
    static constexpr int kTabN = kTab;
    struct Ctx {
        int xbase;  // input offset of this thread's output pixel, -1 past N
    };
    template <class SM>
    __device__ void setup(Ctx &c, SM &sm, int, int n, int tid) const {
        fill_lut<U8>(sm, tid, lo, rng);
        if (n < N) {
            const int ow = n % s.OW, t = n / s.OW, oh = t % s.OH, bb = t / s.OH;
            c.xbase = ((bb * s.Cin) * s.H + oh * s.S) * s.W + ow * s.S;
        } else {
            c.xbase = -1;
        }
    }
    template <class SM>
    __device__ void build(SM &sm, int kc, int kce, int tid) const {  // tabB[k - kc] = im2col offset of k
        for (int k = kc + tid; k < kce; k += NT) {
            const int kw = k % s.KW, t = k / s.KW, kh = t % s.KH, ci = t / s.KH;
            sm.tabB[k - kc] = (ci * s.H + kh) * s.W + kw;
        }
    }
    template <int NA, int NB, int BN, class SM>
    __device__ void gather(const Ctx &c, const SM &sm, int m_blk, int kc, int kb, int k1, int tid, float *ra,
                           float *rb) const {
        const int k = kb + tid % BK;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int m = m_blk + tid / BK + i * (NT / BK);
            ra[i] = (m < M && k < k1) ? w[(size_t)m * K + k] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int kk = kb + tid / BN + i * (NT / BN);
            rb[i] = (c.xbase >= 0 && kk < k1) ? ld_xt<U8>(x, c.xbase + sm.tabB[kk - kc], sm) : 0.f;
        }
    }
    // the epilogue reads a lane's eight row biases up front (unconditional,
    // clamped), not one dependent load per stored element
    static constexpr bool kBias = true;
    __device__ float row_bias(int m) const { return bias ? bias[m < M ? m : M - 1] : 0.f; }
    __device__ void store(int m, int n, float v, int, float b) const {
        if (m >= M || n >= N) return;
        if (bias) v += b;
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
    float *part;         // [groups][splits][Cout][K+1]
    Shape s;
    int M, N, K;         // M = Cout, N = Cin*KH*KW + 1, K = B*OH*OW (split over blockIdx.z)
    long long gx, gy, gp;
    __device__ WgradOps at(int g) const {
        WgradOps o = *this;
        o.x = static_cast<const char *>(x) + (size_t)g * gx * (U8 ? 1 : 4);
        o.dy = dy + (size_t)g * gy;
        o.yact = yact ? yact + (size_t)g * gy : nullptr;
        o.part = part + (size_t)g * gp;
        return o;
    }
    __device__ int kend(int k1) const { return k1; }
    // db (column N - 1) is the row sum of the A operand (dZ), taken from LDS by
    // the n_blk == 0 tiles: a GEMM ones column would cost a whole extra column
    // tile (re-gathering all of A) when Cin*KH*KW is a multiple of the tile width
    static constexpr bool kRowSum = true, kCols = false, kLut = U8, kBias = false;
    __device__ float row_bias(int) const { return 0.f; }
    static constexpr int kTabN = kTab;
    struct Ctx {
        int koff;  // im2col offset of this thread's weight column, -1 past the weights
    };
    template <class SM>
    __device__ void setup(Ctx &c, SM &sm, int, int n, int tid) const {
        fill_lut<U8>(sm, tid, lo, rng);
        if (n < N - 1) {
            const int kw = n % s.KW, t = n / s.KW, kh = t % s.KH, ci = t / s.KH;
            c.koff = (ci * s.H + kh) * s.W + kw;
        } else {
            c.koff = -1;
        }
    }
    template <class SM>
    __device__ void build(SM &sm, int kc, int kce, int tid) const {
        const int ohw = s.OH * s.OW;
        for (int p = kc + tid; p < kce; p += NT) {
            const int r = p % ohw, bb = p / ohw, ow = r % s.OW, oh = r / s.OW;
            sm.tabA[p - kc] = bb * s.Cout * ohw + r;                            // dy offset, channel 0
            sm.tabB[p - kc] = ((bb * s.Cin) * s.H + oh * s.S) * s.W + ow * s.S;  // x offset, column 0
        }
    }
    template <int NA, int NB, int BN, class SM>
    __device__ void gather(const Ctx &c, const SM &sm, int m_blk, int kc, int kb, int k1, int tid, float *ra,
                           float *rb) const {
        const int ohw = s.OH * s.OW;
        const int p = kb + tid % BK;
        const int dbase = p < k1 ? sm.tabA[p - kc] : 0;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int m = m_blk + tid / BK + i * (NT / BK);
            float g = 0.f;
            if (m < M && p < k1) {
                const int o = dbase + m * ohw;
                g = dy[o];
                if (yact && !(yact[o] > 0.f)) g = 0.f;
            }
            ra[i] = g;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int pp = kb + tid / BN + i * (NT / BN);
            float v = 0.f;
            if (pp < k1 && c.koff >= 0) v = ld_xt<U8>(x, sm.tabB[pp - kc] + c.koff, sm);
            rb[i] = v;
        }
    }
    __device__ void store(int m, int n, float v, int z) const {
        if (m < M && n < N) part[((size_t)z * M + m) * N + n] = v;
    }
};

// ---- data gradient -------------------------------------------------------
// Sub-pixel form for stride s > 1: input pixels of one phase (ih mod s, iw mod s)
// = (ph, pw) are reached only by the taps kh = ph + s*a, kw = pw + s*b, at
// output (ih' - a, iw' - b) where ih = ih'*s + ph.  One GEMM per phase over just
// those taps (K / s^2 of the full tap set: no MFMA work on structural zeros).
// All s^2 phases of all groups go out in ONE launch (blockIdx.z = (group * s^2
// + phase) * splits + split): per-phase launches gave a few hundred workgroups
// each, under two per CU, and the gathers' latency went unhidden.  A GEMM too
// short in N to fill the chip splits K (partials summed in a fixed order by
// dgrad_reduce_kernel; the split count depends on the layer shape only, so a
// group's result does not depend on how many groups share the launch).
struct DgradOps {
    const float *w;      // [Cout][Cin][KH][KW]
    const float *dy, *yact;
    float *dx;           // [B][Cin][H][W]
    float *part;         // split-K partials [group*nph + phase][split][M][Nmax], or null (one split)
    Shape s;
    int M, N, K;         // M = Cin, N = B*Hp*Wp (this phase's pixels), K = Cout*nA*nB (its taps)
    int ph, pw, Hp, Wp, nA, nB;
    int nph, Nmax, splits;
    long long gw, gy, gx;
    __device__ DgradOps at(int gi) const {
        DgradOps o = *this;
        const int g = gi / nph, phase = gi % nph;
        o.ph = phase / s.S;
        o.pw = phase % s.S;
        o.Hp = (s.H - o.ph + s.S - 1) / s.S;
        o.Wp = (s.W - o.pw + s.S - 1) / s.S;
        o.nA = s.KH > o.ph ? (s.KH - o.ph + s.S - 1) / s.S : 0;
        o.nB = s.KW > o.pw ? (s.KW - o.pw + s.S - 1) / s.S : 0;
        o.N = s.B * o.Hp * o.Wp;
        o.K = s.Cout * o.nA * o.nB;
        o.w = w + (size_t)g * gw;
        o.dy = dy + (size_t)g * gy;
        o.yact = yact ? yact + (size_t)g * gy : nullptr;
        o.dx = dx + (size_t)g * gx;
        o.part = part ? part + (size_t)gi * splits * M * Nmax : nullptr;
        return o;
    }
    __device__ int kend(int) const { return K; }  // this phase's taps (0: zeros)
    static constexpr bool kRowSum = false, kCols = true, kLut = false, kBias = false;
    __device__ float row_bias(int) const { return 0.f; }
    static constexpr int kTabN = kTab / 2;  // with the tap table: 4 (32x128) / 5 (64x64) workgroups per CU
    struct Ctx {
        int dbase;  // dy offset of this thread's image (channel 0), -1 past N
        int c;      // column within the tile
    };
    template <class SM>
    __device__ void setup(Ctx &c, SM &sm, int n_local, int n, int tid) const {
        c.c = n_local;
        int ihp = 0, iwp = 0;
        c.dbase = -1;
        if (n < N) {
            iwp = n % Wp;
            const int t = n / Wp;
            ihp = t % Hp;
            c.dbase = (t / Hp) * s.Cout * s.OH * s.OW;
        }
        if (tid == n_local) {  // one thread per column fills its tap table
            for (int a = 0; a < nA; ++a) {
                const int oh = ihp - a;
                sm.col[n_local][a] = (oh >= 0 && oh < s.OH) ? oh : -1;
            }
            for (int b = 0; b < nB; ++b) {
                const int ow = iwp - b;
                sm.col[n_local][kTapMax + b] = (ow >= 0 && ow < s.OW) ? ow : -1;
            }
        }
    }
    template <class SM>
    __device__ void build(SM &sm, int kc, int kce, int tid) const {
        const int khw = s.KH * s.KW, nab = nA * nB;
        for (int k = kc + tid; k < kce; k += NT) {
            const int r = k % nab, co = k / nab, a = r / nB, b = r % nB;
            sm.tabA[k - kc] = co * s.Cin * khw + (ph + s.S * a) * s.KW + pw + s.S * b;  // weight offset, channel 0
            sm.tabB[k - kc] = co | (a << 16) | (b << 24);
        }
    }
    template <int NA, int NB, int BN, class SM>
    __device__ void gather(const Ctx &c, const SM &sm, int m_blk, int kc, int kb, int k1, int tid, float *ra,
                           float *rb) const {
        const int khw = s.KH * s.KW, ohw = s.OH * s.OW;
        const int k = kb + tid % BK;
        const int wb = k < k1 ? sm.tabA[k - kc] : 0;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int ci = m_blk + tid / BK + i * (NT / BK);
            ra[i] = (ci < M && k < k1) ? w[wb + ci * khw] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int kk = kb + tid / BN + i * (NT / BN);
            float g = 0.f;
            if (kk < k1 && c.dbase >= 0) {
                const int pk = sm.tabB[kk - kc];
                const int oh = sm.col[c.c][(pk >> 16) & 255], ow = sm.col[c.c][kTapMax + (pk >> 24)];
                if (oh >= 0 && ow >= 0) {
                    const int o = c.dbase + (pk & 0xffff) * ohw + oh * s.OW + ow;
                    g = dy[o];
                    if (yact && !(yact[o] > 0.f)) g = 0.f;
                }
            }
            rb[i] = g;
        }
    }
    __device__ void store(int ci, int n, float v, int z) const {
        if (ci >= M || n >= N) return;
        if (part) {
            part[((size_t)z * M + ci) * Nmax + n] = v;
            return;
        }
        const int iwp = n % Wp, t2 = n / Wp, ihp = t2 % Hp, bb = t2 / Hp;
        dx[(((size_t)bb * s.Cin + ci) * s.H + ihp * s.S + ph) * s.W + iwp * s.S + pw] = v;
    }
};

// dx of every (group, phase) from its split partials, summed in split order
__global__ void dgrad_reduce_kernel(DgradOps o_g) {
    const DgradOps o = o_g.at((int)blockIdx.y);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ci = i / o.Nmax, n = i % o.Nmax;
    if (ci >= o.M || n >= o.N) return;
    const size_t MN = (size_t)o.M * o.Nmax;
    float t = 0.f;
    for (int z = 0; z < o.splits; ++z) t += o.part[z * MN + i];
    const int iwp = n % o.Wp, t2 = n / o.Wp, ihp = t2 % o.Hp, bb = t2 / o.Hp;
    o.dx[(((size_t)bb * o.s.Cin + ci) * o.s.H + ihp * o.s.S + o.ph) * o.s.W + iwp * o.s.S + o.pw] = t;
}

// K range [k0, k1); chunk > 0 splits it over blockIdx.z (split-K, partial tiles per z)
// blockIdx.z = group * zsub + split: groups are the population's agents (each
// its own weights and activations, one launch for all of them)
template <int BM, int BN, class Ops>
__global__ __launch_bounds__(NT) void igemm_kernel(Ops ops_g, int k0, int k1, int chunk, int zsub) {
    static_assert((BM / 32) * (BN / 32) == NT / 64 && NT % BN == 0, "4 waves of 32x32");
    constexpr int NA = BM * BK / NT, NB = BK * BN / NT;
    const int split = (int)blockIdx.z % zsub;
    const Ops ops = ops_g.at((int)blockIdx.z / zsub);
    k1 = ops.kend(k1);
    if (chunk > 0) {
        k0 += split * chunk;
        k1 = k0 + chunk < k1 ? k0 + chunk : k1;
    }
    if (k0 >= k1) k1 = k0;  // empty split: stores zeros
    __shared__ Smem<BM, BN, Ops::kCols, Ops::kLut, Ops::kTabN> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m_blk = blockIdx.y * BM, n_blk = blockIdx.x * BN;
    typename Ops::Ctx ctx;
    ops.setup(ctx, sm, tid % BN, n_blk + tid % BN, tid);
    float ra[NA], rb[NB];
    // As columns are XOR-swizzled by k (swz): the stash writes (16 k rows x 4
    // columns per wave) and the MFMA operand reads (4 k rows x 16 columns) both
    // land in 64 distinct banks
    auto swz = [](int k) { return ((k >> 2) & 3) << 2; };
    auto stash = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NA; ++i) sm.As[buf][tid % BK][(tid / BK + i * (NT / BK)) ^ swz(tid % BK)] = ra[i];
#pragma unroll
        for (int i = 0; i < NB; ++i) sm.Bs[buf][tid / BN + i * (NT / BN)][tid % BN] = rb[i];
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int wm = (wave % (BM / 32)) * 32, wn = (wave / (BM / 32)) * 32;  // this wave's 32x32 sub-tile
    const int r = lane & 15, q = lane >> 4;
    const bool rsum = Ops::kRowSum && n_blk == 0 && tid < BM;  // wgrad db: A's row sums
    float rs = 0.f;
    for (int kc = k0; kc < k1; kc += Ops::kTabN) {
        const int kce = kc + Ops::kTabN < k1 ? kc + Ops::kTabN : k1;
        __syncthreads();  // previous chunk's tables and operands consumed
        ops.build(sm, kc, kce, tid);
        __syncthreads();
        int buf = 0;
        ops.template gather<NA, NB, BN>(ctx, sm, m_blk, kc, kc, kce, tid, ra, rb);
        stash(0);
        __syncthreads();
        for (int kb = kc; kb < kce; kb += BK) {
            const bool more = kb + BK < kce;
            if (more) ops.template gather<NA, NB, BN>(ctx, sm, m_blk, kc, kb + BK, kce, tid, ra, rb);
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                const int sw = swz(kk + q);
                const float a0 = sm.As[buf][kk + q][(wm + r) ^ sw], a1 = sm.As[buf][kk + q][(wm + 16 + r) ^ sw];
                const float b0 = sm.Bs[buf][kk + q][wn + r], b1 = sm.Bs[buf][kk + q][wn + 16 + r];
                acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
            }
            if constexpr (Ops::kRowSum)
                if (rsum) {
#pragma unroll
                    for (int kk = 0; kk < BK; ++kk) rs += sm.As[buf][kk][tid ^ swz(kk)];
                }
            if (more) {
                stash(buf ^ 1);
                __syncthreads();
                buf ^= 1;
            }
        }
    }
    // C layout: lane holds rows 4q + i, column r of each 16x16 tile
    float rb_[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) rb_[i][e] = ops.row_bias(m_blk + wm + 16 * i + 4 * q + e);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int n = n_blk + wn + 16 * j + r;
                if constexpr (Ops::kBias) {
                    ops.store(m_blk + wm + 16 * i + 4 * q + e, n, acc[i][j][e], split, rb_[i][e]);
                } else if (!Ops::kRowSum || n < ops.N - 1) {  // column N - 1 (db) belongs to the row sums
                    ops.store(m_blk + wm + 16 * i + 4 * q + e, n, acc[i][j][e], split);
                }
            }
    if constexpr (Ops::kRowSum)
        if (rsum) ops.store(m_blk + tid, ops.N - 1, rs, split);
}

// fixed-order sum of the wgrad split partials, in two parallel stages (a
// single pass had one thread walk every split of its element: a long chain of
// dependent-latency loads over few threads):
//   stage 1: group g of kRedG consecutive splits -> part[g * kRedG] (in place)
//   stage 2: dW (+)= sum_g part[g * kRedG], db (+)= the last column
constexpr int kRedG = 16;
__global__ void wgrad_reduce1_kernel(float *__restrict__ part, int splits, int MN) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int z0 = (int)blockIdx.y * kRedG;
    if (i >= MN) return;
    part += (size_t)blockIdx.z * splits * MN;
    const int nz = splits - z0 < kRedG ? splits - z0 : kRedG;
    float v[kRedG];
#pragma unroll
    for (int z = 0; z < kRedG; ++z) v[z] = z < nz ? part[(size_t)(z0 + z) * MN + i] : 0.f;
    float t = 0.f;
#pragma unroll
    for (int z = 0; z < kRedG; ++z) t += v[z];
    part[(size_t)z0 * MN + i] = t;
}
__global__ void wgrad_reduce2_kernel(const float *__restrict__ part, int splits, int groups, int M, int N,
                                     float *__restrict__ dw, float *__restrict__ db, int accumulate) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const size_t grp = blockIdx.y;  // population group
    part += grp * splits * M * N;
    dw += grp * M * (N - 1);
    if (db) db += grp * M;
    float v = 0.f;
    for (int g = 0; g < groups; ++g) v += part[(size_t)g * kRedG * M * N + i];
    const int m = i / N, n = i % N;
    if (n < N - 1) {
        float *d = dw + (size_t)m * (N - 1) + n;
        *d = accumulate ? *d + v : v;
    } else if (db) {
        db[m] = accumulate ? db[m] + v : v;
    }
}

// a 32 x 128 tile for GEMMs with at most 32 rows (32-channel layers), else 64 x 64
template <class Ops>
static void launch(const Ops &o, int M, int N, int k0, int k1, int chunk, int splits, int groups, hipStream_t st) {
    const unsigned z = (unsigned)(splits * groups);
    if (M <= 32) {
        dim3 grid((unsigned)ceil_div(N, 128), (unsigned)ceil_div(M, 32), z);
        igemm_kernel<32, 128><<<grid, NT, 0, st>>>(o, k0, k1, chunk, splits);
    } else {
        dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(M, 64), z);
        igemm_kernel<64, 64><<<grid, NT, 0, st>>>(o, k0, k1, chunk, splits);
    }
}

// wgrad split-K plan: enough (group, tile, split) workgroups to fill 256 CUs
// several times over, each split a multiple of BK and at least 64 reduction
// steps long
static void wgrad_plan(const Shape &s, int groups, int &splits, int &chunk) {
    const int M = s.Cout, N = s.Cin * s.KH * s.KW, P = s.B * s.OH * s.OW;  // N: the GEMM's weight columns
    const int tiles = (M <= 32 ? (int)ceil_div(N, 128) : (int)(ceil_div(N, 64) * ceil_div(M, 64))) * groups;
    int want = (int)ceil_div(1024, tiles);
    chunk = (int)(ceil_div(ceil_div(P, want), BK) * BK);
    if (chunk < 64) chunk = 64;
    splits = (int)ceil_div(P, chunk);
}

// dgrad: the largest phase's GEMM (phase 0) and a split-K plan from the layer
// shape alone: one group's (phase, tile, split) workgroups >= kDgradFill, each
// split at least 16 K steps
constexpr int kDgradFill = 384;
struct DgradPlan {
    int nph, Nmax, Kmax, splits, chunk;
};
static DgradPlan dgrad_plan(const Shape &s) {
    DgradPlan d;
    d.nph = s.S * s.S;
    d.Nmax = s.B * (int)ceil_div(s.H, s.S) * (int)ceil_div(s.W, s.S);
    d.Kmax = s.Cout * (int)ceil_div(s.KH, s.S) * (int)ceil_div(s.KW, s.S);
    const int M = s.Cin;
    const int tiles = (M <= 32 ? (int)ceil_div(d.Nmax, 128) : (int)(ceil_div(d.Nmax, 64) * ceil_div(M, 64))) * d.nph;
    int want = (int)ceil_div(kDgradFill, tiles);
    const int most = d.Kmax / (16 * BK);
    if (want > most) want = most;
    if (want < 1) want = 1;
    d.chunk = (int)(ceil_div(ceil_div(d.Kmax, want), BK) * BK);
    d.splits = (int)ceil_div(d.Kmax, d.chunk);
    if (d.splits <= 1) {
        d.splits = 1;
        d.chunk = 0;
    }
    return d;
}
static size_t dgrad_workspace_bytes(const Shape &s, int groups) {
    const DgradPlan d = dgrad_plan(s);
    return d.splits > 1 ? (size_t)groups * d.nph * d.splits * s.Cin * d.Nmax * sizeof(float) : 0;
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
    AGX_REQUIRE(s.KH <= kTapMax && s.KW <= kTapMax && s.Cout < 65536, "%s: kernel taps > %d or > 65535 channels",
                who, kTapMax);
    s.OH = (s.H - s.KH) / s.S + 1;
    s.OW = (s.W - s.KW) / s.S + 1;
    AGX_REQUIRE(s.OH < 32768 && s.OW < 32768, "%s: output height / width >= 32768 (int16 tap tables)", who);
    AGX_REQUIRE((int64_t)s.B * s.Cout * s.OH * s.OW < (1ll << 31) && (int64_t)s.B * s.Cin * s.H * s.W < (1ll << 31),
                "%s: tensor too large for 32-bit indexing", who);
    return AGX_OK;
}

extern "C" int agx_conv2d_forward_grouped(const agx_conv2d_shape *shape, int64_t groups, const void *x,
                                          int64_t x_gstride, int x_is_u8, float x_low, float x_high, const float *w,
                                          int64_t w_gstride, const float *bias, int64_t b_gstride, int relu, float *y,
                                          int64_t y_gstride, void *stream) {
    Shape s;
    if (int rc = check_shape(shape, s, "agx_conv2d_forward")) return rc;
    AGX_REQUIRE(x && w && y && groups >= 1 && groups < 65536, "agx_conv2d_forward: null pointer or bad groups");
    AGX_REQUIRE(!x_is_u8 || x_high > x_low, "agx_conv2d_forward: u8 input needs high > low");
    const int M = s.Cout, N = s.B * s.OH * s.OW, K = s.Cin * s.KH * s.KW;
    hipStream_t st = as_stream(stream);
    if (x_is_u8) {
        FwdOps<true> o{w, x, bias, y, x_low, x_high - x_low, relu, s, M, N, K, x_gstride, w_gstride, b_gstride,
                       y_gstride};
        launch(o, M, N, 0, K, 0, 1, (int)groups, st);
    } else {
        FwdOps<false> o{w, x, bias, y, 0.f, 1.f, relu, s, M, N, K, x_gstride, w_gstride, b_gstride, y_gstride};
        launch(o, M, N, 0, K, 0, 1, (int)groups, st);
    }
    return check_launch("agx_conv2d_forward");
}

extern "C" int agx_conv2d_forward_grouped2(const agx_conv2d_shape *shape, int64_t groups, int64_t g1_count,
                                           const void *x, int64_t x_stride1, int64_t x_stride2, int x_is_u8,
                                           float x_low, float x_high, const float *w, int64_t w_stride1,
                                           int64_t w_stride2, const float *bias, int64_t b_stride1, int64_t b_stride2,
                                           int relu, float *y, int64_t y_stride1, int64_t y_stride2, void *stream) {
    Shape s;
    if (int rc = check_shape(shape, s, "agx_conv2d_forward_grouped2")) return rc;
    AGX_REQUIRE(x && w && y && groups >= 1 && groups < 65536 && g1_count >= 1 && g1_count <= groups,
                "agx_conv2d_forward_grouped2: null pointer or bad groups");
    AGX_REQUIRE(!x_is_u8 || x_high > x_low, "agx_conv2d_forward_grouped2: u8 input needs high > low");
    const int M = s.Cout, N = s.B * s.OH * s.OW, K = s.Cin * s.KH * s.KW;
    hipStream_t st = as_stream(stream);
    if (x_is_u8) {
        FwdOps<true> o{w, x, bias, y, x_low, x_high - x_low, relu, s, M, N, K, x_stride1, w_stride1, b_stride1,
                       y_stride1, x_stride2, w_stride2, b_stride2, y_stride2, (int)g1_count};
        launch(o, M, N, 0, K, 0, 1, (int)groups, st);
    } else {
        FwdOps<false> o{w, x, bias, y, 0.f, 1.f, relu, s, M, N, K, x_stride1, w_stride1, b_stride1, y_stride1,
                        x_stride2, w_stride2, b_stride2, y_stride2, (int)g1_count};
        launch(o, M, N, 0, K, 0, 1, (int)groups, st);
    }
    return check_launch("agx_conv2d_forward_grouped2");
}

extern "C" int agx_conv2d_forward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low,
                                  float x_high, const float *w, const float *bias, int relu, float *y, void *stream) {
    return agx_conv2d_forward_grouped(shape, 1, x, 0, x_is_u8, x_low, x_high, w, 0, bias, 0, relu, y, 0, stream);
}

extern "C" size_t agx_conv2d_wgrad_workspace_bytes_grouped(const agx_conv2d_shape *shape, int64_t groups) {
    Shape s;
    if (check_shape(shape, s, "agx_conv2d_wgrad_workspace_bytes") || groups < 1) return 0;
    int splits = 1, chunk = 0;
    wgrad_plan(s, (int)groups, splits, chunk);
    // one workspace serves the wgrad partials and then (stream-ordered) the dgrad ones
    const size_t wb = (size_t)groups * splits * s.Cout * (s.Cin * s.KH * s.KW + 1) * sizeof(float);
    const size_t db = dgrad_workspace_bytes(s, (int)groups);
    return wb > db ? wb : db;
}

extern "C" size_t agx_conv2d_wgrad_workspace_bytes(const agx_conv2d_shape *shape) {
    return agx_conv2d_wgrad_workspace_bytes_grouped(shape, 1);
}

extern "C" int agx_conv2d_backward_grouped(const agx_conv2d_shape *shape, int64_t groups, const void *x,
                                           int64_t x_gstride, int x_is_u8, float x_low, float x_high, const float *w,
                                           int64_t w_gstride, const float *y_act, const float *dy, int64_t y_gstride,
                                           float *dx, float *dw, float *db, int accumulate, void *workspace,
                                           void *stream) {
    Shape s;
    if (int rc = check_shape(shape, s, "agx_conv2d_backward")) return rc;
    AGX_REQUIRE(x && w && dy && dw && workspace && groups >= 1 && groups < 65536,
                "agx_conv2d_backward: null pointer or bad groups");
    hipStream_t st = as_stream(stream);
    const int G = (int)groups;
    const int K = s.Cin * s.KH * s.KW;
    const int P = s.B * s.OH * s.OW;
    int splits = 1, chunk = 0;
    wgrad_plan(s, G, splits, chunk);
    float *part = static_cast<float *>(workspace);
    const int M = s.Cout, N = K + 1;
    const long long gp = (long long)splits * M * N;
    if (x_is_u8) {
        WgradOps<true> o{dy, y_act, x, x_low, x_high - x_low, part, s, M, N, P, x_gstride, y_gstride, gp};
        launch(o, M, N - 1, 0, P, chunk, splits, G, st);
    } else {
        WgradOps<false> o{dy, y_act, x, 0.f, 1.f, part, s, M, N, P, x_gstride, y_gstride, gp};
        launch(o, M, N - 1, 0, P, chunk, splits, G, st);
    }
    // dW / db of group g land densely at dw + g*Cout*K, db + g*Cout
    const int rgroups = (int)ceil_div(splits, kRedG);
    wgrad_reduce1_kernel<<<dim3((unsigned)ceil_div(M * N, 256), (unsigned)rgroups, (unsigned)G), 256, 0, st>>>(
        part, splits, M * N);
    wgrad_reduce2_kernel<<<dim3((unsigned)ceil_div(M * N, 256), (unsigned)G), 256, 0, st>>>(part, splits, rgroups, M,
                                                                                          N, dw, db, accumulate);
    if (int rc = check_launch("agx_conv2d_backward wgrad")) return rc;
    if (dx) {
        AGX_REQUIRE(!x_is_u8, "agx_conv2d_backward: no data gradient for a u8 input layer");
        const DgradPlan d = dgrad_plan(s);
        DgradOps o{w, dy, y_act, dx, d.splits > 1 ? part : nullptr, s, s.Cin, 0, 0, 0, 0, 0, 0, 0, 0,
                   d.nph, d.Nmax, d.splits, w_gstride, y_gstride, x_gstride};
        const int gp_ = G * d.nph;  // (group, phase) pairs
        launch(o, o.M, d.Nmax, 0, d.Kmax, d.chunk, d.splits, gp_, st);
        if (d.splits > 1)
            dgrad_reduce_kernel<<<dim3((unsigned)ceil_div((size_t)s.Cin * d.Nmax, 256), (unsigned)gp_), 256, 0, st>>>(o);
        if (int rc = check_launch("agx_conv2d_backward dgrad")) return rc;
    }
    return AGX_OK;
}

extern "C" int agx_conv2d_backward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low,
                                   float x_high, const float *w, const float *y_act, const float *dy, float *dx,
                                   float *dw, float *db, int accumulate, void *workspace, void *stream) {
    return agx_conv2d_backward_grouped(shape, 1, x, 0, x_is_u8, x_low, x_high, w, 0, y_act, dy, 0, dx, dw, db,
                                       accumulate, workspace, stream);
}
