// Fused PPO learner + rollout policy step for a population of shared-encoder
// MLP actor-critics.
//
// agx_ppo_learn: ONE persistent workgroup per agent runs every epoch x
// minibatch update of PPO._learn_from_rollout_buffer_flat
// (agilerl/algorithms/ppo.py:836-915) — forward, categorical log-prob /
// entropy, clipped-surrogate + clipped-value loss, backward, two-group
// gradient-norm clip (ppo.py:910-911) and Adam (optimizer_wrapper.py:444-452)
// — without leaving the chip.  A prologue kernel first gathers the rollout
// SoA into per-epoch minibatch order (the reference's shuffled TensorDict
// indexing, ppo.py:842-848) and applies the global advantage normalisation
// (ppo.py:829-834), so the learner streams contiguous 32-row sub-batches.
//
// agx_ppo_act: the rollout policy step (PPO.get_action, ppo.py:567-633 ->
// _get_action_and_values :400-492): forward, Gumbel-max categorical sample
// from a counter-based Philox stream, log-prob, entropy and value, written
// straight into the (P, T, N) rollout SoA.
//
// Network (agilerl/utils/evolvable_networks.py:527-644 create_mlp,
// agilerl/networks/base.py:541-561):
//   encoder: ne-1 x [Linear -> LayerNorm(affine) -> ReLU], Linear(->lat) ->
//            LayerNorm(plain) -> ReLU
//   heads  : actor  Linear(lat->ha) -> LN(affine) -> ReLU -> Linear(->A)
//            critic Linear(lat->hc) -> LN(affine) -> ReLU -> Linear(->1)
//   The two head hidden layers run as ONE merged [ha+hc] layer (same input,
//   per-half LayerNorm); d(latent) = [dz_a | dz_c] . [Wa; Wc] is one GEMM.
//
// Kernels are instantiated per network shape (compile-time plan: every
// offset, trip count and tile->register assignment is a constant, which is
// what keeps ~200 live VGPRs spill-free).  Mapping (512 threads = 8 waves,
// sub-batches of SB = 32 rows):
//   * parameters live in LDS (weight rows padded by 2 floats: conflict-free
//     MFMA operand reads); Adam moments live in REGISTERS — thread t owns
//     LDS parameter slots t, t+512, ... for the whole learn();
//   * every Linear (incl. the output layers, padded to 16 rows, with the bias
//     as an extra ones-column) is an f32 MFMA v_mfma_f32_16x16x4_f32 GEMM;
//     each wave owns fixed 16x16 dW tiles whose accumulators stay in
//     registers over the sub-batches of a minibatch;
//   * LayerNorm forward/backward and the loss are row passes with 16 lanes
//     per row (4 rows per wave): row reductions are DPP (quad_perm,
//     row_half_mirror, row_mirror); bias / LN-affine gradients are reduced
//     across the 4 rows by ds_swizzle + permlane32_swap and accumulated per
//     wave in LDS, summed in a fixed order (deterministic);
//   * minibatch end: dump dW tiles + vector grads into an LDS gradient image
//     of the parameter region (aliasing the dead activations), two-group
//     norm, Adam from registers.
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "agx_common.h"
#include "rollout.h"

namespace agx {

// Partner ownership of the parameter image: uniform chunks (1, default) or the
// proportional n4s * kk / K split of rounds 2-4 (0; A/B builds)
#ifndef AGX_LEARN_UNIFORM
#define AGX_LEARN_UNIFORM 1
#endif
// Reduce-scatter over all 8 waves (two partner halves per owned chunk, summed
// lower + upper through LDS; 1) or one thread per owned chunk over all K
// partners (0, default: measured 1.116 vs 1.133 ms per learn() on one box)
#ifndef AGX_LEARN_RS2
#define AGX_LEARN_RS2 0
#endif

constexpr int kNT = 512;
constexpr int kNW = kNT / kWave;  // 8 waves
constexpr int kSB = 32;           // rows per sub-batch
constexpr int kMaxSlot = 10;      // dW tiles per wave
constexpr int kMaxK = 16;         // partner workgroups per agent
constexpr int kMaxPT = 32;        // LDS parameter slots per thread: 8 float4 chunks
constexpr int kMaxA = 16;
constexpr int kMaxBlk = 28;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

struct NetDims {
    int D, A, ne, eo[3], ha, hc;
};

struct Blk {
    int f0, len, rowlen, l0, ldst;  // flat [f0, f0+len) <-> LDS l0 + (i / rowlen) * ldst + i % rowlen
};

struct LearnPlan {
    int ok;
    int D, A, ne, ein[3], eout[3], eaff[3], lat, ha, hc, H, n;
    // flat offsets (nets.py layout): per encoder layer W, b, [g, be]; actor W, b,
    // g, be, Wout, bout; critic W, b, g, be, Wout, bout
    int f_ew[3], f_eb[3], f_eg[3], f_ebe[3];
    int f_aw, f_ab, f_ag, f_abe, f_aow, f_aob, f_cw, f_cb, f_cg, f_cbe, f_cow, f_cob;
    // LDS (floats)
    int l_ew[3], l_eld[3], l_eb[3], l_eg[3], l_ebe[3];
    int l_hw, l_hld, l_hb, l_hg, l_hbe;
    int l_aow, l_aold, l_aob, l_cow, l_cold, l_cob;
    int param_end;
    int l_x0, ld_x0, l_xe[3], ld_xe[3], l_re[3], l_xh, ld_xh, l_rh;
    int l_s1, l_s2, ld_s;
    int l_lg, l_dlg, l_dvb, l_val, l_row;
    int l_red, red_e[3], red_h, l_stat, l_stamp;
    int l_grad;  // gradient image of [0, param_end) (aliases the activations)
    int lds_floats, act_floats;
    int slab;  // floats per cross-workgroup gradient slab (parameter image + loss)
    // dW tiles per layer group g: enc 0..ne-1, head ne, out-actor ne+1, out-critic ne+2
    int nt[6], ncol[6], slot0[6], nslot[6], nslots;
    int nblk;
    Blk blk[kMaxBlk];
};

constexpr int rup(int x, int m) { return (x + m - 1) / m * m; }

constexpr LearnPlan make_plan(NetDims d) {
    LearnPlan pl{};
    pl.ok = 0;
    pl.D = d.D;
    pl.A = d.A;
    pl.ne = d.ne;
    if (pl.ne < 2 || pl.ne > 3 || pl.A < 1 || pl.A > kMaxA || pl.D < 1 || pl.D > 128) return pl;
    int prev = pl.D;
    for (int e = 0; e < pl.ne; ++e) {
        pl.ein[e] = prev;
        pl.eout[e] = d.eo[e];
        pl.eaff[e] = e < pl.ne - 1;
        if (pl.eout[e] % 16 || pl.eout[e] > 128 || pl.eout[e] < 16) return pl;
        prev = pl.eout[e];
    }
    pl.lat = prev;
    pl.ha = d.ha;
    pl.hc = d.hc;
    pl.H = pl.ha + pl.hc;
    if (pl.ha % 16 || pl.hc % 16 || pl.ha < 16 || pl.hc < 16 || pl.H > 128) return pl;
    // ---- flat layout
    int f = 0;
    for (int e = 0; e < pl.ne; ++e) {
        pl.f_ew[e] = f;
        f += pl.eout[e] * pl.ein[e];
        pl.f_eb[e] = f;
        f += pl.eout[e];
        pl.f_eg[e] = pl.f_ebe[e] = -1;
        if (pl.eaff[e]) {
            pl.f_eg[e] = f;
            f += pl.eout[e];
            pl.f_ebe[e] = f;
            f += pl.eout[e];
        }
    }
    pl.f_aw = f; f += pl.ha * pl.lat;
    pl.f_ab = f; f += pl.ha;
    pl.f_ag = f; f += pl.ha;
    pl.f_abe = f; f += pl.ha;
    pl.f_aow = f; f += pl.A * pl.ha;
    pl.f_aob = f; f += pl.A;
    pl.f_cw = f; f += pl.hc * pl.lat;
    pl.f_cb = f; f += pl.hc;
    pl.f_cg = f; f += pl.hc;
    pl.f_cbe = f; f += pl.hc;
    pl.f_cow = f; f += pl.hc;
    pl.f_cob = f; f += 1;
    pl.n = f;
    // ---- LDS: parameters
    int off = 0;
    for (int e = 0; e < pl.ne; ++e) {
        pl.l_eld[e] = rup(pl.ein[e], 16) + 2;
        pl.l_ew[e] = off; off += rup(pl.eout[e] * pl.l_eld[e], 4);
        pl.l_eb[e] = off; off += rup(pl.eout[e], 4);
        pl.l_eg[e] = off; off += pl.eaff[e] ? rup(pl.eout[e], 4) : 0;
        pl.l_ebe[e] = off; off += pl.eaff[e] ? rup(pl.eout[e], 4) : 0;
    }
    pl.l_hld = pl.lat + 2;
    pl.l_hw = off; off += rup(pl.H * pl.l_hld, 4);
    pl.l_hb = off; off += rup(pl.H, 4);
    pl.l_hg = off; off += rup(pl.H, 4);
    pl.l_hbe = off; off += rup(pl.H, 4);
    pl.l_aold = pl.ha + 2;
    pl.l_aow = off; off += rup(pl.A * pl.l_aold, 4);
    pl.l_aob = off; off += kMaxA;
    pl.l_cold = pl.hc + 2;
    pl.l_cow = off; off += rup(pl.l_cold, 4);
    pl.l_cob = off; off += 4;
    pl.param_end = off;
    if (pl.param_end > kNT * kMaxPT) return pl;
    // ---- LDS: activations (the gradient image aliases them)
    pl.ld_x0 = rup(pl.D, 16) + 2;
    pl.l_x0 = off; off += rup(kSB * pl.ld_x0, 4);
    for (int e = 0; e < pl.ne; ++e) {
        pl.ld_xe[e] = pl.eout[e] + 2;
        pl.l_xe[e] = off; off += kSB * pl.ld_xe[e];
        pl.l_re[e] = off; off += 2 * kSB;
    }
    pl.ld_xh = pl.H + 2;
    pl.l_xh = off; off += kSB * pl.ld_xh;
    pl.l_rh = off; off += 2 * kSB;
    int wmax = pl.H;
    for (int e = 0; e < pl.ne; ++e) wmax = wmax > pl.eout[e] ? wmax : pl.eout[e];
    pl.ld_s = wmax + 2;
    pl.l_s1 = off; off += kSB * pl.ld_s;
    pl.l_s2 = off; off += kSB * pl.ld_s;
    pl.l_lg = off; off += kSB * kMaxA;
    pl.l_val = off; off += kSB;
    pl.act_floats = off;  // the policy-step kernel needs only this much
    pl.l_dlg = off; off += kSB * kMaxA;
    pl.l_dvb = off; off += kSB * kMaxA;
    pl.l_row = off; off += 6 * kSB;  // old_logp, adv, ret, old_v, action, legal-action mask
    pl.l_grad = pl.l_x0;
    if (off - pl.l_x0 < pl.param_end) off = pl.l_x0 + pl.param_end;  // room for the gradient image
    int red = 0;
    for (int e = 0; e < pl.ne; ++e) {
        pl.red_e[e] = red;
        red += (pl.eaff[e] ? 3 : 1) * kNW * pl.eout[e];
    }
    pl.red_h = red;
    red += 3 * kNW * pl.H;
    pl.l_red = off; off += red;
    pl.l_stat = off; off += 5 * kNW;
    off = rup(off, 2);
    pl.l_stamp = off; off += 2 * 80;  // diagnostic phase stamps (agx_debug_learn_stamps)
    pl.lds_floats = off;
    if (pl.lds_floats * 4 > 160 * 1024) return pl;
    // + the loss / approx_kl chunk + the partners' per-wave partial gradient norms
    pl.slab = rup(pl.param_end + 4 + 2 * kNW * kMaxK, 64);
    // ---- dW tile groups
    int slot = 0;
    for (int g = 0; g < pl.ne + 3; ++g) {
        int fo = 0, fi = 0;
        if (g < pl.ne) { fo = pl.eout[g]; fi = pl.ein[g]; }
        else if (g == pl.ne) { fo = pl.H; fi = pl.lat; }
        else if (g == pl.ne + 1) { fo = 16; fi = pl.ha + 1; }   // + bias column
        else { fo = 16; fi = pl.hc + 1; }
        pl.ncol[g] = (fi + 15) / 16;
        pl.nt[g] = (fo / 16) * pl.ncol[g];
        pl.slot0[g] = slot;
        pl.nslot[g] = (pl.nt[g] + kNW - 1) / kNW;
        slot += pl.nslot[g];
    }
    pl.nslots = slot;
    if (slot > kMaxSlot) return pl;
    // ---- flat <-> LDS blocks
    int nb = 0;
    auto blk = [&](int f0, int len, int rowlen, int l0, int ldst) {
        if (len > 0) pl.blk[nb++] = Blk{f0, len, rowlen, l0, ldst};
    };
    for (int e = 0; e < pl.ne; ++e) {
        const int fo = pl.eout[e], fi = pl.ein[e];
        blk(pl.f_ew[e], fo * fi, fi, pl.l_ew[e], pl.l_eld[e]);
        blk(pl.f_eb[e], fo, fo, pl.l_eb[e], fo);
        if (pl.eaff[e]) {
            blk(pl.f_eg[e], fo, fo, pl.l_eg[e], fo);
            blk(pl.f_ebe[e], fo, fo, pl.l_ebe[e], fo);
        }
    }
    blk(pl.f_aw, pl.ha * pl.lat, pl.lat, pl.l_hw, pl.l_hld);
    blk(pl.f_ab, pl.ha, pl.ha, pl.l_hb, pl.ha);
    blk(pl.f_ag, pl.ha, pl.ha, pl.l_hg, pl.ha);
    blk(pl.f_abe, pl.ha, pl.ha, pl.l_hbe, pl.ha);
    blk(pl.f_aow, pl.A * pl.ha, pl.ha, pl.l_aow, pl.l_aold);
    blk(pl.f_aob, pl.A, pl.A, pl.l_aob, pl.A);
    blk(pl.f_cw, pl.hc * pl.lat, pl.lat, pl.l_hw + pl.ha * pl.l_hld, pl.l_hld);
    blk(pl.f_cb, pl.hc, pl.hc, pl.l_hb + pl.ha, pl.hc);
    blk(pl.f_cg, pl.hc, pl.hc, pl.l_hg + pl.ha, pl.hc);
    blk(pl.f_cbe, pl.hc, pl.hc, pl.l_hbe + pl.ha, pl.hc);
    blk(pl.f_cow, pl.hc, pl.hc, pl.l_cow, pl.l_cold);
    blk(pl.f_cob, 1, 1, pl.l_cob, 1);
    pl.nblk = nb;
    pl.ok = 1;
    return pl;
}

// ---------------------------------------------------------------------------
// instantiated shapes: (obs_dim, actions, encoder widths..., head_actor, head_critic)
// ---------------------------------------------------------------------------
#ifdef AGX_BENCH_SHAPE_ONLY  // diagnostic builds (tools/): the config-2 shape alone, a quarter of the compile time
#define AGX_PPO_SHAPES(X) X(8, 4, 2, 64, 64, 0, 64, 64)
#else
#define AGX_PPO_SHAPES(X)                 \
    X(8, 4, 2, 64, 64, 0, 64, 64)  /* LunarLander config 2 (ppo.yaml) */ \
    X(4, 2, 2, 64, 64, 0, 64, 64)  /* CartPole */                        \
    X(6, 3, 2, 64, 64, 0, 64, 64)  /* Acrobot */                         \
    X(8, 4, 2, 64, 64, 0, 64, 16)  /* reference PPO default critic head [16] */ \
    X(4, 2, 2, 64, 64, 0, 64, 16)                                        \
    X(8, 4, 3, 64, 64, 32, 32, 16) /* PPO with no net_config: encoder [64, 64] -> latent 32, heads [32] / [16] */ \
    X(4, 2, 3, 64, 64, 32, 32, 16)
#endif

template <int D_, int A_, int NE_, int E0, int E1, int E2, int HA, int HC>
struct Shape {
    static constexpr NetDims dims{D_, A_, NE_, {E0, E1, E2}, HA, HC};
    static constexpr LearnPlan plan = make_plan(dims);
};

// ---------------------------------------------------------------------------
// cross-lane helpers
// ---------------------------------------------------------------------------
template <int C>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), C, 0xf, 0xf, true));
}
// sum / max over the 16 lanes of a DPP row; result in every lane of the row
__device__ __forceinline__ float row_sum(float v) {
    v += dpp<0xb1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4e>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    return v;
}
__device__ __forceinline__ float row_max(float v) {
    v = fmaxf(v, dpp<0xb1>(v));
    v = fmaxf(v, dpp<0x4e>(v));
    v = fmaxf(v, dpp<0x141>(v));
    v = fmaxf(v, dpp<0x140>(v));
    return v;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// DPP row broadcast (GFX9 row_bcast:15 = 0x142, row_bcast:31 = 0x143): the
// rows enabled in RM receive lane 15 (resp. 31) of the preceding row(s); the
// other rows keep `old`
template <int C, int RM>
__device__ __forceinline__ float bcast(float v, float old) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                 C, RM, 0xf, false));
}
// W-lane row sum (W = 16: one DPP row; W = 32: + the other 16-lane half,
// lane ^ 16; W = 64: the whole wave, by DPP alone — row sums, then row 1 +=
// row 0 and row 3 += row 2 (row_bcast:15), then rows 2-3 += lane 31
// (row_bcast:31): lane 63 holds (r3 + r2) + (r1 + r0), read back as a
// wave-uniform value.  No LDS-crossbar (ds_swizzle) round trip on the chain.)
template <int W>
__device__ __forceinline__ float wrow_sum(float v) {
    v = row_sum(v);
    if constexpr (W == 32)
        v += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401f));
    if constexpr (W == 64) {
        v += bcast<0x142, 0xa>(v, 0.f);
        v += bcast<0x143, 0xc>(v, 0.f);
        v = readlane_f(v, 63);
    }
    return v;
}
template <int W>
__device__ __forceinline__ float wrow_max(float v) {
    v = row_max(v);
    if constexpr (W == 32)
        v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401f)));
    if constexpr (W == 64) {
        v = fmaxf(v, bcast<0x142, 0xa>(v, -__builtin_huge_valf()));
        v = fmaxf(v, bcast<0x143, 0xc>(v, -__builtin_huge_valf()));
        v = readlane_f(v, 63);
    }
    return v;
}
// row slot of this lane: W = 16: wave + 8 * (lane / 16) (4 rows per wave);
// W = 32: 2 * wave + lane / 32 (2 rows per wave, a 16-row sub-batch fills all lanes);
// W = 64: the wave (one row per wave, an 8-row sub-batch fills all lanes)
template <int W>
__device__ __forceinline__ int wrow(int lane, int wave) {
    return W == 64 ? wave : (W == 32 ? wave * 2 + (lane >> 5) : wave + kNW * (lane >> 4));
}
// M tiles (16 rows each) of a sub-batch's GEMMs: an 8-row sub-batch fills
// rows 0-7 of one tile (rows 8-15 are zero and never stored)
template <int SB>
constexpr int m_tiles() { return SB < 16 ? 1 : SB / 16; }
// sum over the 4 row-groups (lanes l, l^16, l^32, l^48) of a wave
__device__ __forceinline__ float rowgroup_sum(float v) {
    // ds_swizzle bit mode (offset[15] = 0): and_mask 0x1f, xor_mask 0x10 -> lane ^ 16
    v += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401f));
    // lane ^ 32 through the LDS crossbar (v_permlane32_swap's second result is
    // mis-allocated by this toolchain's builtin lowering: both results land in
    // one register)
    const int l = (int)(threadIdx.x & 63);
    return v + __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute((l ^ 32) << 2, __builtin_bit_cast(int, v)));
}
// A uniform pointer kept in a VGPR pair (opaque to the compiler): kernel-argument
// pointers otherwise live as 8-SGPR tuples (s_load_dwordx8) that are spilled and
// restored whole whenever one of them is used
template <class T>
__device__ __forceinline__ T *in_vgpr(T *ptr) {
    asm volatile("" : "+v"(ptr));
    return ptr;
}
// ... and back to SGPRs where an instruction needs a scalar base (buffer resources)
template <class T>
__device__ __forceinline__ T *to_sgpr(T *ptr) {
    const unsigned long long u = reinterpret_cast<unsigned long long>(ptr);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    return reinterpret_cast<T *>(((unsigned long long)hi << 32) | lo);
}
// Lane / wave ids re-derived through an opaque asm at the start of each phase:
// otherwise LICM hoists every lane-dependent LDS address of the whole
// learner out of the epoch/minibatch loops and they all stay live (spills).
__device__ __forceinline__ int vlane() {
    int v = (int)threadIdx.x;
    asm volatile("" : "+v"(v));
    return v & 63;
}
__device__ __forceinline__ int vtid() {
    int v = (int)threadIdx.x;
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ int swave() {
    int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    asm volatile("" : "+s"(w));
    return w;
}
// Row passes: wave w owns rows w, w+8, w+16, w+24 (16 lanes per row), so the
// two rows of a 32-lane LDS group are 8 rows apart: 8 * ld = 16 (mod 32) for
// every padded stride here -> conflict-free ds_read_b32 (rows 1 apart were 2-way).
#define AGX_IDS                                             \
    const int lane = vlane(), wave = swave();               \
    const int lr16 = lane & 15, lq = lane >> 4;             \
    const int rrow = wave + kNW * lq, sub = lr16;           \
    (void)lr16, (void)lq, (void)rrow, (void)sub, (void)lane

// workgroup-uniform sums of two values (fixed order); uses stat[slot*kNW .. +2*kNW)
__device__ __forceinline__ void block_sum2(float &a, float &b, float *stat, int slot, int lane, int wave) {
    a = row_sum(a);
    b = row_sum(b);
    const float wa = readlane_f(a, 0) + readlane_f(a, 16) + readlane_f(a, 32) + readlane_f(a, 48);
    const float wb = readlane_f(b, 0) + readlane_f(b, 16) + readlane_f(b, 32) + readlane_f(b, 48);
    if (lane == 0) {
        stat[slot * kNW + wave] = wa;
        stat[(slot + 1) * kNW + wave] = wb;
    }
    __syncthreads();
    float ta = 0.f, tb = 0.f;
    for (int i = 0; i < kNW; ++i) {
        ta += stat[slot * kNW + i];
        tb += stat[(slot + 1) * kNW + i];
    }
    a = ta;
    b = tb;
}

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// C[16x16] += A[16 x K] B[K x 16], K % 4 == 0.  Software-pipelined: the
// operands of k-batch i+1 (KB k values, KB/2 LDS reads per lane) are issued
// before the MFMAs of batch i, and scheduling barriers keep the compiler from
// sinking each read next to its MFMA (left alone it serialises every MFMA
// behind its own LDS round trip: read -> lgkmcnt(0) -> MFMA).
#ifndef AGX_MFMA_KB
#define AGX_MFMA_KB 16
#endif
template <int K, class FA, class FB>
__device__ __forceinline__ f4 mfma_tile(f4 acc, FA a, FB b) {
    const int lane = vlane();
    const int r = lane & 15, q = lane >> 4;
    constexpr int KB = K < AGX_MFMA_KB ? K : AGX_MFMA_KB;  // k values whose operands are loaded per batch
    constexpr int NB = K / KB;
    static_assert(K % KB == 0 && KB % 4 == 0, "k batches");
    float av[2][KB / 4], bv[2][KB / 4];
#pragma unroll
    for (int j = 0; j < KB / 4; ++j) {
        av[0][j] = a(r, 4 * j + q);
        bv[0][j] = b(4 * j + q, r);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        if (i + 1 < NB) {
#pragma unroll
            for (int j = 0; j < KB / 4; ++j) {
                av[(i + 1) & 1][j] = a(r, (i + 1) * KB + 4 * j + q);
                bv[(i + 1) & 1][j] = b((i + 1) * KB + 4 * j + q, r);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < KB / 4; ++j)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i & 1][j], bv[i & 1][j], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

// flat parameter index -> LDS offset (compile-time block table)
template <class C>
__device__ __forceinline__ int flat_to_lds(int f) {
    constexpr LearnPlan pl = C::plan;
    int l = 0;
#pragma unroll
    for (int b = 0; b < pl.nblk; ++b) {
        constexpr int dummy = 0;
        (void)dummy;
        const Blk k = pl.blk[b];
        if (f >= k.f0 && f < k.f0 + k.len) {
            const int i = f - k.f0;
            l = k.l0 + (i / k.rowlen) * k.ldst + i % k.rowlen;
        }
    }
    return l;
}
// LDS offset -> flat index (-1 for padding) and clip group
template <class C>
__device__ __forceinline__ int lds_to_flat(int l, int &group) {
    constexpr LearnPlan pl = C::plan;
    int f = -1;
    group = 0;
#pragma unroll
    for (int b = 0; b < pl.nblk; ++b) {
        const Blk k = pl.blk[b];
        const int rows = k.len / k.rowlen;
        if (l >= k.l0 && l < k.l0 + rows * k.ldst) {
            const int i = l - k.l0;
            const int c = i % k.ldst;
            if (c < k.rowlen) {
                f = k.f0 + (i / k.ldst) * k.rowlen + c;
                group = f >= pl.f_cw ? 1 : 0;
            }
        }
    }
    return f;
}

// ---------------------------------------------------------------------------
// shared forward (X0 in LDS -> y_h in S1, logits in lg, value in val)
// ---------------------------------------------------------------------------
template <class C, int SB = kSB>
struct Fwd {
    static constexpr LearnPlan pl = C::plan;
    static_assert(SB == 8 || SB == 16 || SB == 32, "sub-batch rows");
    float *sm;

    // LayerNorm(+affine)+ReLU of Z (S2, width F; LN groups [0,split), [split,F))
    // -> xhat to xb (stride ldx), y to S1, rstd to rb[2r + group]
    // OUT (the merged head layer): the output layers ride along as row dot
    // products — logits[a] = y_actor . W_out[a] + b[a] and value = y_critic .
    // w_v + b_v, each a per-lane partial over the lane's 16-strided columns
    // then a DPP row sum — and land in lg / val: no separate output phase.
    template <int F, int split, int xb, int ldx, int rb, int gb, int bb, bool OUT = false>
    __device__ __forceinline__ void ln_rows() {
        // 16-row sub-batches: 32 lanes per row (every lane busy, half the columns
        // per lane); 8-row sub-batches: 64 lanes per row (one row per wave)
        constexpr int W = (!OUT && split >= F) ? ((SB == 8 && F % 64 == 0) ? 64 : (SB <= 16 && F % 32 == 0) ? 32 : 16)
                                               : 16;
        constexpr int NC = F / W;
        constexpr int F0 = split < F ? split : F, F1 = F - F0;
        const int lane = vlane(), wave = swave();
        const int sub = lane & (W - 1);
        const int r = wrow<W>(lane, wave);
        if (SB < kSB && r >= SB) return;  // whole W-lane rows beyond the sub-batch idle
        float z[NC];
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            z[i] = sm[pl.l_s2 + r * pl.ld_s + sub + W * i];
            if (W * i < split) s0 += z[i];
            else s1 += z[i];
        }
        const float m0 = wrow_sum<W>(s0) * (1.f / (float)F0);
        const float m1 = F1 > 0 ? wrow_sum<W>(s1) * (1.f / (float)(F1 > 0 ? F1 : 1)) : 0.f;
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            if (W * i < split) v0 += (z[i] - m0) * (z[i] - m0);
            else v1 += (z[i] - m1) * (z[i] - m1);
        }
        const float r0 = 1.f / sqrtf(wrow_sum<W>(v0) / (float)F0 + 1e-5f);
        const float r1 = F1 > 0 ? 1.f / sqrtf(wrow_sum<W>(v1) / (float)(F1 > 0 ? F1 : 1) + 1e-5f) : 0.f;
        if (sub == 0) {
            sm[rb + 2 * r] = r0;
            sm[rb + 2 * r + 1] = r1;
        }
        constexpr int NA = OUT ? pl.A : 1;
        float pa[NA], pv = 0.f;
#pragma unroll
        for (int a = 0; a < NA; ++a) pa[a] = 0.f;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int j = sub + W * i;
            const float xh = W * i < split ? (z[i] - m0) * r0 : (z[i] - m1) * r1;
            sm[xb + r * ldx + j] = xh;
            const float y = gb >= 0 ? relu(xh * sm[gb + j] + sm[bb + j]) : relu(xh);
            sm[pl.l_s1 + r * pl.ld_s + j] = y;
            if constexpr (OUT) {
                if (W * i < split) {
#pragma unroll
                    for (int a = 0; a < NA; ++a) pa[a] += y * sm[pl.l_aow + a * pl.l_aold + j];
                } else {
                    pv += y * sm[pl.l_cow + j - split];
                }
            }
        }
        if constexpr (OUT) {
            float mine = 0.f;
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const float t = row_sum(pa[a]);
                mine = sub == a ? t : mine;
            }
            pv = row_sum(pv);
            if (sub < NA) sm[pl.l_lg + r * kMaxA + sub] = mine + sm[pl.l_aob + sub];
            if (sub == 0) sm[pl.l_val + r] = pv + sm[pl.l_cob];
        }
    }

    // Z[SB x fout] = X W^T + b  -> S2 (rows beyond an 8-row sub-batch are not
    // stored: they stay zero, so no garbage circulates through the padding rows)
    template <int xb, int ldx, int K, int wb, int ldw, int bias, int fout>
    __device__ __forceinline__ void gemm_fwd() {
        constexpr int MT = m_tiles<SB>();
        constexpr int nt = MT * (fout / 16);
        AGX_IDS;
        for (int t = wave; t < nt; t += kNW) {
            const int m0 = (t % MT) * 16, n0 = (t / MT) * 16;
            f4 c = f4{0.f, 0.f, 0.f, 0.f};
            c = mfma_tile<K>(c, [&](int m, int k) { return sm[xb + (m0 + m) * ldx + k]; },
                             [&](int k, int n) { return sm[wb + (n0 + n) * ldw + k]; });
            const float bv = sm[bias + n0 + lr16];
            if (SB >= 16 || lq * 4 < SB) {
#pragma unroll
                for (int i = 0; i < 4; ++i) sm[pl.l_s2 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i] + bv;
            }
        }
    }

    template <int L, class F>
    __device__ __forceinline__ void enc_layer(F st) {
        constexpr int K = rup(pl.ein[L], 16);
        gemm_fwd<L == 0 ? pl.l_x0 : pl.l_s1, L == 0 ? pl.ld_x0 : pl.ld_s, K, pl.l_ew[L], pl.l_eld[L], pl.l_eb[L],
                 pl.eout[L]>();
        __syncthreads();
        st(8 + 2 * L);
        ln_rows<pl.eout[L], pl.eout[L], pl.l_xe[L], pl.ld_xe[L], pl.l_re[L], pl.eaff[L] ? pl.l_eg[L] : -1,
                pl.l_ebe[L]>();
        __syncthreads();
        st(9 + 2 * L);
        if constexpr (L + 1 < pl.ne) enc_layer<L + 1>(st);
    }

    // encoder + the merged head GEMM (Z_h in S2); st(slot): diagnostic phase
    // stamps of the learner's stamped build (a no-op elsewhere)
    template <class F = void (*)(int)>
    __device__ __forceinline__ void trunk(F st = [](int) {}) {
        enc_layer<0>(st);
        gemm_fwd<pl.l_s1, pl.ld_s, pl.lat, pl.l_hw, pl.l_hld, pl.l_hb, pl.H>();
        __syncthreads();
    }

    __device__ __forceinline__ void run() {
        trunk();
        ln_rows<pl.H, pl.ha, pl.l_xh, pl.ld_xh, pl.l_rh, pl.l_hg, pl.l_hbe, true>();  // + output layers
        __syncthreads();
    }
};

template <class C, int B>
__device__ __forceinline__ void blk_copy(float *sm, const float *gp, int tid) {
    constexpr LearnPlan pl = C::plan;
    if constexpr (B < pl.nblk) {
        constexpr Blk k = pl.blk[B];
#pragma unroll 4
        for (int i = tid; i < k.len; i += kNT) sm[k.l0 + (i / k.rowlen) * k.ldst + i % k.rowlen] = gp[k.f0 + i];
        blk_copy<C, B + 1>(sm, gp, tid);
    }
}

template <class C>
__device__ __forceinline__ void load_params(float *sm, const float *gp, int tid) {
    // block by block (compile-time table): one division by a constant row
    // length per element instead of a search over all blocks
    blk_copy<C, 0>(sm, gp, tid);
}

struct LearnArgs {
    float *params, *m, *v;
    const float *lr;
    float b1, b2, eps;
    long long *step;       // [P] Adam steps taken (in/out)
    const float *gobs;     // [E][P][S][D] minibatch-ordered
    const int *gact;       // [E][P][S]
    const unsigned *gmask; // [E][P][S] legal-action bitmask, or null (no masks)
    const float *grow;     // [E][P][4][S]: old_logp, adv_norm, ret, old_v
    long long S;
    int E, B, P;
    float clip, vf, ent, max_norm;
    double target_kl;      // <= 0: no early stop
    const int *batch_p;    // [P] per-agent minibatch size, or null (B)
    const int *epochs_p;   // [P] per-agent update epochs (<= E), or null (E)
    const float *ent_p;    // [P] per-agent entropy coefficient, or null (ent)
    float *loss_out, *kl_out;
    int *epochs_out;
    unsigned *err;         // sticky error word (partner timeout)
    long long *stamps;
    int K;                 // workgroups per agent (data-parallel over sub-batches)
    int Q;                 // agent stride of the block index (>= P; blocks with b % Q >= P exit)
    float *slabs;          // [P][2][K][slab] gradient hand-off (double-buffered)
    float *sums;           // [P][2][slab] reduce-scattered gradient sums (double-buffered)
    unsigned *cnt;         // [P] arrival counters, [P] timeout word, [P+1+p] second-barrier,
                           // [2P+1+p] setup-barrier counters, [3P+1 + p*kMaxK + kk] XCC ids,
                           // [3P+1 + P*kMaxK + p] third-barrier (parameter hand-off) counters
                           // (zeroed per call)
    int debug_stall;       // test hook: partner 1 of agent 0 never arrives
    int write_through;     // 1: always sc1 stores (AGX_LEARN_WRITETHROUGH=1; tests the cross-XCD form)
    const unsigned *skip;  // non-null and nonzero when the learner starts: return untouched
};

#define IC(x) std::integral_constant<int, (x)>()
#define BC(x) std::integral_constant<bool, (x)>()

constexpr unsigned kSpinMax = 1u << 23;  // ~ seconds of s_sleep polling: a missing partner is a bug

// phase stamps go to LDS (a global store would sit in vmcnt and every
// s_waitcnt vmcnt(0) after it would wait for its write); flushed at the end
#define AGX_STAMP(slot)                                                          \
    do {                                                                         \
        if constexpr (ST)                                                        \
            if (b == 0 && e == (Ep > 1) && mb == (nmb > 1) && tid == 0 && (slot) < 80) \
                reinterpret_cast<long long *>(sm + pl.l_stamp)[(slot)] = (long long)__builtin_readcyclecounter(); \
    } while (0)

// ---------------------------------------------------------------------------
// learner
// ---------------------------------------------------------------------------
// JN > 0: every partner owns at most JN float4 chunk rounds (kNT chunks each) —
// with 8 partners one round, and the per-slot Adam / norm code is instantiated
// for that round only (a smaller kernel body); JN = 0: any split (K = 1 owns all)
// ST: the diagnostic build with phase stamps (agx_debug_learn_stamps; the bench
// shape only) — the product kernel carries no stamp code
template <class C, int SB, int JN = 0, bool ST = false>
__global__ __launch_bounds__(kNT, 1) void ppo_learn_kernel(LearnArgs g) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr LearnPlan pl = C::plan;
    // partners per agent this instantiation handles: 16 with 8-row sub-batches,
    // else 8 (the register arrays of the exchange are sized by it)
    constexpr int KM = SB == 8 ? kMaxK : 8;
    // block b -> agent b % Q, partner kk = b / Q with Q = P rounded up to a
    // multiple of the 8 XCDs (partners only): under round-robin dispatch an
    // agent's K workgroups then share one XCD (and its L2) for every P, the
    // strong-scaling shards P = 1, 2, 4 included; padding blocks exit at once
    // an aborted / timed-out rollout queued ahead of this learn leaves its
    // control word set: the partial rollout must not update anything
    if (g.skip && __hip_atomic_load(g.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    const int b = blockIdx.x;
    const int p = b % g.Q, kk = b / g.Q;
    if (p >= g.P) return;
    const int tid = threadIdx.x;
    float *gp = in_vgpr(g.params + (size_t)p * pl.n);
    float *gm = in_vgpr(g.m + (size_t)p * pl.n);
    float *gv = in_vgpr(g.v + (size_t)p * pl.n);
    // cold arguments (timeout path, per-epoch test, end-of-learn outputs) in VGPRs
    unsigned *const err_v = in_vgpr(g.err);
    unsigned *const tmo_v = in_vgpr(g.cnt + g.P);
    float *const loss_out_v = in_vgpr(g.loss_out);
    float *const kl_out_v = in_vgpr(g.kl_out);
    int *const epochs_out_v = in_vgpr(g.epochs_out);
    long long *const step_v = in_vgpr(g.step + p);
    double tkl_v = g.target_kl;
    asm volatile("" : "+v"(tkl_v));
    const long long S = g.S;
    Fwd<C, SB> fw{sm};

    for (int i = tid; i < pl.lds_floats; i += kNT) sm[i] = 0.f;
    __syncthreads();
    load_params<C>(sm, gp, tid);
    // Parameter ownership (Adam is distributed over the partners): partner kk
    // owns the float4 chunks [oc0, oc1) of the LDS parameter image + loss chunk
    // (n4s chunks split K ways); thread tid owns chunks oc0 + tid + kNT*j of it,
    // i.e. slot i is float (i & 3) of chunk oc0 + tid + kNT*(i >> 2).  K == 1:
    // every chunk, thread t owning t, t + kNT, ...
    constexpr int n4 = pl.param_end / 4, n4s = n4 + 1;
#if AGX_LEARN_UNIFORM
    // uniform chunks of cs = ceil(n4s / K): chunk c belongs to partner c / cs,
    // which the parameter hand-off computes per chunk without a table
    const int cs = (n4s + g.K - 1) / g.K;
    int oc0 = kk * cs < n4s ? kk * cs : n4s, oc1 = oc0 + cs < n4s ? oc0 + cs : n4s;
    const float inv_cs = 1.f / (float)cs;  // c / cs = floor((c + 0.5) * inv_cs) exactly for c < 2^16
#else
    int oc0 = n4s * kk / g.K, oc1 = n4s * (kk + 1) / g.K;
#endif
    int pc1 = oc1 < n4 ? oc1 : n4;  // own parameter chunks [oc0, pc1)
    constexpr int kUsed4 = JN > 0 ? JN : (n4 + kNT - 1) / kNT;  // owned chunk rounds per thread, at most
    static_assert(pl.param_end % 4 == 0 && pl.slab >= pl.param_end + 4 + 2 * kNW * kMaxK, "sum slab layout");
    static_assert(4 * kUsed4 <= kMaxPT, "owned slots");
    auto own_c = [&](int j) { return oc0 + vtid() + kNT * j; };
    // owned chunk rounds: a block-uniform trip count (1 with 8 partners), so the
    // unrolled per-slot loops below skip the rounds no thread owns
    const int jn_own = __builtin_amdgcn_readfirstlane((oc1 - oc0 + kNT - 1) / kNT);
    // the bounds only enter per-lane index math: VGPRs (not spilled SGPR pairs)
    asm volatile("" : "+v"(oc0), "+v"(oc1), "+v"(pc1));
    // Adam moments of the owned LDS parameter slots -> registers; group bits
    float am[kMaxPT], av[kMaxPT];
    unsigned gbits = 0, vbits = 0;
#pragma unroll
    for (int i = 0; i < kMaxPT; ++i) {
        if (i >= 4 * kUsed4) {
            am[i] = av[i] = 0.f;
            continue;
        }
        const int c = own_c(i >> 2), l = 4 * c + (i & 3);
        int grp = 0;
        const int f = c < pc1 ? lds_to_flat<C>(l, grp) : -1;
        am[i] = f >= 0 ? gm[f] : 0.f;
        av[i] = f >= 0 ? gv[f] : 0.f;
        if (f >= 0) vbits |= 1u << i;
        if (grp) gbits |= 1u << i;
    }
    // keep the ownership bits as plain VGPR data: left transparent, the compiler
    // re-materialises them as 60 live SGPR-pair lane masks (SGPR spills)
    asm volatile("" : "+v"(vbits), "+v"(gbits));
    __syncthreads();

    constexpr int nmb_dummy = 0;
    (void)nmb_dummy;
    // per-agent hyperparameters (HPO mutations, mutation.py:413-453) or the population's
    const int Bp = g.batch_p ? g.batch_p[p] : g.B;
    const int Ep = g.epochs_p ? g.epochs_p[p] : g.E;
    const float entp = g.ent_p ? g.ent_p[p] : g.ent;
    const int nmb = (int)((S + Bp - 1) / Bp);
    float loss_total = 0.f;
    double kl_total = 0.0;  // sum of per-minibatch approx_kl (np.mean over all minibatches so far, ppo.py:917)
    int n_done = 0, epochs_done = 0;
    const long long step0 = *step_v;
    double pb1 = pow((double)g.b1, (double)step0), pb2 = pow((double)g.b2, (double)step0);
    const float lr_p = g.lr[p];
    float *rowf = sm + pl.l_row;  // [4][SB]: old_logp, adv, ret, old_v
    float *stat = sm + pl.l_stat;
    int *acts = reinterpret_cast<int *>(sm + pl.l_row + 4 * kSB);
    unsigned *legal = reinterpret_cast<unsigned *>(sm + pl.l_row + 5 * kSB);
    if (g.debug_stall && p == 0 && kk == 1) return;  // test hook: a partner that never arrives

    // one thread's share of a sub-batch's inputs: obs words (the SB x D real
    // columns, contiguous in the minibatch-ordered rows; the padding columns of
    // the LDS x0 image are zero-filled on commit) and one row word
    // (old_logp/adv/ret/old_v, action or legal mask)
    constexpr int kPreObs = (SB * pl.D + kNT - 1) / kNT;
    constexpr bool kPrefetch = kPreObs == 1;  // carried in registers across the update
    struct Pre {
        int e, mb, sb;
        float ob[kPreObs];
        unsigned rv;
    };
    // Every load is unconditional from an always-valid address (rows beyond the
    // sub-batch read row 0 of the (epoch, agent) block) and the row predicates
    // are applied on commit: a zero-then-masked-load form makes the next write
    // of those registers wait (vmcnt) for the prefetch just issued.
    // per-thread pointers of this thread's words at epoch 0 (VGPRs) and their
    // per-epoch strides: threads < 4*kSB one row of old_logp/adv/ret/old_v, then
    // the actions, then the legal-action masks (actions again without masks)
    const bool has_mask = g.gmask != nullptr;
    const int tid0 = vtid();
    const int rw_rr = tid0 < 4 * kSB ? tid0 % kSB : (tid0 < 5 * kSB ? tid0 - 4 * kSB : tid0 - 5 * kSB);
    const bool rw_on = tid0 < 6 * kSB;
    const unsigned *rw0 = in_vgpr(tid0 < 4 * kSB ? reinterpret_cast<const unsigned *>(g.grow) + ((size_t)p * 4 + tid0 / kSB) * S
                                  : (tid0 < 5 * kSB || !has_mask) ? reinterpret_cast<const unsigned *>(g.gact) + (size_t)p * S
                                                                   : g.gmask + (size_t)p * S);
    const size_t rw_es = (size_t)g.P * S * (tid0 < 4 * kSB ? 4 : 1);
    const float *ob0 = in_vgpr(g.gobs + (size_t)p * S * pl.D);
    const size_t ob_es = (size_t)g.P * S * pl.D;
    auto fetch = [&](int e_, int mb_, int sb_) {
        Pre r;
        r.e = e_;
        r.mb = mb_;
        r.sb = sb_;
        const int tid = vtid();
        const long long s0_ = (long long)mb_ * Bp;
        const int bsz_ = (int)((s0_ + Bp <= S) ? Bp : S - s0_);
        const int nrow_ = e_ >= Ep ? 0 : (bsz_ - sb_ < SB ? bsz_ - sb_ : SB);
        const size_t ee = (size_t)(e_ < Ep ? e_ : 0);
        const size_t row0 = (size_t)(s0_ + sb_);
        const float *eo = ob0 + ee * ob_es;
#pragma unroll
        for (int k = 0; k < kPreObs; ++k) {
            const int i = tid + k * kNT;
            r.ob[k] = eo[i < nrow_ * pl.D ? row0 * pl.D + i : 0];
        }
        r.rv = rw0[ee * rw_es + ((rw_on && rw_rr < nrow_) ? row0 + rw_rr : 0)];
        return r;
    };
    Pre pre{};
    if constexpr (kPrefetch) pre = fetch(0, 0, kk * SB);

    // Partners that share one XCD share its L2: plain stores (the line stays in
    // that L2) + sc1 loads (L1 bypassed) hand data over without the write-through
    // to memory that sc1 stores cost.  Placement is not guaranteed, so it is
    // checked here: each workgroup publishes HW_REG_XCC_ID and, after one setup
    // barrier, uses the L2-local form only if all K ids agree.
    bool local = false;
    if (g.K > 1) {
        unsigned *xc = g.cnt + 3 * g.P + 1 + (size_t)p * kMaxK;
        if (tid == 0) {
            int x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            __hip_atomic_store(xc + kk, (unsigned)(x & 15) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned *ctr = g.cnt + 2 * g.P + 1 + p;
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned spins = 0;
            int ok = 1;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)g.K) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinMax) {
                    __hip_atomic_store(tmo_v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (err_v) __hip_atomic_fetch_or(err_v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
            stat[4 * kNW] = ok ? 1.f : 0.f;
        }
        __syncthreads();
        if (stat[4 * kNW] == 0.f) return;
        const int ln = vlane();
        const unsigned v = ln < g.K ? __hip_atomic_load(xc + ln, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned v0 = __builtin_amdgcn_readlane(v, 0);
        bool same = v0 != 0u;
        for (int q = 1; q < g.K; ++q) same = same && __builtin_amdgcn_readlane(v, q) == v0;
        local = same && !g.write_through;
    }

    // this agent's slab / sum slab pairs and barrier counters (VGPR-held, see in_vgpr)
    float *slab_p = in_vgpr(g.slabs + (g.K > 1 ? (size_t)p * 2 * g.K * pl.slab : 0));
    float *sum_p = in_vgpr(g.sums + (g.K > 1 ? (size_t)p * 2 * pl.slab : 0));
    unsigned *ctr1 = in_vgpr(g.cnt + p);
    unsigned *ctr2 = in_vgpr(g.cnt + g.P + 1 + p);
    unsigned *ctr3 = in_vgpr(g.cnt + 3 * g.P + 1 + (size_t)g.P * kMaxK + p);
    for (int e = 0; e < Ep; ++e) {
        for (int mb = 0; mb < nmb; ++mb) {
            const long long s0 = (long long)mb * Bp;
            const int bsz = (int)((s0 + Bp <= S) ? Bp : S - s0);
            const float inv_b = 1.f / (float)bsz;
            const int tid = vtid();
            f4 acc[kMaxSlot];
#pragma unroll
            for (int s = 0; s < kMaxSlot; ++s) acc[s] = f4{0.f, 0.f, 0.f, 0.f};
            for (int i = tid; i < pl.l_stat - pl.l_red; i += kNT) sm[pl.l_red + i] = 0.f;
            float lsum = 0.f, klsum = 0.f;
            // this update's gradient slabs (double-buffered by update parity)
            const int upd = e * nmb + mb;
            float *base = g.K > 1 ? to_sgpr(slab_p + (size_t)(upd & 1) * g.K * pl.slab) : nullptr;
            const auto slab_rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)kk * pl.slab, 0,
                                                                     __builtin_amdgcn_readfirstlane(pl.slab * 4),
                                                                     0x00020000);
            // dW tiles of group gg -> fn(LDS-image offset, value) (padding columns skipped)
            auto emit_tiles = [&](auto gc, auto fn) {
                constexpr int gg = decltype(gc)::value;
                AGX_IDS;
#pragma unroll
                for (int j = 0; j < pl.nslot[gg]; ++j) {
                    const int t = wave + kNW * j;
                    if (t < pl.nt[gg]) {
                        const int o0 = (t / pl.ncol[gg]) * 16, i0 = (t % pl.ncol[gg]) * 16;
                        const int col = i0 + lr16;
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int o = o0 + lq * 4 + i;
                            const float x = acc[pl.slot0[gg] + j][i];
                            if constexpr (gg < pl.ne) {
                                if (col < pl.ein[gg]) fn(pl.l_ew[gg] + o * pl.l_eld[gg] + col, x);
                            } else if constexpr (gg == pl.ne) {
                                fn(pl.l_hw + o * pl.l_hld + col, x);
                            } else if constexpr (gg == pl.ne + 1) {
                                if (o < pl.A) {
                                    if (col < pl.ha) fn(pl.l_aow + o * pl.l_aold + col, x);
                                    else if (col == pl.ha) fn(pl.l_aob + o, x);
                                }
                            } else {
                                if (o == 0) {
                                    if (col < pl.hc) fn(pl.l_cow + col, x);
                                    else if (col == pl.hc) fn(pl.l_cob, x);
                                }
                            }
                        }
                    }
                }
            };
            // write-through (sc1) store of one gradient word into this workgroup's slab
            // (plain store when the partners share this XCD's L2, else write-through)
            auto put_l = [&](int l, float x) {
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), slab_rsrc, l * 4, 0, 0);
            };
            auto put_w = [&](int l, float x) {
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), slab_rsrc, l * 4, 0, 16);
            };
            auto slab_put = [&](int l, float x) {
                if (local) put_l(l, x);
                else put_w(l, x);
            };
            // a group's dW tiles -> the slab: the store form is chosen once per group
            // (the cache-policy operand is an immediate; a branch per store cost
            // ~90 scalar branches per update)
            auto emit_slab = [&](auto gc) {
                if (local) emit_tiles(gc, put_l);
                else emit_tiles(gc, put_w);
            };
            // this agent's summed-gradient slab (written by the reduce-scatter)
            const auto sum_rsrc = __builtin_amdgcn_make_buffer_rsrc(
                g.K > 1 ? to_sgpr(sum_p + (size_t)(upd & 1) * pl.slab) : nullptr, 0,
                __builtin_amdgcn_readfirstlane(pl.slab * 4), 0x00020000);
            // Partner barrier (MI355X_MICROARCH visibility rules): every wave drains its
            // write-through (sc1) stores (vmcnt) -> workgroup barrier -> one relaxed
            // agent-scope ticket; relaxed poll with s_sleep -> barrier -> readers use
            // sc1 loads (no fences, cdna_hip_programming.md §6 G16 R1).  Bounded: on
            // timeout the timeout word and the caller's error word are set and the
            // caller's whole block exits.
            auto partner_sync = [&](unsigned *ctr, unsigned target, int st0, int st1) -> bool {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                const int tid = vtid();
                if (tid == 0) {
                    // the last partner to arrive learns it from its own ticket: no
                    // poll round trip on the critical path of the hand-off
                    const unsigned before = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    AGX_STAMP(st0);
                    unsigned spins = 0;
                    int ok = 1;
                    while (before + 1u < target &&
                           __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinMax) {
                            __hip_atomic_store(tmo_v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (err_v) __hip_atomic_fetch_or(err_v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            ok = 0;
                            break;
                        }
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    stat[4 * kNW] = ok ? 1.f : 0.f;
                    AGX_STAMP(st1);
                }
                __syncthreads();
                return stat[4 * kNW] != 0.f;
            };
            // partners publish each group's dW straight from registers as soon as the
            // group is final (last sub-batch), overlapping the stores with the rest of
            // the backward pass
            const bool direct = g.K > 1;

            for (int sb = kk * SB; sb < bsz; sb += g.K * SB) {
                const bool last_sb = sb + g.K * SB >= bsz;
                const int nrow = bsz - sb < SB ? bsz - sb : SB;
                const int jsb = (sb / SB) / g.K;
                const int stb = jsb < 4 ? jsb * 16 : 80;
                const int tid = vtid();
                AGX_STAMP(stb + 0);
                // ---- P0: the sub-batch -> LDS (prefetched into registers during the
                // previous sub-batch; fetched here only when the prefetch guessed
                // another one).  Then the next sub-batch in this partner's sequence is
                // prefetched: its loads fly under this sub-batch's compute.
                // (padding columns rewritten too: the gradient image aliases them)
                {
                    auto commit = [&](const Pre &x) {
                        // the prefetch landed during the previous update (nothing is
                        // outstanding here): an explicit vmcnt(0) the waitcnt pass sees,
                        // so the commit's reads of the prefetch registers do not wait
                        // on the next prefetch's loads (memory ops stay ordered after it)
                        __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
                        for (int k = 0; k < kPreObs; ++k) {
                            const int i = tid + k * kNT;
                            if (i < SB * pl.D) sm[pl.l_x0 + (i / pl.D) * pl.ld_x0 + i % pl.D] = i < nrow * pl.D ? x.ob[k] : 0.f;
                        }
                        constexpr int npad = pl.ld_x0 - pl.D;
#pragma unroll
                        for (int k = 0; k < (SB * npad + kNT - 1) / kNT; ++k) {
                            const int i = tid + k * kNT;
                            if (i < SB * npad) sm[pl.l_x0 + (i / npad) * pl.ld_x0 + pl.D + i % npad] = 0.f;
                        }
                        if (tid < 4 * kSB) rowf[tid] = tid % kSB < nrow ? __builtin_bit_cast(float, x.rv) : 0.f;
                        else if (tid < 5 * kSB) acts[tid - 4 * kSB] = tid - 4 * kSB < nrow ? (int)x.rv : 0;
                        else if (tid < 6 * kSB) legal[tid - 5 * kSB] = (has_mask && tid - 5 * kSB < nrow) ? x.rv : 0xffffffffu;
                    };
                    if constexpr (!kPrefetch) {  // wide observations: registers too tight to carry
                        commit(fetch(e, mb, sb));
                    } else {
                        if (pre.e != e || pre.mb != mb || pre.sb != sb) pre = fetch(e, mb, sb);
                        commit(pre);
                        AGX_STAMP(stb + 4);
                        int ne = e, nm = mb, ns = sb + g.K * SB;
                        if (ns >= bsz) {
                            ns = kk * SB;
                            if (++nm >= nmb) {
                                nm = 0;
                                ++ne;
                            }
                        }
                        pre = fetch(ne, nm, ns);
                        AGX_STAMP(stb + 5);
                    }
                }
                __syncthreads();
                AGX_STAMP(stb + 1);

                // ---- P1-P3: forward trunk (encoder + merged head GEMM) ------------
                fw.trunk([&](int k) { AGX_STAMP(stb + k); });
                AGX_STAMP(stb + 2);

                // ---- P4: ONE row pass over the head (W lanes per row, nothing leaves
                // the row's registers): LayerNorm(+affine)+ReLU forward, the output
                // layers (logits, value), the loss and d(logits) / d(value), and the
                // LayerNorm backward to dZ_h (S2) with the bias / LN-affine column sums.
                // y_h goes to S1 and d(logits) / d(value) to LDS for the output-layer dW.
                // 16-row sub-batches use 32 lanes per row (2 rows per wave, every lane
                // busy, half the per-lane columns: the pass is VALU-issue bound); the
                // row sums then add the other 16-lane half by ds_swizzle (lane ^ 16).
                {
                    // 8-row sub-batches: 64 lanes per row (one row per wave)
                    constexpr int W = (SB == 8 && pl.H % 64 == 0 && pl.ha % 64 == 0)
                                          ? 64
                                          : ((SB <= 16 && pl.H % 32 == 0 && pl.ha % 32 == 0) ? 32 : 16);
                    const int lane = vlane(), wave = swave();
                    const int sub = lane & (W - 1);
                    const int r = wrow<W>(lane, wave);
                    constexpr int F = pl.H, split = pl.ha, NC = F / W, NA = pl.A;
                    constexpr int F0 = split, F1 = F - split;
                    const int a = sub;
                    auto swz16 = [](float v) {
                        return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401f));
                    };
                    auto rsum = [&](float v) { return wrow_sum<W>(v); };
                    auto rmax = [&](float v) { return wrow_max<W>(v); };
                    // rows beyond the sub-batch (W-lane rows past SB) compute on zeros
                    // and contribute exact zeros to the column reductions
                    const bool rl = r < SB;
                    const bool live = rl && r < nrow;
                    float z[NC], xh[NC];
                    float s0 = 0.f, s1 = 0.f;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        z[i] = rl ? sm[pl.l_s2 + r * pl.ld_s + sub + W * i] : 0.f;
                        if (W * i < split) s0 += z[i];
                        else s1 += z[i];
                    }
                    const float m0 = rsum(s0) * (1.f / (float)F0);
                    const float m1 = rsum(s1) * (1.f / (float)F1);
                    float v0 = 0.f, v1 = 0.f;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        if (W * i < split) v0 += (z[i] - m0) * (z[i] - m0);
                        else v1 += (z[i] - m1) * (z[i] - m1);
                    }
                    const float r0 = 1.f / sqrtf(rsum(v0) / (float)F0 + 1e-5f);
                    const float r1 = 1.f / sqrtf(rsum(v1) / (float)F1 + 1e-5f);
                    float pa[NA], pv = 0.f;
#pragma unroll
                    for (int k = 0; k < NA; ++k) pa[k] = 0.f;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        const int j = sub + W * i;
                        xh[i] = W * i < split ? (z[i] - m0) * r0 : (z[i] - m1) * r1;
                        const float y = relu(xh[i] * sm[pl.l_hg + j] + sm[pl.l_hbe + j]);
                        if (rl) sm[pl.l_s1 + r * pl.ld_s + j] = y;
                        if (W * i < split) {
#pragma unroll
                            for (int k = 0; k < NA; ++k) pa[k] += y * sm[pl.l_aow + k * pl.l_aold + j];
                        } else {
                            pv += y * sm[pl.l_cow + j - split];
                        }
                    }
                    float mine = 0.f;
#pragma unroll
                    for (int k = 0; k < NA; ++k) {
                        const float t = rsum(pa[k]);
                        mine = sub == k ? t : mine;
                    }
                    const float v = rsum(pv) + sm[pl.l_cob];
                    // loss + d(logits), d(value) (ppo.py:876-908); illegal actions:
                    // logits -> -1e8 (apply_action_mask_discrete, distributions.py:16-28)
                    const bool ok_a = (legal[rl ? r : 0] >> a) & 1u;
                    const float lg = a < NA ? (ok_a ? mine + sm[pl.l_aob + sub] : -1.0e8f) : -3.0e38f;
                    const float mx = rmax(lg);
                    const float ex = a < NA ? expf(lg - mx) : 0.f;
                    const float lse = mx + logf(rsum(ex));
                    const float pa_ = a < NA ? expf(lg - lse) : 0.f;
                    const float lpe = logf(pa_ + 1e-8f);
                    const float Hs = -rsum(a < NA ? pa_ * lpe : 0.f);  // H = -sum p log(p+1e-8)
                    const float gh = -(lpe + pa_ / (pa_ + 1e-8f));          // dH/dp_a
                    const float pg_dot = rsum(a < NA ? pa_ * gh : 0.f);
                    const int a_t = acts[rl ? r : 0];
                    const float logp = __builtin_bit_cast(
                                           float, __builtin_amdgcn_ds_bpermute((lane - sub + a_t) * 4,
                                                                               __builtin_bit_cast(int, lg))) -
                                       lse;
                    const int rr = rl ? r : 0;
                    const float olp = rowf[rr], A = rowf[kSB + rr], R = rowf[2 * kSB + rr], ov = rowf[3 * kSB + rr];
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
                    const float g_H = -entp * inv_b;
                    const float dl = g_logp * ((a == a_t ? 1.f : 0.f) - pa_) + g_H * pa_ * (gh - pg_dot);
                    const float dlm = (a < NA && live && ok_a) ? dl : 0.f;
                    const float dvr = live ? g.vf * 0.5f * inv_b * (gu * 2.f * eu + gc * 2.f * ec * inv) : 0.f;
                    if (rl) {
                        if (a < NA) sm[pl.l_dlg + r * kMaxA + a] = dlm;
                        if (a == 0) sm[pl.l_dvb + r * kMaxA] = dvr;
                    }
                    if (a == 0 && live) {
                        lsum += (fmaxf(p1, p2) + g.vf * 0.5f * fmaxf(lu, lc) - entp * Hs) * inv_b;
                        klsum += ((ratio - 1.f) - lrt) * inv_b;  // approx_kl (ppo.py:899-902)
                    }
                    // LayerNorm backward: dY[j] = sum_a dlg[a] W_out[a][j] (actor columns)
                    // or dv w_v[j] (critic columns)
                    float dla[NA];
#pragma unroll
                    for (int k = 0; k < NA; ++k)
                        dla[k] = __builtin_bit_cast(
                            float, __builtin_amdgcn_ds_bpermute((lane - sub + k) * 4, __builtin_bit_cast(int, dlm)));
                    float dxh[NC], dyp[NC];
                    float a1 = 0.f, a2 = 0.f, c1 = 0.f, c2 = 0.f;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        const int j = sub + W * i;
                        float dy;
                        if (W * i < split) {
                            dy = 0.f;
#pragma unroll
                            for (int k = 0; k < NA; ++k) dy += dla[k] * sm[pl.l_aow + k * pl.l_aold + j];
                        } else {
                            dy = dvr * sm[pl.l_cow + j - split];
                        }
                        xh[i] = rl ? xh[i] : 0.f;
                        const float gam = sm[pl.l_hg + j];
                        const float y = xh[i] * gam + sm[pl.l_hbe + j];
                        dyp[i] = y > 0.f ? dy : 0.f;
                        dxh[i] = dyp[i] * gam;
                        if (W * i < split) {
                            a1 += dxh[i];
                            a2 += dxh[i] * xh[i];
                        } else {
                            c1 += dxh[i];
                            c2 += dxh[i] * xh[i];
                        }
                    }
                    const float rs0 = rl ? r0 : 0.f, rs1 = rl ? r1 : 0.f;
                    const float ma1 = rsum(a1) * (1.f / (float)F0), ma2 = rsum(a2) * (1.f / (float)F0);
                    const float mc1 = rsum(c1) * (1.f / (float)F1), mc2 = rsum(c2) * (1.f / (float)F1);
                    float *rd = sm + pl.l_red + pl.red_h;
                    float cs[3][NC];
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        const int j = sub + W * i;
                        const bool g0 = W * i < split;
                        const float dz = (g0 ? rs0 : rs1) * (dxh[i] - (g0 ? ma1 : mc1) - xh[i] * (g0 ? ma2 : mc2));
                        if (rl) sm[pl.l_s2 + r * pl.ld_s + j] = dz;
                        cs[0][i] = rl ? dz : 0.f;
                        cs[1][i] = dyp[i] * xh[i];
                        cs[2][i] = dyp[i];
                    }
                    if constexpr (W == 16) {  // the two rows of a 32-lane group
#pragma unroll
                        for (int k = 0; k < 3; ++k)
#pragma unroll
                            for (int i = 0; i < NC; ++i) cs[k][i] += swz16(cs[k][i]);  // lane ^ 16
                    }
                    if constexpr (W == 32 || (W == 16 && SB > 16)) {  // rows in lanes 32-63 too
#pragma unroll
                        for (int k = 0; k < 3; ++k)
#pragma unroll
                            for (int i = 0; i < NC; ++i)
                                cs[k][i] += __builtin_bit_cast(
                                    float, __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, __builtin_bit_cast(int, cs[k][i])));
                    }
                    if (lane < W) {
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            float o[NC];
#pragma unroll
                            for (int i = 0; i < NC; ++i) o[i] = rd[(k * kNW + wave) * F + sub + W * i];
#pragma unroll
                            for (int i = 0; i < NC; ++i) rd[(k * kNW + wave) * F + sub + W * i] = o[i] + cs[k][i];
                        }
                    }
                }
                __syncthreads();
                AGX_STAMP(stb + 3);

                // backward row pass through LN(+affine)+ReLU of an encoder layer:
                // dY (dyb, stride ldy) -> dZ (S2)
                auto ln_bwd = [&](auto Fc, auto dybc, auto ldyc, auto xbc, auto ldxc, auto rbc, auto gbc, auto bbc,
                                  auto redc, auto affc) {
                    constexpr int F = decltype(Fc)::value;
                    constexpr int dyb = decltype(dybc)::value, ldy = decltype(ldyc)::value;
                    constexpr int xb = decltype(xbc)::value, ldx = decltype(ldxc)::value;
                    constexpr int rb = decltype(rbc)::value, gb = decltype(gbc)::value, bb = decltype(bbc)::value;
                    constexpr int red = decltype(redc)::value;
                    constexpr bool aff = decltype(affc)::value;
                    // 16-row sub-batches: 32 lanes per row, 8-row: 64 (as the forward pass)
                    constexpr int W = (SB == 8 && F % 64 == 0) ? 64 : ((SB <= 16 && F % 32 == 0) ? 32 : 16);
                    constexpr int NC = F / W;
                    const int lane = vlane(), wave = swave();
                    const int sub = lane & (W - 1);
                    const int r = wrow<W>(lane, wave);
                    // rows beyond the sub-batch hold stale LDS data: they contribute
                    // exact zeros to the column reductions
                    const bool rl = r < SB;
                    float xh[NC], dxh[NC], dyp[NC];
                    float a1 = 0.f, a2 = 0.f;
                    const float rs0 = rl ? sm[rb + 2 * r] : 0.f;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        const int j = sub + W * i;
                        const float dy = rl ? sm[dyb + r * ldy + j] : 0.f;
                        xh[i] = rl ? sm[xb + r * ldx + j] : 0.f;
                        const float gam = aff ? sm[gb + j] : 1.f;
                        const float y = aff ? xh[i] * gam + sm[bb + j] : xh[i];
                        dyp[i] = y > 0.f ? dy : 0.f;
                        dxh[i] = dyp[i] * gam;
                        a1 += dxh[i];
                        a2 += dxh[i] * xh[i];
                    }
                    const float ma1 = wrow_sum<W>(a1) * (1.f / (float)F), ma2 = wrow_sum<W>(a2) * (1.f / (float)F);
                    float *rd = sm + pl.l_red + red;
                    // dZ row pass; the column sums (bias, gamma, beta gradients) of the
                    // wave's rows are batched: all cross-row reductions, then all LDS
                    // loads of the per-wave accumulators, then all stores (one LDS
                    // round trip instead of a read-modify-write chain per column)
                    constexpr int NV = aff ? 3 : 1;
                    float cs[NV][NC];
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        const int j = sub + W * i;
                        const float dz = rs0 * (dxh[i] - ma1 - xh[i] * ma2);
                        if (rl) sm[pl.l_s2 + r * pl.ld_s + j] = dz;
                        cs[0][i] = rl ? dz : 0.f;
                        if constexpr (aff) {
                            cs[1][i] = dyp[i] * xh[i];
                            cs[2][i] = dyp[i];
                        }
                    }
                    if constexpr (W == 16) {  // the two rows of a 32-lane group
#pragma unroll
                        for (int k = 0; k < NV; ++k)
#pragma unroll
                            for (int i = 0; i < NC; ++i)
                                cs[k][i] += __builtin_bit_cast(
                                    float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, cs[k][i]), 0x401f));  // lane ^ 16
                    }
                    if constexpr (W == 32 || (W == 16 && SB > 16)) {  // rows in lanes 32-63 too
#pragma unroll
                        for (int k = 0; k < NV; ++k)
#pragma unroll
                            for (int i = 0; i < NC; ++i)
                                cs[k][i] += __builtin_bit_cast(
                                    float, __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, __builtin_bit_cast(int, cs[k][i])));
                    }
                    if (lane < W) {
#pragma unroll
                        for (int k = 0; k < NV; ++k) {
                            float o[NC];
#pragma unroll
                            for (int i = 0; i < NC; ++i) o[i] = rd[(k * kNW + wave) * F + sub + W * i];
#pragma unroll
                            for (int i = 0; i < NC; ++i) rd[(k * kNW + wave) * F + sub + W * i] = o[i] + cs[k][i];
                        }
                    }
                };
                // ---- P6/P7: output-layer dW (bias = ones column; reads d(logits) /
                // d(value) and y_h), head dW += dZ^T latent, d(latent) = dZ . W_h ->
                // the dead head-xhat region (nothing in this phase reads it)
                {
                    AGX_IDS;
                    constexpr int ga = pl.ne + 1, gc = pl.ne + 2;
#pragma unroll
                    for (int j = 0; j < pl.nslot[ga]; ++j) {
                        const int t = wave + kNW * j;
                        if (t < pl.nt[ga]) {
                            const int i0 = (t % pl.ncol[ga]) * 16;
                            acc[pl.slot0[ga] + j] = mfma_tile<SB>(
                                acc[pl.slot0[ga] + j], [&](int m, int k) { return sm[pl.l_dlg + k * kMaxA + m]; },
                                [&](int k, int n) {
                                    // branch-free: a clamped load (a finite y) scaled to the
                                    // ones / zero columns (a select would be sunk into a branch)
                                    const int c = i0 + n;
                                    const float x = sm[pl.l_s1 + k * pl.ld_s + (c < pl.ha ? c : pl.ha - 1)];
                                    return x * (c < pl.ha ? 1.f : 0.f) + (c == pl.ha ? 1.f : 0.f);
                                });
                        }
                    }
#pragma unroll
                    for (int j = 0; j < pl.nslot[gc]; ++j) {
                        const int t = wave + kNW * j;
                        if (t < pl.nt[gc]) {
                            const int i0 = (t % pl.ncol[gc]) * 16;
                            acc[pl.slot0[gc] + j] = mfma_tile<SB>(
                                acc[pl.slot0[gc] + j], [&](int m, int k) { return sm[pl.l_dvb + k * kMaxA + m]; },
                                [&](int k, int n) {
                                    const int c = i0 + n;
                                    const float x = sm[pl.l_s1 + k * pl.ld_s + pl.ha + (c < pl.hc ? c : pl.hc - 1)];
                                    return x * (c < pl.hc ? 1.f : 0.f) + (c == pl.hc ? 1.f : 0.f);
                                });
                        }
                    }
                    if (direct && last_sb) {
                        emit_slab(IC(pl.ne + 1));
                        emit_slab(IC(pl.ne + 2));
                    }
                    constexpr int gh = pl.ne, Le = pl.ne - 1;
#pragma unroll
                    for (int j = 0; j < pl.nslot[gh]; ++j) {
                        const int t = wave + kNW * j;
                        if (t < pl.nt[gh]) {
                            const int o0 = (t / pl.ncol[gh]) * 16, i0 = (t % pl.ncol[gh]) * 16;
                            acc[pl.slot0[gh] + j] = mfma_tile<SB>(
                                acc[pl.slot0[gh] + j], [&](int m, int k) { return sm[pl.l_s2 + k * pl.ld_s + o0 + m]; },
                                [&](int k, int n) { return relu(sm[pl.l_xe[Le] + k * pl.ld_xe[Le] + i0 + n]); });
                        }
                    }
                    if (direct && last_sb) emit_slab(IC(gh));
                    constexpr int MT = m_tiles<SB>();
                    constexpr int nt = MT * (pl.lat / 16);
                    for (int t = wave; t < nt; t += kNW) {
                        const int m0 = (t % MT) * 16, n0 = (t / MT) * 16;
                        f4 c = f4{0.f, 0.f, 0.f, 0.f};
                        c = mfma_tile<pl.H>(c, [&](int m, int k) { return sm[pl.l_s2 + (m0 + m) * pl.ld_s + k]; },
                                            [&](int k, int n) { return sm[pl.l_hw + k * pl.l_hld + n0 + n]; });
                        if (SB >= 16 || lq * 4 < SB) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) sm[pl.l_xh + (m0 + lq * 4 + i) * pl.ld_xh + n0 + lr16] = c[i];
                        }
                    }
                }
                __syncthreads();
                AGX_STAMP(stb + 6);

                // ---- P8: encoder backward, last layer first ----------------------
                auto enc_bwd = [&](auto Lc) {
                    constexpr int L = decltype(Lc)::value;
                    constexpr int fin = pl.ein[L], fout = pl.eout[L];
                    AGX_IDS;
                    constexpr int dyb = L == pl.ne - 1 ? pl.l_xh : pl.l_s1;
                    constexpr int ldy = L == pl.ne - 1 ? pl.ld_xh : pl.ld_s;
                    ln_bwd(IC(fout), IC(dyb), IC(ldy), IC(pl.l_xe[L]), IC(pl.ld_xe[L]), IC(pl.l_re[L]), IC(pl.l_eg[L]),
                           IC(pl.l_ebe[L]), IC(pl.red_e[L]), BC(pl.eaff[L] != 0));
                    __syncthreads();
                    constexpr bool in_aff = L > 0 && pl.eaff[L > 0 ? L - 1 : 0];
                    constexpr int xb = L == 0 ? pl.l_x0 : pl.l_xe[L > 0 ? L - 1 : 0];
                    constexpr int ldx = L == 0 ? pl.ld_x0 : pl.ld_xe[L > 0 ? L - 1 : 0];
                    constexpr int gbase = L > 0 ? pl.l_eg[L > 0 ? L - 1 : 0] : 0;
                    constexpr int bbase = L > 0 ? pl.l_ebe[L > 0 ? L - 1 : 0] : 0;
#pragma unroll
                    for (int j = 0; j < pl.nslot[L]; ++j) {
                        const int t = wave + kNW * j;
                        if (t < pl.nt[L]) {
                            const int o0 = (t / pl.ncol[L]) * 16, i0 = (t % pl.ncol[L]) * 16;
                            const int col = i0 + lr16;
                            const bool cv = col < fin;
                            const float gam = (in_aff && cv) ? sm[gbase + col] : 1.f;
                            const float bet = (in_aff && cv) ? sm[bbase + col] : 0.f;
                            acc[pl.slot0[L] + j] = mfma_tile<SB>(
                                acc[pl.slot0[L] + j], [&](int m, int k) { return sm[pl.l_s2 + k * pl.ld_s + o0 + m]; },
                                [&](int k, int n) {
                                    const float x = sm[xb + k * ldx + i0 + n];
                                    if constexpr (L == 0) return x;
                                    else return cv ? relu(x * gam + bet) : 0.f;
                                });
                        }
                    }
                    if (direct && last_sb) emit_slab(IC(L));
                    if constexpr (L > 0) {
                        constexpr int MT = m_tiles<SB>();
                        constexpr int nt = MT * (fin / 16);
                        for (int t = wave; t < nt; t += kNW) {
                            const int m0 = (t % MT) * 16, n0 = (t / MT) * 16;
                            f4 c = f4{0.f, 0.f, 0.f, 0.f};
                            c = mfma_tile<fout>(c, [&](int m, int k) { return sm[pl.l_s2 + (m0 + m) * pl.ld_s + k]; },
                                                [&](int k, int n) { return sm[pl.l_ew[L] + k * pl.l_eld[L] + n0 + n]; });
                            if (SB >= 16 || lq * 4 < SB) {
#pragma unroll
                                for (int i = 0; i < 4; ++i) sm[pl.l_s1 + (m0 + lq * 4 + i) * pl.ld_s + n0 + lr16] = c[i];
                            }
                        }
                    }
                    __syncthreads();
                };
                if constexpr (pl.ne == 3) enc_bwd(IC(2));
                enc_bwd(IC(1));
                enc_bwd(IC(0));
                AGX_STAMP(stb + 7);
            }  // sub-batches

            // ---- P9: gradients -> the LDS image (K == 1) or the slab (partners) --
            float *G = sm + pl.l_grad;
            auto gput = [&](int l, float x) { G[l] = x; };
            if (!direct) {
                emit_tiles(IC(0), gput);
                emit_tiles(IC(1), gput);
                if constexpr (pl.ne == 3) emit_tiles(IC(2), gput);
                emit_tiles(IC(pl.ne), gput);
                emit_tiles(IC(pl.ne + 1), gput);
                emit_tiles(IC(pl.ne + 2), gput);
            } else if (kk * SB >= bsz) {  // no sub-batch this update: publish zeros
                emit_slab(IC(0));
                emit_slab(IC(1));
                if constexpr (pl.ne == 3) emit_slab(IC(2));
                emit_slab(IC(pl.ne));
                emit_slab(IC(pl.ne + 1));
                emit_slab(IC(pl.ne + 2));
            }
            // LN / bias vectors: fixed-order sums of the per-wave partials
            auto vdump = [&](auto Lc, auto put) {
                constexpr int L = decltype(Lc)::value;
                constexpr int F = L < pl.ne ? pl.eout[L < pl.ne ? L : 0] : pl.H;
                constexpr int nv = (L < pl.ne && !pl.eaff[L < pl.ne ? L : 0]) ? 1 : 3;
                constexpr int red = L < pl.ne ? pl.red_e[L < pl.ne ? L : 0] : pl.red_h;
                const int tid = vtid();
                // compile-time rounds; all kNW partial loads issued before the
                // fixed-order sum (a load-add chain waited on every LDS round trip)
#pragma unroll
                for (int rnd = 0; rnd < (nv * F + kNT - 1) / kNT; ++rnd) {
                    const int idx = tid + rnd * kNT;
                    if (idx >= nv * F) break;
                    const int k = idx / F, j = idx % F;
                    float pv[kNW];
#pragma unroll
                    for (int w = 0; w < kNW; ++w) pv[w] = sm[pl.l_red + red + (k * kNW + w) * F + j];
                    float x = 0.f;
#pragma unroll
                    for (int w = 0; w < kNW; ++w) x += pv[w];
                    int l;
                    if constexpr (L < pl.ne) {
                        l = (k == 0 ? pl.l_eb[L < pl.ne ? L : 0] : (k == 1 ? pl.l_eg[L < pl.ne ? L : 0] : pl.l_ebe[L < pl.ne ? L : 0])) + j;
                    } else {
                        l = (k == 0 ? pl.l_hb : (k == 1 ? pl.l_hg : pl.l_hbe)) + j;
                    }
                    put(l, x);
                }
            };
            auto vdump_all = [&](auto put) {
                vdump(IC(0), put);
                vdump(IC(1), put);
                if constexpr (pl.ne == 3) vdump(IC(2), put);
                vdump(IC(pl.ne), put);
            };
            if (!direct) vdump_all(gput);
            else if (local) vdump_all(put_l);
            else vdump_all(put_w);
            AGX_STAMP(64 + 9);
            __syncthreads();
            float lmb = lsum, klmb = klsum;
            {
                AGX_IDS;
                block_sum2(lmb, klmb, stat, 2, lane, wave);
            }
            float gr[kMaxPT];  // summed gradients of the owned slots
            constexpr int NQ = (2 * kNW * KM + 63) / 64;
            float vq[NQ];  // partners: this lane's words of the published partial norms
            if (g.K > 1) {
                // ---- P9b: exchange partial gradients with the agent's partners --------
                // every gradient word went out as a write-through (sc1) store from the
                // backward pass / vdump; the loss words follow.  Drained by every storing
                // wave before the barrier (partner_sync), so no release fence
                if (tid == 0) {
                    slab_put(pl.param_end, lmb);
                    slab_put(pl.param_end + 1, klmb);
                }
                if (!partner_sync(ctr1, (unsigned)(g.K * (upd + 1)), 64 + 11, 64 + 12)) return;
                // ---- reduce-scatter: partner kk sums its own float4 chunks [oc0, oc1)
                // of the parameter image (+ the chunk holding the loss / approx_kl
                // words) over the K slabs in partner order; the sums stay in its
                // registers (it alone runs Adam on them), only the loss chunk and the
                // per-wave partial gradient norms go to the agent's sum slab
                {
                    const int tid = vtid();
                    // one buffer descriptor over the K consecutive slabs
                    const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                        base, 0, __builtin_amdgcn_readfirstlane(g.K * pl.slab * 4), 0x00020000);
                    bool rs_done = false;
#if AGX_LEARN_RS2
                    // all 8 waves load: thread t sums chunk oc0 + (t mod kNT/2) over one
                    // half of the partners (half t / (kNT/2): partners [KM/2 h, KM/2 h +
                    // KM/2), in order), the upper half hands its sum over through the
                    // dead activation region of LDS, and the owner adds the two halves
                    // (fixed order: lower + upper)
                    if constexpr (JN == 1) {
                        if (oc1 - oc0 <= kNT / 2) {  // workgroup-uniform
                            constexpr int KH = KM / 2;
                            const int h = tid >= kNT / 2 ? 1 : 0;
                            const int c = oc0 + (tid & (kNT / 2 - 1));
                            const int cl = c < oc1 ? c : oc0;
                            f4 x[KH];
#pragma unroll
                            for (int q = 0; q < KH; ++q) {
                                const int qq = KH * h + q, qs = qq < g.K ? qq : g.K - 1;
                                const f4 v = __builtin_bit_cast(
                                    f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (qs * pl.slab + 4 * cl) * 4, 0, 16));
                                x[q] = qq < g.K ? v : f4{0.f, 0.f, 0.f, 0.f};
                            }
                            f4 t = x[0];
#pragma unroll
                            for (int q = 1; q < KH; ++q) t += x[q];
                            f4 *xch = reinterpret_cast<f4 *>(sm + pl.l_x0);
                            if (h) xch[tid - kNT / 2] = t;
                            __syncthreads();
                            if (!h) {
                                t += xch[tid];
                                if (c == n4) {  // the loss / approx_kl chunk: every partner reads it
                                    if (local) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, t), sum_rsrc, c * 16, 0, 0);
                                    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, t), sum_rsrc, c * 16, 0, 16);
                                }
                            }
#pragma unroll
                            for (int cc = 0; cc < 4; ++cc) gr[cc] = (!h && c < pc1) ? t[cc] : 0.f;
                            rs_done = true;
                        }
                    }
#endif
#pragma unroll
                    for (int j = 0; j < kUsed4; ++j) {
                        if (rs_done) break;  // uniform
                        const int c = oc0 + tid + kNT * j;
                        f4 t = f4{0.f, 0.f, 0.f, 0.f};
                        if (j >= jn_own) {  // uniform: no thread owns round j
#pragma unroll
                            for (int cc = 0; cc < 4; ++cc) gr[4 * j + cc] = 0.f;
                            continue;
                        }
                        if (c < oc1) {
                            f4 x[KM];  // all K loads in flight at once
#pragma unroll
                            for (int q = 0; q < KM; ++q)
                                x[q] = q < g.K ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                           rs, (q * pl.slab + 4 * c) * 4, 0, 16))
                                               : f4{0.f, 0.f, 0.f, 0.f};
                            t = x[0];  // partner order
#pragma unroll
                            for (int q = 1; q < KM; ++q)
                                if (q < g.K) t += x[q];
                            if (c == n4) {  // the loss / approx_kl chunk: every partner reads it
                                if (local) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, t), sum_rsrc, c * 16, 0, 0);
                                else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, t), sum_rsrc, c * 16, 0, 16);
                            }
                        }
#pragma unroll
                        for (int cc = 0; cc < 4; ++cc) gr[4 * j + cc] = c < pc1 ? t[cc] : 0.f;
                    }
                    AGX_STAMP(64 + 3);
                    // partial two-group squared norms of the owned (valid) slots, per wave
                    float n0 = 0.f, n1 = 0.f;
#pragma unroll
                    for (int i = 0; i < 4 * kUsed4; ++i) {
                        if ((i >> 2) >= jn_own) break;
                        const bool valid = (vbits >> i) & 1u, crit = (gbits >> i) & 1u;
                        gr[i] = valid ? gr[i] : 0.f;
                        const float x2 = gr[i] * gr[i];
                        n1 += crit ? x2 : 0.f;
                        n0 += crit ? 0.f : x2;
                    }
                    const int lane = vlane(), wave = swave();
                    const float r0 = row_sum(n0), r1 = row_sum(n1);
                    const float w0 = readlane_f(r0, 0) + readlane_f(r0, 16) + readlane_f(r0, 32) + readlane_f(r0, 48);
                    const float w1 = readlane_f(r1, 0) + readlane_f(r1, 16) + readlane_f(r1, 32) + readlane_f(r1, 48);
                    if (lane < 2) {
                        const float w = lane ? w1 : w0;
                        const int o = (pl.param_end + 4 + (kk * kNW + wave) * 2 + lane) * 4;
                        if (local) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, w), sum_rsrc, o, 0, 0);
                        else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, w), sum_rsrc, o, 0, 16);
                    }
                }
                AGX_STAMP(64 + 13);
                if (!partner_sync(ctr2, (unsigned)(g.K * (upd + 1)), 64 + 8, 64 + 15)) return;
                // ONE round trip for everything the second barrier published: the
                // K x kNW per-wave partial norms (unconditional loads; the slab
                // always holds the kMaxK-partner area, words past this split's are
                // masked) and the minibatch loss / approx_kl words
                {
                    const int lane = vlane();
                    const int np = 2 * kNW * g.K;  // <= 256: word lane + 64 q holds [partner][wave][group]
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const float x = __builtin_bit_cast(
                            float, __builtin_amdgcn_raw_buffer_load_b32(sum_rsrc, (pl.param_end + 4 + 64 * q + lane) * 4, 0, 16));
                        vq[q] = lane + 64 * q < np ? x : 0.f;
                    }
                }
                // the minibatch loss and approx_kl: partner-order sums of the K words
                // (uniform: the early-stop branch depends on it)
                const unsigned lw = __builtin_amdgcn_raw_buffer_load_b32(sum_rsrc, pl.param_end * 4, 0, 16);
                const unsigned kw = __builtin_amdgcn_raw_buffer_load_b32(sum_rsrc, (pl.param_end + 1) * 4, 0, 16);
                lmb = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(lw));
                klmb = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(kw));
            }

            // ---- P10: two-group norm, Adam from registers -------------------------
            // Branch-free over the owned slots: slots entirely inside the parameter
            // region need no bounds test (padding slots carry g = m = v = 0, so
            // Adam writes their value back unchanged); per-slot branches cost
            // exec-mask traffic and SGPR spills.
            float t0 = 0.f, t1 = 0.f;
            if (!direct) {
                const f4 *G4 = reinterpret_cast<const f4 *>(G);
#pragma unroll
                for (int j = 0; j < kUsed4; ++j) {
                    const int c = own_c(j);
                    const f4 x = c < pc1 ? G4[c] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc) gr[4 * j + cc] = x[cc];
                }
                float n0 = 0.f, n1 = 0.f;
#pragma unroll
                for (int i = 0; i < 4 * kUsed4; ++i) {
                    const bool valid = (vbits >> i) & 1u, crit = (gbits >> i) & 1u;
                    gr[i] = valid ? gr[i] : 0.f;
                    const float x2 = gr[i] * gr[i];
                    n1 += crit ? x2 : 0.f;
                    n0 += crit ? 0.f : x2;
                }
                AGX_IDS;
                // both group norms in one reduction round (fixed order)
                {
                    const float r0 = row_sum(n0), r1 = row_sum(n1);
                    const float w0 = readlane_f(r0, 0) + readlane_f(r0, 16) + readlane_f(r0, 32) + readlane_f(r0, 48);
                    const float w1 = readlane_f(r1, 0) + readlane_f(r1, 16) + readlane_f(r1, 32) + readlane_f(r1, 48);
                    if (lane == 0) {
                        stat[wave] = w0;
                        stat[kNW + wave] = w1;
                    }
                }
                __syncthreads();
                for (int i = 0; i < kNW; ++i) {
                    t0 += stat[i];
                    t1 += stat[kNW + i];
                }
            } else {
                // the K x kNW per-wave partials of both groups from the sum slab
                // ([partner][wave][group]: group = index parity, loaded right after the
                // second barrier), summed in one fixed order by every wave of every
                // partner -> identical clip
                const int lane = vlane();
                float v = vq[0];
#pragma unroll
                for (int q = 1; q < NQ; ++q) v += vq[q];
                const float x0 = row_sum((lane & 1) ? 0.f : v), x1 = row_sum((lane & 1) ? v : 0.f);
                t0 = readlane_f(x0, 0) + readlane_f(x0, 16) + readlane_f(x0, 32) + readlane_f(x0, 48);
                t1 = readlane_f(x1, 0) + readlane_f(x1, 16) + readlane_f(x1, 32) + readlane_f(x1, 48);
            }
            if (tid == 0) loss_total += lmb;
            kl_total += (double)klmb;
            ++n_done;
            AGX_STAMP(64 + 14);
            const float c0 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t0) + 1e-6f), 1.f) : 1.f;
            const float c1 = g.max_norm > 0.f ? fminf(g.max_norm / (sqrtf(t1) + 1e-6f), 1.f) : 1.f;
            // bias corrections 1 - beta^step from running f64 products (the
            // host/torch form is pow(); products agree to an ulp of f64, i.e.
            // to the f32 results used here)
            pb1 *= (double)g.b1;
            pb2 *= (double)g.b2;
            const float bc1 = (float)(1.0 - pb1);
            const float bc2s = (float)sqrt(1.0 - pb2);
            const float step_size = lr_p / bc1;
            const float inv_bc2s = 1.f / bc2s;
            // Adam on the owned float4 chunks: LDS b128 reads/writes; the elementwise
            // math on 4-vectors lowers to packed-f32 VALU ops (v_pk_mul/add_f32)
            f4 pv[kMaxPT / 4];  // all parameter reads issued before any write
            f4 *sm4 = reinterpret_cast<f4 *>(sm);
#pragma unroll
            for (int j = 0; j < kUsed4; ++j) {
                const int c = own_c(j);
                pv[j] = (j < jn_own && c < pc1) ? sm4[c] : f4{0.f, 0.f, 0.f, 0.f};
            }
            const float ob1 = 1.f - g.b1, ob2 = 1.f - g.b2;
#pragma unroll
            for (int j = 0; j < kUsed4; ++j) {
                if (j >= jn_own) break;  // uniform
                f4 gc, m, v;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * j + c;
                    gc[c] = ((gbits >> i) & 1u) ? c1 : c0;
                    m[c] = am[i];
                    v[c] = av[i];
                }
                gc = f4{gr[4 * j], gr[4 * j + 1], gr[4 * j + 2], gr[4 * j + 3]} * gc;
                m = m + ob1 * (gc - m);
                v = v * g.b2 + ob2 * gc * gc;
                // hardware sqrt / reciprocal (1 ulp) instead of the IEEE expansions:
                // the update m/(sqrt(v)+eps) is compared within tolerance, never
                // bit-exactly (summation order already differs)
                f4 r;
#pragma unroll
                for (int c = 0; c < 4; ++c) r[c] = __builtin_amdgcn_sqrtf(v[c]);
                r = r * inv_bc2s + g.eps;
#pragma unroll
                for (int c = 0; c < 4; ++c) r[c] = __builtin_amdgcn_rcpf(r[c]);
                const f4 nv = pv[j] - step_size * (m * r);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    am[4 * j + c] = m[c];
                    av[4 * j + c] = v[c];
                }
                const int c = own_c(j);
                if (c < pc1) {
                    sm4[c] = nv;
                    // partners: the updated chunk goes to this workgroup's slab (its
                    // gradient words there were consumed before the second barrier)
                    if (direct) {
                        if (local) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, nv), slab_rsrc, c * 16, 0, 0);
                        else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, nv), slab_rsrc, c * 16, 0, 16);
                    }
                }
            }
            if (direct) {
                // ---- P11: every partner's updated chunks -> this LDS image --------
                if (!partner_sync(ctr3, (unsigned)(g.K * (upd + 1)), 64 + 0,
                                  64 + 1))
                    return;
                const int tid = vtid();
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    base, 0, __builtin_amdgcn_readfirstlane(g.K * pl.slab * 4), 0x00020000);
#if AGX_LEARN_UNIFORM
                // every thread of the workgroup takes chunks tid, tid + kNT, ...
                // of the whole image from their owners' slabs: all loads issued
                // unconditionally (the clamped chunk of a thread past the image
                // re-reads a valid word), then the other partners' chunks -> LDS
                constexpr int NR = (n4 + kNT - 1) / kNT;
                f4 x[NR];
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    const int c0 = tid + kNT * j, c = c0 < n4 ? c0 : n4 - 1;
                    const int q = (int)(((float)c + 0.5f) * inv_cs);
                    x[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (q * pl.slab + 4 * c) * 4, 0, 16));
                }
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    const int c = tid + kNT * j;
                    const int q = (int)(((float)c + 0.5f) * inv_cs);
                    if (c < n4 && q != kk) sm4[c] = x[j];
                }
#else
                // round r: chunk qc0 + tid + kNT*r of every other partner q, all loads in flight
                const int span = (n4s + g.K - 1) / g.K + 1;
                for (int r0 = 0; r0 < span; r0 += kNT) {
                    f4 x[KM];
                    int cq[KM];
#pragma unroll
                    for (int q = 0; q < KM; ++q) {
                        const int qc0 = (int)((long long)n4s * q / g.K), qc1 = (int)((long long)n4s * (q + 1) / g.K);
                        const int c = qc0 + tid + r0;
                        cq[q] = (q < g.K && q != kk && c < qc1 && c < n4) ? c : -1;
                        x[q] = cq[q] >= 0 ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                        rs, (q * pl.slab + 4 * c) * 4, 0, 16))
                                          : f4{0.f, 0.f, 0.f, 0.f};
                    }
#pragma unroll
                    for (int q = 0; q < KM; ++q)
                        if (cq[q] >= 0) sm4[cq[q]] = x[q];
                }
#endif
                AGX_STAMP(64 + 2);
            }
            __syncthreads();
            AGX_STAMP(64 + 10);
        }  // minibatches
        ++epochs_done;
        // target-KL early stop after the epoch (ppo.py:917-918); every partner
        // holds the same fixed-order kl words, so all take the same branch
        {
            const unsigned long long tb = __builtin_bit_cast(unsigned long long, tkl_v);
            const unsigned thi = __builtin_amdgcn_readfirstlane((unsigned)(tb >> 32));
            const unsigned tlo = __builtin_amdgcn_readfirstlane((unsigned)tb);  // unsigned: no sign extension
            const double tkl = __builtin_bit_cast(double, ((unsigned long long)thi << 32) | tlo);
            if (tkl > 0.0 && kl_total / (double)n_done > tkl) break;
        }
    }  // epochs

    // ---- write parameters and moments back (partners hold identical parameter
    // images; each writes its own chunks, whose moments it holds) -------------------
#pragma unroll
    for (int i = 0; i < 4 * kUsed4; ++i) {
        const int l = 4 * own_c(i >> 2) + (i & 3);
        if ((vbits >> i) & 1u) {
            int grp;
            const int f = lds_to_flat<C>(l, grp);
            gp[f] = sm[l];
            gm[f] = am[i];
            gv[f] = av[i];
        }
    }
    if constexpr (ST)
        if (g.stamps && b == 0 && tid < 80) g.stamps[tid] = reinterpret_cast<const long long *>(sm + pl.l_stamp)[tid];
    if (tid == 0 && kk == 0) {
        if (loss_out_v) loss_out_v[p] = loss_total / ((float)S * (float)Ep);
        if (kl_out_v) kl_out_v[p] = n_done ? (float)(kl_total / (double)n_done) : 0.f;
        if (epochs_out_v) epochs_out_v[p] = epochs_done;
        *step_v = step0 + n_done;
    }
#undef IC
#undef BC
}

// ---------------------------------------------------------------------------
// prologue: permute the rollout SoA into minibatch order, normalise advantages
// ---------------------------------------------------------------------------
__global__ void ppo_gather_kernel(const float *__restrict__ obs, const long long *__restrict__ act,
                                  const float *__restrict__ old_logp, const float *__restrict__ adv,
                                  const float *__restrict__ ret, const float *__restrict__ old_v,
                                  const double *__restrict__ adv_stats, const long long *__restrict__ perms,
                                  const unsigned char *__restrict__ masks, int A,
                                  long long S, int D, int P, float *__restrict__ gobs, int *__restrict__ gact,
                                  unsigned *__restrict__ gmask, float *__restrict__ grow,
                                  unsigned *__restrict__ counters, int ncounters, const int *__restrict__ epochs_p,
                                  unsigned *__restrict__ err) {
    const int ep = blockIdx.y;  // e * P + p
    const int p = ep % P;
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    // the learner's arrival counters + timeout word (stream-ordered before it;
    // replaces a separate memset launch)
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < ncounters; i += blockDim.x) counters[i] = 0u;
    if (j >= S) return;
    // epochs beyond an agent's own update_epochs: the learner never reads
    // them, and their perms rows are not part of the contract (agx.h)
    if (epochs_p && ep / P >= epochs_p[p]) return;
    long long src = perms[(size_t)ep * S + j];
    if (src < 0 || src >= S) {
        // a host-side slip must not become a device fault: flag it in the
        // caller's sticky error word (bit 2; PPOPopulation.check_errors raises
        // AgxError) and gather row 0 in its place
        if (err) __hip_atomic_fetch_or(err, AGX_LEARN_ERR_PERM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        src = 0;
    }
    const size_t sp = (size_t)p * S + src;
    for (int d = 0; d < D; ++d) gobs[((size_t)ep * S + j) * D + d] = obs[sp * D + d];
    gact[(size_t)ep * S + j] = (int)act[sp];
    if (masks) {  // [P][S][A] u8 -> one bit per action
        unsigned bits = 0;
        for (int a = 0; a < A; ++a) bits |= (masks[sp * A + a] != 0 ? 1u : 0u) << a;
        gmask[(size_t)ep * S + j] = bits;
    }
    float *gr = grow + (size_t)ep * 4 * S;
    double a = adv[sp];
    if (adv_stats) a = (a - adv_stats[2 * p]) * (1.0 / (adv_stats[2 * p + 1] + 1e-8));  // == adv_normalize_kernel
    gr[j] = old_logp[sp];
    gr[S + j] = (float)a;
    gr[2 * S + j] = ret[sp];
    gr[3 * S + j] = old_v[sp];
}

// ---------------------------------------------------------------------------
// rollout policy step
// ---------------------------------------------------------------------------
// One policy step of workgroup (p, n0).  resident: the parameters (and the
// zeroed padding of the parameter region) are already in LDS from an earlier
// step of the same persistent launch; only the activations are re-zeroed.
// st (diagnostic, may be null): s_memrealtime after the host reads landed,
// after the forward, after the outputs were issued (thread 0 only)
template <class C>
__device__ __forceinline__ void act_body(const ActArgs &g, float *sm, bool resident, long long *st = nullptr) {
    constexpr LearnPlan pl = C::plan;
    const int p = blockIdx.y, n0 = blockIdx.x * kSB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nrow = g.N - n0 < kSB ? g.N - n0 : kSB;
    // every host read of the step is issued up front (one round trip)
    const float *ob = g.obs + (size_t)p * g.obs_pstride + (size_t)n0 * pl.D;
    constexpr int kObsIt = (kSB * pl.D + kNT - 1) / kNT;
    float obv[kObsIt];
#pragma unroll
    for (int k = 0; k < kObsIt; ++k) {
        const int i = tid + k * kNT;
        obv[k] = i < nrow * pl.D ? ld_sys(ob + i) : 0.f;
    }
    const bool prev = g.st_rew && tid < nrow;
    const size_t idx = (size_t)p * g.N + n0 + tid;
    float rw = 0.f;
    unsigned char dn = 0;
    if (prev) {
        rw = ld_sys(g.st_rew + idx);
        dn = ld_sys_u8(g.st_done + idx);
    }
    if (st && tid == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        st[0] = (long long)__builtin_amdgcn_s_memrealtime() + (long long)(obv[0] != obv[0]);
    }
    if (prev) {  // reward/done of the previous step -> slot t-1, episode accounting
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
    if (g.obs_copy) {
        float *oc = g.obs_copy + (size_t)p * g.obs_copy_pstride + (size_t)n0 * pl.D;
#pragma unroll
        for (int k = 0; k < kObsIt; ++k)
            if (tid + k * kNT < nrow * pl.D) oc[tid + k * kNT] = obv[k];
    }
    if (!g.act) return;
    for (int i = resident ? pl.param_end + tid : tid; i < pl.act_floats; i += kNT) sm[i] = 0.f;
    __syncthreads();
    if (!resident) load_params<C>(sm, g.params + (size_t)p * pl.n, tid);
#pragma unroll
    for (int k = 0; k < kObsIt; ++k) {
        const int i = tid + k * kNT;
        if (i < kSB * pl.D) sm[pl.l_x0 + (i / pl.D) * pl.ld_x0 + i % pl.D] = obv[k];
    }
    __syncthreads();
    Fwd<C> fw{sm};
    fw.run();
    if (st && tid == 0) st[1] = (long long)__builtin_amdgcn_s_memrealtime();
    // categorical over 16 lanes per row
    const int r = wave + kNW * (lane >> 4), a = lane & 15;
    const bool live = r < nrow;
    float lg = a < pl.A ? sm[pl.l_lg + r * kMaxA + a] : -3.0e38f;
    if (g.mask && a < pl.A && live) {  // illegal -> -1e8 (apply_action_mask_discrete, distributions.py:16-28)
        const size_t mo = (size_t)p * g.mask_pstride + (size_t)(n0 + r) * pl.A + a;
        const unsigned char ok = ld_sys_u8(g.mask + mo);
        if (g.mask_copy) g.mask_copy[(size_t)p * g.mask_copy_pstride + (size_t)(n0 + r) * pl.A + a] = ok;
        if (!ok) lg = -1.0e8f;
    }
    const float mx = row_max(lg);
    const float lse = mx + logf(row_sum(a < pl.A ? expf(lg - mx) : 0.f));
    const float pa = a < pl.A ? expf(lg - lse) : 0.f;
    const float H = -row_sum(a < pl.A ? pa * logf(pa + 1e-8f) : 0.f);
    float score = lg;
    if (g.sample) {
        const unsigned long long env =
            (g.env_base ? (unsigned long long)g.env_base[p] : (unsigned long long)p * g.N) + n0 + r;
        const uint4 rnd = philox(make_uint4((unsigned)env, (unsigned)(env >> 32), (unsigned)g.counter,
                                            (unsigned)(g.counter >> 32) ^ ((unsigned)(a >> 2) << 24)),
                                 make_uint2((unsigned)g.seed, (unsigned)(g.seed >> 32)));
        const unsigned w = (a & 3) == 0 ? rnd.x : (a & 3) == 1 ? rnd.y : (a & 3) == 2 ? rnd.z : rnd.w;
        const float u = ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
        score = a < pl.A ? lg - logf(-logf(u)) : -3.0e38f;                  // Gumbel-max
    }
    const float best = row_max(score);
    const unsigned long long ball = __ballot(score == best);
    const int choice = __builtin_ctz((unsigned)((ball >> (lane & ~15)) & 0xffffu));  // first maximum
    const float lgc = __builtin_bit_cast(
        float, __builtin_amdgcn_ds_bpermute(((lane & ~15) + choice) * 4, __builtin_bit_cast(int, lg)));
    if (live && a == 0) {
        const size_t o = (size_t)p * g.out_pstride + n0 + r;
        if (g.act_out) g.act_out[o] = choice;
        if (g.logp_out) g.logp_out[o] = lgc - lse;
        if (g.ent_out) g.ent_out[o] = H;
        if (g.value_out) g.value_out[o] = sm[pl.l_val + r];
        if (g.act_flat)  // host memory: system-scope (write-through) store
            __hip_atomic_store(g.act_flat + (size_t)p * g.N + n0 + r, (long long)choice, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (st && tid == 0) st[2] = (long long)__builtin_amdgcn_s_memrealtime();
}

template <class C>
__global__ __launch_bounds__(kNT, 1) void ppo_act_kernel(ActArgs g) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    act_body<C>(g, sm, false);
}

// Persistent rollout: ONE launch runs all nsteps policy steps of a rollout
// (agx_ppo_rollout_persistent).  Step t's arguments are read from
// steps[t] (host memory) while the workgroup waits for the host to publish
// sequence number base+t+1 in ctl->seq (the env step has written the staging);
// after the step every thread's host stores are released at system scope and
// thread 0 writes done[block] = base+t+1 (sequence numbers are offset by the
// rollout's base so the control block is never reset).  Parameters are loaded into LDS once.
// The wait is bounded: after timeout_ticks of s_memrealtime (100 MHz) or on
// ctl->seq == kSeqAbort the workgroup sets ctl->timeout and exits.
template <class C>
__global__ __launch_bounds__(kNT, 1) void ppo_rollout_persistent_kernel(const ActArgs *steps, int nsteps,
                                                                        agx_rollout_ctl *ctl,
                                                                        unsigned long long timeout_ticks,
                                                                        unsigned base, long long *stamps) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr LearnPlan pl = C::plan;
    __shared__ ActArgs s_args;
    __shared__ int s_go;
    const int tid = threadIdx.x;
    const int blk = blockIdx.y * gridDim.x + blockIdx.x;
    unsigned *rel = rollout_release_word(ctl, gridDim.x * gridDim.y, blk);  // this workgroup's own line
    constexpr int kArgWords = (int)(sizeof(ActArgs) / 4);
    if (tid == 0)  // this workgroup is resident (agx_rollout_ctl.started counts them): a host pacing
        __hip_atomic_fetch_add(&ctl->started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // several can tell
    for (int t = 0; t < nsteps; ++t) {
        long long *st = stamps && blk == 0 && t < 32 ? stamps + 8 * t : nullptr;
        if (st && tid == 0) st[0] = (long long)__builtin_amdgcn_s_memrealtime();
        if (tid < kArgWords)
            reinterpret_cast<unsigned *>(&s_args)[tid] = reinterpret_cast<const unsigned *>(steps + t)[tid];
        if (tid == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int go = 1;
            for (;;) {
                // relaxed: an acquire at system scope would invalidate the
                // caches on every poll; one invalidate follows the wait
                const unsigned v = __hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v == AGX_ROLLOUT_ABORT) {  // host exception: the rollout is partial
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                if (v == AGX_ROLLOUT_STOP) {  // clean early end (an evaluation whose episodes all finished)
                    go = 0;
                    break;
                }
                if (v >= base + (unsigned)(t + 1)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                    go = 0;
                    __hip_atomic_store(&ctl->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
            if (st) st[1] = (long long)__builtin_amdgcn_s_memrealtime();
            if (stamps && t == 5 && blk < 64) stamps[256 + blk] = (long long)__builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
        if (!s_go) return;
        const ActArgs g = s_args;
        act_body<C>(g, sm, t > 0 && pl.param_end > 0, st ? st + 2 : nullptr);
        // the host-memory stores (actions) are system-scope write-through;
        // wait for their acknowledgements (no L2 write-back: a release fence
        // would flush every dirty L2 line per wave)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (st && tid == 0) st[5] = (long long)__builtin_amdgcn_s_memrealtime();
        if (stamps && tid == 0 && t == 5 && blk < 64) stamps[320 + blk] = (long long)__builtin_amdgcn_s_memrealtime();
        if (tid == 0)
            __hip_atomic_store(rollout_done_words(ctl) + blk, base + (unsigned)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch over the instantiated shapes
// ---------------------------------------------------------------------------
static bool same_layout(const agx_ppo_net *net, const LearnPlan &pl) {
    if (!pl.ok || net->n_params != pl.n || net->critic_start != pl.f_cw) return false;
    for (int e = 0; e < pl.ne; ++e) {
        if (net->enc_w[e] != pl.f_ew[e] || net->enc_b[e] != pl.f_eb[e]) return false;
        if (pl.eaff[e] && (net->enc_ln_w[e] != pl.f_eg[e] || net->enc_ln_b[e] != pl.f_ebe[e])) return false;
    }
    return net->actor_w == pl.f_aw && net->actor_b == pl.f_ab && net->actor_ln_w == pl.f_ag &&
           net->actor_ln_b == pl.f_abe && net->actor_out_w == pl.f_aow && net->actor_out_b == pl.f_aob &&
           net->critic_w == pl.f_cw && net->critic_b == pl.f_cb && net->critic_ln_w == pl.f_cg &&
           net->critic_ln_b == pl.f_cbe && net->critic_out_w == pl.f_cow && net->critic_out_b == pl.f_cob;
}

static bool dims_match(const agx_ppo_net *net, const NetDims &d) {
    if (net->obs_dim != d.D || net->n_actions != d.A || net->n_enc != d.ne) return false;
    if (net->enc_dim[0] != d.D) return false;
    for (int e = 0; e < d.ne; ++e)
        if (net->enc_dim[e + 1] != d.eo[e]) return false;
    return net->head_actor == d.ha && net->head_critic == d.hc;
}

struct Launcher {
    const LearnPlan *plan;
    void (*learn)(const LearnArgs &, int nblocks, size_t lds, hipStream_t, int sb);
    void (*act)(const ActArgs &, dim3 grid, size_t lds, hipStream_t);
    void (*persist)(const ActArgs *, int, agx_rollout_ctl *, unsigned long long, unsigned, long long *, dim3 grid,
                    size_t lds, hipStream_t);
    int (*persist_occupancy)(size_t lds);  // co-resident persistent workgroups per CU
};

template <class C>
static void launch_learn(const LearnArgs &a, int nblocks, size_t lds, hipStream_t s, int sb) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    // one owned chunk round per thread when the K-way split leaves <= kNT chunks per partner
    constexpr int n4s = C::plan.param_end / 4 + 1;
    const bool one_round = (n4s + a.K - 1) / a.K + 1 <= kNT;
    if constexpr (std::is_same_v<C, Shape<8, 4, 2, 64, 64, 0, 64, 64>>) {
        if (a.stamps && sb == 8 && one_round) {
            (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 8, 1, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            ppo_learn_kernel<C, 8, 1, true><<<(unsigned)nblocks, kNT, lds, s>>>(a);
            return;
        }
        if (a.stamps && sb == 16 && one_round) {
            (void)hipFuncSetAttribute((const void *)ppo_learn_kernel<C, 16, 1, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            ppo_learn_kernel<C, 16, 1, true><<<(unsigned)nblocks, kNT, lds, s>>>(a);
            return;
        }
    }
    if (sb == 8 && one_round) ppo_learn_kernel<C, 8, 1><<<(unsigned)nblocks, kNT, lds, s>>>(a);
    else if (sb == 8) ppo_learn_kernel<C, 8><<<(unsigned)nblocks, kNT, lds, s>>>(a);
    else if (sb == 16 && one_round) ppo_learn_kernel<C, 16, 1><<<(unsigned)nblocks, kNT, lds, s>>>(a);
    else if (sb == 16) ppo_learn_kernel<C, 16><<<(unsigned)nblocks, kNT, lds, s>>>(a);
    else ppo_learn_kernel<C, 32><<<(unsigned)nblocks, kNT, lds, s>>>(a);
}
template <class C>
static void launch_act(const ActArgs &a, dim3 grid, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)ppo_act_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    ppo_act_kernel<C><<<grid, kNT, lds, s>>>(a);
}

// Co-resident persistent workgroups per CU, queried once per shape: a launch
// may be issued while another persistent launch (a group evaluated in lock
// step) waits for the host, so the launch path calls nothing that could wait
// for the device.
template <class C>
static int persist_occupancy(size_t lds) {
    static size_t cached_lds = 0;
    static int cached = -1;
    if (cached >= 0 && cached_lds == lds) return cached;
    (void)hipFuncSetAttribute((const void *)ppo_rollout_persistent_kernel<C>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ppo_rollout_persistent_kernel<C>, kNT, lds) != hipSuccess)
        return 0;
    cached_lds = lds;
    cached = n;
    return n;
}

template <class C>
static void launch_persist(const ActArgs *steps, int nsteps, agx_rollout_ctl *ctl, unsigned long long ticks,
                           unsigned base, long long *stamps, dim3 grid, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)ppo_rollout_persistent_kernel<C>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        attr = true;
    }
    ppo_rollout_persistent_kernel<C><<<grid, kNT, lds, s>>>(steps, nsteps, ctl, ticks, base, stamps);
}

static bool find_launcher(const agx_ppo_net *net, Launcher &out) {
    if (!net) return false;
#define AGX_TRY(D_, A_, NE_, E0, E1, E2, HA, HC)                                                      \
    {                                                                                                 \
        using C = Shape<D_, A_, NE_, E0, E1, E2, HA, HC>;                                             \
        static_assert(C::plan.ok, "instantiated PPO shape must have a valid plan");                   \
        if (dims_match(net, C::dims) && same_layout(net, C::plan)) {                                  \
            out = Launcher{&C::plan, &launch_learn<C>, &launch_act<C>, &launch_persist<C>, &persist_occupancy<C>};                               \
            return true;                                                                              \
        }                                                                                             \
    }
    AGX_PPO_SHAPES(AGX_TRY)
#undef AGX_TRY
    return false;
}

static long long *&g_stamps_ptr() {  // learner phase stamps, int64[80]
    static long long *p = nullptr;
    return p;
}
static long long *&g_roll_stamps_ptr() {  // persistent-rollout stamps, int64[384]
    static long long *p = nullptr;
    return p;
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_ppo_learn_lds_bytes(const agx_ppo_net *net) {
    Launcher L;
    if (!find_launcher(net, L)) return 0;
    return (size_t)L.plan->lds_floats * sizeof(float);
}

// Workgroups per agent: the learner spreads an agent's sub-batches over up to
// kMaxK = 16 partner workgroups (one CU each) when the population leaves CUs idle.
static int cu_count() {
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
// Partner workgroups per agent: all partners must be co-resident (1 block per
// CU), so K <= CUs / P; AGX_LEARN_SPLIT lowers the cap (tests, diagnostics).
static int max_partners(int64_t P) {
    int k = kMaxK;
    if (const char *e = getenv("AGX_LEARN_SPLIT")) k = atoi(e);
    if (k < 1) k = 1;
    if (k > kMaxK) k = kMaxK;
    const int64_t fit = cu_count() / (P > 0 ? P : 1);
    if (fit < k) k = fit < 1 ? 1 : (int)fit;
    return k;
}
// Sub-batch rows and partner count of one learn: 8-row sub-batches over up to
// 16 partners when the population leaves that many CUs per agent (row passes
// at 64 lanes per row, half the dW contraction per CU), 16-row sub-batches over
// up to 8, else 32-row sub-batches over up to 4.  AGX_LEARN_SB = 8 / 16 / 32
// forces the row count.
static void pick_split(int64_t P, int64_t batch, int &K, int &SB) {
    const int kmax = max_partners(P);
    int sb = kmax >= 16 ? 8 : (kmax >= 8 ? 16 : 32);
    if (const char *e = getenv("AGX_LEARN_SB")) {
        const int v = atoi(e);
        if (v == 8 || v == 16 || v == 32) sb = v;
    }
    const int64_t nsb = (batch + sb - 1) / sb;
    K = sb == 32 ? (kmax > 4 ? 4 : kmax) : (sb == 16 ? (kmax > 8 ? 8 : kmax) : kmax);
    if (K > nsb) K = (int)nsb;
    if (K < 1) K = 1;
    SB = sb;
}
struct LearnWs {
    size_t cnt, gobs, gact, gmask, grow, slabs, sums, total;
};
static LearnWs learn_ws(const LearnPlan &pl, int64_t P, int64_t S, int64_t epochs) {
    LearnWs w;
    const size_t per = (size_t)epochs * P * S;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    w.cnt = 0;
    w.gobs = up(((size_t)(4 + kMaxK) * P + 1) * 4);  // barrier counters, timeout word, XCC ids
    w.gact = w.gobs + up(per * pl.D * 4);
    w.gmask = w.gact + up(per * 4);
    w.grow = w.gmask + up(per * 4);
    w.slabs = w.grow + up(per * 4 * 4);
    // partners of any split pick_split can choose (AGX_LEARN_SPLIT only lowers it)
    const int64_t fit = cu_count() / (P > 0 ? P : 1);
    const int K = fit < 1 ? 1 : (fit > kMaxK ? kMaxK : (int)fit);
    w.sums = w.slabs + (K > 1 ? up((size_t)P * 2 * K * pl.slab * 4) : 0);
    w.total = w.sums + (K > 1 ? (size_t)P * 2 * pl.slab * 4 : 0);
    return w;
}

extern "C" size_t agx_ppo_learn_workspace_bytes(const agx_ppo_net *net, int64_t P, int64_t S, int64_t epochs) {
    Launcher L;
    if (!find_launcher(net, L) || P <= 0 || S <= 0 || epochs <= 0) return 0;
    return learn_ws(*L.plan, P, S, epochs).total;
}

extern "C" int agx_debug_learn_stamps(int64_t *buf) {
    static_assert(sizeof(long long) == sizeof(int64_t), "");
    g_stamps_ptr() = reinterpret_cast<long long *>(buf);
    return AGX_OK;
}

extern "C" int agx_debug_rollout_stamps(int64_t *buf) {
    g_roll_stamps_ptr() = reinterpret_cast<long long *>(buf);
    return AGX_OK;
}

extern "C" int agx_ppo_learn_prepare(const agx_ppo_net *net, void *workspace, void *stream) {
    (void)workspace;
    (void)stream;
    AGX_REQUIRE(net, "agx_ppo_learn_prepare: null pointer");
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_learn_prepare: network shape not instantiated for the fused learner");
        return AGX_EUNSUPPORTED;
    }
    return AGX_OK;
}

static int &g_debug_stall() {
    static int v = 0;
    return v;
}
extern "C" int agx_debug_learn_stall(int on) {
    g_debug_stall() = on;
    return AGX_OK;
}

extern "C" int agx_ppo_learn(const agx_ppo_net *net, const agx_ppo_learn_args *x, void *workspace, void *stream) {
    AGX_REQUIRE(net && x && workspace, "agx_ppo_learn: null net / args / workspace");
    AGX_REQUIRE(x->params && x->exp_avg && x->exp_avg_sq && x->adam_step && x->lr && x->obs && x->actions &&
                    x->old_logp && x->adv && x->ret && x->old_value && x->perms,
                "agx_ppo_learn: null pointer");
    const int64_t P = x->P, S = x->S, epochs = x->epochs, batch = x->batch;
    AGX_REQUIRE(P > 0 && P <= 65535 && S > 0 && S < (1ll << 31) && epochs > 0 && batch > 0 && epochs * P <= 65535,
                "agx_ppo_learn: bad sizes P=%lld S=%lld epochs=%lld batch=%lld", (long long)P, (long long)S,
                (long long)epochs, (long long)batch);
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_learn: network shape not instantiated for the fused learner");
        return AGX_EUNSUPPORTED;
    }
    const LearnPlan &pl = *L.plan;
    hipStream_t s = as_stream(stream);
    const LearnWs w = learn_ws(pl, P, S, epochs);
    char *ws = static_cast<char *>(workspace);
    float *gobs = reinterpret_cast<float *>(ws + w.gobs);
    int *gact = reinterpret_cast<int *>(ws + w.gact);
    unsigned *gmask = x->action_masks ? reinterpret_cast<unsigned *>(ws + w.gmask) : nullptr;
    float *grow = reinterpret_cast<float *>(ws + w.grow);
    int K = 1, SB = kSB;
    pick_split(P, batch, K, SB);
    // partners: agents strided by a multiple of 8 blocks (one XCD per agent, see
    // the kernel) while the padded grid still fits the CUs
    long long Q = K > 1 ? (P + 7) / 8 * 8 : P;
    if (Q * K > cu_count()) Q = P;
    AGX_REQUIRE(Q * K <= 65535, "agx_ppo_learn: too many workgroups");
    // counters + timeout word: one 16-byte-multiple block at the workspace start, zeroed by the gather
    dim3 ggrid((unsigned)ceil_div(S, 256), (unsigned)(epochs * P));
    ppo_gather_kernel<<<ggrid, 256, 0, s>>>(x->obs, reinterpret_cast<const long long *>(x->actions), x->old_logp,
                                            x->adv, x->ret, x->old_value, x->adv_stats,
                                            reinterpret_cast<const long long *>(x->perms), x->action_masks, pl.A, S,
                                            pl.D, (int)P, gobs, gact, gmask, grow, reinterpret_cast<unsigned *>(ws),
                                            (int)(w.gobs / sizeof(unsigned)), x->epochs_per_agent, x->error_word);
    const int rc2 = check_launch("agx_ppo_learn gather");
    if (rc2) return rc2;
    LearnArgs a;
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
    a.B = (int)batch;
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
    a.err = x->error_word;
    a.stamps = g_stamps_ptr();
    a.K = K;
    a.Q = (int)Q;
    a.slabs = reinterpret_cast<float *>(ws + w.slabs);
    a.sums = reinterpret_cast<float *>(ws + w.sums);
    a.cnt = reinterpret_cast<unsigned *>(ws);
    a.debug_stall = K > 1 ? g_debug_stall() : 0;
    a.skip = x->skip_if_set;
    {
        const char *wt = getenv("AGX_LEARN_WRITETHROUGH");
        a.write_through = wt && atoi(wt) != 0;
    }
    L.learn(a, (int)(Q * K), (size_t)pl.lds_floats * sizeof(float), s, SB);
    return check_launch("agx_ppo_learn");
}

extern "C" int agx_ppo_act(const agx_ppo_net *net, int64_t P, int64_t N, const float *params, const float *obs,
                           int64_t obs_agent_stride, const uint8_t *action_mask, int64_t mask_agent_stride,
                           int sample, uint64_t seed, uint64_t counter,
                           int64_t *actions, float *log_probs, float *values, float *entropy,
                           int64_t out_agent_stride, int64_t *actions_flat, const int64_t *agent_env_base,
                           void *stream) {
    AGX_REQUIRE(net && params && obs && P > 0 && N > 0 && P <= 65535, "agx_ppo_act: bad arguments");
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_act: network shape not instantiated");
        return AGX_EUNSUPPORTED;
    }
    ActArgs a;
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
    a.act = 1;
    a.obs_copy = nullptr;
    a.obs_copy_pstride = 0;
    a.st_rew = nullptr;
    a.st_done = nullptr;
    a.rew_prev = nullptr;
    a.done_prev = nullptr;
    a.prev_pstride = 0;
    a.scores = nullptr;
    a.ret_sum = nullptr;
    a.episodes = nullptr;
    a.mask = action_mask;
    a.mask_pstride = mask_agent_stride;
    a.mask_copy = nullptr;
    a.mask_copy_pstride = 0;
    a.env_base = reinterpret_cast<const long long *>(agent_env_base);
    dim3 grid((unsigned)ceil_div(N, kSB), (unsigned)P);
    L.act(a, grid, (size_t)L.plan->act_floats * sizeof(float), as_stream(stream));
    return check_launch("agx_ppo_act");
}

extern "C" int agx_ppo_rollout_step(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                                    const agx_rollout_io *io, int act, int sample, uint64_t seed,
                                    uint64_t counter, void *stream) {
    AGX_REQUIRE(net && io && P > 0 && N > 0 && P <= 65535, "agx_ppo_rollout_step: bad arguments");
    if (int rc = check_rollout_io(io, act, params, "agx_ppo_rollout_step")) return rc;
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_rollout_step: network shape not instantiated");
        return AGX_EUNSUPPORTED;
    }
    ActArgs a;
    fill_rollout_args(a, L.plan->D, L.plan->A, P, N, params, io, act, sample, seed, counter);
    dim3 grid((unsigned)ceil_div(N, kSB), (unsigned)P);
    L.act(a, grid, (size_t)L.plan->act_floats * sizeof(float), as_stream(stream));
    return check_launch("agx_ppo_rollout_step");
}

extern "C" int64_t agx_rollout_workgroups(int64_t P, int64_t N) { return P * ceil_div(N, kSB); }

// Every workgroup of a persistent rollout must be resident at once: the host
// releases step t only after EVERY workgroup has finished step t-1, while the
// resident ones spin on the release word — a grid larger than the GPU holds
// would deadlock until the timeout.
extern "C" int64_t agx_rollout_max_workgroups(const agx_ppo_net *net) {
    Launcher L;
    if (!find_launcher(net, L)) return 0;
    return (int64_t)L.persist_occupancy((size_t)L.plan->act_floats * sizeof(float)) * cu_count();
}
extern "C" size_t agx_rollout_ctl_bytes(int64_t P, int64_t N) {
    const unsigned nwg = (unsigned)agx_rollout_workgroups(P, N);
    return (size_t)rollout_release_offset(nwg, nwg) * sizeof(unsigned);
}
extern "C" size_t agx_rollout_args_bytes(int64_t nsteps) { return (size_t)nsteps * sizeof(ActArgs); }

static int persistent_fits(const Launcher &L, int64_t P, int64_t N, const char *who) {
    const int64_t nwg = agx_rollout_workgroups(P, N);
    const int64_t cap = (int64_t)L.persist_occupancy((size_t)L.plan->act_floats * sizeof(float)) * cu_count();
    if (nwg > cap) {
        set_error("%s: %lld workgroups cannot all be resident (the GPU holds %lld of this kernel at once); use "
                  "per-step launches", who, (long long)nwg, (long long)cap);
        return AGX_EUNSUPPORTED;
    }
    return AGX_OK;
}

extern "C" int agx_ppo_eval_persistent(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                                       const float *stage_obs, const uint8_t *stage_mask, int64_t *actions_flat,
                                       const int64_t *agent_env_base, int64_t nsteps, uint32_t base, uint64_t seed,
                                       uint64_t counter0, void *args_host, agx_rollout_ctl *ctl, double timeout_s,
                                       void *stream) {
    AGX_REQUIRE(net && params && stage_obs && actions_flat && args_host && ctl && P > 0 && N > 0 && P <= 65535 &&
                    nsteps >= 1,
                "agx_ppo_eval_persistent: bad arguments");
    AGX_REQUIRE((uint64_t)base + (uint64_t)nsteps < AGX_ROLLOUT_STOP, "agx_ppo_eval_persistent: base wraps");
    AGX_REQUIRE(timeout_s > 0 && timeout_s < 3600, "agx_ppo_eval_persistent: timeout_s out of range");
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_eval_persistent: network shape not instantiated");
        return AGX_EUNSUPPORTED;
    }
    if (int rc = persistent_fits(L, P, N, "agx_ppo_eval_persistent")) return rc;
    const LearnPlan &pl = *L.plan;
    ActArgs *steps = static_cast<ActArgs *>(args_host);
    for (int64_t t = 0; t < nsteps; ++t) {
        ActArgs a{};
        a.params = params;
        a.obs = stage_obs;
        a.obs_pstride = N * (int64_t)pl.D;
        a.N = (int)N;
        a.P = (int)P;
        a.sample = 1;
        a.seed = seed;
        a.counter = counter0 + (uint64_t)t;
        a.act_flat = reinterpret_cast<long long *>(actions_flat);
        a.act = 1;
        a.mask = stage_mask;
        a.mask_pstride = N * (int64_t)pl.A;
        a.env_base = reinterpret_cast<const long long *>(agent_env_base);
        steps[t] = a;
    }
    const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    ctl->nwg = (uint32_t)agx_rollout_workgroups(P, N);
    dim3 grid((unsigned)ceil_div(N, kSB), (unsigned)P);
    L.persist(steps, (int)nsteps, ctl, ticks, base, nullptr, grid, (size_t)pl.act_floats * sizeof(float),
              as_stream(stream));
    return check_launch("agx_ppo_eval_persistent");
}

extern "C" int agx_ppo_rollout_persistent(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                                          const agx_rollout_io *ios, int64_t nsteps, uint32_t base, uint64_t seed,
                                          uint64_t counter0, void *args_host, agx_rollout_ctl *ctl,
                                          double timeout_s, void *stream) {
    AGX_REQUIRE(net && ios && params && args_host && ctl && P > 0 && N > 0 && P <= 65535 && nsteps >= 1,
                "agx_ppo_rollout_persistent: bad arguments");
    AGX_REQUIRE((uint64_t)base + (uint64_t)nsteps < AGX_ROLLOUT_STOP, "agx_ppo_rollout_persistent: base wraps");
    AGX_REQUIRE(timeout_s > 0 && timeout_s < 3600, "agx_ppo_rollout_persistent: timeout_s out of range");
    Launcher L;
    if (!find_launcher(net, L)) {
        set_error("agx_ppo_rollout_persistent: network shape not instantiated");
        return AGX_EUNSUPPORTED;
    }
    if (int rc = persistent_fits(L, P, N, "agx_ppo_rollout_persistent")) return rc;
    ActArgs *steps = static_cast<ActArgs *>(args_host);
    for (int64_t t = 0; t < nsteps; ++t) {
        const bool last = t + 1 == nsteps;
        if (int rc = check_rollout_io(ios + t, 1, params, "agx_ppo_rollout_persistent")) return rc;
        fill_rollout_args(steps[t], L.plan->D, L.plan->A, P, N, params, ios + t, 1, last ? 0 : 1, seed,
                          last ? 0 : counter0 + 1 + (uint64_t)t);
    }
    const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    ctl->nwg = (uint32_t)agx_rollout_workgroups(P, N);
    dim3 grid((unsigned)ceil_div(N, kSB), (unsigned)P);
    L.persist(steps, (int)nsteps, ctl, ticks, base, g_roll_stamps_ptr(), grid, (size_t)L.plan->act_floats * sizeof(float),
              as_stream(stream));
    return check_launch("agx_ppo_rollout_persistent");
}
