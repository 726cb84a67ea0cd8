// DQN TD target and Rainbow C51 categorical projection + cross entropy.
//
// TD target — agilerl/algorithms/dqn.py:296-314 (DQN.update):
//   q_t = max_a Qtgt(s')  |  Qtgt(s')[argmax_a Q(s')] (double)
//   y   = r + (gamma*q_t)*(1-d)        (f32, one rounding per op)
//   loss = MSE(Q(s)[a], y);  dloss/dQ(s)[a] = 2 (Q[a]-y) / B
//
// C51 — agilerl/algorithms/dqn_rainbow.py:313-367 (RainbowDQN._dqn_loss), f32:
//   a* = argmax Q_online(s') (first maximum, like torch.argmax)
//   t_z = clamp(r + ((1-d)*gamma)*z, vmin, vmax);  b = (t_z - vmin) / f32(dz)
//   L = floor(b), U = ceil(b); L[(U>0)&(U==L)] -= 1; U[(Z-1>L)&(U==L)] += 1
//   proj.index_add_(L, p*(U-b)); proj.index_add_(U, p*(b-L))   (serial order)
//   loss_i = -sum_z proj_z * log_p[a_i, z]
// The serial index_add_ adds, per bin, all lower masses in atom order and
// then all upper masses in atom order.  When b is monotone in z (support
// ascending, (1-d)*gamma >= 0 — always the case in Rainbow) the atoms feeding
// a bin form a contiguous run, found by a binary search in LDS; the bin's
// lane then adds that run in order — bit-identical to the reference's
// projection.  A row whose b is not monotone falls back to the full ordered
// scan.  One wave per row, lane z <-> atom z (Z <= 64 per pass, Z <= 256).
// Algorithmic bytes per row: 4A (q row) + 4Z (target row a*) + 4Z (log_p row
// a_i) + 8 (r, d) + 4 (loss) = 444 B at A = 6, Z = 51.
#include <cmath>

#include "agx_common.h"

namespace agx {

constexpr int kTdBlock = 256;

// one row per lane; the squared TD errors are reduced per block (f64, fixed
// order) into partials[blockIdx] and summed by td_loss_finalize
__global__ __launch_bounds__(kTdBlock) void td_target_kernel(
    const float *__restrict__ qno, const float *__restrict__ qnt, const float *__restrict__ qc,
    const int64_t *__restrict__ act, const float *__restrict__ r, const float *__restrict__ d, int64_t B, int A,
    float g, int dbl, float *__restrict__ y, float *__restrict__ g_q, double *__restrict__ partials) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sq = 0.0;
    if (i < B) {
        const float *tn = qnt + i * A;
        float qt;
        if (dbl) {
            const float *on = qno + i * A;
            int best = 0;
            float bv = on[0];
            for (int a = 1; a < A; ++a)
                if (on[a] > bv) {
                    bv = on[a];
                    best = a;
                }
            qt = tn[best];
        } else {
            qt = tn[0];
            for (int a = 1; a < A; ++a) qt = fmaxf(qt, tn[a]);
        }
        const float yi = r[i] + (g * qt) * (1.0f - d[i]);
        y[i] = yi;
        if (qc) {
            const int64_t ai = act[i];
            const float qa = qc[i * A + ai];
            if (g_q) {
                const float diff = qa - yi;
                const float scale = 2.0f / (float)B;
                for (int a = 0; a < A; ++a) g_q[i * A + a] = (a == ai) ? diff * scale : 0.0f;
            }
            const double dd = (double)qa - (double)yi;
            sq = dd * dd;
        }
    }
    if (partials) {
        __shared__ double red[kTdBlock / kWave];
        sq = wave_sum(sq);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = sq;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int w = 0; w < kTdBlock / kWave; ++w) t += red[w];
            partials[blockIdx.x] = t;
        }
    }
}

// MADDPG critic target (agilerl/algorithms/maddpg.py:764-781): NaN rewards ->
// 0, NaN dones -> 1, dones cast to uint8 (truncation), then
//   y = r + ((1 - d) * gamma) * q'        ((1 - d) in uint8 arithmetic)
//   loss = MSE(q, y);  dloss/dq = 2 (q - y) / B
// One row per lane, squared errors reduced like td_target_kernel.
__global__ __launch_bounds__(kTdBlock) void maddpg_critic_kernel(
    const float *__restrict__ q, const float *__restrict__ qn, const float *__restrict__ r,
    const float *__restrict__ d, int64_t B, float g, float *__restrict__ y, float *__restrict__ g_q,
    double *__restrict__ partials) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sq = 0.0;
    if (i < B) {
        const float ri = __builtin_isnan(r[i]) ? 0.0f : r[i];
        const float di = __builtin_isnan(d[i]) ? 1.0f : d[i];
        const unsigned char du = (unsigned char)(int)di;           // .to(torch.uint8)
        const float nd = (float)(unsigned char)(1u - du);           // 1 - uint8 tensor (wraps)
        const float yi = ri + (nd * g) * qn[i];
        if (y) y[i] = yi;
        const float diff = q[i] - yi;
        if (g_q) g_q[i] = diff * (2.0f / (float)B);
        const double dd = (double)q[i] - (double)yi;
        sq = dd * dd;
    }
    __shared__ double red[kTdBlock / kWave];
    sq = wave_sum(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kTdBlock / kWave; ++w) t += red[w];
        partials[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void td_loss_finalize(const double *__restrict__ partials, int64_t nblk,
                                                         int64_t B, float *__restrict__ loss) {
    __shared__ double red[1024 / kWave];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < nblk; i += blockDim.x) s += partials[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) t += red[w];
        *loss = (float)(t / (double)B);
    }
}

constexpr int kC51Waves = 4;   // rows per block
constexpr int kC51MaxZ = 256;  // atoms per row (lane handles Z/64 of them)

__device__ __forceinline__ int lower_bound_i(const int *a, int n, int key) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kC51Waves * 64) void c51_kernel(
    const float *__restrict__ qno, const float *__restrict__ tdist, const float *__restrict__ logp,
    const int64_t *__restrict__ act, const float *__restrict__ rew, const float *__restrict__ dn,
    const float *__restrict__ support, int64_t B, int A, int Z, float vmin, float vmax, float dz,
    float g, float *__restrict__ loss, float *__restrict__ proj) {
    __shared__ int sL[kC51Waves][kC51MaxZ];
    __shared__ int sU[kC51Waves][kC51MaxZ];
    __shared__ float sml[kC51Waves][kC51MaxZ];
    __shared__ float smu[kC51Waves][kC51MaxZ];
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * kC51Waves + w;
    const bool live = row < B;            // dead waves shadow the last row and store nothing,
    const int64_t i = live ? row : B - 1;  // so every wave reaches the barrier
    // a* = argmax_a Q_online(s'), first maximum
    float bv = -__builtin_inff();
    int ba = 0x7fffffff;
    for (int a = lane; a < A; a += 64) {
        const float q = qno[i * A + a];
        if (q > bv || (q == bv && a < ba)) {
            bv = q;
            ba = a;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float q2 = __shfl_xor(bv, o, 64);
        const int a2 = __shfl_xor(ba, o, 64);
        if (q2 > bv || (q2 == bv && a2 < ba)) {
            bv = q2;
            ba = a2;
        }
    }
    const int astar = ba;
    const float k = (1.0f - dn[i]) * g;
    const float r = rew[i];
    const float *prow = tdist + ((size_t)i * A + astar) * Z;
    bool mono = true;
    for (int z = lane; z < Z; z += 64) {
        float tz = r + k * support[z];
        tz = fminf(fmaxf(tz, vmin), vmax);  // clamp(min=vmin, max=vmax)
        const float b = (tz - vmin) / dz;
        int L = (int)floorf(b), U = (int)ceilf(b);
        if (U > 0 && U == L) L -= 1;
        if (Z - 1 > L && U == L) U += 1;
        L = L < 0 ? 0 : (L > Z - 1 ? Z - 1 : L);  // guard (never taken for valid inputs)
        U = U < 0 ? 0 : (U > Z - 1 ? Z - 1 : U);
        const float p = prow[z];
        sL[w][z] = L;
        sU[w][z] = U;
        sml[w][z] = p * ((float)U - b);
        smu[w][z] = p * (b - (float)L);
    }
    __syncthreads();
    for (int z = lane; z + 1 < Z; z += 64)
        if (sL[w][z + 1] < sL[w][z] || sU[w][z + 1] < sU[w][z]) mono = false;
    mono = __all(mono);
    const float *lrow = logp + ((size_t)i * A + act[i]) * Z;
    float part = 0.0f;
    for (int bin = lane; bin < Z; bin += 64) {
        float acc = 0.0f;
        if (mono) {
            int z0 = lower_bound_i(sL[w], Z, bin), z1 = lower_bound_i(sL[w], Z, bin + 1);
            for (int z = z0; z < z1; ++z) acc += sml[w][z];
            z0 = lower_bound_i(sU[w], Z, bin);
            z1 = lower_bound_i(sU[w], Z, bin + 1);
            for (int z = z0; z < z1; ++z) acc += smu[w][z];
        } else {
            for (int z = 0; z < Z; ++z)
                if (sL[w][z] == bin) acc += sml[w][z];
            for (int z = 0; z < Z; ++z)
                if (sU[w][z] == bin) acc += smu[w][z];
        }
        if (proj && live) proj[(size_t)i * Z + bin] = acc;
        part += acc * lrow[bin];
    }
    part = wave_sum(part);
    if (lane == 0 && live) loss[i] = -part;
}

// Z <= 64 (Rainbow: Z = 51): R rows per wave, processed in lock-step so the
// dependent load levels (Q(s') row -> a* -> target row; a -> log_p row)
// overlap.  The serial index_add_ order is kept without a search: L (and U)
// is monotone in z, so the atoms feeding bin b form one run [s_b, e_b);
// the atom that starts (ends) a run writes s_b (e_b) into per-wave LDS, and
// bin lane b then folds its run left to right, reading the run's masses from
// the atom lanes with ds_bpermute — the same additions, in the same order,
// as the reference's two index_add_ calls.  Rows whose L/U are not monotone
// take the ordered scan of c51_kernel.
constexpr int kC51RowWaves = 4;

__device__ __forceinline__ float bperm_f(int src_lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane << 2, __builtin_bit_cast(int, v)));
}
// acc += mass[s], mass[s+1], ..., mass[e-1] in that order (mass[z] lives in
// lane z); nmax = wave max of e - s.  The usual run is 1-2 atoms; a d = 1 row
// sends all Z atoms to one bin, so long runs keep 8 permutes in flight.
__device__ __forceinline__ float fold_run(float acc, int s, int e, int nmax, float mass) {
    if (nmax <= 2) {
        const float m0 = bperm_f(s & 63, mass), m1 = bperm_f((s + 1) & 63, mass);
        acc = s < e ? acc + m0 : acc;
        return s + 1 < e ? acc + m1 : acc;
    }
    for (int t = 0; t < nmax; t += 8) {
        float m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = bperm_f((s + t + j) & 63, mass);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = s + t + j < e ? acc + m[j] : acc;
    }
    return acc;
}

template <int C>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), C, 0xf, 0xf, true));
}
// wave-wide sum (DPP within rows of 16, then the 4 row results)
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_f<0xb1>(v);
    v += dpp_f<0x4e>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    const int vi = __builtin_bit_cast(int, v);
    return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(vi, 0)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(vi, 16))) +
           (__builtin_bit_cast(float, __builtin_amdgcn_readlane(vi, 32)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(vi, 48)));
}

template <int R>
__global__ __launch_bounds__(kC51RowWaves * 64) void c51_rows_kernel(
    const float *__restrict__ qno, const float *__restrict__ tdist, const float *__restrict__ logp,
    const int64_t *__restrict__ act, const float *__restrict__ rew, const float *__restrict__ dn,
    const float *__restrict__ support, int64_t B, int A, int Z, float vmin, float vmax, float dz, float g,
    float *__restrict__ loss, float *__restrict__ proj) {
    // per row: monotone -> L-run start, L-run end, U-run start, U-run end per bin;
    // otherwise (ordered-scan fallback) L, U, lower mass, upper mass per atom
    __shared__ int sRun[kC51RowWaves][R][4][64];
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * kC51RowWaves + __builtin_amdgcn_readfirstlane(w)) * R;
    int64_t ri[R];
    int astar[R];
    float rr[R], kk[R];
    int64_t ai[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ri[r] = row0 + r < B ? row0 + r : B - 1;  // dead rows shadow the last row, store nothing
        ai[r] = act[ri[r]];
        rr[r] = rew[ri[r]];
        kk[r] = (1.0f - dn[ri[r]]) * g;
        // a* = argmax_a Q_online(s'), first maximum; the row is wave-uniform
        const float *qr = qno + ri[r] * A;
        float bv = qr[0];
        int ba = 0;
        if (A <= 8) {  // all (scalar) loads issued together
            float qv[8];
#pragma unroll
            for (int a = 1; a < 8; ++a) qv[a] = a < A ? qr[a] : -__builtin_inff();
#pragma unroll
            for (int a = 1; a < 8; ++a)
                if (qv[a] > bv) {
                    bv = qv[a];
                    ba = a;
                }
        } else {
            for (int a = 1; a < A; ++a) {
                const float qa = qr[a];
                if (qa > bv) {
                    bv = qa;
                    ba = a;
                }
            }
        }
        astar[r] = ba;
    }
    const float sup = lane < Z ? support[lane] : 0.f;
    float p[R], lp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        p[r] = lane < Z ? tdist[((size_t)ri[r] * A + astar[r]) * Z + lane] : 0.f;
        lp[r] = lane < Z ? logp[((size_t)ri[r] * A + ai[r]) * Z + lane] : 0.f;
    }
    int Lr[R], Ur[R];
    float mlr[R], mur[R];
    bool mono[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int L = 0x7fffffff, U = 0x7fffffff;  // lanes >= Z: beyond every bin
        float ml = 0.f, mu = 0.f;
        if (lane < Z) {
            float tz = rr[r] + kk[r] * sup;
            tz = fminf(fmaxf(tz, vmin), vmax);
            const float b = (tz - vmin) / dz;
            L = (int)floorf(b);
            U = (int)ceilf(b);
            if (U > 0 && U == L) L -= 1;
            if (Z - 1 > L && U == L) U += 1;
            L = L < 0 ? 0 : (L > Z - 1 ? Z - 1 : L);
            U = U < 0 ? 0 : (U > Z - 1 ? Z - 1 : U);
            ml = p[r] * ((float)U - b);
            mu = p[r] * (b - (float)L);
        }
        Lr[r] = L;
        Ur[r] = U;
        mlr[r] = ml;
        mur[r] = mu;
        const int Lp = __shfl_up(L, 1, 64), Up = __shfl_up(U, 1, 64);
        const int Ln = __shfl_down(L, 1, 64), Un = __shfl_down(U, 1, 64);
        mono[r] = __all(!(lane + 1 < Z) || (Ln >= L && Un >= U));
        // empty runs by default; run starts / ends written by their atoms
        sRun[w][r][0][lane] = 0;
        sRun[w][r][1][lane] = 0;
        sRun[w][r][2][lane] = 0;
        sRun[w][r][3][lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (mono[r] && lane < Z) {
            if (lane == 0 || Lp != L) sRun[w][r][0][L] = lane;
            if (lane + 1 == Z || Ln != L) sRun[w][r][1][L] = lane + 1;
            if (lane == 0 || Up != U) sRun[w][r][2][U] = lane;
            if (lane + 1 == Z || Un != U) sRun[w][r][3][U] = lane + 1;
        }
        if (!mono[r]) {
            sRun[w][r][0][lane] = L;
            sRun[w][r][1][lane] = U;
            sRun[w][r][2][lane] = __builtin_bit_cast(int, ml);
            sRun[w][r][3][lane] = __builtin_bit_cast(int, mu);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int bin = lane;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float acc = 0.f;
        if (mono[r]) {
            const int l0 = sRun[w][r][0][bin], l1 = sRun[w][r][1][bin];
            const int u0 = sRun[w][r][2][bin], u1 = sRun[w][r][3][bin];
            // wave-uniform trip counts; masses come from the atom lanes
            int nl = l1 - l0, nu = u1 - u0;
            for (int o = 32; o > 0; o >>= 1) {
                nl = max(nl, __shfl_xor(nl, o, 64));
                nu = max(nu, __shfl_xor(nu, o, 64));
            }
            acc = fold_run(acc, l0, l1, nl, mlr[r]);
            acc = fold_run(acc, u0, u1, nu, mur[r]);
        } else if (bin < Z) {
            for (int z = 0; z < Z; ++z)
                if (sRun[w][r][0][z] == bin) acc += __builtin_bit_cast(float, sRun[w][r][2][z]);
            for (int z = 0; z < Z; ++z)
                if (sRun[w][r][1][z] == bin) acc += __builtin_bit_cast(float, sRun[w][r][3][z]);
        }
        const bool live = row0 + r < B;
        if (proj && live && bin < Z) proj[(size_t)ri[r] * Z + bin] = acc;
        const float part = wave_sum_dpp(bin < Z ? acc * lp[r] : 0.f);
        if (lane == 0 && live) loss[ri[r]] = -part;
    }
}


// Z <= 64, A <= 64 (Rainbow: Z = 51, A = 6): one wave per 64 rows, one lane
// per row.  The per-row serial order of the reference's two index_add_ calls
// is then simply the lane's own loop over z:
//   1. lane k finds a*_k = argmax Q_online(s'_k) from its own Q row;
//   2. the wave gathers the 64 selected target rows by LDS-DMA
//      (buffer_load ... lds, flattened (row, atom) order, a* of the row taken
//      from its lane): they land in LDS as [row][z] without passing through
//      VGPRs, and lane k reads its own row at pitch Z (odd: conflict-free);
//   3. the same LDS region becomes the projection [bin][row] (pitch 64: a
//      lane's bin never conflicts with another lane's).  Pass L: lane k walks
//      z = 0..Z-1 and adds m_l to bin L_z; pass U adds m_u to bin U_z.  L and U
//      are monotone in z for a valid support, so pass L keeps the running bin
//      sum in a register (each step stores the partial; the last store of a
//      run is the sum) and pass U reads a bin's pass-L value only when a new
//      run starts — those reads are issued 8 atoms ahead, which is exact
//      because a new U bin has not yet been written by pass U.  A lane whose
//      row turns out not to be monotone redoes both passes as plain
//      read-modify-writes;
//   4. the projection goes to registers, the region receives the log_p rows
//      (LDS-DMA again), lane k folds its loss.
// One Z x 64 region (13 KB) for all three lives and ~150 VGPRs: 3 waves per
// SIMD hide the dependent q -> a* -> gather chain (the register-staged
// version, 26 KB and 341 registers, ran 1 wave per SIMD: 258 -> 151 us at
// 2^20 rows).  Opaque copies of the lane id / bin words per group of 8
// atoms keep the scheduler from hoisting all Z address computations.
constexpr int kC51LaneRows = 64;

// ROWS: the caller hands over the two selected rows per batch element already
// gathered ([B][Z] target distribution of a*, [B][Z] log p of the taken
// action — agx_dueling_head_forward_rows emits exactly these), so both LDS-DMA
// gathers read one contiguous Z x 64-float span per wave: no 128-B line is
// fetched for a neighbouring action's atoms, and no Q row / action is read.
// Z atoms at compile time (the gather's (row, atom) split is a multiply-shift,
// the atom loops unroll into independent chains).  POW2: Δz is a power of two
// (±200 or ±100 over 51 atoms: 8 or 4), so (tz − v_min)/Δz is the exact
// product with 1/Δz and the f32 division sequence is skipped.
template <int Z, bool POW2, bool ROWS = false>
__global__ __launch_bounds__(64) void c51_dma_kernel(
    const float *__restrict__ qno, const float *__restrict__ tdist, const float *__restrict__ logp,
    const int64_t *__restrict__ act, const float *__restrict__ rew, const float *__restrict__ dn,
    const float *__restrict__ support, int64_t B, int A, float vmin, float vmax, float dz, float inv_dz,
    float g, float *__restrict__ loss, float *__restrict__ proj) {
    static_assert(Z >= 2 && Z <= 64, "one lane per atom of the support");
    __shared__ float sA[Z * 64];
    const int lane = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * kC51LaneRows;
    const int nrows = (int)(B - row0 < kC51LaneRows ? B - row0 : kC51LaneRows);
    const bool live = lane < nrows;
    const int64_t i = row0 + (live ? lane : nrows - 1);  // dead lanes shadow the last row
    const int a_cur = ROWS ? 0 : (int)act[i];
    const float r = rew[i];
    const float kk = (1.0f - dn[i]) * g;
    int astar = 0;
    if constexpr (!ROWS) {
        const float *qr = qno + i * A;
        float bv = qr[0];
        for (int a = 1; a < A; ++a) {  // first maximum
            const float q = qr[a];
            if (q > bv) {
                bv = q;
                astar = a;
            }
        }
    }
    const float supv = lane < Z ? support[lane] : 0.f;
    const uint32_t blk = (uint32_t)((ROWS ? 1 : A) * Z * 4);
    // rows (row0 + rk, sel of lane rk) of a [B][A][Z] array -> sA[rk * Z + z];
    // rows past B read as 0 (buffer range = this wave's nrows rows)
    auto dma_rows = [&](const float *__restrict__ src, int sel) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src) + row0 * (ROWS ? 1 : A) * Z, 0,
                                                          (int)(blk * (uint32_t)nrows), 0x00020000);
        // opaque lane id: keeps the Z offset computations here instead of
        // hoisted (and held in registers) across the passes
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int j = 0; j < Z; ++j) {
            const int e = ln + 64 * j, rk = e / Z, z = e - rk * Z;
            const int srow = ROWS ? 0 : __shfl(sel, rk & 63, 64);
            const uint32_t off = (uint32_t)rk * blk + (uint32_t)((srow * Z + z) * 4);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void *)(sA + 64 * j), 4, off, 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    // rv / kv: copies of r / kk re-made opaque every 8 atoms, so the
    // scheduler cannot hoist all Z atom computations (3 Z live values) ahead
    float rv = r, kv = kk;
    int lf = lane;
    auto fence = [&](int z) {
        if (z % 8 == 0) asm volatile("" : "+v"(rv), "+v"(kv), "+v"(lf));
    };
    auto atom = [&](int z, int &L, int &U, float &b) {
        const float sup = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, supv), z));
        float tz = rv + kv * sup;
        tz = fminf(fmaxf(tz, vmin), vmax);  // clamp(min=vmin, max=vmax)
        b = POW2 ? (tz - vmin) * inv_dz : (tz - vmin) / dz;
        L = (int)floorf(b);
        U = (int)ceilf(b);
        if (U > 0 && U == L) L -= 1;
        if (Z - 1 > L && U == L) U += 1;
        L = L < 0 ? 0 : (L > Z - 1 ? Z - 1 : L);  // guard (never taken for valid inputs)
        U = U < 0 ? 0 : (U > Z - 1 ? Z - 1 : U);
    };
    dma_rows(tdist, astar);
    float pm[Z];  // p_z, then the upper mass mu_z
#pragma unroll
    for (int z = 0; z < Z; ++z) pm[z] = sA[lane * Z + z];
    __syncthreads();  // every row read before sA becomes the projection
#pragma unroll
    for (int bin = 0; bin < Z; ++bin) sA[bin * 64 + lane] = 0.f;
    // pass L (runs of equal L are consecutive; every partial stored, the last
    // store of a run is its sum), then pass U from the pass-L bin values
    bool mono = true;
    uint32_t ub4[(Z + 3) / 4] = {};
    {
        int prev = -1;
        float acc = 0.f;
#pragma unroll
        for (int z = 0; z < Z; ++z) {
            int L, U;
            float b;
            fence(z);
            atom(z, L, U, b);
            ub4[z / 4] |= (uint32_t)U << (8 * (z % 4));
            const float p = pm[z];
            const float ml = p * ((float)U - b);
            pm[z] = p * (b - (float)L);
            mono = mono && L >= prev;
            acc = (L == prev ? acc : 0.f) + ml;
            sA[L * 64 + lf] = acc;
            prev = L;
        }
    }
    {
        int prev = -1;
        float acc = 0.f;
#pragma unroll
        for (int z0 = 0; z0 < Z; z0 += 8) {
            // opaque per group: the bin decode and addresses of one group of 8
            // atoms at a time (hoisted for all Z they cost ~140 VGPRs)
            int lu = lane;
            uint32_t w0 = ub4[z0 / 4], w1 = z0 / 4 + 1 < (Z + 3) / 4 ? ub4[z0 / 4 + 1] : 0u;
            asm volatile("" : "+v"(lu), "+v"(w0), "+v"(w1));
            auto ubin = [&](int j) { return (int)(((j < 4 ? w0 : w1) >> (8 * (j % 4))) & 255u); };
            float base[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (z0 + j < Z) base[j] = sA[ubin(j) * 64 + lu];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (z0 + j < Z) {
                    const int U = ubin(j);
                    mono = mono && U >= prev;
                    acc = (U == prev ? acc : base[j]) + pm[z0 + j];
                    sA[U * 64 + lu] = acc;
                    prev = U;
                }
            }
        }
    }
    if (!mono) {  // never for a sorted support and gamma >= 0: ordered read-modify-writes, p re-read
        const float *trow = tdist + ((size_t)i * (ROWS ? 1 : A) + astar) * Z;
        for (int bin = 0; bin < Z; ++bin) sA[bin * 64 + lane] = 0.f;
        for (int z = 0; z < Z; ++z) {
            int L, U;
            float b;
            atom(z, L, U, b);
            sA[L * 64 + lane] += trow[z] * ((float)U - b);
        }
        for (int z = 0; z < Z; ++z) {
            int L, U;
            float b;
            atom(z, L, U, b);
            sA[U * 64 + lane] += trow[z] * (b - (float)L);
        }
    }
    __syncthreads();
    float pr[Z];
#pragma unroll
    for (int bin = 0; bin < Z; ++bin) pr[bin] = sA[bin * 64 + lane];
    if (proj) {  // optional projection output, coalesced over (row, bin)
        for (int e = lane; e < nrows * Z; e += 64) {
            const int rk = e / Z, z = e - rk * Z;
            proj[(size_t)row0 * Z + e] = sA[z * 64 + rk];
        }
    }
    __syncthreads();  // projection read out before the log_p rows land
    dma_rows(logp, a_cur);
    float part = 0.f;
#pragma unroll
    for (int bin = 0; bin < Z; ++bin) part += pr[bin] * sA[lane * Z + bin];
    if (live) loss[i] = -part;
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_td_workspace_bytes(int64_t B) {
    return B > 0 ? (size_t)ceil_div(B, kTdBlock) * sizeof(double) : 0;
}

extern "C" int agx_td_target(const float *q_next_online, const float *q_next_target,
                             const float *q_cur, const int64_t *actions, const float *rewards,
                             const float *dones, int64_t B, int64_t A, double gamma, int double_q,
                             float *y, float *g_q, float *loss, void *workspace, void *stream) {
    AGX_REQUIRE(q_next_target && rewards && dones && y && B >= 0 && A > 0 && A < 65536,
                "agx_td_target: bad arguments");
    AGX_REQUIRE(!double_q || q_next_online, "agx_td_target: double_q needs q_next_online");
    AGX_REQUIRE(!(g_q || loss) || (q_cur && actions), "agx_td_target: loss needs q_cur/actions");
    AGX_REQUIRE(!loss || workspace, "agx_td_target: loss needs the workspace (agx_td_workspace_bytes)");
    if (B == 0) return AGX_OK;
    hipStream_t s = as_stream(stream);
    const int64_t nblk = ceil_div(B, kTdBlock);
    double *part = loss ? static_cast<double *>(workspace) : nullptr;
    td_target_kernel<<<(unsigned)nblk, kTdBlock, 0, s>>>(q_next_online, q_next_target, q_cur, actions, rewards,
                                                         dones, B, (int)A, (float)gamma, double_q, y, g_q, part);
    int rc = check_launch("agx_td_target");
    if (rc || !loss) return rc;
    td_loss_finalize<<<1, 1024, 0, s>>>(part, nblk, B, loss);
    return check_launch("agx_td_target loss");
}

extern "C" int agx_maddpg_critic_target(const float *q, const float *q_next, const float *rewards,
                                        const float *dones, int64_t B, double gamma, float *y, float *g_q,
                                        float *loss, void *workspace, void *stream) {
    AGX_REQUIRE(q && q_next && rewards && dones && loss && workspace && B >= 0,
                "agx_maddpg_critic_target: bad arguments");
    if (B == 0) return AGX_OK;
    hipStream_t s = as_stream(stream);
    const int64_t nblk = ceil_div(B, kTdBlock);
    double *part = static_cast<double *>(workspace);
    maddpg_critic_kernel<<<(unsigned)nblk, kTdBlock, 0, s>>>(q, q_next, rewards, dones, B, (float)gamma, y, g_q,
                                                            part);
    int rc = check_launch("agx_maddpg_critic_target");
    if (rc) return rc;
    td_loss_finalize<<<1, 1024, 0, s>>>(part, nblk, B, loss);
    return check_launch("agx_maddpg_critic_target loss");
}

extern "C" int agx_c51_project_loss_rows(const float *target_rows, const float *logp_rows, const float *rewards,
                                         const float *dones, const float *support, int64_t B, int64_t Z,
                                         double v_min, double v_max, double gamma, float *loss, float *proj,
                                         void *stream) {
    AGX_REQUIRE(target_rows && logp_rows && rewards && dones && support && loss,
                "agx_c51_project_loss_rows: null pointer");
    AGX_REQUIRE(B >= 0 && Z == 51, "agx_c51_project_loss_rows: Z must be 51 (Rainbow's atoms)");
    if (B == 0) return AGX_OK;
    const float dz = (float)((v_max - v_min) / (double)(Z - 1));
    int e2 = 0;
    const double m = std::frexp((v_max - v_min) / (double)(Z - 1), &e2);
    const bool pow2 = m == 0.5 && (double)dz == std::ldexp(1.0, e2 - 1) && e2 > -60 && e2 < 60;
    const float inv = pow2 ? (float)std::ldexp(1.0, 1 - e2) : 0.f;
    auto kern = pow2 ? c51_dma_kernel<51, true, true> : c51_dma_kernel<51, false, true>;
    kern<<<(unsigned)ceil_div(B, kC51LaneRows), 64, 0, as_stream(stream)>>>(
        nullptr, target_rows, logp_rows, nullptr, rewards, dones, support, B, 1, (float)v_min, (float)v_max, dz, inv,
        (float)gamma, loss, proj);
    return check_launch("agx_c51_project_loss_rows");
}

extern "C" int agx_c51_project_loss(const float *q_next_online, const float *target_dist,
                                    const float *logp_cur, const int64_t *actions,
                                    const float *rewards, const float *dones, const float *support,
                                    int64_t B, int64_t A, int64_t Z, double v_min, double v_max,
                                    double gamma, float *loss, float *proj, void *stream) {
    AGX_REQUIRE(q_next_online && target_dist && logp_cur && actions && rewards && dones && support &&
                    loss,
                "agx_c51_project_loss: null pointer");
    AGX_REQUIRE(B >= 0 && A > 0 && Z >= 2 && Z <= kC51MaxZ, "agx_c51_project_loss: need 2 <= Z <= %d",
                kC51MaxZ);
    if (B == 0) return AGX_OK;
    const float dz = (float)((v_max - v_min) / (double)(Z - 1));  // python float -> f32 operand
    if (Z == 51 && A <= 64) {  // Rainbow's 51 atoms
        int e2 = 0;
        const double m = std::frexp((v_max - v_min) / (double)(Z - 1), &e2);
        const bool pow2 = m == 0.5 && (double)dz == std::ldexp(1.0, e2 - 1) && e2 > -60 && e2 < 60;
        const float inv = pow2 ? (float)std::ldexp(1.0, 1 - e2) : 0.f;
        auto kern = pow2 ? c51_dma_kernel<51, true> : c51_dma_kernel<51, false>;
        kern<<<(unsigned)ceil_div(B, kC51LaneRows), 64, 0, as_stream(stream)>>>(
            q_next_online, target_dist, logp_cur, actions, rewards, dones, support, B, (int)A, (float)v_min,
            (float)v_max, dz, inv, (float)gamma, loss, proj);
        return check_launch("agx_c51_project_loss");
    }
    if (Z <= 64 && A <= 64) {
        constexpr int R = 4;
        const int64_t rows_per_block = (int64_t)kC51RowWaves * R;
        c51_rows_kernel<R><<<(unsigned)ceil_div(B, rows_per_block), kC51RowWaves * 64, 0, as_stream(stream)>>>(
            q_next_online, target_dist, logp_cur, actions, rewards, dones, support, B, (int)A, (int)Z,
            (float)v_min, (float)v_max, dz, (float)gamma, loss, proj);
        return check_launch("agx_c51_project_loss");
    }
    c51_kernel<<<(unsigned)ceil_div(B, kC51Waves), kC51Waves * 64, 0, as_stream(stream)>>>(
        q_next_online, target_dist, logp_cur, actions, rewards, dones, support, B, (int)A, (int)Z,
        (float)v_min, (float)v_max, dz, (float)gamma, loss, proj);
    return check_launch("agx_c51_project_loss");
}
