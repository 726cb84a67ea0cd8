// Prioritized-replay sum/min segment trees in HBM (f64), batched.
//
// Reference: agilerl/components/segment_tree.py (SumSegmentTree /
// MinSegmentTree: 1-indexed heap of 2*capacity floats, __setitem__ :81-95,
// retrieve :136-156) and agilerl/components/replay_buffer.py:261-428
// (PrioritizedReplayBuffer: add :296-309, _update_priority :311-329,
// _sample_proportional :357-381, _calculate_weights :383-409,
// update_priorities :411-428).
//
// Exactness argument: the reference recomputes every ancestor of a written
// leaf as op(left, right) of its CURRENT children, so after any sequence of
// writes every internal node equals op(children) — the tree is a pure
// function of the leaves.  We therefore (1) resolve the batch to its final
// leaf values (last duplicate wins, as the sequential loop does),
// (2) rebuild the dirty paths level-synchronously.  Identical f64 adds/mins
// in identical operand order => bit-identical nodes.
//
// Small batches (<= 1024: config-3 inserts and learn-step updates) run in
// ONE workgroup: LDS dedup, __syncthreads between levels, child reads via
// agent-scope (L1-bypassing) loads.  Large batches run level-per-launch with
// a global "last writer" table; the last 11 levels (<= 2047 nodes) are redone
// whole by one workgroup.
//
// Sampling: one lane per stratum; the top kTopLevels levels of the sum tree
// are staged into LDS once per 1024 samples when the batch is large, the
// rest of the walk reads HBM/L2.  Algorithmic bytes:
// 8 B x depth (left-child reads) + 4 B uniform + 8 B index per sample.
#include "agx_common.h"
#include "libm_pow.h"

namespace agx {

constexpr int kSmallBatch = 1024;
constexpr int kTopLevels = 11;  // nodes 1 .. 2047 (16 KiB) staged in LDS
constexpr int kTopNodes = (1 << kTopLevels) - 1;

__device__ __forceinline__ double ld_agent(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void atomic_max_pos_double(double *addr, double v) {
    // positive doubles order like their bit patterns
    atomicMax(reinterpret_cast<unsigned long long *>(addr), (unsigned long long)__double_as_longlong(v));
}

__global__ void per_fill(double *__restrict__ sum_tree, double *__restrict__ min_tree, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
         i += (int64_t)gridDim.x * blockDim.x) {
        sum_tree[i] = 0.0;
        min_tree[i] = __builtin_inf();
    }
}

__device__ __forceinline__ void recompute(double *sum_tree, double *min_tree, int64_t k) {
    const double a = ld_agent(sum_tree + 2 * k), b = ld_agent(sum_tree + 2 * k + 1);
    sum_tree[k] = a + b;
    const double c = ld_agent(min_tree + 2 * k), d = ld_agent(min_tree + 2 * k + 1);
    min_tree[k] = (d < c) ? d : c;  // Python min(c, d): c unless d < c
}

// ---- one-workgroup path ---------------------------------------------------
// mode 0: update (per-index priorities, floor, max update); mode 1: add
// (ring positions, every leaf = max_priority ** alpha).
template <int kMode>
__global__ __launch_bounds__(kSmallBatch) void per_small(
    double *__restrict__ sum_tree, double *__restrict__ min_tree, int64_t cap, int levels,
    int64_t max_size, const int64_t *__restrict__ indices, const float *__restrict__ pri,
    int64_t start, int n, double alpha, double floor_, double *__restrict__ max_priority) {
    __shared__ int64_t s_idx[kSmallBatch];
    __shared__ double s_max[kSmallBatch / kWave];
    const int i = threadIdx.x;
    const bool act = i < n;
    int64_t idx = 0;
    double p = 0.0;
    if (act) {
        if (kMode == 0) {
            idx = indices[i];
            p = (double)pri[i];
            if (p < floor_) p = floor_;  // max(priority.item(), floor)
        } else {
            idx = (start + i) % max_size;
        }
    }
    s_idx[i] = act ? idx : -1;
    // batch max priority (order-free)
    double pm = act ? p : 0.0;
    for (int o = 32; o > 0; o >>= 1) pm = fmax(pm, __shfl_xor(pm, o, 64));
    if ((i & 63) == 0) s_max[i / 64] = pm;
    __syncthreads();
    bool writer = act;
    if (kMode == 0 && act) {
        for (int j = i + 1; j < n; ++j)
            if (s_idx[j] == idx) {
                writer = false;
                break;
            }
    }
    double leaf = 0.0;
    if (kMode == 0) {
        if (writer) leaf = libm_pow(p, alpha);
    } else {
        leaf = libm_pow(*max_priority, alpha);
    }
    if (writer) {
        sum_tree[cap + idx] = leaf;
        min_tree[cap + idx] = leaf;
    }
    __syncthreads();
    if (kMode == 0 && i == 0) {
        double m = *max_priority;
        for (int w = 0; w < kSmallBatch / kWave; ++w) m = fmax(m, s_max[w]);
        *max_priority = m;
    }
    int64_t node = cap + idx;
    for (int l = 0; l < levels; ++l) {
        node >>= 1;
        if (act) recompute(sum_tree, min_tree, node);  // duplicates write identical values
        __syncthreads();
    }
}

// ---- multi-launch path ----------------------------------------------------
__global__ void per_mark(int32_t *__restrict__ win, const int64_t *__restrict__ indices, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) win[indices[i]] = -1;
}

// The running max priority is one address: an atomic per wave serialises
// ~1k same-address atomics at L2 (14 us at 2^16 updates).  One per block, and
// only when the block's max exceeds the value already there (max only grows).
__global__ __launch_bounds__(256) void per_claim(int32_t *__restrict__ win, const int64_t *__restrict__ indices,
                                                 const float *__restrict__ pri, int64_t n, double floor_,
                                                 double *__restrict__ max_priority) {
    __shared__ double red[256 / kWave];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double pm = 0.0;
    if (i < n) {
        atomicMax(win + indices[i], (int32_t)i);
        double p = (double)pri[i];
        pm = p < floor_ ? floor_ : p;
    }
    for (int o = 32; o > 0; o >>= 1) pm = fmax(pm, __shfl_xor(pm, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pm;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 256 / kWave; ++w) pm = fmax(pm, red[w]);
        if (pm > 0.0 && pm > __hip_atomic_load(max_priority, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomic_max_pos_double(max_priority, pm);
    }
}

__global__ void per_write_leaves(double *__restrict__ sum_tree, double *__restrict__ min_tree,
                                 int64_t cap, const int32_t *__restrict__ win,
                                 const int64_t *__restrict__ indices, const float *__restrict__ pri,
                                 int64_t n, double alpha, double floor_) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t idx = indices[i];
    if (win[idx] != (int32_t)i) return;
    double p = (double)pri[i];
    if (p < floor_) p = floor_;
    const double leaf = libm_pow(p, alpha);
    sum_tree[cap + idx] = leaf;
    min_tree[cap + idx] = leaf;
}

__global__ void per_add_leaves(double *__restrict__ sum_tree, double *__restrict__ min_tree,
                               int64_t cap, int64_t max_size, int64_t start, int64_t n,
                               double alpha, const double *__restrict__ max_priority) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double leaf = libm_pow(*max_priority, alpha);
    const int64_t idx = (start + i) % max_size;
    sum_tree[cap + idx] = leaf;
    min_tree[cap + idx] = leaf;
}

// recompute level `shift` ancestors of the touched leaves
__global__ void per_level(double *__restrict__ sum_tree, double *__restrict__ min_tree, int64_t cap,
                          const int64_t *__restrict__ indices, int64_t max_size, int64_t start,
                          int64_t n, int shift) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t idx = indices ? indices[i] : (start + i) % max_size;
    const int64_t node = (cap + idx) >> shift;
    const double a = sum_tree[2 * node], b = sum_tree[2 * node + 1];
    sum_tree[node] = a + b;
    const double c = min_tree[2 * node], d = min_tree[2 * node + 1];
    min_tree[node] = (d < c) ? d : c;
}

// recompute every node of the top `levels` levels (nodes 1 .. 2^levels - 1)
// from the 2^levels nodes below them, staged once in LDS (one HBM round trip
// instead of one per level)
__global__ __launch_bounds__(1024) void per_top(double *__restrict__ sum_tree,
                                                double *__restrict__ min_tree, int levels) {
    __shared__ double s_sum[1 << kTopLevels], s_min[1 << kTopLevels];
    const int tid = threadIdx.x;
    const int nin = 1 << levels;
    for (int j = tid; j < nin; j += 1024) {
        s_sum[j] = ld_agent(sum_tree + nin + j);
        s_min[j] = ld_agent(min_tree + nin + j);
    }
    __syncthreads();
    for (int l = levels - 1; l >= 0; --l) {
        const int m = 1 << l;
        const bool act = tid < m;
        double a = 0.0, c = 0.0;
        if (act) {
            a = s_sum[2 * tid] + s_sum[2 * tid + 1];
            const double c0 = s_min[2 * tid], d0 = s_min[2 * tid + 1];
            c = (d0 < c0) ? d0 : c0;  // Python min(c, d)
            sum_tree[m + tid] = a;
            min_tree[m + tid] = c;
        }
        __syncthreads();
        if (act) {
            s_sum[tid] = a;
            s_min[tid] = c;
        }
        __syncthreads();
    }
}

// recompute EVERY node of levels [r, r + k) from the (final) nodes of level
// r + k: workgroup w owns the subtree rooted at node 2^r + w, stages its 2^k
// inputs of both trees in LDS and writes each level back with coalesced
// stores.  The tree is a pure function of the leaves, so a whole-band rebuild
// gives the same bits as the dirty-path walk (same operands, same order).
constexpr int kBandLevels = 9;  // 512 inputs per subtree: 8 KiB of LDS for both trees
__global__ __launch_bounds__(256) void per_band(double *__restrict__ sum_tree, double *__restrict__ min_tree,
                                               int r, int k) {
    static_assert((1 << kBandLevels) <= 2 * 256, "one node per thread on the first level");
    __shared__ double s_sum[1 << kBandLevels], s_min[1 << kBandLevels];
    const int w = blockIdx.x, tid = threadIdx.x;
    const int64_t root = ((int64_t)1 << r) + w;
    const int64_t in0 = root << k;  // first input node (level r + k)
    for (int j = tid; j < (1 << k); j += 256) {
        s_sum[j] = sum_tree[in0 + j];
        s_min[j] = min_tree[in0 + j];
    }
    __syncthreads();
    for (int l = k - 1; l >= 0; --l) {  // level r + l: 2^l <= 256 nodes of this subtree
        const bool act = tid < (1 << l);
        double a = 0.0, c = 0.0;
        if (act) {
            a = s_sum[2 * tid] + s_sum[2 * tid + 1];
            const double c0 = s_min[2 * tid], d0 = s_min[2 * tid + 1];
            c = (d0 < c0) ? d0 : c0;  // Python min(c, d): c unless d < c
            sum_tree[(root << l) + tid] = a;
            min_tree[(root << l) + tid] = c;
        }
        __syncthreads();
        if (act) {
            s_sum[tid] = a;
            s_min[tid] = c;
        }
        __syncthreads();
    }
}

// ---- sampling ---------------------------------------------------------------
template <bool kStage>
__global__ __launch_bounds__(256) void per_sample_kernel(
    const double *__restrict__ sum_tree, const double *__restrict__ min_tree, int64_t cap,
    int levels, const float *__restrict__ u, int64_t B, double size, double beta,
    int64_t *__restrict__ out_idx, float *__restrict__ weights, int32_t *__restrict__ err) {
    __shared__ double top[kStage ? kTopNodes + 1 : 1];
    const int stage_levels = kStage ? (levels < kTopLevels ? levels : kTopLevels) : 0;
    if (kStage) {
        const int nodes = (1 << stage_levels);  // copies nodes 0 .. 2^s - 1
        for (int k = threadIdx.x; k < nodes; k += blockDim.x) top[k] = sum_tree[k];
        __syncthreads();
    }
    const double total = sum_tree[1];
    const double segment = total / (double)B;
    double max_w = 0.0;
    if (weights) max_w = libm_pow(min_tree[1] / total * size, -beta);
    int32_t bad = 0;
    // kPer independent walks per lane advance level by level in lock step: each
    // level issues kPer independent loads, so a lane's latency chain is one
    // walk deep instead of kPer walks (identical arithmetic per walk)
    constexpr int kPer = 4;
    int64_t i[kPer], k[kPer];
    double ub[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        i[r] = ((int64_t)blockIdx.x * kPer + r) * blockDim.x + threadIdx.x;
        k[r] = 1;
        ub[r] = 0.0;
        if (i[r] < B) {
            const double a = segment * (double)i[r];
            const double b = segment * (double)(i[r] + 1);
            ub[r] = (double)u[i[r]] * (b - a) + a;
            if (!(ub[r] >= 0.0 && ub[r] <= total + 1e-5)) ++bad;
        }
    }
    // children of node k live at 2k, 2k+1; the LDS copy holds nodes < 2^s;
    // every walk takes exactly `levels` steps (cap = 2^levels)
    for (int lev = 0; lev < levels; ++lev) {
        double left[kPer];
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int64_t l = 2 * k[r];
            // l = 2k lies at depth lev + 1: in the LDS copy iff it is < 2^s
            left[r] = (kStage && lev + 1 < stage_levels) ? top[l] : sum_tree[l];
        }
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int64_t l = 2 * k[r];
            if (left[r] > ub[r]) {
                k[r] = l;
            } else {
                ub[r] -= left[r];
                k[r] = l + 1;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        if (i[r] >= B) continue;
        out_idx[i[r]] = k[r] - cap;
        if (weights) {
            const double ps = sum_tree[k[r]] / total;
            weights[i[r]] = (float)(libm_pow(ps * size, -beta) / max_w);
        }
    }
    if (err && bad) atomicAdd(err, bad);
}

__global__ void per_gather_kernel(const double *__restrict__ tree, const int64_t *__restrict__ nodes,
                                  int64_t n, double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = tree[nodes[i]];
}

__global__ void pow_kernel(const double *x, const double *y, double *o, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = libm_pow(x[i], y[i]);
}

static inline int log2_exact(int64_t cap) {
    int l = 0;
    while (((int64_t)1 << l) < cap) ++l;
    return l;
}

static int rebuild_large(double *sum_tree, double *min_tree, int64_t cap, const int64_t *indices,
                         int64_t max_size, int64_t start, int64_t n, hipStream_t s) {
    const int levels = log2_exact(cap);
    const int top = levels < kTopLevels ? levels : kTopLevels;
    const unsigned blocks = (unsigned)ceil_div(n, 256);
    if (n * 32 >= cap && levels > top) {
        // dense batch: nearly every subtree is dirty; rebuild whole bands of
        // kBandLevels levels bottom-up (one launch per band, no per-level launches)
        for (int lo = levels; lo > top;) {
            const int k = lo - top < kBandLevels ? lo - top : kBandLevels;
            per_band<<<(unsigned)((int64_t)1 << (lo - k)), 256, 0, s>>>(sum_tree, min_tree, lo - k, k);
            lo -= k;
        }
        per_top<<<1, 1024, 0, s>>>(sum_tree, min_tree, top);
        return check_launch("agx_per rebuild");
    }
    // levels whose nodes lie below the top block: shift 1 .. levels - top
    for (int shift = 1; shift <= levels - top; ++shift)
        per_level<<<blocks, 256, 0, s>>>(sum_tree, min_tree, cap, indices, max_size, start, n, shift);
    per_top<<<1, 1024, 0, s>>>(sum_tree, min_tree, top);
    return check_launch("agx_per rebuild");
}

}  // namespace agx

using namespace agx;

static bool pow2(int64_t c) { return c > 0 && (c & (c - 1)) == 0; }

extern "C" size_t agx_per_workspace_bytes(int64_t capacity, int64_t max_batch) {
    (void)max_batch;
    return (size_t)capacity * sizeof(int32_t);
}

extern "C" int agx_per_init(double *sum_tree, double *min_tree, int64_t capacity, void *stream) {
    AGX_REQUIRE(sum_tree && min_tree && pow2(capacity), "agx_per_init: capacity must be a power of 2");
    const int64_t n2 = 2 * capacity;
    const int64_t blocks = ceil_div(n2, 256);
    per_fill<<<(unsigned)(blocks > 4096 ? 4096 : blocks), 256, 0, as_stream(stream)>>>(sum_tree, min_tree, n2);
    return check_launch("agx_per_init");
}

extern "C" int agx_per_add(double *sum_tree, double *min_tree, int64_t capacity, int64_t max_size,
                           int64_t start, int64_t n, double alpha, const double *max_priority,
                           void *workspace, void *stream) {
    (void)workspace;
    AGX_REQUIRE(sum_tree && min_tree && max_priority && pow2(capacity) && max_size > 0 &&
                    max_size <= capacity && start >= 0 && start < max_size && n >= 0,
                "agx_per_add: bad arguments");
    if (n == 0) return AGX_OK;
    hipStream_t s = as_stream(stream);
    if (n > max_size) {  // a ring longer than the buffer: only the last max_size writes survive
        start = (start + (n - max_size)) % max_size;
        n = max_size;
    }
    if (n <= kSmallBatch) {
        per_small<1><<<1, kSmallBatch, 0, s>>>(sum_tree, min_tree, capacity, log2_exact(capacity),
                                                max_size, nullptr, nullptr, start, (int)n, alpha, 0.0,
                                                const_cast<double *>(max_priority));
        return check_launch("agx_per_add");
    }
    per_add_leaves<<<(unsigned)ceil_div(n, 256), 256, 0, s>>>(sum_tree, min_tree, capacity, max_size,
                                                             start, n, alpha, max_priority);
    int rc = check_launch("agx_per_add leaves");
    if (rc) return rc;
    return rebuild_large(sum_tree, min_tree, capacity, nullptr, max_size, start, n, s);
}

extern "C" int agx_per_update(double *sum_tree, double *min_tree, int64_t capacity, int64_t max_size,
                              const int64_t *indices, const float *priorities, int64_t n, double alpha,
                              double floor_, double *max_priority, void *workspace, void *stream) {
    AGX_REQUIRE(sum_tree && min_tree && indices && priorities && max_priority && pow2(capacity) &&
                    max_size > 0 && max_size <= capacity && n >= 0 && n < ((int64_t)1 << 31),
                "agx_per_update: bad arguments");
    if (n == 0) return AGX_OK;
    hipStream_t s = as_stream(stream);
    if (n <= kSmallBatch) {
        per_small<0><<<1, kSmallBatch, 0, s>>>(sum_tree, min_tree, capacity, log2_exact(capacity),
                                                max_size, indices, priorities, 0, (int)n, alpha,
                                                floor_, max_priority);
        return check_launch("agx_per_update");
    }
    AGX_REQUIRE(workspace, "agx_per_update: batches > %d need agx_per_workspace_bytes() of workspace",
                kSmallBatch);
    int32_t *win = static_cast<int32_t *>(workspace);
    const unsigned blocks = (unsigned)ceil_div(n, 256);
    per_mark<<<blocks, 256, 0, s>>>(win, indices, n);
    per_claim<<<blocks, 256, 0, s>>>(win, indices, priorities, n, floor_, max_priority);
    per_write_leaves<<<blocks, 256, 0, s>>>(sum_tree, min_tree, capacity, win, indices, priorities, n,
                                           alpha, floor_);
    int rc = check_launch("agx_per_update leaves");
    if (rc) return rc;
    return rebuild_large(sum_tree, min_tree, capacity, indices, max_size, 0, n, s);
}

extern "C" int agx_per_sample(const double *sum_tree, const double *min_tree, int64_t capacity,
                              const float *uniforms, int64_t B, int64_t size, double beta,
                              int64_t *indices, float *weights, int32_t *err, void *stream) {
    AGX_REQUIRE(sum_tree && uniforms && indices && pow2(capacity) && B >= 0,
                "agx_per_sample: bad arguments");
    AGX_REQUIRE(!weights || (min_tree && size > 0), "agx_per_sample: weights need min_tree and size");
    if (B == 0) return AGX_OK;
    hipStream_t s = as_stream(stream);
    const int levels = log2_exact(capacity);
    const int64_t per_block = 256 * 4;
    const unsigned blocks = (unsigned)ceil_div(B, per_block);
    if (B >= 8192)
        per_sample_kernel<true><<<blocks, 256, 0, s>>>(sum_tree, min_tree, capacity, levels, uniforms, B,
                                                       (double)size, beta, indices, weights, err);
    else
        per_sample_kernel<false><<<blocks, 256, 0, s>>>(sum_tree, min_tree, capacity, levels, uniforms,
                                                        B, (double)size, beta, indices, weights, err);
    return check_launch("agx_per_sample");
}

extern "C" int agx_per_gather(const double *tree, const int64_t *nodes, int64_t n, double *out,
                              void *stream) {
    AGX_REQUIRE(tree && nodes && out && n >= 0, "agx_per_gather: bad arguments");
    if (n == 0) return AGX_OK;
    per_gather_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(tree, nodes, n, out);
    return check_launch("agx_per_gather");
}

extern "C" int agx_debug_pow(const double *x, const double *y, double *out, int64_t n, void *stream) {
    AGX_REQUIRE(x && y && out && n >= 0, "agx_debug_pow: bad arguments");
    if (n == 0) return AGX_OK;
    pow_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(x, y, out, n);
    return check_launch("agx_debug_pow");
}
