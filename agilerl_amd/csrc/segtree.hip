// Single segment trees (sum or min) in HBM: the generic SegmentTree /
// SumSegmentTree / MinSegmentTree API (agilerl/components/segment_tree.py)
// for callers that use one tree on its own.  The prioritized-replay pair goes
// through agx_per_* (per.hip), which updates both trees in one pass.
//
//   agx_segtree_set      SegmentTree.__setitem__ (:81-95) for a batch of
//                        (idx, value) in order: last duplicate wins; every
//                        ancestor recomputed as op(left, right) of its final
//                        children (the tree is a pure function of its leaves,
//                        so this equals the sequential walks bit-for-bit).
//   agx_segtree_operate  SegmentTree.operate (:61-79): the reference's
//                        recursion (_operate_helper :30-59), same operand
//                        order, one lane.
//   agx_segtree_retrieve SumSegmentTree.retrieve (:136-156) for a batch of
//                        f64 upper bounds; err counts failed asserts.
#include "agx_common.h"

namespace agx {

constexpr int kSetBlock = 1024;

__device__ __forceinline__ double seg_ld(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double seg_op(int op, double a, double b) {
    return op == 0 ? a + b : ((b < a) ? b : a);  // Python min(a, b): a unless b < a
}

__global__ void segtree_fill(double *tree, int64_t n2, double v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        tree[i] = v;
}

// n <= kSetBlock: one workgroup, dirty paths rebuilt level by level
__global__ __launch_bounds__(kSetBlock) void segtree_set_small(double *tree, int64_t cap, int op,
                                                               const int64_t *__restrict__ idx,
                                                               const double *__restrict__ val, int n, int depth) {
    __shared__ int64_t sidx[kSetBlock];
    const int t = threadIdx.x;
    if (t < n) sidx[t] = idx[t];
    __syncthreads();
    bool win = t < n;
    if (win)
        for (int j = t + 1; j < n; ++j)
            if (sidx[j] == sidx[t]) {
                win = false;
                break;
            }
    int64_t k = t < n ? cap + sidx[t] : 0;
    if (win) __hip_atomic_store(tree + k, val[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int l = 0; l < depth; ++l) {
        __threadfence_block();
        __syncthreads();
        k >>= 1;
        if (win) {
            const double a = seg_ld(tree + 2 * k), b = seg_ld(tree + 2 * k + 1);
            __hip_atomic_store(tree + k, seg_op(op, a, b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// large batches: winners through a last-writer table, then whole-level rebuilds
__global__ void segtree_claim(int32_t *win, const int64_t *__restrict__ idx, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicMax(win + idx[i], (int32_t)i);
}
__global__ void segtree_write(double *tree, int64_t cap, const int32_t *win, const int64_t *__restrict__ idx,
                              const double *__restrict__ val, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && win[idx[i]] == (int32_t)i) tree[cap + idx[i]] = val[i];
}
__global__ void segtree_level(double *tree, int op, int64_t first, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const int64_t k = first + i;
        tree[k] = seg_op(op, tree[2 * k], tree[2 * k + 1]);
    }
}

// the reference recursion, verbatim in structure (depth <= 2 log2(cap))
__device__ double seg_operate(const double *tree, int op, int64_t start, int64_t end, int64_t node, int64_t ns,
                              int64_t ne) {
    if (start == ns && end == ne) return tree[node];
    const int64_t mid = (ns + ne) / 2;
    if (end <= mid) return seg_operate(tree, op, start, end, 2 * node, ns, mid);
    if (mid + 1 <= start) return seg_operate(tree, op, start, end, 2 * node + 1, mid + 1, ne);
    const double a = seg_operate(tree, op, start, mid, 2 * node, ns, mid);
    const double b = seg_operate(tree, op, mid + 1, end, 2 * node + 1, mid + 1, ne);
    return seg_op(op, a, b);
}
__global__ void segtree_operate_kernel(const double *tree, int64_t cap, int op, int64_t start, int64_t end,
                                       double *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = seg_operate(tree, op, start, end, 1, 0, cap - 1);
}

__global__ void segtree_retrieve_kernel(const double *__restrict__ tree, int64_t cap, const double *__restrict__ ub,
                                        int64_t n, int64_t *__restrict__ out, int32_t *err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double u = ub[i];
    if (err && !(0.0 <= u && u <= tree[1] + 1e-5)) atomicAdd(err, 1);
    int64_t k = 1;
    while (k < cap) {
        const double l = tree[2 * k];
        if (l > u) {
            k = 2 * k;
        } else {
            u -= l;
            k = 2 * k + 1;
        }
    }
    out[i] = k - cap;
}

static bool pow2(int64_t c) { return c > 0 && (c & (c - 1)) == 0; }
static int log2i(int64_t c) {
    int d = 0;
    while (((int64_t)1 << d) < c) ++d;
    return d;
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_segtree_workspace_bytes(int64_t capacity) {
    return capacity > 0 ? (size_t)capacity * sizeof(int32_t) : 0;
}

extern "C" int agx_segtree_init(double *tree, int64_t capacity, int op, void *stream) {
    AGX_REQUIRE(tree && pow2(capacity) && (op == 0 || op == 1),
                "agx_segtree_init: capacity must be positive and a power of 2");
    const int64_t n2 = 2 * capacity;
    const int64_t blocks = ceil_div(n2, 256);
    segtree_fill<<<(unsigned)(blocks > 4096 ? 4096 : blocks), 256, 0, as_stream(stream)>>>(
        tree, n2, op == 0 ? 0.0 : __builtin_inf());
    return check_launch("agx_segtree_init");
}

extern "C" int agx_segtree_set(double *tree, int64_t capacity, int op, const int64_t *indices, const double *values,
                               int64_t n, void *workspace, void *stream) {
    AGX_REQUIRE(tree && pow2(capacity) && (op == 0 || op == 1) && n >= 0, "agx_segtree_set: bad arguments");
    if (n == 0) return AGX_OK;
    AGX_REQUIRE(indices && values, "agx_segtree_set: null pointer");
    hipStream_t s = as_stream(stream);
    const int depth = log2i(capacity);
    if (n <= kSetBlock) {
        segtree_set_small<<<1, kSetBlock, 0, s>>>(tree, capacity, op, indices, values, (int)n, depth);
        return check_launch("agx_segtree_set");
    }
    AGX_REQUIRE(workspace && n < ((int64_t)1 << 31), "agx_segtree_set: large batches need the workspace");
    int32_t *win = static_cast<int32_t *>(workspace);
    if (hipMemsetAsync(win, 0xff, (size_t)capacity * sizeof(int32_t), s) != hipSuccess)
        return check_launch("agx_segtree_set memset");
    const unsigned gb = (unsigned)ceil_div(n, 256);
    segtree_claim<<<gb, 256, 0, s>>>(win, indices, n);
    segtree_write<<<gb, 256, 0, s>>>(tree, capacity, win, indices, values, n);
    for (int64_t first = capacity / 2; first >= 1; first /= 2)
        segtree_level<<<(unsigned)ceil_div(first, 256), 256, 0, s>>>(tree, op, first, first);
    return check_launch("agx_segtree_set");
}

extern "C" int agx_segtree_operate(const double *tree, int64_t capacity, int op, int64_t start, int64_t end,
                                   double *out, void *stream) {
    AGX_REQUIRE(tree && out && pow2(capacity) && (op == 0 || op == 1), "agx_segtree_operate: bad arguments");
    // SegmentTree.operate: end <= 0 counts from capacity; the range is [start, end)
    if (end <= 0) end += capacity;
    end -= 1;
    AGX_REQUIRE(0 <= start && start <= end && end < capacity, "agx_segtree_operate: empty or out-of-range segment");
    segtree_operate_kernel<<<1, 64, 0, as_stream(stream)>>>(tree, capacity, op, start, end, out);
    return check_launch("agx_segtree_operate");
}

extern "C" int agx_segtree_retrieve(const double *tree, int64_t capacity, const double *upperbounds, int64_t n,
                                    int64_t *indices, int32_t *err, void *stream) {
    AGX_REQUIRE(tree && pow2(capacity) && n >= 0, "agx_segtree_retrieve: bad arguments");
    if (n == 0) return AGX_OK;
    AGX_REQUIRE(upperbounds && indices, "agx_segtree_retrieve: null pointer");
    segtree_retrieve_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(tree, capacity, upperbounds,
                                                                                       n, indices, err);
    return check_launch("agx_segtree_retrieve");
}
