// Population row gather in place (the single-rank generation step's clone,
// hpo/population_sync.py; tournament.py:71-119 + core/base.py clone): every
// per-agent buffer (parameters, both Adam moments, lr, Adam step, per-agent
// hyperparameters — rows of 4-byte words) gets row j := old row idx[j], for all
// buffers in two launches (gather into a workspace, copy back) instead of a
// gather + copy per buffer.  idx may repeat rows (a parent cloned twice).
#include "agx_common.h"

namespace agx {

struct RowBufs {
    float *ptr[AGX_ROWS_MAX_BUFS];
    int64_t width[AGX_ROWS_MAX_BUFS];  // 4-byte words per row
    int64_t off[AGX_ROWS_MAX_BUFS + 1];  // prefix sums of width
    int n;
};

template <bool kBack>
__global__ void rows_copy_kernel(RowBufs b, const int64_t *__restrict__ idx, int64_t P, float *__restrict__ ws) {
    const int64_t j = blockIdx.y;  // destination row
    const int64_t total = b.off[b.n];
    const int64_t src = kBack ? j : idx[j];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int k = 0;
        while (k + 1 < b.n && i >= b.off[k + 1]) ++k;
        const int64_t c = i - b.off[k];
        if (kBack) b.ptr[k][j * b.width[k] + c] = ws[j * total + i];
        else ws[j * total + i] = b.ptr[k][src * b.width[k] + c];
    }
}

}  // namespace agx

using namespace agx;

extern "C" size_t agx_rows_gather_workspace_bytes(const int64_t *widths, int nbuf, int64_t P) {
    if (!widths || nbuf < 1 || nbuf > AGX_ROWS_MAX_BUFS || P < 1) return 0;
    int64_t t = 0;
    for (int k = 0; k < nbuf; ++k) t += widths[k];
    return (size_t)t * (size_t)P * sizeof(float);
}

extern "C" int agx_rows_gather(float *const *bufs, const int64_t *widths, int nbuf, int64_t P, const int64_t *idx,
                               void *workspace, void *stream) {
    AGX_REQUIRE(bufs && widths && idx && workspace && nbuf >= 1 && nbuf <= AGX_ROWS_MAX_BUFS && P >= 1 && P <= 65535,
                "agx_rows_gather: bad arguments (1 <= nbuf <= %d)", AGX_ROWS_MAX_BUFS);
    RowBufs b{};
    b.n = nbuf;
    b.off[0] = 0;
    for (int k = 0; k < nbuf; ++k) {
        AGX_REQUIRE(bufs[k] && widths[k] > 0, "agx_rows_gather: buffer %d null or empty", k);
        b.ptr[k] = bufs[k];
        b.width[k] = widths[k];
        b.off[k + 1] = b.off[k] + widths[k];
    }
    const int64_t total = b.off[nbuf];
    const unsigned gx = (unsigned)(ceil_div(total, 256) < 64 ? ceil_div(total, 256) : 64);
    dim3 grid(gx, (unsigned)P);
    hipStream_t s = as_stream(stream);
    float *ws = static_cast<float *>(workspace);
    rows_copy_kernel<false><<<grid, 256, 0, s>>>(b, idx, P, ws);
    if (int rc = check_launch("agx_rows_gather")) return rc;
    rows_copy_kernel<true><<<grid, 256, 0, s>>>(b, idx, P, ws);
    return check_launch("agx_rows_gather");
}
