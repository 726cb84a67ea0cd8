// Replay-buffer batch gather (include/agx_replay.h): dst[f][b] = src[f][idx[b]]
// for every stored field in one launch.  Workgroup (chunk c, row b): its lanes
// walk the concatenation of the fields' rows in units of each field's width
// (16 bytes when the field's row size and both base addresses allow it, else
// 4, else 1), so the big uint8 frame rows move as 16-byte vector copies and
// the scalar fields ride in the same launch.
#include <cstdint>

#include "agx_common.h"
#include "../../include/agx_replay.h"

namespace agx {

namespace rg {

struct Fields {
    const unsigned char *src[AGX_REPLAY_MAX_FIELDS];
    unsigned char *dst[AGX_REPLAY_MAX_FIELDS];
    long long row_bytes[AGX_REPLAY_MAX_FIELDS];
    long long unit_start[AGX_REPLAY_MAX_FIELDS + 1];  // prefix sums of units per row
    int width[AGX_REPLAY_MAX_FIELDS];
    int n;
};

__global__ __launch_bounds__(256) void gather_kernel(Fields fs, const int64_t *idx, long long rows, int *err) {
    const long long b = blockIdx.y;
    const long long r = idx[b];
    if (r < 0 || r >= rows) {
        if (err && threadIdx.x == 0 && blockIdx.x == 0) *err = 1;
        return;
    }
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < fs.unit_start[fs.n];
         u += (long long)gridDim.x * blockDim.x) {
        int f = 0;
#pragma unroll
        for (int k = 1; k < AGX_REPLAY_MAX_FIELDS; ++k) f += (k < fs.n && u >= fs.unit_start[k]) ? 1 : 0;
        const long long off = (u - fs.unit_start[f]) * fs.width[f];
        const unsigned char *s = fs.src[f] + r * fs.row_bytes[f] + off;
        unsigned char *d = fs.dst[f] + b * fs.row_bytes[f] + off;
        switch (fs.width[f]) {
            case 16: *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(s); break;
            case 4: *reinterpret_cast<unsigned *>(d) = *reinterpret_cast<const unsigned *>(s); break;
            default: *d = *s; break;
        }
    }
}

}  // namespace rg

extern "C" int agx_replay_gather(const void *const *src, void *const *dst, const int64_t *row_bytes, int nfields,
                                 const int64_t *idx, int64_t B, int64_t rows, int *err, void *stream) {
    AGX_REQUIRE(src && dst && row_bytes && idx && nfields >= 1 && nfields <= AGX_REPLAY_MAX_FIELDS && B >= 0 &&
                    rows >= 1,
                "agx_replay_gather: bad arguments (1..%d fields)", AGX_REPLAY_MAX_FIELDS);
    if (B == 0) return AGX_OK;
    AGX_REQUIRE(B < 65536, "agx_replay_gather: batch %lld too large", (long long)B);
    rg::Fields fs{};
    fs.n = nfields;
    long long units = 0;
    for (int f = 0; f < nfields; ++f) {
        AGX_REQUIRE(src[f] && dst[f] && row_bytes[f] >= 1, "agx_replay_gather: field %d incomplete", f);
        const uintptr_t a = reinterpret_cast<uintptr_t>(src[f]) | reinterpret_cast<uintptr_t>(dst[f]);
        const long long rb = row_bytes[f];
        const int w = (rb % 16 == 0 && a % 16 == 0) ? 16 : (rb % 4 == 0 && a % 4 == 0) ? 4 : 1;
        fs.src[f] = static_cast<const unsigned char *>(src[f]);
        fs.dst[f] = static_cast<unsigned char *>(dst[f]);
        fs.row_bytes[f] = rb;
        fs.width[f] = w;
        fs.unit_start[f] = units;
        units += rb / w;
    }
    fs.unit_start[nfields] = units;
    const unsigned chunks = (unsigned)ceil_div(units, 256);
    dim3 grid(chunks < 64 ? chunks : 64, (unsigned)B);
    rg::gather_kernel<<<grid, 256, 0, as_stream(stream)>>>(fs, idx, rows, err);
    return check_launch("agx_replay_gather");
}

}  // namespace agx
