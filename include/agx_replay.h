/* Replay-buffer batch gather: every field of the sampled transitions in one
 * launch.  ReplayBuffer.sample / PrioritizedReplayBuffer.sample
 * (agilerl/components/replay_buffer.py:97-137, 361-409) index each stored
 * field with the sampled indices (one index op per field in torch); here the
 * fields' rows move together, 16 bytes per lane where a field's rows allow
 * it.  Binding: INTEGRATION.md. */
#ifndef AGX_REPLAY_H
#define AGX_REPLAY_H

#include "agx.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AGX_REPLAY_MAX_FIELDS 8

/* For each field f < nfields: dst[f] row b (row_bytes[f] bytes) = src[f] row
 * idx[b]; idx device int64 [B], each in [0, rows) (checked: a bad index sets
 * *err to 1 and its rows are left unwritten; err may be NULL). */
int agx_replay_gather(const void *const *src, void *const *dst, const int64_t *row_bytes, int nfields,
                      const int64_t *idx, int64_t B, int64_t rows, int *err, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* AGX_REPLAY_H */
