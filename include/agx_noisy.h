/* Rainbow's dueling head streams: the value and advantage MLPs of
 * DuelingDistributionalMLP (agilerl/networks/custom_modules.py:20-162), each
 * a stack of NoisyLinear -> LayerNorm -> ReLU hidden layers and a NoisyLinear
 * output layer (agilerl/modules/mlp.py create_mlp, noisy = True,
 * layer_norm = True), forward and backward for all streams in one launch
 * per layer depth.
 *
 * The reference runs every layer as torch ops: the noisy weight
 * mu + sigma * eps (custom_components.py:124-131), the Linear, LayerNorm and
 * ReLU, each stream separately, and autograd's matching backward ops.  At
 * the batch sizes of a Rainbow update (B = 64 rows) each of those is a
 * launch-latency-bound kernel; here one launch per depth forms the noisy
 * weights in the operand loads (mu + sigma * eps rounded as torch rounds
 * it), normalises the previous layer's output in the loads, and runs the
 * GEMM on f32 MFMA tiles.  The backward launch of a depth computes the
 * weight / bias / LayerNorm gradients (d mu = dW, d sigma = dW * eps) and
 * the input gradient (summed over the streams at depth 0, where every
 * stream reads the same latent).
 *
 * Replaces the calls DuelingDistributionalMLP.forward makes into its two
 * streams (agilerl/networks/custom_modules.py:127-162, self.model(x) and
 * self.advantage_net(x)) and autograd's backward through them; binding:
 * INTEGRATION.md. */
#ifndef AGX_NOISY_H
#define AGX_NOISY_H

#include "agx.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AGX_NOISY_MAX_STREAMS 6
#define AGX_NOISY_MAX_LAYERS 4
#define AGX_NOISY_MAX_ROWS 1024

/* One layer of one stream, nn.Linear layout.  Weight [fout][fin] =
 * w_mu + w_sigma * w_eps (w_sigma == NULL: the plain weight w_mu, e.g. a
 * NoisyLinear in eval mode); bias [fout] likewise.  Hidden layers carry the
 * LayerNorm(fout) affine (ln_gamma, ln_beta), applied with ReLU before the
 * next layer; the output layer has ln_gamma == NULL.  out [B][fout]: the
 * layer's output before normalisation — written by the forward, read by the
 * backward.  ln_part [B][ceil(fout / 16)][2] (hidden layers): the forward's
 * LayerNorm statistics of out per 16-feature tile (mean, sum of squared
 * deviations), combined in tile order wherever a row's mean / rstd is needed
 * (forward and backward alike).  grad_*: backward outputs (grad_w_sigma /
 * grad_b_sigma only with w_sigma, grad_ln_* only on hidden layers). */
typedef struct agx_noisy_stream_layer {
    const float *w_mu, *w_sigma, *w_eps;
    const float *b_mu, *b_sigma, *b_eps;
    const float *ln_gamma, *ln_beta;
    float *out;
    float *ln_part;
    float *grad_w_mu, *grad_w_sigma, *grad_b_mu, *grad_b_sigma, *grad_ln_gamma, *grad_ln_beta;
    int32_t fin, fout;
} agx_noisy_stream_layer;

/* layers [n_streams][n_layers]; every stream's layer 0 reads x [B][fin].
 * 1 <= n_streams <= 6, 1 <= n_layers <= 4, 0 <= B <= 1024. */
int agx_noisy_streams_forward(const agx_noisy_stream_layer *layers, int32_t n_streams, int32_t n_layers, const float *x,
                              int64_t B, float ln_eps, void *stream);

/* The same forward with stream s's layer 0 reading xs[s] [B][fin] (no-grad
 * passes over several networks at once: RainbowDQN's online and target
 * heads on the next observations, each on its own network's latent, and
 * the online head on the observations whose backward follows). */
int agx_noisy_streams_forward_each(const agx_noisy_stream_layer *layers, int32_t n_streams, int32_t n_layers,
                                   const float *const *xs, int64_t B, float ln_eps, void *stream);

/* Bytes of device workspace agx_noisy_streams_backward needs (the gradients
 * of the hidden activations and their per-tile LayerNorm-backward sums). */
size_t agx_noisy_streams_workspace_bytes(const agx_noisy_stream_layer *layers, int32_t n_streams, int32_t n_layers,
                                         int64_t B);

/* grad_out[s] [B][fout of the last layer]: d loss / d (stream s's output);
 * grad_x [B][fin] (NULL: not needed): d loss / d x summed over the streams.
 * Reads the forward's out and ln_part buffers; writes every grad_* of
 * every layer. */
int agx_noisy_streams_backward(const agx_noisy_stream_layer *layers, int32_t n_streams, int32_t n_layers, const float *x,
                               int64_t B, float ln_eps, const float *const *grad_out, float *grad_x, void *workspace,
                               void *stream);

#ifdef __cplusplus
}
#endif

#endif /* AGX_NOISY_H */
