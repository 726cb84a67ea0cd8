/*
 * agx.h — C ABI of libagx.so, the MI355X (gfx950) hot path of a
 * population-based RL trainer (drop-in for the mcx/AgileRL hot path).
 *
 * Conventions (every entry point):
 *   - all array pointers are DEVICE pointers owned by the caller
 *     (e.g. torch.Tensor.data_ptr()); layouts are dense, row-major;
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous
 *     on it, does no allocation, no host<->device copy and no synchronisation
 *     (graph-capturable);
 *   - scratch, where needed, is caller-provided; *_workspace_bytes() sizes it;
 *   - return 0 (AGX_OK) or a negative status; agx_last_error() returns a
 *     thread-local message for the last failing call on this thread;
 *   - no C++ exception crosses the ABI; calls on distinct streams are
 *     independent and thread-safe.
 *
 * Each entry point cites the reference (mcx/AgileRL 2.7.0) interface it
 * replaces; paths are relative to the reference checkout.
 */
#ifndef AGX_H
#define AGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AGX_OK 0
#define AGX_EINVAL (-1)       /* bad shape / pointer / argument             */
#define AGX_EHIP (-2)         /* HIP runtime error (launch or device fault) */
#define AGX_EUNSUPPORTED (-3) /* configuration not implemented             */

/* ---- library ------------------------------------------------------------ */
const char *agx_last_error(void);
int agx_version(void); /* major*10000 + minor*100 + patch */
/* Device properties of the current device (CU count, HBM peak guess);
 * fills out[0]=multiProcessorCount, out[1]=gcnArch (950), out[2]=warpSize. */
int agx_device_info(int *out3);

/* ---- GAE / Monte-Carlo returns -------------------------------------------
 * Replaces RolloutBuffer.compute_returns_and_advantages
 * (agilerl/components/rollout_buffer.py:413-481), batched over a population.
 * Layout: P agents x (T, N) time-major SoA, i.e. x[p][t][n].
 * rewards/values f32, dones u8 (the reference's torch.bool), last_value
 * f32 [P][N], last_done u8 [P][N].  Outputs advantages/returns f32 [P][T][N],
 * bit-exact to the reference (f64 carry, the NumPy-2 dtype flow).
 * If adv_stats != NULL, also writes per-agent [mean, unbiased std] (f64) of
 * the advantages, as used by PPO's normalisation (agilerl/algorithms/
 * ppo.py:829-834); this needs `workspace` of agx_gae_workspace_bytes(). */
size_t agx_gae_workspace_bytes(int64_t P, int64_t T, int64_t N);
int agx_gae(const float *rewards, const uint8_t *dones, const float *values,
            const float *last_value, const uint8_t *last_done, int64_t P, int64_t T,
            int64_t N, double gamma, double gae_lambda, int use_gae, float *advantages,
            float *returns, double *adv_stats, void *workspace, void *stream);

/* In-place (a - mean) / (std + 1e-8) per agent (ppo.py:829-834);
 * adv_stats as written by agx_gae.  adv is [P][count]. */
int agx_adv_normalize(float *adv, const double *adv_stats, int64_t P, int64_t count, void *stream);

/* ---- PPO clipped-surrogate loss, forward + backward ----------------------
 * Replaces the loss block of PPO._learn_from_rollout_buffer_flat
 * (agilerl/algorithms/ppo.py:868-902) and its autograd backward.
 * num_minibatches contiguous minibatches of `batch` samples.  logp / value /
 * entropy are the network outputs in minibatch order; old_logp / adv / ret /
 * old_value are read at index[j] when index != NULL (the shuffled minibatch
 * gather of ppo.py:842-848), else at j.
 * Writes d loss / d{logp, value, entropy} per sample and, per minibatch,
 * stats[m*8 + {0:loss, 1:policy_loss, 2:value_loss, 3:entropy_loss,
 *              4:approx_kl, 5:clip_fraction}]. */
int agx_ppo_loss_fwd_bwd(const float *logp, const float *old_logp, const float *adv,
                         const float *ret, const float *old_value, const float *value,
                         const float *entropy, const int64_t *index, int64_t batch,
                         int64_t num_minibatches, float clip_coef, float vf_coef,
                         float ent_coef, float *g_logp, float *g_value, float *g_entropy,
                         float *stats, void *stream);

/* ---- fused PPO learner ----------------------------------------------------
 * Replaces PPO._learn_from_rollout_buffer_flat (agilerl/algorithms/ppo.py:
 * 836-921) end to end for the shared-encoder MLP actor-critic the reference
 * builds (create_mlp, agilerl/utils/evolvable_networks.py:527-644): per
 * agent one workgroup runs all epochs x minibatches (gather -> forward ->
 * loss -> backward -> 2-group grad clip -> Adam) with parameters in LDS and
 * f32 MFMA GEMMs.  Offsets below index one agent's flat parameter row
 * [encoder | actor head | critic head] in state-dict order.
 * Supported: 2-3 encoder Linear layers (hidden: LayerNorm(affine)+ReLU,
 * output: LayerNorm(plain)+ReLU), one hidden layer per head (LN affine +
 * ReLU), widths multiples of 16 (<= 128, heads <= 128 together),
 * obs_dim <= 128, n_actions <= 16, <= 14336 parameters and the LDS plan
 * within 160 KiB; otherwise AGX_EUNSUPPORTED. */
typedef struct agx_ppo_net {
    int32_t obs_dim, n_actions, n_enc;
    int32_t enc_dim[4]; /* enc_dim[0] = obs_dim, enc_dim[i] = width of encoder layer i */
    int32_t enc_w[3], enc_b[3], enc_ln_w[3], enc_ln_b[3];
    int32_t head_actor, head_critic;
    int32_t actor_w, actor_b, actor_ln_w, actor_ln_b, actor_out_w, actor_out_b;
    int32_t critic_w, critic_b, critic_ln_w, critic_ln_b, critic_out_w, critic_out_b;
    int32_t n_params, critic_start;
} agx_ppo_net;

/* LDS bytes the fused learner needs for `net` (0: unsupported). */
size_t agx_ppo_learn_lds_bytes(const agx_ppo_net *net);
/* Device workspace bytes for agx_ppo_learn: arrival counters, the
 * minibatch-ordered copy of the rollout for `epochs` epochs of P agents x S
 * samples, and the gradient hand-off slabs of the partner workgroups (an
 * agent's sub-batches are spread over up to 8 workgroups when P leaves CUs
 * idle; AGX_LEARN_SPLIT=1..8 lowers the choice). */
size_t agx_ppo_learn_workspace_bytes(const agx_ppo_net *net, int64_t P, int64_t S, int64_t epochs);
/* Validates that `net` is one of the instantiated shapes (the kernel plan is
 * compile-time); no device work.  AGX_EUNSUPPORTED otherwise. */
int agx_ppo_learn_prepare(const agx_ppo_net *net, void *workspace, void *stream);
/* Arguments of one agx_ppo_learn call (all device pointers, caller-owned).
 *   params / exp_avg / exp_avg_sq  [P][n_params] f32, updated in place;
 *   adam_step   [P] int64, in/out: Adam steps each agent has taken (the
 *               1-based step of the next update is adam_step[p] + 1; an agent
 *               that stops early on target_kl takes fewer);
 *   lr          [P] f32 per-agent learning rate (HPO-mutable);
 *   obs [P][S][obs_dim] f32, actions [P][S] int64, old_logp / adv / ret /
 *   old_value [P][S] f32 — the rollout SoA flattened as get_tensor_batch
 *   does (rollout_buffer.py:525-577), row t*N + n;
 *   adv_stats   [P][2] f64 (mean, unbiased std; agx_gae) normalises adv on
 *               the fly as ppo.py:829-834, or NULL when adv is normalised;
 *   action_masks [P][S][n_actions] u8 (1 = legal) or NULL: illegal logits
 *               become -1e8 before the log-softmax (distributions.py:16-28);
 *   perms       [epochs][P][S] int64: epoch e, agent p visits rows
 *               perms[e][p][0..S) in order (the reference's cumulative
 *               np.random.shuffle stream, ppo.py:838-842);
 *   target_kl   <= 0: off; else after every epoch an agent stops when the
 *               mean approx_kl over all its minibatches so far exceeds it
 *               (ppo.py:899-902, 917-918);
 *   loss_out    [P] f32 = sum of minibatch losses / (S * epochs) (ppo.py:920);
 *   kl_out      [P] f32 mean approx_kl over the minibatches run, or NULL;
 *   epochs_out  [P] int32 epochs run, or NULL;
 *   error_word  one uint32, sticky: the kernel ORs in
 *               AGX_LEARN_ERR_TIMEOUT (1) when a partner workgroup gave up
 *               waiting (the agent's update is then incomplete) and the
 *               gather prologue ORs in AGX_LEARN_ERR_PERM (2) when a perms
 *               entry it reads lies outside [0, S) (row 0 is gathered in
 *               its place: the update is then invalid, but nothing faults);
 *               never cleared by the library — the caller checks and resets
 *               it (PPOPopulation raises AgxError). */
#define AGX_LEARN_ERR_TIMEOUT 1u
#define AGX_LEARN_ERR_PERM 2u
typedef struct agx_ppo_learn_args {
    int64_t P, S, epochs, batch;
    float *params, *exp_avg, *exp_avg_sq;
    int64_t *adam_step;
    const float *lr;
    float beta1, beta2, eps, max_grad_norm;
    const float *obs;
    const int64_t *actions;
    const float *old_logp, *adv, *ret, *old_value;
    const double *adv_stats;
    const uint8_t *action_masks;
    const int64_t *perms;
    float clip_coef, vf_coef, ent_coef;
    double target_kl;
    float *loss_out, *kl_out;
    int32_t *epochs_out;
    uint32_t *error_word;
    /* heterogeneous population (RL-hyperparameter mutations, mutation.py:
     * 413-453), each NULL = the scalar above for every agent: per-agent
     * minibatch size (<= batch, which sizes the partner split), update
     * epochs (<= epochs; perms rows e >= epochs_per_agent[p] are not read)
     * and entropy coefficient.  loss_out divides by S * epochs_per_agent[p]. */
    const int32_t *batch_per_agent, *epochs_per_agent;
    const float *ent_coef_per_agent;
    /* NULL, or a word the learner reads when it starts (device or coherent
     * host memory): nonzero -> the call leaves params, moments, steps and
     * outputs untouched.  The pipelined PPO iteration passes the persistent
     * rollout's agx_rollout_ctl.timeout word, so a learn queued behind a
     * rollout the host aborted (env exception) or that timed out never runs
     * on the partial rollout. */
    const uint32_t *skip_if_set;
} agx_ppo_learn_args;
int agx_ppo_learn(const agx_ppo_net *net, const agx_ppo_learn_args *args, void *workspace, void *stream);
/* Rollout policy step (PPO.get_action / _get_action_and_values, ppo.py:
 * 400-633) for all P agents x N envs: obs of agent p, env n at
 * obs + p*obs_agent_stride + n*obs_dim; writes (each output may be NULL)
 * actions int64, log_probs, values, entropy at + p*out_agent_stride + n and
 * actions_flat[p*N + n].  sample=1: Gumbel-max draw from Philox4x32-10
 * keyed by seed, counter = (env index, step counter); sample=0: argmax.
 * action_mask: NULL, or legal-action flags of agent p, env n at
 * action_mask + p*mask_agent_stride + n*n_actions (u8, 1 = legal): illegal
 * logits become -1e8 first (ppo.py:529-565, distributions.py:16-28).
 * agent_env_base: NULL, or [P] int64 device array — the global index of
 * agent p's env 0: the Philox stream of its env n is that of global env
 * agent_env_base[p] + n (NULL: p*N + n).  A population sharded over ranks,
 * or split into groups of agents with equal networks, samples exactly what
 * the whole population samples in one launch. */
int agx_ppo_act(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                const float *obs, int64_t obs_agent_stride, const uint8_t *action_mask,
                int64_t mask_agent_stride, int sample, uint64_t seed,
                uint64_t counter, int64_t *actions, float *log_probs, float *values,
                float *entropy, int64_t out_agent_stride, int64_t *actions_flat,
                const int64_t *agent_env_base, void *stream);
/* One vector step of rollout collection for all P agents x N envs
 * (rollouts/on_policy.py:23-203 loop body + RolloutBuffer.add,
 * rollout_buffer.py:235-411), fused into ONE launch:
 *  - stage_obs [P][N][obs_dim] (the packed H2D staging of the env's new
 *    observations) is copied to obs_slot (agent stride obs_agent_stride);
 *  - if stage_rew: reward/done of the PREVIOUS step go to rewards_prev /
 *    dones_prev (slot t-1) and, if scores, the per-env episode accounting
 *    (score += r; on done: return_sum += score, episodes += 1, score = 0;
 *    on_policy.py:147-172) is updated;
 *  - if act: the policy step of agx_ppo_act on stage_obs writes actions /
 *    log_probs / values (slot t, agent stride slot_agent_stride) and the
 *    contiguous actions_flat [P*N] (may be NULL) for the D2H.  stage_* and
 *    actions_flat may be pinned host memory (device-accessible, zero-copy:
 *    the kernel reads the env's staging and writes the actions over the host
 *    link, so a vector step is one launch and one wait).  The call after
 *    the last step uses act=1 with only `values` set for the bootstrap value
 *    (on_policy.py:184-196). */
typedef struct agx_rollout_io {
    const float *stage_obs;
    const float *stage_rew;           /* [P*N] or NULL */
    const uint8_t *stage_done;        /* [P*N] */
    float *obs_slot;                  /* or NULL */
    int64_t obs_agent_stride;
    float *rewards_prev;              /* slot t-1, agent stride prev_agent_stride */
    uint8_t *dones_prev;
    int64_t prev_agent_stride;
    int64_t *actions;                 /* each may be NULL; agent stride slot_agent_stride */
    float *log_probs, *values;
    int64_t slot_agent_stride;
    int64_t *actions_flat;
    float *scores;                    /* [P*N] or NULL */
    double *return_sum;               /* [P*N] */
    int64_t *episodes;                /* [P*N] */
    /* legal-action masks of this step ([P*N][n_actions] u8, 1 = legal, the
     * env's info["action_mask"], on_policy.py:82-110) or NULL; illegal
     * logits become -1e8 before sampling; copied to mask_slot (rollout
     * slot t, agent stride mask_agent_stride) when that is set */
    const uint8_t *stage_mask;
    uint8_t *mask_slot;
    int64_t mask_agent_stride;
    /* [P] global index of each agent's env 0 for the Philox stream, or NULL
     * (agx_ppo_act's agent_env_base) */
    const int64_t *agent_env_base;
} agx_rollout_io;
int agx_ppo_rollout_step(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                         const agx_rollout_io *io, int act, int sample, uint64_t seed,
                         uint64_t counter, void *stream);

/* Persistent rollout: ONE launch runs a whole rollout of nsteps = T + 1
 * agx_ppo_rollout_step calls (ios[0..T]; steps 0..T-1 sample with Philox
 * counters counter0 + 1 + t, step T is the bootstrap step: act, no sample),
 * paced by the host through a control block in coherent host memory
 * (agx_host_alloc):
 *   host:   env step writes the staging  ->  agx_host_signal(ctl, base + t + 1)
 *           -> agx_host_wait(ctl, nwg, base + t + 1) -> actions_flat is ready;
 *   device: each workgroup waits for ctl->seq >= base + t + 1, runs step t
 *           with the parameters resident in LDS, releases its host stores and
 *           sets its done word (uint32 after the header) to base + t + 1.
 * `base` grows by nsteps per rollout, so the block is never reset.  Replaces
 * the per-step launch + event wait of rollouts/on_policy.py:23-203's loop.
 * args_host: agx_rollout_args_bytes(nsteps) of agx_host_alloc memory (the
 * per-step arguments, read by the device as the host releases each step).
 * A workgroup gives up after timeout_s or on seq == AGX_ROLLOUT_ABORT and
 * sets ctl->timeout. */
#define AGX_ROLLOUT_ABORT 0xffffffffu
typedef struct agx_rollout_ctl {
    uint32_t seq;     /* host -> device: last released step (base + t + 1) */
    uint32_t timeout; /* device -> host: a workgroup stopped waiting (1:
                         timeout, 2: abort); agx_ppo_learn_args.skip_if_set */
    uint32_t nwg;     /* workgroups (set by agx_ppo_rollout_persistent)    */
    uint32_t started; /* device -> host: workgroups resident so far (each
                         adds 1 when it starts; the host clears it before
                         launching): a host pacing several launches paces
                         only those whose nwg workgroups all run */
    /* followed by nwg uint32 done words, then (64-byte aligned) one 64-byte
     * release line per workgroup: each workgroup polls its own copy of seq */
} agx_rollout_ctl;
/* seq value that ends a persistent launch early and cleanly (an evaluation
 * whose episodes have all finished): every workgroup waiting for its next
 * step exits without touching ctl->timeout. */
#define AGX_ROLLOUT_STOP 0xfffffffeu
int64_t agx_rollout_workgroups(int64_t P, int64_t N);
/* Workgroups of the persistent rollout kernel for `net` the GPU holds at once
 * (occupancy x CUs; 0: shape not instantiated).  Every workgroup of a
 * persistent rollout must be resident together (the host paces them in lock
 * step), so agx_ppo_rollout_persistent returns AGX_EUNSUPPORTED when
 * agx_rollout_workgroups(P, N) exceeds this; callers then use per-step
 * launches (agx_ppo_rollout_step). */
int64_t agx_rollout_max_workgroups(const agx_ppo_net *net);
size_t agx_rollout_ctl_bytes(int64_t P, int64_t N);
size_t agx_rollout_args_bytes(int64_t nsteps);
int agx_ppo_rollout_persistent(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                               const agx_rollout_io *ios, int64_t nsteps, uint32_t base, uint64_t seed,
                               uint64_t counter0, void *args_host, agx_rollout_ctl *ctl, double timeout_s,
                               void *stream);
/* Persistent evaluation: PPO.test's loop (agilerl/algorithms/ppo.py:1113-
 * 1289) for P agents x N envs in ONE launch of the persistent rollout kernel,
 * paced like agx_ppo_rollout_persistent.  Step t reads the observations from
 * stage_obs (coherent host memory, [P*N][D]; legal-action masks from
 * stage_mask [P*N][A] or NULL), samples with Philox counter counter0 + t
 * (agx_ppo_act's stream) and writes the P*N actions to actions_flat (host).
 * Nothing else is stored: no rollout slots, no episode accounting (the host
 * tallies the evaluation episodes from its env step).  The host ends the
 * launch early with agx_host_signal(ctl, AGX_ROLLOUT_STOP) once every episode
 * has finished; a launch that runs all nsteps ends by itself.
 * args_host: agx_rollout_args_bytes(nsteps) of agx_host_alloc memory. */
int agx_ppo_eval_persistent(const agx_ppo_net *net, int64_t P, int64_t N, const float *params,
                            const float *stage_obs, const uint8_t *stage_mask, int64_t *actions_flat,
                            const int64_t *agent_env_base, int64_t nsteps, uint32_t base, uint64_t seed,
                            uint64_t counter0, void *args_host, agx_rollout_ctl *ctl, double timeout_s,
                            void *stream);
/* ---- reference RNG streams (host) ----------------------------------------
 * The minibatch permutations PPO._learn_from_rollout_buffer_flat draws from
 * numpy's global legacy MT19937 (ppo.py:836-842: indices = arange(S) once
 * per learn, np.random.shuffle(indices) per epoch), for P agents learning
 * one after another as train_on_policy's agent loop does
 * (train_on_policy.py:210): perms [epochs][P][S] in HOST memory.  mt_key
 * [624] / mt_pos are numpy's state (np.random.get_state()[1:3]), advanced in
 * place (the caller writes them back with np.random.set_state).
 * epochs_per_agent (host, [P]) or NULL: agent p draws only its own
 * epochs_per_agent[p] <= epochs shuffles (rows beyond are left as they are).
 * Host code, no device work. */
int agx_host_shuffle_perms(uint32_t *mt_key, int32_t *mt_pos, int64_t P, int64_t epochs, int64_t S,
                           const int64_t *epochs_per_agent, int64_t *perms);
/* Coherent (fine-grained) pinned host memory, device-accessible at the same
 * address; NULL on failure. */
void *agx_host_alloc(size_t bytes);
int agx_host_free(void *ptr);
/* A dedicated non-blocking stream (hipStreamNonBlocking: never ordered with
 * the legacy NULL stream) for a persistent launch that must run beside
 * others — the groups of an evaluation paced in lock step each keep one
 * resident, so each needs a stream of its own.  NULL on failure. */
void *agx_stream_create(void);
/* release-store seq into ctl->seq and every workgroup's release line */
int agx_host_signal(agx_rollout_ctl *ctl, uint32_t seq);
/* spin until every done word >= target; AGX_EHIP on ctl->timeout or after
 * timeout_s */
int agx_host_wait(const agx_rollout_ctl *ctl, int64_t nwg, uint32_t target, double timeout_s);
/* the same for workgroups [w0, w1) only (ctl->seq untouched): a host that
 * paces two halves of a launch, stepping one half's envs while the other
 * half's workgroups run */
int agx_host_signal_range(agx_rollout_ctl *ctl, int64_t w0, int64_t w1, uint32_t seq);
int agx_host_wait_range(const agx_rollout_ctl *ctl, int64_t w0, int64_t w1, uint32_t target, double timeout_s);
/* agx_host_signal_range(ctl, s0, s1, seq) then agx_host_wait_range(ctl, w0, w1,
 * target, timeout_s): one call where a part's release hands over to the next
 * part's wait */
int agx_host_signal_wait_range(agx_rollout_ctl *ctl, int64_t s0, int64_t s1, uint32_t seq, int64_t w0, int64_t w1,
                               uint32_t target, double timeout_s);

/* ---- prioritized replay segment trees -----------------------------------
 * Replaces SumSegmentTree / MinSegmentTree (agilerl/components/
 * segment_tree.py) and the priority half of PrioritizedReplayBuffer
 * (agilerl/components/replay_buffer.py:261-428).
 * Trees are 1-indexed heaps of 2*capacity doubles (node k has children 2k,
 * 2k+1; leaf i at capacity+i), capacity a power of two >= max_size.
 * max_priority is a device f64 scalar (initialise to 1.0).
 * Leaves hold priority**alpha computed by glibc's own pow algorithm
 * (csrc/libm_pow.h: the reference's Python float ** is glibc pow, which is
 * not correctly rounded), bit for bit; the tree is a pure function of the
 * leaves, so batched updates are identical to the reference's sequential
 * path walks. */
size_t agx_per_workspace_bytes(int64_t capacity, int64_t max_batch);
int agx_per_init(double *sum_tree, double *min_tree, int64_t capacity, void *stream);
/* PrioritizedReplayBuffer.add (replay_buffer.py:296-309): n leaves at ring
 * positions (start + i) % max_size get max_priority**alpha. */
int agx_per_add(double *sum_tree, double *min_tree, int64_t capacity, int64_t max_size,
                int64_t start, int64_t n, double alpha, const double *max_priority,
                void *workspace, void *stream);
/* PrioritizedReplayBuffer.update_priorities (replay_buffer.py:411-428):
 * in order, p = max(priority, floor), leaf = p**alpha (last duplicate wins),
 * max_priority = max(max_priority, p).  Indices must be in [0, max_size). */
int agx_per_update(double *sum_tree, double *min_tree, int64_t capacity, int64_t max_size,
                   const int64_t *indices, const float *priorities, int64_t n, double alpha,
                   double floor, double *max_priority, void *workspace, void *stream);
/* _sample_proportional (replay_buffer.py:357-381) + SumSegmentTree.retrieve
 * (segment_tree.py:136-156): uniforms are the caller's torch.rand(B) stream.
 * If weights != NULL also _calculate_weights (replay_buffer.py:383-409) with
 * the buffer's current `size`.  err (device int32, may be NULL) gets the count
 * of samples whose upper bound failed the reference's assert. */
int agx_per_sample(const double *sum_tree, const double *min_tree, int64_t capacity,
                   const float *uniforms, int64_t B, int64_t size, double beta,
                   int64_t *indices, float *weights, int32_t *err, void *stream);
/* SegmentTree.__getitem__ / reductions helper: copies tree[k] for given
 * nodes (used for sum()/min() and leaf reads without a host round trip). */
int agx_per_gather(const double *tree, const int64_t *nodes, int64_t n, double *out, void *stream);

/* ---- single segment trees ------------------------------------------------
 * SegmentTree / SumSegmentTree / MinSegmentTree used on their own
 * (agilerl/components/segment_tree.py): op 0 = sum (init 0.0), 1 = min
 * (init +inf); tree = 2*capacity doubles, capacity a power of two.
 * set: SegmentTree.__setitem__ (:81-95) for n (index, value) pairs in order
 *   (last duplicate wins); workspace (agx_segtree_workspace_bytes) is needed
 *   only for n > 1024.
 * operate: SegmentTree.operate(start, end) (:61-79), the reference recursion
 *   and operand order; end <= 0 counts from capacity; result to *out (device).
 * retrieve: SumSegmentTree.retrieve (:136-156) for n f64 upper bounds; err
 *   (device int32, may be NULL) counts failed `0 <= ub <= sum + 1e-5`. */
size_t agx_segtree_workspace_bytes(int64_t capacity);
int agx_segtree_init(double *tree, int64_t capacity, int op, void *stream);
int agx_segtree_set(double *tree, int64_t capacity, int op, const int64_t *indices, const double *values,
                    int64_t n, void *workspace, void *stream);
int agx_segtree_operate(const double *tree, int64_t capacity, int op, int64_t start, int64_t end,
                        double *out, void *stream);
int agx_segtree_retrieve(const double *tree, int64_t capacity, const double *upperbounds, int64_t n,
                         int64_t *indices, int32_t *err, void *stream);

/* ---- DQN TD target -------------------------------------------------------
 * Replaces DQN.update's target + loss (agilerl/algorithms/dqn.py:296-314):
 * y = r + gamma*q_t*(1-d), q_t = max_a Qtgt(s') or Qtgt(s')[argmax Q(s')]
 * (double_q); loss = mean((Q(s)[a] - y)^2); g_q = d loss / d Q(s) (B,A). */
size_t agx_td_workspace_bytes(int64_t B);
int agx_td_target(const float *q_next_online, const float *q_next_target, const float *q_cur,
                  const int64_t *actions, const float *rewards, const float *dones, int64_t B,
                  int64_t A, double gamma, int double_q, float *y, float *g_q, float *loss,
                  void *workspace, void *stream);

/* ---- MADDPG critic target + MSE ------------------------------------------
 * Replaces the critic half of MADDPG._learn_individual
 * (agilerl/algorithms/maddpg.py:764-790): NaN rewards -> 0, NaN dones -> 1,
 * dones cast to uint8; y = r + ((1 - d) * gamma) * q_next; loss =
 * mean((q - y)^2) and dloss/dq = 2 (q - y) / B.  q, q_next, rewards, dones,
 * y, g_q: (B) f32 (y, g_q may be NULL).  workspace: agx_td_workspace_bytes(B). */
int agx_maddpg_critic_target(const float *q, const float *q_next, const float *rewards,
                             const float *dones, int64_t B, double gamma, float *y, float *g_q,
                             float *loss, void *workspace, void *stream);

/* ---- Rainbow C51 projection + cross entropy ------------------------------
 * Replaces RainbowDQN._dqn_loss (agilerl/algorithms/dqn_rainbow.py:313-367).
 * q_next_online (B,A) picks a*; target_dist (B,A,Z) are the clamped target
 * probabilities; logp_cur (B,A,Z) the online log-softmax on s; support (Z).
 * Writes the elementwise loss (B) and, if proj != NULL, the projected
 * distribution (B,Z) bit-exact to the serial index_add_. */
int agx_c51_project_loss(const float *q_next_online, const float *target_dist,
                         const float *logp_cur, const int64_t *actions, const float *rewards,
                         const float *dones, const float *support, int64_t B, int64_t A,
                         int64_t Z, double v_min, double v_max, double gamma, float *loss,
                         float *proj, void *stream);
/* The same projection + loss on the two selected rows already gathered
 * (agx_dueling_head_forward_rows): target_rows [B][Z] = target_dist[b][a*_b],
 * logp_rows [B][Z] = logp_cur[b][action_b].  Both stream contiguously: the
 * 128-B lines of the neighbouring actions' atoms are never fetched.  Z = 51. */
int agx_c51_project_loss_rows(const float *target_rows, const float *logp_rows, const float *rewards,
                              const float *dones, const float *support, int64_t B, int64_t Z, double v_min,
                              double v_max, double gamma, float *loss, float *proj, void *stream);

/* ---- optimiser -----------------------------------------------------------
 * Fused per-agent gradient-norm clip + Adam over a population's flat
 * parameter buffers (replaces clip_grad_norm_ ppo.py:910-911 /
 * dqn_rainbow.py:479 and torch.optim.Adam via OptimizerWrapper.step,
 * agilerl/algorithms/core/optimizer_wrapper.py:444-452).
 * params/grads/exp_avg/exp_avg_sq: [P][n]; the n parameters are split into
 * G clip groups by group_offsets[0..G] (host array, G <= 8); with
 * max_norm <= 0 nothing is clipped.  lr: device f32 [P] (per-agent learning
 * rates, mutable by HPO without recompiling a graph); steps: device int64
 * [P], in/out — each agent's Adam step count (this update uses steps[p]+1
 * for the bias corrections and advances the counts of the agents it
 * updates); active: device u8 [P] or NULL (all) — inactive agents' rows
 * and counts are left untouched (agents stopped early by target_kl). */
size_t agx_adam_workspace_bytes(int64_t P, int64_t n);
int agx_clip_adam(float *params, float *grads, float *exp_avg, float *exp_avg_sq, int64_t P,
                  int64_t n, const int64_t *group_offsets, int G, float max_norm,
                  const float *lr, float beta1, float beta2, float eps, int64_t *steps,
                  const uint8_t *active, void *workspace, void *stream);
/* Polyak soft update target <- tau*online + (1-tau)*target
 * (dqn.py:349-358, dqn_rainbow.py:492-501). */
int agx_polyak(float *target, const float *online, int64_t n, float tau, void *stream);
/* NoisyLinear.reset_noise (agilerl/modules/custom_components.py:116-131) for
 * up to 16 noisy layers of a network in one launch.  eps_in [in_features] and
 * eps_out [out_features] are the layer's two torch.randn draws (the caller
 * draws them in the reference's order); with f(x) = sign(x) * sqrt(|x|):
 * weight_epsilon [out][in] = f(eps_out) outer f(eps_in), bias_epsilon = f(eps_out). */
typedef struct agx_noisy_layer {
    const float *eps_in;
    const float *eps_out;
    float *weight_epsilon;
    float *bias_epsilon;
    int64_t in_features, out_features;
} agx_noisy_layer;
int agx_noisy_reset(const agx_noisy_layer *layers, int n_layers, void *stream);

/* ---- convolutional encoder (EvolvableCNN) -----------------------------------
 * Conv2d layers of agilerl/modules/cnn.py:224-552 (create_cnn,
 * utils/evolvable_networks.py:460-525) as implicit GEMMs on the f32 matrix
 * cores; NCHW f32 tensors, weights [Cout][Cin][KH][KW], no padding, square
 * stride (the Atari encoders: 8x8/4, 4x4/2, 3x3/1).  The first layer may
 * read uint8 frames directly (x_is_u8): each pixel becomes
 * (x - x_low) / (x_high - x_low) on load, the reference's image
 * normalisation (utils/algo_utils.py:1134-1183), in f32 with an IEEE divide. */
typedef struct agx_conv2d_shape {
    int64_t batch;
    int32_t in_channels, height, width, out_channels, kernel_h, kernel_w, stride;
} agx_conv2d_shape;
/* y = act(conv(x, w) + bias), act = ReLU when relu != 0 (bias may be NULL). */
int agx_conv2d_forward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low, float x_high,
                       const float *w, const float *bias, int relu, float *y, void *stream);
size_t agx_conv2d_wgrad_workspace_bytes(const agx_conv2d_shape *shape);
/* Gradients of that layer from dy = dL/d(output): y_act (the forward's
 * post-ReLU output, or NULL for no activation) masks dy; dw, db (db may be
 * NULL) receive (or with accumulate += ) the weight / bias gradients — a
 * split-K reduction summed in a fixed order; dx (NULL: skip; not available
 * for u8 inputs) receives the input gradient. */
int agx_conv2d_backward(const agx_conv2d_shape *shape, const void *x, int x_is_u8, float x_low, float x_high,
                        const float *w, const float *y_act, const float *dy, float *dx, float *dw, float *db,
                        int accumulate, void *workspace, void *stream);

/* Population-batched forms (no reference counterpart: the reference runs one
 * agent's nn.Conv2d at a time): `groups` independent convolutions of one shape
 * in ONE launch — group g reads x + g*x_gstride, w + g*w_gstride,
 * bias + g*b_gstride and writes y + g*y_gstride (element strides; dy / y_act
 * share y_gstride, dx shares x_gstride).  The weight / bias gradients of group
 * g land densely at dw + g*Cout*Cin*KH*KW and db + g*Cout.  groups = 1 is the
 * single-agent call above. */
int agx_conv2d_forward_grouped(const agx_conv2d_shape *shape, int64_t groups, const void *x, int64_t x_gstride,
                               int x_is_u8, float x_low, float x_high, const float *w, int64_t w_gstride,
                               const float *bias, int64_t b_gstride, int relu, float *y, int64_t y_gstride,
                               void *stream);
/* The grouped forward over a two-level group index g = g1 + g1_count * g2
 * (g1 < g1_count): group g reads x + g1*x_stride1 + g2*x_stride2 and likewise
 * w, bias, y.  RainbowDQN's update runs its three no-padding CNN forwards
 * (online on s', online on s, target on s': g1 picks the frames, g2 the
 * network) as one launch per layer (dqn_rainbow.py:284-367). */
int agx_conv2d_forward_grouped2(const agx_conv2d_shape *shape, int64_t groups, int64_t g1_count, const void *x,
                                int64_t x_stride1, int64_t x_stride2, int x_is_u8, float x_low, float x_high,
                                const float *w, int64_t w_stride1, int64_t w_stride2, const float *bias,
                                int64_t b_stride1, int64_t b_stride2, int relu, float *y, int64_t y_stride1,
                                int64_t y_stride2, void *stream);
size_t agx_conv2d_wgrad_workspace_bytes_grouped(const agx_conv2d_shape *shape, int64_t groups);
int agx_conv2d_backward_grouped(const agx_conv2d_shape *shape, int64_t groups, const void *x, int64_t x_gstride,
                                int x_is_u8, float x_low, float x_high, const float *w, int64_t w_gstride,
                                const float *y_act, const float *dy, int64_t y_gstride, float *dx, float *dw,
                                float *db, int accumulate, void *workspace, void *stream);

/* ---- Rainbow dueling distributional head ------------------------------------
 * DuelingDistributionalMLP.forward (agilerl/networks/custom_modules.py:127-162)
 * after its value [B][Z] and advantage [B][A][Z] streams:
 * x = (v + adv) - mean_a adv; mode 2 (log=True) out = log_softmax_z(x)
 * [B][A][Z]; mode 1 (q=False) out = clamp(softmax_z(x), min=1e-3) [B][A][Z];
 * mode 0 (q=True) out[b][a] = sum_z clamp(softmax_z(x), 1e-3) * support[z].
 * 1 <= Z <= 64.  The backward maps dL/d(out) of the same mode to
 * dL/d(value) [B][Z] and dL/d(advantage) [B][A][Z]. */
int agx_dueling_head_forward(const float *value, const float *advantage, const float *support, int64_t B, int64_t A,
                             int64_t Z, int mode, float *out, void *stream);
int agx_dueling_head_backward(const float *value, const float *advantage, const float *support,
                              const float *grad_out, int64_t B, int64_t A, int64_t Z, int mode, float *grad_value,
                              float *grad_advantage, void *stream);
/* Selected rows (dqn_rainbow.py:313-367 target_dist[range(B), a*] and
 * log_p[range(B), action], fused into the head): out [B][Z] = the full form's
 * out[b][sel[b]][:] bit for bit, mode 1 (clamped probabilities) or 2 (log);
 * sel: device int64 [B].  The backward (log mode) takes dL/d(out rows) [B][Z]
 * (zero gradient on every other action, as autograd through the gather). */
int agx_dueling_head_forward_rows(const float *value, const float *advantage, const int64_t *sel, int64_t B,
                                  int64_t A, int64_t Z, int mode, float *out, void *stream);
int agx_dueling_head_backward_rows(const float *value, const float *advantage, const int64_t *sel,
                                   const float *grad_rows, int64_t B, int64_t A, int64_t Z, float *grad_value,
                                   float *grad_advantage, void *stream);

/* ---- population row gather ---------------------------------------------------
 * The single-rank generation step's clone (tournament.py:71-119 + clone,
 * core/base.py): for each of nbuf buffers of P rows (widths[k] 4-byte words
 * per row, row-major), row j becomes the old row idx[j] (device int64[P], may
 * repeat).  All buffers in two launches through a caller-owned workspace of
 * agx_rows_gather_workspace_bytes. */
#define AGX_ROWS_MAX_BUFS 8
size_t agx_rows_gather_workspace_bytes(const int64_t *widths, int nbuf, int64_t P);
int agx_rows_gather(float *const *bufs, const int64_t *widths, int nbuf, int64_t P, const int64_t *idx,
                    void *workspace, void *stream);

/* ---- diagnostics ---------------------------------------------------------
 * out[i] = pow(x[i], y[i]) by the routine the PER leaves and IS weights use
 * (glibc's pow algorithm, bit-identical to the host libm); for parity tests. */
int agx_debug_pow(const double *x, const double *y, double *out, int64_t n, void *stream);
/* Fused-learner phase timing: subsequent agx_ppo_learn calls write shader
 * cycle stamps of agent 0's first minibatch into buf (device int64[80]:
 * [sub_batch*16 + phase], phases 0-8 per sub-batch, 9-11 at slot 64+);
 * buf = NULL disables. */
int agx_debug_learn_stamps(int64_t *buf);
/* Persistent-rollout phase timing: subsequent agx_ppo_rollout_persistent
 * launches write s_memrealtime stamps into buf (device int64[384]: workgroup
 * 0's phases [step*8 + k] for steps < 32, per-workgroup stamps of step 5 at
 * 256 + wg and 320 + wg for wg < 64); buf = NULL disables. */
int agx_debug_rollout_stamps(int64_t *buf);
/* Test hook: on != 0 makes partner workgroup 1 of agent 0 skip every
 * hand-off of subsequent agx_ppo_learn calls (when the call splits agents
 * over partners), so the bounded partner wait times out and sets
 * args->error_word — the failure path tests/test_population_gpu.py checks. */
int agx_debug_learn_stall(int on);
/* STREAM-style bandwidth probes for bench.py's measured HBM peak: mode 0
 * copies `bytes` (read + write, nontemporal stores), mode 1 reads them
 * (dst receives at most one float4 per block).  grid = 0: one block per
 * 16 KiB tile, else a grid-stride loop over `grid` blocks.  bytes % 16 == 0. */
int agx_debug_stream(const void *src, void *dst, int64_t bytes, int mode, int64_t grid, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AGX_H */
