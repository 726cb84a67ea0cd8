/* Runtime-shape PPO learner: any MLP actor-critic the reference's
 * architecture mutations produce (agilerl/hpo/mutation.py:829-885 ->
 * EvolvableMLP add/remove layer/node, EvolvableNetwork latent nodes).
 *
 * agx_ppo_learn (agx.h) runs a compile-time plan per network shape; after an
 * architecture mutation an agent's shape is one of thousands, so this entry
 * point takes the network as a runtime LAYER LIST instead and runs the same
 * PPO.learn (agilerl/algorithms/ppo.py:836-920: every epoch x minibatch
 * update, clipped loss, two-group gradient clip ppo.py:910-911, Adam
 * optimizer_wrapper.py:444-452) in one launch, one workgroup per agent.
 * Same argument block, same outputs and error behaviour as agx_ppo_learn.
 *
 * Replaces, for mutated architectures, the call PPO.learn makes
 * (agilerl/algorithms/ppo.py:787-920); binding: INTEGRATION.md. */
#ifndef AGX_GRAPH_H
#define AGX_GRAPH_H

#include "agx.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AGX_PPO_GRAPH_MAX_LAYERS 16
#define AGX_PPO_GRAPH_MAX_WIDTH 512   /* widest LayerNorm / ReLU layer */
#define AGX_PPO_GRAPH_MAX_ACTIONS 32

/* One Linear [-> LayerNorm] [-> ReLU] of the network, nn.Linear layout:
 * weight [fout][fin] at flat offset w, bias [fout] at b; ln 0: none,
 * 1: LayerNorm without affine, 2: LayerNorm with affine (weight at ln_w,
 * bias at ln_b); src: -1 = the observation, else the index of the layer
 * whose output this layer reads (layers are listed in topological order). */
typedef struct agx_ppo_layer {
    int32_t fin, fout, w, b, ln_w, ln_b, ln, relu, src;
} agx_ppo_layer;

/* The actor-critic: layers[actor_out] produces the n_actions logits,
 * layers[critic_out] the value (both plain Linear); flat parameter rows of
 * n_params floats; clip groups [0, critic_start) and [critic_start, n_params). */
typedef struct agx_ppo_graph {
    int32_t obs_dim, n_actions, n_layers, actor_out, critic_out, n_params, critic_start;
    agx_ppo_layer layers[AGX_PPO_GRAPH_MAX_LAYERS];
} agx_ppo_graph;

/* AGX_OK when the graph is one agx_ppo_learn_graph runs (AGX_EINVAL with the
 * reason in agx_last_error otherwise).  Host-side only. */
int agx_ppo_graph_check(const agx_ppo_graph *net);
/* Device workspace bytes of agx_ppo_learn_graph for P agents x S samples,
 * `epochs` epochs and minibatches of at most `batch` rows (0: bad graph). */
size_t agx_ppo_learn_graph_workspace_bytes(const agx_ppo_graph *net, int64_t P, int64_t S, int64_t epochs,
                                           int64_t batch);
/* agx_ppo_learn over a runtime layer list (args as for agx_ppo_learn;
 * args->batch must not exceed the workspace's batch). */
int agx_ppo_learn_graph(const agx_ppo_graph *net, const agx_ppo_learn_args *args, void *workspace, void *stream);

/* The rollout policy step of agx_ppo_act (agx.h: same arguments, outputs,
 * Philox stream and masks) over a runtime layer list, for n_actions <= 32;
 * `workspace` holds agx_ppo_act_graph_workspace_bytes(net, P, N) bytes of
 * activation scratch.  Replaces, for mutated architectures, PPO.get_action
 * (agilerl/algorithms/ppo.py:567-633). */
size_t agx_ppo_act_graph_workspace_bytes(const agx_ppo_graph *net, int64_t P, int64_t N);
int agx_ppo_act_graph(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params, const float *obs,
                      int64_t obs_agent_stride, const uint8_t *action_mask, int64_t mask_agent_stride, int sample,
                      uint64_t seed, uint64_t counter, int64_t *actions, float *log_probs, float *values,
                      float *entropy, int64_t out_agent_stride, int64_t *actions_flat,
                      const int64_t *agent_env_base, void *workspace, void *stream);

/* Partnered-learner phase timing: subsequent agx_ppo_learn_graph calls that
 * split minibatches over partners write shader-cycle stamps of agent 0,
 * partner 0, update 1 into buf (device int64[10]: start, gradients done,
 * loss words, barrier 1, reduce-scatter, barrier 2, norms, Adam, barrier 3,
 * acquire); NULL disables. */
int agx_debug_graph_stamps(int64_t *buf);
/* Persistent rollout / evaluation of a runtime-shape population: the
 * host-paced loops of agx_ppo_rollout_persistent and agx_ppo_eval_persistent
 * (agx.h: same agx_rollout_io steps, control block protocol, Philox counters,
 * AGX_ROLLOUT_ABORT / AGX_ROLLOUT_STOP) around agx_ppo_act_graph's step, one
 * launch per rollout (replaces rollouts/on_policy.py:23-203's per-step
 * forward for mutated architectures).  The grid is
 * agx_ppo_rollout_graph_workgroups(P, N) workgroups (16 env rows each), all of
 * which must be co-resident (AGX_EUNSUPPORTED beyond
 * agx_ppo_rollout_graph_max_workgroups()); the control block holds
 * agx_ppo_rollout_graph_ctl_bytes(P, N) bytes; `workspace` as
 * agx_ppo_act_graph. */
int64_t agx_ppo_rollout_graph_workgroups(int64_t P, int64_t N);
int64_t agx_ppo_rollout_graph_max_workgroups(void);
size_t agx_ppo_rollout_graph_ctl_bytes(int64_t P, int64_t N);
int agx_ppo_rollout_graph_persistent(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params,
                                     const agx_rollout_io *ios, int64_t nsteps, uint32_t base, uint64_t seed,
                                     uint64_t counter0, void *args_host, agx_rollout_ctl *ctl, double timeout_s,
                                     void *workspace, void *stream);
int agx_ppo_eval_graph_persistent(const agx_ppo_graph *net, int64_t P, int64_t N, const float *params,
                                  const float *stage_obs, const uint8_t *stage_mask, int64_t *actions_flat,
                                  const int64_t *agent_env_base, int64_t nsteps, uint32_t base, uint64_t seed,
                                  uint64_t counter0, void *args_host, agx_rollout_ctl *ctl, double timeout_s,
                                  void *workspace, void *stream);

/* Evaluation pass of a WHOLE population in ONE persistent launch (replaces
 * the per-agent agent.test loop of train_on_policy.py:363-373 and PPO.test,
 * ppo.py:1113-1289, for every group of a population at once): agent p of P
 * runs its own network nets[p] (any MLP actor-critic, compiled shapes
 * included; one obs_dim / n_actions for all) on its parameter row params[p]
 * over envs [p N, (p + 1) N) of the packed host staging (stage_obs [P N][D],
 * actions_flat [P N], coherent host memory), sampled from its own Philox
 * stream: seed seeds[p], env env_base[p] + n, counter counters[p] + t at step
 * t.  Host-paced like agx_ppo_eval_graph_persistent (control block of
 * agx_ppo_rollout_graph_ctl_bytes(P, N) bytes, release word t + 1 + base,
 * AGX_ROLLOUT_STOP ends it early).  agents_host / agents_dev:
 * agx_ppo_eval_multi_bytes(P) bytes of coherent host memory / device memory
 * for the per-agent plans (copied on `stream` before the launch).
 * agx_ppo_eval_multi_supported: 1 when every network's policy-step tiles fit
 * in LDS and the P x ceil(N / 16) workgroups can all be resident (else the
 * groups' own passes run: agx_ppo_eval_persistent / _graph_persistent). */
/* Optional episode tally of the pass on the device: at each step the
 * previous env step's reward / done (host staging, P N each) go into the env's
 * running score (f64, as the reference's numpy tally) and its first finished
 * episode's score; each workgroup stores its count of finished envs into
 * fin_words[w] (coherent host memory) before its done word, so the host ends
 * the pass once they sum to P N (one step after the last episode ended).
 * prev: the staging already holds a reward / done when the launch starts (a
 * pass continued by a second launch). */
typedef struct agx_eval_tally {
    const float *stage_rew;
    const uint8_t *stage_done;
    double *scores, *completed; /* [P N] device, zeroed by the caller */
    uint8_t *finished;          /* [P N] device, zeroed by the caller */
    uint32_t *fin_words;        /* [workgroups] coherent host memory */
    int prev;
} agx_eval_tally;
size_t agx_ppo_eval_multi_bytes(int64_t P);
/* diagnostic: workgroup 0's stamps of steps 2..33 of the next
 * agx_ppo_eval_multi_persistent launches into buf (int64[128], s_memrealtime
 * ticks of 10 ns: release seen, observations staged, forward done, done word
 * written per step); null stops. */
int agx_debug_eval_stamps(int64_t *buf);
int agx_ppo_eval_multi_supported(const agx_ppo_graph *const *nets, int64_t P, int64_t N);
int agx_ppo_eval_multi_persistent(const agx_ppo_graph *const *nets, const float *const *params,
                                  const int64_t *env_base, const uint64_t *seeds, const uint64_t *counters, int64_t P,
                                  int64_t N, const float *stage_obs, int64_t *actions_flat, int64_t nsteps,
                                  uint32_t base, void *agents_host, void *agents_dev, agx_rollout_ctl *ctl,
                                  double timeout_s, const agx_eval_tally *tally, void *stream);

#ifdef __cplusplus
}
#endif

#endif
