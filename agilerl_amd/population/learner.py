"""Host side of the fused PPO learners: agx_ppo_learn (learner.hip, the
compiled network shapes) and agx_ppo_learn_graph (graph_learner.hip, any MLP
actor-critic as a runtime layer list: the shapes architecture mutations
produce)."""

from __future__ import annotations

import ctypes

import torch

from .. import _lib
from .. import kernels as K
from .nets import ActorCriticSpec

_i32 = ctypes.c_int32


class AgxPPONet(ctypes.Structure):
    """Mirror of ``agx_ppo_net`` (include/agx.h)."""

    _fields_ = [
        ("obs_dim", _i32), ("n_actions", _i32), ("n_enc", _i32), ("enc_dim", _i32 * 4),
        ("enc_w", _i32 * 3), ("enc_b", _i32 * 3), ("enc_ln_w", _i32 * 3), ("enc_ln_b", _i32 * 3),
        ("head_actor", _i32), ("head_critic", _i32),
        ("actor_w", _i32), ("actor_b", _i32), ("actor_ln_w", _i32), ("actor_ln_b", _i32),
        ("actor_out_w", _i32), ("actor_out_b", _i32),
        ("critic_w", _i32), ("critic_b", _i32), ("critic_ln_w", _i32), ("critic_ln_b", _i32),
        ("critic_out_w", _i32), ("critic_out_b", _i32),
        ("n_params", _i32), ("critic_start", _i32),
    ]


def net_descriptor(spec: ActorCriticSpec) -> AgxPPONet | None:
    """The fused-kernel descriptor, or None when the architecture is outside
    what agx_ppo_learn covers (then the torch learner runs)."""
    if (len(spec.actor) != 2 or len(spec.critic) != 2 or not spec.layer_norm
            or not 2 <= len(spec.encoder) <= 3 or not getattr(spec, "share_encoders", True)):
        return None
    d = AgxPPONet()
    d.obs_dim, d.n_actions, d.n_enc = spec.obs_dim, spec.n_actions, len(spec.encoder)
    d.enc_dim[0] = spec.obs_dim
    for i, lay in enumerate(spec.encoder):
        d.enc_dim[i + 1] = lay.fout
        d.enc_w[i], d.enc_b[i] = lay.w, lay.b
        d.enc_ln_w[i], d.enc_ln_b[i] = lay.g, lay.beta
    a1, ao = spec.actor
    c1, co = spec.critic
    d.head_actor, d.head_critic = a1.fout, c1.fout
    d.actor_w, d.actor_b, d.actor_ln_w, d.actor_ln_b = a1.w, a1.b, a1.g, a1.beta
    d.actor_out_w, d.actor_out_b = ao.w, ao.b
    d.critic_w, d.critic_b, d.critic_ln_w, d.critic_ln_b = c1.w, c1.b, c1.g, c1.beta
    d.critic_out_w, d.critic_out_b = co.w, co.b
    d.n_params, d.critic_start = spec.n_params, spec.actor_end
    lib = _lib.load(require_gpu=False)  # pure host-side planning query
    if lib.agx_ppo_learn_lds_bytes(ctypes.byref(d)) == 0:
        return None
    return d


class AgxPPOLayer(ctypes.Structure):
    """Mirror of ``agx_ppo_layer`` (include/agx_graph.h)."""

    _fields_ = [(n, _i32) for n in ("fin", "fout", "w", "b", "ln_w", "ln_b", "ln", "relu", "src")]


GRAPH_MAX_LAYERS = 16


class AgxPPOGraph(ctypes.Structure):
    """Mirror of ``agx_ppo_graph`` (include/agx_graph.h)."""

    _fields_ = [("obs_dim", _i32), ("n_actions", _i32), ("n_layers", _i32), ("actor_out", _i32),
                ("critic_out", _i32), ("n_params", _i32), ("critic_start", _i32),
                ("layers", AgxPPOLayer * GRAPH_MAX_LAYERS)]


_LN_KIND = {None: 0, "plain": 1, "affine": 2}


def graph_descriptor(spec) -> AgxPPOGraph | None:
    """The runtime layer list of an MLP actor-critic (encoder chain -> latent;
    actor head and critic head on the latent, or the critic on its own encoder
    chain when share_encoders is off), or None when agx_ppo_learn_graph does
    not cover it (more than 16 layers, a LayerNorm / ReLU layer wider than 512,
    more than 32 actions): then the torch learner runs."""
    if not isinstance(spec, ActorCriticSpec):
        return None
    layers: list[tuple] = []

    def chain(lays, src):
        for lay in lays:
            layers.append((lay, src))
            src = len(layers) - 1
        return src

    latent = chain(spec.encoder, -1)
    actor_out = chain(spec.actor, latent)
    critic_latent = chain(spec.critic_encoder, -1) if spec.critic_encoder else latent
    critic_out = chain(spec.critic, critic_latent)
    if len(layers) > GRAPH_MAX_LAYERS:
        return None
    d = AgxPPOGraph()
    d.obs_dim, d.n_actions, d.n_layers = spec.obs_dim, spec.n_actions, len(layers)
    d.actor_out, d.critic_out, d.n_params, d.critic_start = actor_out, critic_out, spec.n_params, spec.actor_end
    for i, (lay, src) in enumerate(layers):
        x = d.layers[i]
        x.fin, x.fout, x.w, x.b = lay.fin, lay.fout, lay.w, lay.b
        x.ln_w, x.ln_b, x.ln, x.relu, x.src = lay.g, lay.beta, _LN_KIND[lay.ln], int(lay.act), src
    lib = _lib.load(require_gpu=False)  # pure host-side validation
    if lib.agx_ppo_graph_check(ctypes.byref(d)) != 0:
        return None
    return d


class AgxPPOLearnArgs(ctypes.Structure):
    """Mirror of ``agx_ppo_learn_args`` (include/agx.h)."""

    _fields_ = [
        ("P", ctypes.c_int64), ("S", ctypes.c_int64), ("epochs", ctypes.c_int64), ("batch", ctypes.c_int64),
        ("params", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
        ("adam_step", ctypes.c_void_p), ("lr", ctypes.c_void_p),
        ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
        ("max_grad_norm", ctypes.c_float),
        ("obs", ctypes.c_void_p), ("actions", ctypes.c_void_p), ("old_logp", ctypes.c_void_p),
        ("adv", ctypes.c_void_p), ("ret", ctypes.c_void_p), ("old_value", ctypes.c_void_p),
        ("adv_stats", ctypes.c_void_p), ("action_masks", ctypes.c_void_p), ("perms", ctypes.c_void_p),
        ("clip_coef", ctypes.c_float), ("vf_coef", ctypes.c_float), ("ent_coef", ctypes.c_float),
        ("target_kl", ctypes.c_double),
        ("loss_out", ctypes.c_void_p), ("kl_out", ctypes.c_void_p), ("epochs_out", ctypes.c_void_p),
        ("error_word", ctypes.c_void_p),
        ("batch_per_agent", ctypes.c_void_p), ("epochs_per_agent", ctypes.c_void_p),
        ("ent_coef_per_agent", ctypes.c_void_p), ("skip_if_set", ctypes.c_void_p),
    ]


class FusedLearner:
    batch_ws = None  # the graph learner's scratch is sized by the minibatch

    def __init__(self, pop):
        self.desc = net_descriptor(pop.spec)
        if self.desc is None:
            raise _lib.AgxError("network outside the fused learner's coverage")
        lib = _lib.load()
        nbytes = lib.agx_ppo_learn_workspace_bytes(ctypes.byref(self.desc), pop.P, pop.S, pop.update_epochs)
        self.ws = torch.empty(max(16, nbytes), dtype=torch.uint8, device=pop.device)
        _lib.check(lib.agx_ppo_learn_prepare(ctypes.byref(self.desc), self.ws.data_ptr(), _lib.stream()),
                   "agx_ppo_learn_prepare")
        self._outputs(pop)
        self.fn = lib.agx_ppo_learn

    def _outputs(self, pop) -> None:
        self.epochs_ws = pop.update_epochs
        self.loss = torch.zeros(pop.P, dtype=torch.float32, device=pop.device)
        self.kl = torch.zeros(pop.P, dtype=torch.float32, device=pop.device)
        self.epochs_run = torch.zeros(pop.P, dtype=torch.int32, device=pop.device)
        self.args = AgxPPOLearnArgs()
        self.key = None

    def learn(self, pop, perms: torch.Tensor | None = None, skip_if_set: int | None = None) -> torch.Tensor:
        """All epochs x minibatches of every agent in two launches (gather +
        learner).  Advantages are normalised on the fly from pop.adv_stats
        (ppo.py:829-834); pop.advantages itself is left untouched."""
        if perms is None:
            perms = pop.permutations()
        opt = pop.opt
        b1, b2 = opt.betas
        masks = pop.action_masks
        # the argument block is rebuilt only when a buffer or hyperparameter
        # changes; per call only the permutations and the stream change (host
        # time between the rollout and the learner is on the critical path)
        key = (pop.params.data.data_ptr(), opt.exp_avg.data_ptr(), opt.exp_avg_sq.data_ptr(), opt.lr.data_ptr(),
               opt.steps.data_ptr(), pop.obs.data_ptr(), pop.advantages.data_ptr(), pop.returns.data_ptr(),
               pop.values.data_ptr(), pop.log_probs.data_ptr(), pop.actions.data_ptr(), pop.adv_stats.data_ptr(),
               None if masks is None else masks.data_ptr(), float(b1), float(b2), float(opt.eps), pop.split_batch,
               pop.update_epochs, float(pop.clip_coef), float(pop.vf_coef), float(pop.ent_coef),
               float(pop.max_grad_norm), float(pop.target_kl or 0.0), pop.err_word.data_ptr(),
               *((None, None, None) if pop._hp_dev is None else (t.data_ptr() for t in pop._hp_dev)))
        if self.key != key:
            a = self.args
            a.P, a.S, a.epochs, a.batch = pop.P, pop.S, pop.update_epochs, pop.split_batch
            a.params, a.exp_avg, a.exp_avg_sq = key[0], key[1], key[2]
            a.lr, a.adam_step = key[3], key[4]
            a.beta1, a.beta2, a.eps, a.max_grad_norm = key[13], key[14], key[15], key[21]
            a.obs, a.actions, a.old_logp = key[5], key[10], key[9]
            a.adv, a.ret, a.old_value, a.adv_stats = key[6], key[7], key[8], key[11]
            a.action_masks = key[12]
            a.clip_coef, a.vf_coef, a.ent_coef, a.target_kl = key[18], key[19], key[20], key[22]
            a.loss_out, a.kl_out = self.loss.data_ptr(), self.kl.data_ptr()
            a.epochs_out, a.error_word = self.epochs_run.data_ptr(), key[23]
            a.batch_per_agent, a.epochs_per_agent, a.ent_coef_per_agent = key[24], key[25], key[26]
            self.key = key
            self.aref = ctypes.byref(self.args)
            self.dref = ctypes.byref(self.desc)
        self.args.perms = perms.data_ptr()
        self.args.skip_if_set = skip_if_set
        rc = self.fn(self.dref, self.aref, self.ws.data_ptr(), _lib.stream())
        if rc != 0:
            _lib.check(rc, "agx_ppo_learn")
        return self.loss

    def timed_out(self, pop) -> bool:
        """True if a partner workgroup of the last learn() gave up waiting for
        another (the kernel's bounded spin; the timeout word follows the P
        arrival counters at the start of the workspace).  Synchronises."""
        word = self.ws[4 * pop.P: 4 * pop.P + 4].view(torch.int32)
        return bool(int(word.item()) != 0)


class GraphLearner(FusedLearner):
    """agx_ppo_learn_graph: the same learn() over a runtime layer list (one
    workgroup per agent, scratch sized by the largest minibatch)."""

    def __init__(self, pop):
        self.desc = graph_descriptor(pop.spec)
        if self.desc is None:
            raise _lib.AgxError("network outside the graph learner's coverage")
        lib = _lib.load()
        self.batch_ws = pop.split_batch
        nbytes = lib.agx_ppo_learn_graph_workspace_bytes(ctypes.byref(self.desc), pop.P, pop.S, pop.update_epochs,
                                                         self.batch_ws)
        if nbytes == 0:
            raise _lib.AgxError(f"agx_ppo_learn_graph_workspace_bytes: {lib.agx_last_error().decode()}")
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=pop.device)
        self._outputs(pop)
        self.fn = lib.agx_ppo_learn_graph

    def timed_out(self, pop) -> bool:
        return False  # one workgroup per agent: no partner hand-off to time out


def make_learner(pop) -> FusedLearner:
    return FusedLearner(pop) if pop.fused_descriptor() is not None else GraphLearner(pop)


def learner_stale(pop) -> bool:
    """True when pop has no learner yet or its workspace is too small."""
    L = getattr(pop, "_fused", None)
    return (L is None or L.epochs_ws < pop.update_epochs
            or (L.batch_ws is not None and L.batch_ws < pop.split_batch))


def fused_learn(pop, perms=None, skip_if_set: int | None = None) -> torch.Tensor:
    if learner_stale(pop):
        pop._fused = make_learner(pop)
    return pop._fused.learn(pop, perms, skip_if_set)


def policy_step(pop, desc: AgxPPONet, obs: torch.Tensor, obs_agent_stride: int, *, sample: bool, counter: int,
                actions=None, log_probs=None, values=None, entropy=None, out_agent_stride: int = 0,
                actions_flat=None, action_mask=None, mask_agent_stride: int = 0) -> None:
    """agx_ppo_act over all P agents x N envs (PPO.get_action, ppo.py:567-633)."""
    _lib.call("agx_ppo_act", ctypes.byref(desc), pop.P, pop.N, pop.params.data.data_ptr(), obs.data_ptr(),
              obs_agent_stride, _lib.ptr(action_mask), mask_agent_stride, 1 if sample else 0, pop.act_seed, counter,
              _lib.ptr(actions), _lib.ptr(log_probs), _lib.ptr(values), _lib.ptr(entropy), out_agent_stride,
              _lib.ptr(actions_flat), pop.env_base_d.data_ptr(), _lib.stream())


def graph_act_workspace(pop, desc: AgxPPOGraph):
    """(desc, scratch) of agx_ppo_act_graph for this population, allocated on
    first use.  Callers that keep a persistent launch resident (lock-stepped
    evaluation) take it before launching: an allocation can wait for the
    device."""
    ws = getattr(pop, "_act_ws", None)
    if ws is None or ws[0] is not desc:
        lib = _lib.load()
        nbytes = lib.agx_ppo_act_graph_workspace_bytes(ctypes.byref(desc), pop.P, pop.N)
        if nbytes == 0:
            raise _lib.AgxError(f"agx_ppo_act_graph_workspace_bytes: {lib.agx_last_error().decode()}")
        ws = pop._act_ws = (desc, torch.empty(nbytes, dtype=torch.uint8, device=pop.device))
    return ws


def policy_step_graph(pop, desc: AgxPPOGraph, obs: torch.Tensor, obs_agent_stride: int, *, sample: bool,
                      counter: int, actions=None, log_probs=None, values=None, entropy=None,
                      out_agent_stride: int = 0, actions_flat=None, action_mask=None,
                      mask_agent_stride: int = 0) -> None:
    """agx_ppo_act_graph over all P agents x N envs: the policy step of
    policy_step for a mutated (runtime-shape) network, same Philox stream."""
    ws = graph_act_workspace(pop, desc)
    _lib.call("agx_ppo_act_graph", ctypes.byref(desc), pop.P, pop.N, pop.params.data.data_ptr(), obs.data_ptr(),
              obs_agent_stride, _lib.ptr(action_mask), mask_agent_stride, 1 if sample else 0, pop.act_seed, counter,
              _lib.ptr(actions), _lib.ptr(log_probs), _lib.ptr(values), _lib.ptr(entropy), out_agent_stride,
              _lib.ptr(actions_flat), pop.env_base_d.data_ptr(), ws[1].data_ptr(), _lib.stream())

