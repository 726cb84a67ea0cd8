"""Drop-in ``PPO`` (agilerl/algorithms/ppo.py:108-1290) for discrete-action
MLP actor-critics, backed by the HBM population engine.

A ``PPO`` object is a *view* of one row of a :class:`PPOPopulation` (its
parameters, Adam state and rollout SoA live in HBM, stacked with the other
agents of the population).  ``create_population`` (agilerl_amd.utils) builds
one population and P views, so ``train_on_policy`` can run the whole
population with one launch per kernel; a standalone ``PPO(...)`` owns a
population of one.

Supported: Discrete action spaces, Box observations, ``net_config`` with
``encoder_config`` / ``head_config`` MLP ``hidden_size`` lists and
``latent_dim`` (the reference's defaults: encoder [64, 64] -> latent 32,
actor head [32], critic head [16] unless ``head_config`` is given,
ppo.py:286-320 via networks/base.py and networks/actors.py),
LayerNorm on, shared encoder.  ``get_action`` / ``learn`` / ``test`` keep the
reference's signatures and return types; recurrent policies,
continuous actions and custom ``actor_network`` objects raise
NotImplementedError (outside the hot path).  ``get_action(obs, action_mask)``
applies the reference's legal-action masks (logits of illegal actions ->
-1e8, ppo.py:529-565); ``target_kl`` stops an agent's epochs early exactly
as ppo.py:917-918 does, inside the fused learner.
"""

from __future__ import annotations

import ctypes
from typing import Any

import numpy as np
import torch

from .. import _lib
from ..population.nets import ActorCriticSpec
from ..population.ppo_pop import PPOPopulation


def _hidden(cfg: dict | None, default: list[int]) -> list[int]:
    if cfg is None:
        return list(default)
    if hasattr(cfg, "hidden_size"):
        return list(cfg.hidden_size)
    return list(cfg.get("hidden_size", default))


def _image_spec(observation_space, action_space, net_config: dict, normalize_images: bool):
    """ImageActorCriticSpec for an image Box space (ppo.py:286-320 with
    base.py:521-530): EvolvableCNN encoder from ``encoder_config``
    (channel_size / kernel_size / stride_size; the reference default
    CnnNetConfig [32, 32] 3x3 stride 1), MLP heads from ``head_config``
    (layer_norm as configured; critic default [16])."""
    from ..networks.base import as_config, cnn_net_config, image_norm_bounds
    from ..population.image_nets import ImageActorCriticSpec

    enc = cnn_net_config(**(as_config(net_config.get("encoder_config")) or {}))
    if enc.get("block_type", "Conv2d") != "Conv2d" or enc.get("layer_norm"):
        raise NotImplementedError("agx image PPO: Conv2d blocks without BatchNorm (the Atari encoders)")
    if enc.get("activation", "ReLU") != "ReLU" or enc.get("output_activation", "ReLU") not in (None, "ReLU"):
        raise NotImplementedError("agx image PPO: ReLU encoders")
    head = as_config(net_config.get("head_config"))
    actor_hidden = _hidden(head, [32])
    critic_hidden = _hidden(head, [16])  # ppo.py:292-300 default critic head
    head_ln = bool((head or {}).get("layer_norm", True))
    # architecture-mutation limits: the CNN's (CnnNetConfig defaults 1, 6, 16,
    # 256, modules/configs.py:114-127), the heads' (MlpNetConfig: 1, 3, 16, 500)
    # and the latent's (EvolvableNetwork: 8, 128)
    cnn_limits = (int(enc.get("min_hidden_layers", 1)), int(enc.get("max_hidden_layers", 6)),
                  int(enc.get("min_channel_size", 16)), int(enc.get("max_channel_size", 256)))
    head_limits = _limits(head, head is None or not isinstance(head, dict))
    latent_limits = (int(net_config.get("min_latent_dim", 8)), int(net_config.get("max_latent_dim", 128)))
    dtype = torch.uint8 if np.dtype(observation_space.dtype) == np.uint8 else torch.float32
    norm = image_norm_bounds(observation_space) if normalize_images else None
    return ImageActorCriticSpec(obs_shape=tuple(observation_space.shape), n_actions=int(action_space.n),
                                channel_size=list(enc["channel_size"]), kernel_size=list(enc["kernel_size"]),
                                stride_size=list(enc["stride_size"]), latent_dim=int(net_config.get("latent_dim", 32)),
                                actor_hidden=actor_hidden, critic_hidden=critic_hidden, head_layer_norm=head_ln,
                                obs_dtype=dtype, image_norm=norm, cnn_limits=cnn_limits, actor_limits=head_limits,
                                critic_limits=head_limits, latent_limits=latent_limits)


def _limits(cfg, config_default: bool) -> tuple:
    """(min / max hidden layers, min / max nodes) of an MLP built from ``cfg``:
    a dict falls back on EvolvableMLP's defaults (1, 3, 32, 500,
    modules/mlp.py:61-82), an MlpNetConfig on its own (1, 3, 16, 500,
    modules/configs.py:56-70)."""
    d = (1, 3, 16, 500) if config_default else (1, 3, 32, 500)
    if cfg is None:
        return d
    get = cfg.get if isinstance(cfg, dict) else (lambda k, v: getattr(cfg, k, v))
    return (int(get("min_hidden_layers", d[0])), int(get("max_hidden_layers", d[1])),
            int(get("min_mlp_nodes", d[2])), int(get("max_mlp_nodes", d[3])))


def spec_from_net_config(observation_space, action_space, net_config: dict | None, normalize_images: bool = True,
                         share_encoders: bool = True):
    """The networks ppo.py:286-320 builds, as the reference's defaults fill
    them in: no encoder_config -> get_default_encoder_config's MlpNetConfig
    [64, 64] (utils/evolvable_networks.py:168-217); latent_dim 32 with limits
    8 / 128 (networks/base.py:191-194); no head_config -> actor head
    MlpNetConfig [32] (networks/actors.py:300-303), critic head [16]
    (ppo.py:292-300)."""
    if not hasattr(action_space, "n"):
        raise NotImplementedError("agx PPO supports Discrete action spaces")
    net_config = dict(net_config or {})
    from ..networks.base import is_image_space

    if is_image_space(observation_space):
        if not share_encoders:
            raise NotImplementedError("agx image PPO: the shared CNN encoder (share_encoders=True)")
        return _image_spec(observation_space, action_space, net_config, normalize_images)
    enc_cfg = net_config.get("encoder_config")
    enc = _hidden(enc_cfg, [64, 64])
    head = net_config.get("head_config")
    actor_hidden = _hidden(head, [32])
    critic_hidden = _hidden(head, [16])  # ppo.py:292-300 default critic head
    latent = int(net_config.get("latent_dim", 32))
    obs_dim = int(np.prod(observation_space.shape))
    enc_lim = _limits(enc_cfg, enc_cfg is None or not isinstance(enc_cfg, dict))
    head_lim = _limits(head, head is None or not isinstance(head, dict))
    lat_lim = (int(net_config.get("min_latent_dim", 8)), int(net_config.get("max_latent_dim", 128)))
    return ActorCriticSpec(obs_dim=obs_dim, n_actions=int(action_space.n), encoder_hidden=enc, latent_dim=latent,
                           actor_hidden=actor_hidden, critic_hidden=critic_hidden, encoder_limits=enc_lim,
                           actor_limits=head_lim, critic_limits=head_lim if head is not None else (1, 3, 16, 500),
                           latent_limits=lat_lim, share_encoders=bool(share_encoders),
                           encoder_name="shared_encoder" if share_encoders else "actor_encoder")


class PPO:
    algo = "PPO"

    def __init__(self, observation_space, action_space, index: int = 0, hp_config=None,
                 net_config: dict[str, Any] | None = None, batch_size: int = 64, lr: float = 1e-4,
                 learn_step: int = 2048, gamma: float = 0.99, gae_lambda: float = 0.95, mut=None,
                 action_std_init: float = 0.0, clip_coef: float = 0.2, ent_coef: float = 0.01,
                 vf_coef: float = 0.5, max_grad_norm: float = 0.5, target_kl: float | None = None,
                 normalize_images: bool = True, update_epochs: int = 4, actor_network=None, critic_network=None,
                 share_encoders: bool = True, num_envs: int = 1, use_rollout_buffer: bool = True,
                 rollout_buffer_config=None, recurrent: bool = False, device="cuda", accelerator=None,
                 wrap: bool = True, bptt_sequence_type=None, max_seq_len=None, *, _population=None,
                 _row: int | None = None) -> None:
        if recurrent:
            raise NotImplementedError("recurrent PPO is outside the agx hot path")
        if actor_network is not None or critic_network is not None:
            raise NotImplementedError("custom actor/critic modules: use net_config (MLP) networks")
        self.share_encoders = bool(share_encoders)
        assert isinstance(batch_size, int) and batch_size >= 1, "Batch size must be an integer greater than or equal to one."
        assert lr > 0, "Learning rate must be greater than zero."
        assert isinstance(learn_step, int) and learn_step >= 1, "Learn step rate must be an integer greater than or equal to one."
        from ..hpo.registry import MutationRegistry

        self.observation_space, self.action_space = observation_space, action_space
        self.index = index
        self.net_config = net_config
        self._learn_step = learn_step
        self.gamma, self.gae_lambda, self.mut = gamma, gae_lambda, mut
        self.clip_coef, self.vf_coef = clip_coef, vf_coef
        self.max_grad_norm, self.target_kl = max_grad_norm, target_kl
        self.num_envs = num_envs
        # hyperparameters the HPO may mutate (core/base.py:301, registry.py:190-242)
        self.registry = MutationRegistry(hp_config)
        self.device = torch.device(device)
        self.scores: list[float] = []
        self.fitness: list[float] = []
        self.steps: list[int] = [0]
        if _population is None:
            spec = spec_from_net_config(observation_space, action_space, net_config, normalize_images,
                                        share_encoders=share_encoders)
            _population = PPOPopulation(spec, 1, num_envs, learn_step=learn_step, batch_size=batch_size, lr=lr,
                                        gamma=gamma, gae_lambda=gae_lambda, clip_coef=clip_coef, ent_coef=ent_coef,
                                        vf_coef=vf_coef, max_grad_norm=max_grad_norm, update_epochs=update_epochs,
                                        target_kl=target_kl, seeds=[index], device=self.device)
            _row = 0
        self.population, self.row = _population, int(_row)
        self._counter = 0
        # architecture / learn_step mutations waiting for the population engine
        # to regroup the agents (population/engine.py)
        self._pending_state = None
        self._pending_learn_step = None
        # the networks' own generators for node / layer counts (the reference's
        # EvolvableModule.rng; seeded from the agent's initial index so a run
        # is reproducible and a sharded population draws as the whole one)
        self.module_rng = np.random.default_rng((0x5EED, int(index)))
        self.critic_rng = np.random.default_rng((0x5EEE, int(index)))
        # CNN encoders' kernel-size helpers keep generators of their own
        # (MutableKernelSizes, modules/cnn.py:55-72)
        self.kernel_rng = np.random.default_rng((0x5EEF, int(index)))
        self.critic_kernel_rng = np.random.default_rng((0x5EF0, int(index)))
        pop = self.population
        if _population is not None and (batch_size, update_epochs, ent_coef) != (
                pop.agent_batch[self.row], pop.agent_epochs[self.row], pop.agent_ent[self.row]):
            self.batch_size, self.update_epochs, self.ent_coef = batch_size, update_epochs, ent_coef
        if pop.agent_lr[self.row] != float(lr):
            self.lr = lr

    # ---- per-agent RL hyperparameters: rows of the population's tables ---- #
    @property
    def lr(self) -> float:
        return self.population.agent_lr[self.row]

    @lr.setter
    def lr(self, value: float) -> None:
        self.population.set_agent_hparam(self.row, "lr", value)

    def reinit_optimizers(self, optimizer=None) -> None:
        """core/base.py:760-775: a fresh Adam for this agent (zero moments and
        step, current lr) — after an lr, a parameter or an architecture
        mutation."""
        if self._pending_state is not None:
            s = self._pending_state
            s.exp_avg.zero_()
            s.exp_avg_sq.zero_()
            s.step = 0
            return
        self.population.reinit_agent_optimizer(self.row)

    @property
    def batch_size(self) -> int:
        return int(self.population.agent_batch[self.row])

    @batch_size.setter
    def batch_size(self, value: int) -> None:
        self.population.set_agent_hparam(self.row, "batch_size", int(value))

    @property
    def update_epochs(self) -> int:
        return int(self.population.agent_epochs[self.row])

    @update_epochs.setter
    def update_epochs(self, value: int) -> None:
        self.population.set_agent_hparam(self.row, "update_epochs", int(value))

    @property
    def ent_coef(self) -> float:
        return float(self.population.agent_ent[self.row])

    @ent_coef.setter
    def ent_coef(self, value: float) -> None:
        self.population.set_agent_hparam(self.row, "ent_coef", float(value))

    @property
    def learn_step(self) -> int:
        return self._pending_learn_step or self._learn_step

    @learn_step.setter
    def learn_step(self, value: int) -> None:
        """The rollout length (ppo.py:363 capacity ceil(learn_step / num_envs));
        the population engine moves the agent to a group of its learn_step at
        the next generation (the reference's create_rollout_buffer hook)."""
        value = int(value)
        if value < 1:
            raise ValueError("learn_step must be >= 1")
        self._pending_learn_step = value if value != self._learn_step else None
        if self._pending_state is not None:
            self._pending_state.learn_step = value

    @property
    def can_mutate_architecture(self) -> bool:
        from ..population.image_nets import ImageActorCriticSpec
        from ..population.nets import ActorCriticSpec

        # population/arch.py (MLP) and population/image_arch.py (CNN encoder)
        # mutate the shared-encoder layouts
        return (isinstance(self.spec, ActorCriticSpec) and self.spec.share_encoders) or \
            isinstance(self.spec, ImageActorCriticSpec)

    def architecture_mutation(self, new_layer_prob: float, rng) -> str | None:
        """mutation.py:829-885 on this agent (population/arch.py): -> the
        applied method.  The mutated networks wait in a pending state for the
        engine's regroup (the row layout of the current group is another
        shape's)."""
        from ..population import arch
        from ..population.engine import AgentState

        from ..population import image_arch
        from ..population.image_nets import ImageActorCriticSpec

        spec, pop, r = self.spec, self.population, self.row
        flat = (self._pending_state.params if self._pending_state is not None
                else pop.params.data[r, :spec.n_params]).cpu()
        if isinstance(spec, ImageActorCriticSpec):
            method = image_arch.sample_method(new_layer_prob, rng)
            new_spec, new_flat, applied, _ = image_arch.mutate(spec, flat, method, self.module_rng, self.kernel_rng,
                                                               self.critic_rng, self.critic_kernel_rng)
        else:
            method = arch.sample_method(new_layer_prob, rng)
            new_spec, new_flat, applied, _ = arch.mutate(spec, flat, method, self.module_rng, self.critic_rng)
        n = new_spec.n_params
        zeros = torch.zeros(n, dtype=torch.float32, device=pop.device)
        self._pending_state = AgentState(new_spec, self.learn_step, new_flat.to(pop.device), zeros.clone(),
                                         zeros.clone(), 0, float(pop.agent_lr[r]), int(pop.agent_batch[r]),
                                         int(pop.agent_epochs[r]), float(pop.agent_ent[r]))
        return applied

    def get_lr_names(self) -> list[str]:
        return ["lr"]

    def policy_weights(self) -> dict[str, torch.Tensor]:
        """The policy network's (actor: encoder + head) parameters by the
        reference's actor state-dict names, as views of the HBM row (what
        parameter mutations perturb, mutation.py:536-565; the critic's
        encoder is the same memory, so the shared-encoder copy follows)."""
        out = {}
        for k, t in self.state_dict().items():
            if k.startswith("actor."):
                out[k[len("actor."):]] = t
        return out

    def mutation_hook(self) -> None:
        """Shared-encoder hook (core/base.py): the critic encoder aliases the
        actor encoder in the flat layout, so there is nothing to copy."""

    # ------------------------------------------------------------------ #
    @property
    def spec(self) -> ActorCriticSpec:
        return self._pending_state.spec if self._pending_state is not None else self.population.spec

    def state_dict(self) -> dict[str, torch.Tensor]:
        """Reference-compatible parameter names (actor.encoder / head_net /
        critic.head_net ...) -> tensors (views of the HBM row, or of the
        pending mutated state)."""
        flat = self._pending_state.params if self._pending_state is not None else self.population.params.data[self.row]
        return {k: flat[off:off + int(np.prod(shape))].view(shape)
                for k, (off, shape) in self.spec.state_dict_keys().items()}

    @torch.no_grad()
    def load_state_dict(self, state_dict: dict[str, torch.Tensor], strict: bool = True) -> None:
        """Copy reference-named tensors into this agent's HBM row."""
        keys = self.spec.state_dict_keys()
        if strict:
            missing, unexpected = set(keys) - set(state_dict), set(state_dict) - set(keys)
            if missing or unexpected:
                raise KeyError(f"state_dict mismatch: missing {sorted(missing)}, unexpected {sorted(unexpected)}")
        flat = self.population.params.data[self.row]
        for k, (off, shape) in keys.items():
            if k in state_dict and not self.spec.aliased(k):
                t = torch.as_tensor(state_dict[k])
                if tuple(t.shape) != tuple(shape):
                    raise ValueError(f"{k}: shape {tuple(t.shape)}, expected {tuple(shape)}")
                flat[off:off + t.numel()] = t.reshape(-1).to(flat)

    def _opt_rows(self):
        opt = self.population.opt
        return opt.exp_avg[self.row], opt.exp_avg_sq[self.row]

    def save_checkpoint(self, path: str) -> None:
        """core/base.py:939-949 layout (see algorithms/checkpoint.py)."""
        from . import checkpoint as C

        sd = self.state_dict()
        keys = self.spec.state_dict_keys()
        m, v = self._opt_rows()
        spec = self.spec
        opt = {"exp_avg": {k: m[o:o + int(np.prod(sh))].view(sh) for k, (o, sh) in keys.items()
                           if not spec.aliased(k)},
               "exp_avg_sq": {k: v[o:o + int(np.prod(sh))].view(sh) for k, (o, sh) in keys.items()
                              if not spec.aliased(k)},
               "step": int(self.population.opt.steps[self.row])}
        mods = {net: {k[len(net) + 1:]: t for k, t in sd.items() if k.startswith(net + ".")}
                for net in ("actor", "critic")}
        torch.save(C.checkpoint_dict(self, mods, {"optimizer": opt}), path)

    @torch.no_grad()
    def load_checkpoint(self, path: str) -> None:
        """core/base.py:951-1072 for the agx layout; torch.load(weights_only=True)."""
        from . import checkpoint as C

        ck = C.read(path, self.algo, adam_networks=("actor", "critic"))
        info = ck["network_info"]
        sd = {f"{net}.{k}": t for net in info["network_names"] for k, t in info["modules"][f"{net}_state_dict"].items()}
        self.load_state_dict(sd)
        opt = info["optimizers"]["optimizer_state_dict"]
        keys = self.spec.state_dict_keys()
        m, v = self._opt_rows()
        for k, t in opt["exp_avg"].items():
            if self.spec.aliased(k):  # shares the actor encoder's row (a reference file holds both)
                continue
            o, sh = keys[k]
            m[o:o + t.numel()] = t.reshape(-1).to(m)
            v[o:o + t.numel()] = opt["exp_avg_sq"][k].reshape(-1).to(v)
        self.population.opt.steps[self.row] = int(opt["step"])
        C.restore_attributes(self, ck)

    @classmethod
    def load(cls, path: str, device="cuda", accelerator=None) -> "PPO":
        from . import checkpoint as C

        ck = C.load_file(path, adam_networks=("actor", "critic"))
        obs_space, act_space = C.spaces(ck)
        kw = {k: ck[k] for k in ("batch_size", "lr", "learn_step", "gamma", "gae_lambda", "clip_coef", "ent_coef",
                                 "vf_coef", "max_grad_norm", "target_kl", "update_epochs", "num_envs",
                                 "net_config", "index") if k in ck}
        agent = cls(obs_space, act_space, device=device, **kw)
        agent.load_checkpoint(path)
        return agent

    @torch.no_grad()
    def get_action(self, obs, action_mask=None, hidden_state=None, *args, **kwargs):
        """-> (action, log_prob, entropy, value) numpy arrays (ppo.py:567-633);
        sampling is a Gumbel-max draw from a counter-based Philox stream."""
        pop = self.population
        o = np.asarray(obs)
        keep_u8 = o.dtype == np.uint8 and pop.obs.dtype == torch.uint8  # frames normalised in the conv load
        o = torch.as_tensor(o, dtype=torch.uint8 if keep_u8 else torch.float32, device=self.device)
        o = o.reshape(-1, pop.spec.obs_dim).contiguous()
        n = o.shape[0]
        mask = None
        if action_mask is not None:
            mask = torch.as_tensor(np.asarray(action_mask), device=self.device).reshape(n, pop.spec.n_actions)
            mask = (mask != 0).to(torch.uint8).contiguous()
        out = dict(actions=torch.empty(n, dtype=torch.int64, device=self.device),
                   log_probs=torch.empty(n, device=self.device), values=torch.empty(n, device=self.device),
                   entropy=torch.empty(n, device=self.device))
        desc = pop.fused_descriptor()
        gdesc = pop.learn_descriptor() if desc is None else None
        if gdesc is not None:  # a mutated MLP shape: agx_ppo_act_graph on this agent's row
            self._counter += 1
            ws = getattr(self, "_act_graph_ws", None)
            if ws is None or ws[0] is not gdesc or ws[1] < n:
                nbytes = _lib.load().agx_ppo_act_graph_workspace_bytes(ctypes.byref(gdesc), 1, n)
                ws = self._act_graph_ws = (gdesc, n, torch.empty(nbytes, dtype=torch.uint8, device=self.device))
            params = pop.params.data[self.row]
            _lib.call("agx_ppo_act_graph", ctypes.byref(gdesc), 1, n, params.data_ptr(), o.data_ptr(), 0,
                      _lib.ptr(mask), 0, 1, pop.act_seed + 7919 * pop.agent_ids[self.row], (1 << 40) + self._counter,
                      out["actions"].data_ptr(), out["log_probs"].data_ptr(), out["values"].data_ptr(),
                      out["entropy"].data_ptr(), 0, None, None, ws[2].data_ptr(), _lib.stream())
        elif desc is None:
            logits, value = pop.spec.forward(pop.params.data[self.row:self.row + 1], o.unsqueeze(0))
            from ..population.nets import categorical

            if mask is not None:
                logits = torch.where(mask.bool().unsqueeze(0), logits, torch.full_like(logits, -1e8))
            logp_all, ent = categorical(logits)
            u = torch.rand(logits.shape, device=self.device).clamp_(min=1e-20)
            a = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1)
            out["actions"], out["values"], out["entropy"] = a.view(-1), value.view(-1), ent.view(-1)
            out["log_probs"] = logp_all.gather(-1, a.unsqueeze(-1)).view(-1)
        else:
            self._counter += 1
            params = pop.params.data[self.row]
            _lib.call("agx_ppo_act", ctypes.byref(desc), 1, n, params.data_ptr(), o.data_ptr(), 0, _lib.ptr(mask), 0,
                      1, pop.act_seed + 7919 * pop.agent_ids[self.row], (1 << 40) + self._counter,
                      out["actions"].data_ptr(), out["log_probs"].data_ptr(), out["values"].data_ptr(),
                      out["entropy"].data_ptr(), 0, None, None, _lib.stream())
        return tuple(out[k].cpu().numpy() for k in ("actions", "log_probs", "entropy", "values"))

    @property
    def rollout_buffer(self) -> "AgentRolloutBuffer":
        """The reference's ``agent.rollout_buffer`` (RolloutBuffer API: reset /
        add / compute_returns_and_advantages / size) over this agent's rows
        of the HBM rollout, for custom collectors (``collect_rollouts_fn``)."""
        buf = getattr(self, "_rollout_buffer", None)
        if buf is None or buf.pop is not self.population or buf.row != self.row:
            buf = self._rollout_buffer = AgentRolloutBuffer(self.population, self.row)
        return buf

    def learn(self, experiences=None) -> float:
        """One PPO update of this agent from the HBM rollout (ppo.py:635-921);
        returns the reference's mean loss (sum / (num_samples * epochs))."""
        if experiences is not None:
            return self._learn_from_experiences(experiences)
        # Views of one population learn together: the first view to call learn()
        # after a rollout runs the fused learner for every agent (each agent is
        # updated exactly once per rollout, as in the reference's per-agent loop).
        pop = self.population
        if getattr(pop, "_learned_rollout", None) != pop.rollout_id:
            pop._last_losses = pop.learn().cpu().numpy()
            pop.check_errors()  # a partner timeout would leave the update incomplete: raise, never return it
            pop._learned_rollout = pop.rollout_id
        return float(pop._last_losses[self.row])

    def _learn_from_experiences(self, experiences) -> float:
        """The reference's deprecated ``learn(experiences)``
        (ppo.py:655-812, use_rollout_buffer=False): (observations, actions,
        log_probs, rewards, dones, values, next_obs, next_done) stacked over
        time; GAE with next_non_terminal = 1 - dones[t + 1] (next_done at the
        end) and the critic's value of next_obs; per epoch one numpy shuffle,
        minibatches of ``batch_size`` (singletons skipped) with the advantage
        normalised per minibatch, the clipped loss, the two-group gradient clip
        and Adam (agx_clip_adam on this agent's row); target_kl checked after
        each epoch on the last minibatch's approx_kl.  -> mean_loss /
        (num_samples * update_epochs)."""
        from ..population.nets import categorical

        if not experiences:
            raise ValueError("Experiences must be provided when use_rollout_buffer is False")
        pop, r, spec = self.population, self.row, self.spec
        if pop.fused_descriptor() is None and getattr(spec, "feat_dim", None) is not None:
            raise NotImplementedError("learn(experiences): MLP actor-critics")

        def stack(x, dtype):
            if isinstance(x, torch.Tensor):
                t = x
            elif isinstance(x, (list, tuple)) and len(x) and isinstance(x[0], torch.Tensor):
                t = torch.stack([torch.as_tensor(v) for v in x])
            else:
                t = torch.as_tensor(np.asarray(x))
            return t.to(self.device, dtype)

        obs, actions, log_probs, rewards, dones, values, next_obs, next_done = experiences
        obs = stack(obs, torch.float32)
        actions, log_probs = stack(actions, torch.int64), stack(log_probs, torch.float32)
        rewards, dones, values = stack(rewards, torch.float32), stack(dones, torch.float32), stack(values, torch.float32)
        next_obs, next_done = stack(next_obs, torch.float32), stack(next_done, torch.float32)
        T = rewards.shape[0]
        params = pop.params.data[r:r + 1]
        with torch.no_grad():
            _, next_value = spec.forward(params, next_obs.reshape(1, -1, spec.obs_dim))
            next_value = next_value.reshape(-1)
            adv = torch.zeros_like(rewards)
            last = torch.zeros_like(rewards[0])
            for t in reversed(range(T)):
                nnt = 1.0 - (next_done if t == T - 1 else dones[t + 1])
                nv = next_value if t == T - 1 else values[t + 1]
                delta = rewards[t] + self.gamma * nv * nnt - values[t]
                adv[t] = last = delta + self.gamma * self.gae_lambda * nnt * last
            returns = adv + values
        obs_f = obs.reshape(-1, spec.obs_dim)
        act_f, lp_f, adv_f = actions.reshape(-1), log_probs.reshape(-1), adv.reshape(-1)
        ret_f, val_f = returns.reshape(-1), values.reshape(-1)
        n = obs_f.shape[0]
        idxs = np.arange(n)
        opt = pop.opt
        active = torch.zeros(pop.P, dtype=torch.uint8, device=self.device)
        active[r] = 1
        mean_loss, approx_kl = 0.0, None
        clip, vf, ent = self.clip_coef, self.vf_coef, float(self.ent_coef)
        for _ in range(int(self.update_epochs)):
            np.random.shuffle(idxs)
            for start in range(0, n, int(self.batch_size)):
                mb = idxs[start:start + int(self.batch_size)]
                if len(mb) <= 1:
                    continue
                sel = torch.as_tensor(mb, device=self.device)
                w = pop.params.data[r:r + 1].detach().clone().requires_grad_(True)
                logits, value = spec.forward(w, obs_f[sel].unsqueeze(0))
                logp_all, entropy = categorical(logits[0])
                logp = logp_all.gather(-1, act_f[sel].unsqueeze(-1)).squeeze(-1)
                logratio = logp - lp_f[sel]
                ratio = logratio.exp()
                with torch.no_grad():
                    approx_kl = ((ratio - 1) - logratio).mean()
                a = adv_f[sel]
                a = (a - a.mean()) / (a.std() + 1e-8)
                pg_loss = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
                v = value[0].view(-1)
                v_clipped = val_f[sel] + torch.clamp(v - val_f[sel], -clip, clip)
                v_loss = 0.5 * torch.max((v - ret_f[sel]) ** 2, (v_clipped - ret_f[sel]) ** 2).mean()
                loss = pg_loss - ent * entropy.mean() + v_loss * vf
                loss.backward()
                opt.grads[r].copy_(w.grad[0])
                opt.step(active)
                mean_loss += loss.item()
            if self.target_kl is not None and approx_kl is not None and approx_kl > self.target_kl:
                break
        return mean_loss / (n * int(self.update_epochs))

    @torch.no_grad()
    def test(self, env, swap_channels: bool = False, max_steps: int | None = None, loop: int = 3,
             vectorized: bool = True, callback=None) -> float:
        """Mean score over ``loop`` passes in which every env finishes one
        episode (ppo.py:1113-1289); appends to ``self.fitness``."""
        rewards = []
        num_envs = env.num_envs if hasattr(env, "num_envs") and vectorized else 1
        for _ in range(loop):
            obs, _info = env.reset()
            scores = np.zeros(num_envs)
            completed = np.zeros(num_envs)
            finished = np.zeros(num_envs, dtype=bool)
            step = 0
            while not np.all(finished):
                action, _, _, _ = self.get_action(obs)
                obs, reward, term, trunc, _info = env.step(action)
                step += 1
                scores += np.asarray(reward).reshape(num_envs)
                done = np.logical_or(term, trunc).reshape(num_envs)
                if max_steps is not None and step == max_steps:
                    done = np.ones(num_envs, dtype=bool)
                for i in range(num_envs):
                    if done[i] and not finished[i]:
                        completed[i] = scores[i]
                        finished[i] = True
            rewards.append(float(np.mean(completed)))
        mean_fit = float(np.mean(rewards))
        self.fitness.append(mean_fit)
        return mean_fit


class AgentRolloutBuffer:
    """RolloutBuffer (agilerl/components/rollout_buffer.py:61-481) calls on one
    agent's slice of a population's HBM rollout SoA.  A custom collector
    (train_on_policy's ``collect_rollouts_fn``, on_policy.py:23-203 shape)
    ``reset()``s it, ``add()``s one vector step at a time (obs, action,
    reward, done, value, log_prob of the agent's num_envs envs) and calls
    ``compute_returns_and_advantages(last_value, last_done)``: the agx_gae
    launch of the agent's population.  The population must hold this agent
    alone (train_on_policy runs custom collectors with one agent per group),
    so the GAE and the learn that follows touch no other agent's rollout."""

    def __init__(self, pop, row: int):
        self.pop, self.row = pop, int(row)
        self.capacity, self.num_envs = pop.T, pop.N
        self.pos, self.full = 0, False

    def reset(self) -> None:
        self.pos, self.full = 0, False

    def size(self) -> int:
        return self.capacity * self.num_envs if self.full else self.pos * self.num_envs

    def _put(self, dst: torch.Tensor, value, dtype=None) -> None:
        t = torch.as_tensor(np.asarray(value) if not isinstance(value, torch.Tensor) else value, device=dst.device)
        dst.copy_(t.to(dtype or dst.dtype).reshape(dst.shape))

    def add(self, obs, action, reward, done, value, log_prob, next_obs=None, hidden_state=None, **_kw) -> None:
        if self.pos >= self.capacity:
            raise ValueError(f"rollout buffer full ({self.capacity} vector steps); call reset()")
        p, t = self.pop, self.pos
        self._put(p.obs[self.row, t], obs)
        self._put(p.actions[self.row, t], action)
        self._put(p.rewards[self.row, t], reward)
        self._put(p.dones[self.row, t], np.asarray(done, dtype=np.uint8) if not isinstance(done, torch.Tensor)
                  else done.to(torch.uint8))
        self._put(p.values[self.row, t], value)
        self._put(p.log_probs[self.row, t], log_prob)
        self.pos += 1
        self.full = self.pos == self.capacity

    def compute_returns_and_advantages(self, last_value, last_done) -> None:
        p = self.pop
        if p.P != 1:
            raise NotImplementedError("a custom collector fills one agent's rollout: the agent must be alone in "
                                      "its population (train_on_policy groups agents one per population when "
                                      "collect_rollouts_fn is given)")
        if not self.full:
            raise ValueError(f"the rollout holds {self.pos} of {self.capacity} vector steps; the learner takes a "
                             "full rollout (ceil(learn_step / num_envs) steps)")
        lv = torch.as_tensor(np.asarray(last_value, dtype=np.float32) if not isinstance(last_value, torch.Tensor)
                             else last_value, device=p.device).to(torch.float32).reshape(1, p.N).contiguous()
        ld = torch.as_tensor(np.asarray(last_done) if not isinstance(last_done, torch.Tensor) else last_done,
                             device=p.device).to(torch.uint8).reshape(1, p.N).contiguous()
        p.finish_rollout(None, ld, lv)
