"""Drop-in ``MADDPG`` (agilerl/algorithms/maddpg.py:46-960) for Box
observations and Discrete / Box actions, one network per agent.

Networks are the reference's: ``DeterministicActor`` per agent (EvolvableMLP
encoder + "actor" head, GumbelSoftmax / Tanh output) and a centralised
``ContinuousQNetwork`` critic per agent on the Dict of every agent's
observation (``EvolvableMultiInput``: concatenated vector observations ->
``final_dense`` -> ReLU) plus all agents' actions.  The critic step of
``_learn_individual`` — NaN rewards -> 0, NaN dones -> 1, y = r + (1 - d)
gamma Q'(s', a'), MSE and its gradient — is one libagx launch
(``agx_maddpg_critic_target``); soft updates are ``agx_polyak``.  Grouped
(shared-policy) agents, action masks and env-defined actions are outside the
hot path.
"""

from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Any

import numpy as np
import torch

from .. import kernels as K
from ..envs import Dict as DictSpace
from ..networks import ContinuousQNetwork, DeterministicActor
from ..networks.base import as_config, mlp_net_config
from . import checkpoint as C
from .evolvable import EvolvableAgentMixin


class _CriticLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, q_next, rewards, dones, gamma):
        _, g_q, loss = K.maddpg_critic_target(q.contiguous(), q_next.contiguous(), rewards.contiguous(),
                                              dones.contiguous(), gamma)
        ctx.save_for_backward(g_q.view_as(q))
        return loss.view(())

    @staticmethod
    def backward(ctx, gl):
        (g_q,) = ctx.saved_tensors
        return g_q * gl, None, None, None, None


def _as_dict(spaces, agent_ids):
    if isinstance(spaces, (list, tuple)):
        return OrderedDict(zip(agent_ids, spaces))
    return OrderedDict((a, spaces[a]) for a in agent_ids)


def _action_dim(space) -> int:
    return int(space.n) if hasattr(space, "n") else int(np.prod(space.shape))


class MADDPG(EvolvableAgentMixin):
    algo = "MADDPG"
    # maddpg.py:424-444: the actors are the policy group (targets shared); one
    # optimizer set per learning rate
    _lr_optimizers = {"lr_actor": "actor_optimizers", "lr_critic": "critic_optimizers"}
    _policy_group = ("actors", "actor_targets")

    def __init__(self, observation_spaces, action_spaces, agent_ids: list[str] | None = None,
                 O_U_noise: bool = True, expl_noise: float = 0.1, vect_noise_dim: int = 1, mean_noise: float = 0.0,
                 theta: float = 0.15, dt: float = 1e-2, index: int = 0, hp_config=None,
                 net_config: dict[str, Any] | None = None, batch_size: int = 64, lr_actor: float = 0.001,
                 lr_critic: float = 0.01, learn_step: int = 5, gamma: float = 0.95, tau: float = 0.01, mut=None,
                 normalize_images: bool = True, actor_networks=None, critic_networks=None, device="cuda",
                 accelerator=None, torch_compiler=None, wrap: bool = True) -> None:
        assert learn_step >= 1, "Learn step must be greater than or equal to one."
        assert isinstance(learn_step, int), "Learn step rate must be an integer."
        assert isinstance(batch_size, int), "Batch size must be an integer."
        assert batch_size >= 1, "Batch size must be greater than or equal to one."
        assert isinstance(lr_actor, float), "Actor learning rate must be a float."
        assert lr_actor > 0, "Actor learning rate must be greater than zero."
        assert isinstance(lr_critic, float), "Critic learning rate must be a float."
        assert lr_critic > 0, "Critic learning rate must be greater than zero."
        assert isinstance(gamma, float), "Gamma must be a float."
        assert isinstance(tau, float), "Tau must be a float."
        assert tau > 0, "Tau must be greater than zero."
        if actor_networks is not None or critic_networks is not None:
            raise NotImplementedError("custom actor/critic modules: use net_config (MLP) networks")
        if agent_ids is None:
            agent_ids = list(observation_spaces.keys()) if hasattr(observation_spaces, "keys") else \
                [f"agent_{i}" for i in range(len(observation_spaces))]
        self.agent_ids = list(agent_ids)
        self.observation_space = _as_dict(observation_spaces, self.agent_ids)
        self.action_space = _as_dict(action_spaces, self.agent_ids)
        self.possible_observation_spaces = DictSpace(dict(self.observation_space))
        self.action_dims = {a: _action_dim(s) for a, s in self.action_space.items()}
        self.index, self.hp_config, self.mut = index, hp_config, mut
        self.batch_size, self.lr_actor, self.lr_critic = batch_size, lr_actor, lr_critic
        self.learn_step, self.gamma, self.tau = learn_step, gamma, tau
        self.net_config = net_config
        self.device = torch.device(device)
        self.learn_counter = 0
        self.O_U_noise, self.vect_noise_dim, self.theta, self.dt = O_U_noise, vect_noise_dim, theta, dt
        self.sqdt = dt ** 0.5
        self.training = True
        self.scores: list[float] = []
        self.fitness: list[float] = []
        self.steps: list[int] = [0]
        dev = self.device
        self.sample_gaussian = {a: torch.zeros(vect_noise_dim, d, device=dev) for a, d in self.action_dims.items()}
        self.expl_noise = expl_noise if isinstance(expl_noise, dict) else \
            {a: expl_noise * torch.ones(vect_noise_dim, d, device=dev) for a, d in self.action_dims.items()}
        self.mean_noise = mean_noise if isinstance(mean_noise, dict) else \
            {a: mean_noise * torch.ones(vect_noise_dim, d, device=dev) for a, d in self.action_dims.items()}
        self.current_noise = {a: torch.zeros(vect_noise_dim, d, device=dev) for a, d in self.action_dims.items()}

        agent_cfgs = self._agent_configs(net_config)
        critic_cfg = self._critic_config(agent_cfgs)
        self.actors = torch.nn.ModuleDict({a: self._actor(a, agent_cfgs[a]) for a in self.agent_ids})
        self.actor_targets = torch.nn.ModuleDict({a: self._actor(a, agent_cfgs[a]) for a in self.agent_ids})
        self.critics = torch.nn.ModuleDict({a: self._critic(critic_cfg) for a in self.agent_ids})
        self.critic_targets = torch.nn.ModuleDict({a: self._critic(critic_cfg) for a in self.agent_ids})
        for a in self.agent_ids:
            self.actor_targets[a].load_state_dict(self.actors[a].state_dict())
            self.critic_targets[a].load_state_dict(self.critics[a].state_dict())
        # the networks' own generators (EvolvableModule.rng, shared with their
        # modules; seeded from the agent's initial index so a run is reproducible)
        for i, a in enumerate(self.agent_ids):
            self.actors[a].rng = np.random.default_rng((0x5EED, int(index), i))
            self.critics[a].rng = np.random.default_rng((0x5EEE, int(index), i))
            # maddpg.py:346-347: the actors' encoders do not mutate (the critic's
            # encoder is of another type)
            self.actors[a].encoder.disable_mutations()
            self.actor_targets[a].encoder.disable_mutations()
        self.actor_optimizers = {a: torch.optim.Adam(self.actors[a].parameters(), lr=lr_actor) for a in self.agent_ids}
        self.critic_optimizers = {a: torch.optim.Adam(self.critics[a].parameters(), lr=lr_critic)
                                  for a in self.agent_ids}
        self._init_registry(hp_config)

    def _fresh_optimizer(self, lr_name: str):
        nets, lr = (self.actors, self.lr_actor) if lr_name == "lr_actor" else (self.critics, self.lr_critic)
        return {a: torch.optim.Adam(nets[a].parameters(), lr=lr) for a in self.agent_ids}

    # ---- network construction (maddpg.py:296-380) ---------------------------
    def _agent_configs(self, net_config) -> dict[str, dict]:
        net_config = copy.deepcopy(as_config(net_config) or {})
        per_agent = all(a in net_config for a in self.agent_ids) if net_config else False
        out = {}
        for a in self.agent_ids:
            cfg = copy.deepcopy(net_config[a] if per_agent else net_config)
            head = as_config(cfg.get("head_config"))
            if head is None:
                head = mlp_net_config([64])
                head.pop("output_activation", None)
            cfg["head_config"] = head
            out[a] = cfg
        return out

    def _critic_config(self, agent_cfgs) -> dict:
        heads = [agent_cfgs[a]["head_config"] for a in self.agent_ids]
        deepest = max(heads, key=lambda h: len(h.get("hidden_size", [])))
        encs = [as_config(agent_cfgs[a].get("encoder_config")) for a in self.agent_ids]
        mlp = max([e for e in encs if e and "hidden_size" in e] or [mlp_net_config([64, 64])],
                  key=lambda e: len(e["hidden_size"]))
        return {"encoder_config": {"mlp_config": copy.deepcopy(mlp), "latent_dim": mlp["hidden_size"][-1]},
                "head_config": copy.deepcopy(deepest),
                "latent_dim": max(agent_cfgs[a].get("latent_dim", 32) for a in self.agent_ids),
                "min_latent_dim": min(agent_cfgs[a].get("min_latent_dim", 8) for a in self.agent_ids),
                "max_latent_dim": max(agent_cfgs[a].get("max_latent_dim", 1024) for a in self.agent_ids)}

    def _actor(self, a, cfg) -> DeterministicActor:
        return DeterministicActor(self.observation_space[a], self.action_space[a], device=self.device,
                                  **copy.deepcopy(cfg))

    def _critic(self, cfg) -> ContinuousQNetwork:
        return ContinuousQNetwork(self.possible_observation_spaces, [self.action_space[a] for a in self.agent_ids],
                                  device=self.device, **copy.deepcopy(cfg))

    # ---- architecture mutation (hpo/mutation.py:887-1011, 1163-1203) --------
    @property
    def can_mutate_architecture(self) -> bool:
        # a population sharded over ranks does not replay the module draws
        return not getattr(self, "sharded", False)

    def policy_mutation_methods(self) -> list[str]:
        """The actors ModuleDict's table: every agent's LAYER methods, then
        every agent's NODE methods, each prefixed by its agent id (the
        reference's ModuleDict under PYTHONHASHSEED=0, tests/golden
        maddpgarch*: actor_methods)."""
        layer, node = [], []
        for a in self.agent_ids:
            net = self.actors[a]
            for m in net.mutation_methods:
                (layer if net.is_layer_method(m) else node).append(f"{a}.{m}")
        return layer + node

    @staticmethod
    def _find_analogous_mutation(sampled: str | None, available: list[str], policy_agent: str) -> str | None:
        """Mutations._find_analogous_mutation (hpo/mutation.py:1163-1203)."""
        if not sampled:
            return None
        if sampled in available:
            return sampled
        bottom = sampled.split(".")[-1]
        for method in available:
            parts = method.split(".")
            if parts[-1] == bottom and (policy_agent in parts or "vector_mlp" in parts):
                return method
        return None

    def architecture_mutation(self, new_layer_prob: float, rng) -> str | None:
        """_architecture_mutate_multi (hpo/mutation.py:887-1011): a method
        sampled from the actors' table with ``rng`` (Mutations.rng), applied to
        the sampled agent's actor; the method it applied (with its mutation
        dict) to every other actor that has it; then, per critic and once per
        mutated agent (the reference's repeat guard), the analogous method.
        The targets are re-made from the mutated networks
        (reinit_shared_networks, :104-160).  -> the mutation label (the
        applied method without its agent id) or None."""
        from ..networks.base import mutation_probs

        table = self.policy_mutation_methods()
        mut_method = str(rng.choice(table, p=mutation_probs(table, new_layer_prob), size=1)[0])
        agent, method = mut_method.split(".", 1)
        applied, mut_dict = self.actors[agent].apply_mutation_dict(method)
        mutated = []
        if applied is not None:
            sampled_agent, sampled = agent, applied
            mutated.append(agent)
        else:
            sampled_agent, sampled = agent, None
        for a in self.agent_ids:
            if a == sampled_agent:
                continue
            if sampled in self.actors[a].mutation_methods:
                done, _ = self.actors[a].apply_mutation_dict(sampled, mut_dict)
                if done is not None:
                    mutated.append(a)
        self.critic_mutations = []
        for a in self.agent_ids:
            critic = self.critics[a]
            analogous, last = False, None
            for m_agent in mutated:
                if analogous and last == analogous:
                    continue
                analogous = self._find_analogous_mutation(sampled, critic.mutation_methods, m_agent)
                if analogous is None:
                    raise RuntimeError(f"MADDPG architecture mutation: no analogous method for {sampled!r} in "
                                       f"critic {a!r} ({critic.mutation_methods})")
                last, _ = critic.apply_mutation_dict(analogous, mut_dict)
                self.critic_mutations.append((a, analogous, str(last)))
        for a in self.agent_ids:
            self.actor_targets[a] = copy.deepcopy(self.actors[a])
            self.critic_targets[a] = copy.deepcopy(self.critics[a])
        return sampled

    # ---- acting (maddpg.py:456-625) ---------------------------------------
    def set_training_mode(self, training: bool) -> None:
        self.training = training

    def _obs(self, o) -> torch.Tensor:
        t = o if isinstance(o, torch.Tensor) else torch.as_tensor(np.asarray(o))
        t = t.to(self.device).float()
        return t.unsqueeze(0) if t.dim() == 1 else t

    def action_noise(self, agent_id: str) -> torch.Tensor:
        if self.O_U_noise:
            noise = (self.current_noise[agent_id]
                     + self.theta * (self.mean_noise[agent_id] - self.current_noise[agent_id]) * self.dt
                     + self.expl_noise[agent_id] * self.sqdt * self.sample_gaussian[agent_id].normal_())
            self.current_noise[agent_id] = noise
            return noise
        torch.normal(self.mean_noise[agent_id], self.expl_noise[agent_id], out=self.sample_gaussian[agent_id])
        return self.sample_gaussian[agent_id]

    def reset_action_noise(self, indices: list[int]) -> None:
        for a in self.agent_ids:
            for i in indices:
                self.current_noise[a][i, :] = 0

    @torch.no_grad()
    def get_action(self, obs: dict, infos=None, *args, **kwargs):
        """-> (actions for the env, raw actor outputs), dicts of numpy arrays."""
        raw = {}
        for a in obs:
            actor = self.actors[a]
            actor.eval()
            act = actor(self._obs(obs[a]))
            actor.train()
            if self.training:
                lo, hi = (0.0, 1.0) if hasattr(self.action_space[a], "n") else (-1.0, 1.0)
                act = torch.clamp(act + self.action_noise(a), lo, hi)
            raw[a] = act.cpu()
        processed = OrderedDict()
        for a, act in raw.items():
            if hasattr(self.action_space[a], "n"):
                processed[a] = act.numpy().argmax(axis=-1)
            else:
                actor = self.actors[a]
                processed[a] = DeterministicActor.rescale_action(act, actor.action_low, actor.action_high,
                                                                 actor.output_activation).numpy()
            raw[a] = act.numpy()
        return processed, raw

    # ---- learning (maddpg.py:629-838) ---------------------------------------
    def learn(self, experiences) -> dict[str, tuple[float, float]]:
        states, actions, rewards, next_states, dones = experiences
        dev = self.device
        actions = {a: t.to(dev) for a, t in actions.items()}
        rewards = {a: t.to(dev) for a, t in rewards.items()}
        dones = {a: t.to(dev) for a, t in dones.items()}
        states = {a: self._obs(t) for a, t in states.items()}
        next_states = {a: self._obs(t) for a, t in next_states.items()}
        with torch.no_grad():
            next_actions = [self.actor_targets[a](next_states[a]) for a in self.agent_ids]
        stacked_actions = torch.cat([actions[a] for a in self.agent_ids], dim=1)
        stacked_next_actions = torch.cat(next_actions, dim=1)
        losses = {a: self._learn_individual(a, stacked_actions, stacked_next_actions, states, next_states, actions,
                                            rewards, dones) for a in self.agent_ids}
        for a in self.agent_ids:
            self.soft_update(self.actors[a], self.actor_targets[a])
            self.soft_update(self.critics[a], self.critic_targets[a])
        return losses

    def _learn_individual(self, agent_id, stacked_actions, stacked_next_actions, states, next_states, actions,
                          rewards, dones) -> tuple[float, float]:
        actor, critic = self.actors[agent_id], self.critics[agent_id]
        q_value = critic(states, stacked_actions)
        with torch.no_grad():
            q_next = self.critic_targets[agent_id](next_states, stacked_next_actions)
        # NaN handling, y_j and MSE fused in agx_maddpg_critic_target (maddpg.py:764-781)
        critic_loss = _CriticLoss.apply(q_value, q_next, rewards[agent_id].float().reshape(-1),
                                        dones[agent_id].float().reshape(-1), float(self.gamma))
        opt_c = self.critic_optimizers[agent_id]
        opt_c.zero_grad()
        critic_loss.backward()
        opt_c.step()
        action = actor(states[agent_id])
        detached = {a: (action if a == agent_id else actions[a]) for a in self.agent_ids}
        actor_loss = -critic(states, torch.cat([detached[a] for a in self.agent_ids], dim=1)).mean()
        opt_a = self.actor_optimizers[agent_id]
        opt_a.zero_grad()
        actor_loss.backward()
        opt_a.step()
        return actor_loss.item(), critic_loss.item()

    @torch.no_grad()
    def soft_update(self, net: torch.nn.Module, target: torch.nn.Module) -> None:
        """target <- tau * net + (1 - tau) * target (maddpg.py:822-836), agx_polyak."""
        for e, t in zip(net.parameters(), target.parameters()):
            K.polyak_(t.data.view(-1), e.data.reshape(-1), float(self.tau))

    # ---- evaluation (maddpg.py:838-960) ------------------------------------
    def test(self, env, swap_channels: bool = False, max_steps: int | None = None, loop: int = 3,
             sum_scores: bool = True) -> float:
        self.set_training_mode(False)
        rewards = []
        num_envs = env.num_envs if hasattr(env, "num_envs") else 1
        vec = hasattr(env, "num_envs")
        with torch.no_grad():
            for _ in range(loop):
                obs, info = env.reset()
                width = 1 if sum_scores else len(self.agent_ids)
                scores = np.zeros((num_envs, width))
                completed = np.zeros((num_envs, width))
                finished = np.zeros(num_envs)
                step = 0
                while not np.all(finished):
                    step += 1
                    action, _ = self.get_action(obs, infos=info)
                    if not vec:
                        action = {a: act[0] for a, act in action.items()}
                    obs, reward, term, trunc, info = env.step(action)
                    r = np.array([np.asarray(reward[a]).reshape(num_envs) for a in self.agent_ids]).T
                    r = np.where(np.isnan(r), 0, r)
                    scores += r.sum(-1, keepdims=True) if sum_scores else r
                    done = np.zeros(num_envs, dtype=bool)
                    for a in self.agent_ids:
                        done |= np.asarray(term[a]).reshape(num_envs).astype(bool)
                        done |= np.asarray(trunc[a]).reshape(num_envs).astype(bool)
                    for i in range(num_envs):
                        if (done[i] or (max_steps is not None and step == max_steps)) and not finished[i]:
                            completed[i] = scores[i]
                            finished[i] = 1
                rewards.append(np.mean(completed, axis=0))
        self.set_training_mode(True)
        mean_fit = np.mean(rewards, axis=0)
        mean_fit = float(mean_fit[0]) if sum_scores else mean_fit
        self.fitness.append(mean_fit)
        return mean_fit

    def clone(self, index: int | None = None, wrap: bool = True):
        c = copy.deepcopy(self)
        if index is not None:
            c.index = index
        return c

    # ---- checkpoints (core/base.py:939-1072 layout, see checkpoint.py) --------
    def save_checkpoint(self, path: str) -> None:
        mods = {n: {a: m.state_dict() for a, m in getattr(self, n).items()}
                for n in ("actors", "actor_targets", "critics", "critic_targets")}
        opts = {n: {a: o.state_dict() for a, o in getattr(self, n).items()}
                for n in ("actor_optimizers", "critic_optimizers")}
        ck = C.checkpoint_dict(self, mods, opts, spaces=False)
        ck["lr_actor"], ck["lr_critic"], ck["agent_ids"] = self.lr_actor, self.lr_critic, self.agent_ids
        torch.save(ck, path)

    @torch.no_grad()
    def load_checkpoint(self, path: str) -> None:
        ck = C.read(path, self.algo)
        info = ck["network_info"]
        for n in ("actors", "actor_targets", "critics", "critic_targets"):
            for a, sd in info["modules"][f"{n}_state_dict"].items():
                if sd:  # empty ones are skipped, as the reference (core/base.py:1006-1008)
                    getattr(self, n)[a].load_state_dict(sd)
        for n in ("actor_optimizers", "critic_optimizers"):
            for a, sd in info["optimizers"][f"{n}_state_dict"].items():
                getattr(self, n)[a].load_state_dict(sd)
        C.restore_attributes(self, ck)
