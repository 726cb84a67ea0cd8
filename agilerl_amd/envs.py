"""Host-side synthetic vectorised environments (gymnasium-style API).

``SyntheticVecEnv`` is a LunarLander-v2-shaped stand-in (obs 8 f32, 4
discrete actions, reward ~ N(0,1), termination ~ Bernoulli(1/200)) whose step
costs ~nothing, so benchmarks measure the framework, not box2d (SURVEY §8d;
gymnasium/box2d are not installed on this image).  It returns the
gymnasium 5-tuple ``(obs, reward, terminated, truncated, info)``.

Observations/rewards/dones are written straight into caller-provided
(pinned) host buffers when given, so the H2D copy into the HBM rollout SoA is
a single async hipMemcpy per field per step.
"""

from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def sample(self):
        return np.random.randint(self.n)


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = dtype
        self.low = np.full(self.shape, low, dtype=dtype)
        self.high = np.full(self.shape, high, dtype=dtype)

    def sample(self):
        return np.random.uniform(self.low, self.high).astype(self.dtype)


class Dict:
    """Mapping of named spaces; a plain dict is key-sorted like gymnasium's
    ``spaces.Dict``."""

    def __init__(self, spaces: dict):
        from collections import OrderedDict

        self.spaces = spaces if isinstance(spaces, OrderedDict) else dict(sorted(spaces.items()))

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def values(self):
        return self.spaces.values()

    def __getitem__(self, k):
        return self.spaces[k]

    def __iter__(self):
        return iter(self.spaces)

    def __len__(self):
        return len(self.spaces)


class SyntheticVecEnv:
    """``num_envs`` independent synthetic episodes; data drawn from a ring of
    pre-generated batches (``ring`` steps) so a step is a memcpy.
    ``max_episode_steps`` truncates episodes like gymnasium's TimeLimit
    (LunarLander: 1000); None never truncates (the bench's default)."""

    def __init__(self, num_envs: int, obs_dim: int = 8, n_actions: int = 4, p_done: float = 1 / 200,
                 seed: int = 0, ring: int = 97, max_episode_steps: int | None = None):
        self.num_envs = int(num_envs)
        self.single_observation_space = Box(-np.inf, np.inf, (obs_dim,))
        self.single_action_space = Discrete(n_actions)
        self.observation_space = self.single_observation_space
        self.action_space = self.single_action_space
        rng = np.random.default_rng(seed)
        self._obs = rng.standard_normal((ring, num_envs, obs_dim), dtype=np.float32)
        self._rew = rng.standard_normal((ring, num_envs), dtype=np.float32)
        self._term = rng.random((ring, num_envs)) < p_done
        self._trunc = np.zeros(num_envs, dtype=bool)
        self.max_episode_steps = max_episode_steps
        self._len = np.zeros(num_envs, dtype=np.int64)
        self._k = 0
        self._ring = ring
        self.steps = 0

    def reset(self, seed=None, options=None, out_obs: np.ndarray | None = None):
        self._k = 0
        self._len[:] = 0
        obs = self._obs[0]
        if out_obs is not None:
            np.copyto(out_obs.reshape(obs.shape), obs)
            obs = out_obs
        return obs, {}

    def step(self, actions, out_obs=None, out_rew=None, out_done=None):
        self._k = (self._k + 1) % self._ring
        self.steps += self.num_envs
        obs, rew, term = self._obs[self._k], self._rew[self._k], self._term[self._k]
        if out_obs is not None:
            np.copyto(out_obs.reshape(obs.shape), obs)
            obs = out_obs
        if out_rew is not None:
            np.copyto(out_rew.reshape(rew.shape), rew)
            rew = out_rew
        if out_done is not None:
            np.copyto(out_done.reshape(term.shape), term)
        trunc = self._trunc
        if self.max_episode_steps is not None:
            self._len += 1
            trunc = (self._len >= self.max_episode_steps) & ~term
            self._len[term | trunc] = 0
        return obs, rew, term, trunc, {}

    def close(self):
        pass


class SyntheticMultiAgentVecEnv:
    """PettingZoo-parallel-style vectorised multi-agent stand-in shaped like
    MPE simple_speaker_listener (speaker: obs 3, 3 actions; listener: obs 11,
    5 actions): ``reset() -> (obs, infos)``, ``step(actions) -> (obs,
    rewards, terminations, truncations, infos)``, each a dict agent_id ->
    array with a leading ``num_envs`` dim.  Rewards ~ N(0,1) shared, episodes
    truncate after ``max_cycles`` steps (simple_speaker_listener has no
    terminations)."""

    def __init__(self, num_envs: int, agent_dims: dict | None = None, max_cycles: int = 25, seed: int = 0,
                 ring: int = 61):
        agent_dims = agent_dims or {"speaker_0": (3, 3), "listener_0": (11, 5)}
        self.num_envs = int(num_envs)
        self.agents = list(agent_dims)
        self.possible_agents = list(agent_dims)
        self.observation_spaces = {a: Box(-np.inf, np.inf, (o,)) for a, (o, _) in agent_dims.items()}
        self.action_spaces = {a: Discrete(n) for a, (_, n) in agent_dims.items()}
        rng = np.random.default_rng(seed)
        self._obs = {a: rng.standard_normal((ring, num_envs, o), dtype=np.float32) for a, (o, _) in agent_dims.items()}
        self._rew = rng.standard_normal((ring, num_envs), dtype=np.float32)
        self._ring, self._k, self._t = ring, 0, 0
        self.max_cycles = max_cycles

    def single_observation_space(self, agent):
        return self.observation_spaces[agent]

    def single_action_space(self, agent):
        return self.action_spaces[agent]

    def observation_space(self, agent):
        return self.observation_spaces[agent]

    def action_space(self, agent):
        return self.action_spaces[agent]

    def reset(self, seed=None, options=None):
        self._k, self._t = 0, 0
        return {a: self._obs[a][0].copy() for a in self.agents}, {a: {} for a in self.agents}

    def step(self, actions):
        self._k = (self._k + 1) % self._ring
        self._t += 1
        trunc = np.full(self.num_envs, self._t % self.max_cycles == 0)
        obs = {a: self._obs[a][self._k].copy() for a in self.agents}
        rew = {a: self._rew[self._k].copy() for a in self.agents}
        term = {a: np.zeros(self.num_envs, dtype=bool) for a in self.agents}
        return obs, rew, term, {a: trunc.copy() for a in self.agents}, {a: {} for a in self.agents}

    def close(self):
        pass
