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

    #: the step never touches the GPU (PopulationRunner may pace a persistent rollout)
    agx_device_free = True

    def __init__(self, num_envs: int, obs_dim: int = 8, n_actions: int = 4, p_done: float = 1 / 200,
                 seed: int = 0, ring: int = 97, max_episode_steps: int | None = None):
        self.num_envs = int(num_envs)
        self.single_observation_space = Box(-np.inf, np.inf, (obs_dim,))
        self.single_action_space = Discrete(n_actions)
        self.observation_space = self.single_observation_space
        self.action_space = self.single_action_space
        self._obs_dim, self._p_done, self._ring, self.seed = obs_dim, p_done, ring, seed
        self._generate(seed)
        self._trunc = np.zeros(num_envs, dtype=bool)
        self.max_episode_steps = max_episode_steps
        self._len = np.zeros(num_envs, dtype=np.int64)
        self._k = 0
        self._ring = ring
        self.steps = 0

    def _generate(self, seed: int) -> None:
        rng = np.random.default_rng(seed)
        ring, n = self._ring, self.num_envs
        self._obs = rng.standard_normal((ring, n, self._obs_dim), dtype=np.float32)
        self._rew = rng.standard_normal((ring, n), dtype=np.float32)
        self._term = rng.random((ring, n)) < self._p_done

    def reseed(self, seed: int) -> None:
        """A different episode stream (StackedVecEnv.from_shared gives each
        agent's copy its own)."""
        self.seed = int(seed)
        self._generate(self.seed)

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


class SyntheticAtariVecEnv(SyntheticVecEnv):
    """Pong-shaped stand-in (ALE is not installed): uint8 frame stacks
    ``(4, 84, 84)`` in [0, 255] (AtariPreprocessing + FrameStack, channels
    first), 6 discrete actions, sparse rewards in {-1, 0, +1} (a point every
    ~60 steps), termination ~ Bernoulli(1/800).  Frames come from a ring of
    pre-generated batches, as SyntheticVecEnv."""

    def __init__(self, num_envs: int, frame_shape=(4, 84, 84), n_actions: int = 6, p_done: float = 1 / 800,
                 seed: int = 0, ring: int = 13, max_episode_steps: int | None = None):
        self.num_envs = int(num_envs)
        self.single_observation_space = Box(0, 255, tuple(frame_shape), dtype=np.uint8)
        self.single_action_space = Discrete(n_actions)
        self.observation_space = self.single_observation_space
        self.action_space = self.single_action_space
        self._frame_shape, self._p_done, self._ring, self.seed = tuple(frame_shape), p_done, ring, seed
        self._generate(seed)
        self._trunc = np.zeros(num_envs, dtype=bool)
        self.max_episode_steps = max_episode_steps
        self._len = np.zeros(num_envs, dtype=np.int64)
        self._k = 0
        self.steps = 0

    def _generate(self, seed: int) -> None:
        rng = np.random.default_rng(seed)
        ring, n = self._ring, self.num_envs
        self._obs = rng.integers(0, 256, (ring, n, *self._frame_shape), dtype=np.uint8)
        point = rng.random((ring, n)) < 1 / 60
        self._rew = np.where(point, np.where(rng.random((ring, n)) < 0.5, -1.0, 1.0), 0.0).astype(np.float32)
        self._term = rng.random((ring, n)) < self._p_done


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


def _reseed_copy(env, k: int) -> None:
    """Give a deep-copied env its own random stream: ``reseed(seed)`` when the
    env offers it (the synthetic envs), else a fresh ``np_random`` generator on
    the env and on each gymnasium sub-env."""
    base = int(getattr(env, "seed", 0) or 0) if not callable(getattr(env, "seed", None)) else 0
    seed = (base + 1_000_003 * k) & 0x7FFFFFFF
    if callable(getattr(env, "reseed", None)):
        env.reseed(seed)
        return
    subs = list(getattr(env, "envs", []) or [])
    for j, e in enumerate([env, *subs]):
        if hasattr(e, "np_random"):
            try:
                e.np_random = np.random.default_rng(seed + j)
            except (AttributeError, TypeError):
                pass


class StackedVecEnv:
    """P vector envs side by side as ONE vector env of sum(num_envs) envs, in
    order (agent p of a population owns the p-th block).  Works with any
    gymnasium-style vector env (``reset() -> (obs, info)``, ``step(a) ->
    (obs, reward, terminated, truncated, info)``) and also offers the
    ``out_*`` write-into-staging arguments PopulationRunner uses.  A per-step
    ``info["action_mask"]`` is stacked the same way.

    ``from_shared(env, copies)`` builds it from the reference's call-site env
    (train_on_policy.py:210 shares ONE N-env between agents that take turns,
    each turn starting from env.reset()): the population engine steps all
    agents at once, so each agent gets its own deep copy of that env."""

    def __init__(self, envs: list):
        self.envs = list(envs)
        self.sizes = [int(e.num_envs) for e in self.envs]
        self.num_envs = int(sum(self.sizes))
        e0 = self.envs[0]
        for attr in ("single_observation_space", "single_action_space", "observation_space", "action_space"):
            if hasattr(e0, attr):
                setattr(self, attr, getattr(e0, attr))
        space = getattr(e0, "single_observation_space", None)
        # uint8 image frames stay uint8; everything else is stacked as f32
        self._obs_dtype = np.uint8 if getattr(space, "dtype", None) == np.uint8 else np.float32
        self._fz = None  # the stacked rings of a lock-step SyntheticVecEnv stack (_fusable)

    @classmethod
    def from_shared(cls, env, copies: int, offset: int = 0) -> "StackedVecEnv":
        """``offset``: global index of the first agent (a population sharded
        over ranks): copy k behaves as the unsharded population's copy
        offset + k, copy 0 of the global population being ``env`` itself."""
        import copy

        try:
            clones = [copy.deepcopy(env) for _ in range(copies - (1 if offset == 0 else 0))]
        except Exception as err:  # noqa: BLE001 - e.g. subprocess-backed vector envs
            raise TypeError(f"cannot clone {type(env).__name__} for {copies} agents ({err}); pass a vector env "
                            f"of population_size x num_envs environments or a StackedVecEnv of one env per agent")
        # the reference's agents take turns on one env, so each sees different
        # episodes: give every copy its own random stream instead of the
        # original's (a deep copy would replay it)
        first = 1 if offset == 0 else offset
        for k, c in enumerate(clones, start=first):
            _reseed_copy(c, k)
        return cls(([env] if offset == 0 else []) + clones)

    @property
    def agx_device_free(self) -> bool:
        return all(bool(getattr(e, "agx_device_free", False)) for e in self.envs)

    def _split(self, x):
        out, s = [], 0
        for n in self.sizes:
            out.append(x[s:s + n])
            s += n
        return out

    def _cat(self, parts, out=None, dtype=None):
        if out is not None:  # each env's block straight into its slice of the staging (one copy)
            flat = out.reshape(self.num_envs, -1)
            s = 0
            for n, p in zip(self.sizes, parts):
                np.copyto(flat[s:s + n], np.asarray(p).reshape(n, -1), casting="unsafe")
                s += n
            return out
        return np.concatenate([np.asarray(p, dtype=dtype) for p in parts], axis=0)

    @staticmethod
    def _infos(infos):
        masks = [i.get("action_mask") if isinstance(i, dict) else None for i in infos]
        if all(m is not None for m in masks):
            return {"action_mask": np.concatenate([np.asarray(m) for m in masks], axis=0)}
        return {}

    def reset(self, seed=None, options=None, out_obs: np.ndarray | None = None):
        # a vector env seeds its sub-envs seed, seed + 1, ...: block k starts
        # after the blocks before it, so no two sub-envs share a seed
        offs = np.concatenate([[0], np.cumsum(self.sizes)[:-1]]).tolist()
        res = [e.reset() if seed is None else e.reset(seed=seed + int(o)) for o, e in zip(offs, self.envs)]
        obs = self._cat([r[0] for r in res], out_obs, self._obs_dtype)
        return obs, self._infos([r[1] for r in res])

    #: stacked rings above this size are not built (the blocks step one by one)
    FUSE_BYTES = 256 << 20

    def _fusable(self) -> bool:
        """Every block a SyntheticVecEnv (the flat-vector kind) in lock-step
        (same ring position, ring length and time limit): then one vectorized
        step over stacked copies of the blocks' rings does what stepping each
        block does, with one copy per output instead of one per block.  The
        blocks' episode lengths become views into one stacked array, so a
        block stepped on its own later (after a regroup) stays consistent; a
        reseeded block, a block stepped on its own, or a block re-stacked
        elsewhere drops the stacked rings (rebuilt, or the per-block path)."""
        envs = self.envs
        fz = self._fz
        if fz is not None:
            ids, views, seen = fz[0], fz[4], fz[9]
            k = envs[0]._k
            for e, i, v in zip(envs, ids, views):
                if e._obs is not i or e._len is not v or e._k != k:
                    break
            else:
                if any(e.steps != n for e, n in zip(envs, seen)):
                    # blocks stepped on their own in lock step (ring positions still
                    # agree): their lengths grew in place, the cached bound did not
                    fz[7][0] = int(fz[5].max()) if fz[5].size else 0
                    seen[:] = [e.steps for e in envs]
                return True
            self._fz = None
        e0 = envs[0]
        if any(type(e) is not SyntheticVecEnv for e in envs):
            return False
        if any(e._ring != e0._ring or e.max_episode_steps != e0.max_episode_steps or e._k != e0._k or
               e._obs_dim != e0._obs_dim for e in envs):
            return False
        if sum(e._obs.nbytes + e._rew.nbytes + e._term.nbytes for e in envs) > self.FUSE_BYTES:
            return False
        obs = np.concatenate([e._obs for e in envs], axis=1)
        rew = np.concatenate([e._rew for e in envs], axis=1)
        term = np.concatenate([e._term for e in envs], axis=1)
        lens = np.concatenate([e._len for e in envs])
        views, s = [], 0
        for e in envs:
            e._len = lens[s:s + e.num_envs]
            views.append(e._len)
            s += e.num_envs
        # [6]: an upper bound of the episode lengths (while it stays below the
        # time limit no env can be truncated and the step skips that test)
        # [8]: per ring slot, whether any env's episode ends there (a lookup
        # instead of a test of the slot's terminations every step)
        # [9]: each block's step count as of the last fused step (a block stepped
        # on its own invalidates [6]'s bound)
        self._fz = ([e._obs for e in envs], obs, rew, term, views, lens, np.zeros(self.num_envs, dtype=bool),
                    [int(lens.max()) if lens.size else 0], term.any(axis=1).tolist(), [e.steps for e in envs])
        return True

    def _step_fused(self, out_obs, out_rew, out_done):
        _, robs, rrew, rterm, _, lens, ztrunc, lmax, rany, seen = self._fz
        e0 = self.envs[0]
        k = (e0._k + 1) % e0._ring
        for j, e in enumerate(self.envs):
            e._k = k
            e.steps += e.num_envs
            seen[j] = e.steps
        obs, rew, term = robs[k], rrew[k], rterm[k]
        if out_obs is not None:
            np.copyto(out_obs.reshape(obs.shape), obs)
            obs = out_obs
        if out_rew is not None:
            np.copyto(out_rew.reshape(rew.shape), rew)
            rew = out_rew
        if out_done is not None:
            np.copyto(out_done.reshape(term.shape), term)
        trunc = ztrunc
        if e0.max_episode_steps is not None:
            lens += 1
            lmax[0] += 1
            if lmax[0] < e0.max_episode_steps:  # no env can reach the limit: only episode ends reset
                if rany[k]:
                    lens[term] = 0
            else:
                trunc = (lens >= e0.max_episode_steps) & ~term
                lens[term | trunc] = 0
                lmax[0] = int(lens.max())
        return obs, rew, term, trunc, {}

    def step(self, actions, out_obs=None, out_rew=None, out_done=None):
        if self._fusable():
            return self._step_fused(out_obs, out_rew, out_done)
        res = [e.step(a) for e, a in zip(self.envs, self._split(np.asarray(actions)))]
        obs = self._cat([r[0] for r in res], out_obs, self._obs_dtype)
        rew = self._cat([r[1] for r in res], out_rew, np.float32)
        term = np.concatenate([np.asarray(r[2], dtype=bool) for r in res])
        trunc = np.concatenate([np.asarray(r[3], dtype=bool) for r in res])
        if out_done is not None:
            np.copyto(out_done.reshape(term.shape), term)
        return obs, rew, term, trunc, self._infos([r[4] for r in res])

    def close(self):
        for e in self.envs:
            if hasattr(e, "close"):
                e.close()
