"""Generate golden input/output vectors from the reference's OWN hot-path code.

Test infrastructure only.  Runs in the build container (where the read-only
reference checkout lives at /root/reference); skips cleanly when it is absent.
Nothing from the reference is copied: the reference source files are executed
in place (path-loaded, bytecode writing disabled) with ``sys.modules`` stubs
for the third-party imports that are not installed here (gymnasium,
tensordict, pettingzoo) and for the agilerl sub-packages these files import
but the exercised methods never touch.  Only seeded inputs and the outputs the
reference produced are written, as small ``.npz`` files beside this script.

Reference functions exercised (paths relative to /root/reference):
  * agilerl/components/rollout_buffer.py:413-481  RolloutBuffer.compute_returns_and_advantages
  * agilerl/components/segment_tree.py            SumSegmentTree / MinSegmentTree
  * agilerl/components/replay_buffer.py:261-428   PrioritizedReplayBuffer (_update_priority,
                                                  _sample_proportional, _calculate_weights,
                                                  update_priorities)
  * agilerl/algorithms/ppo.py:814-921             PPO._learn_from_rollout_buffer_flat (loss math;
                                                  and end to end on a real actor-critic built by
                                                  create_mlp, agilerl/utils/evolvable_networks.py:
                                                  527-644, with log_prob_discrete / entropy_discrete,
                                                  agilerl/utils/torch_utils.py:142-199, and
                                                  apply_action_mask_discrete,
                                                  agilerl/networks/distributions.py:16-28)
  * agilerl/algorithms/dqn.py:274-324             DQN.update (TD target)
  * agilerl/algorithms/dqn_rainbow.py:284-367     RainbowDQN._dqn_loss (C51 projection)
  * agilerl/hpo/tournament.py:41-119              TournamentSelection
  * agilerl/components/replay_buffer.py:206-258   MultiStepReplayBuffer._get_n_step_info
  * agilerl/components/multi_agent_replay_buffer.py:155-167  MultiAgentReplayBuffer.sample
                                                  (Python random.sample + _process_transition)
  * agilerl/algorithms/maddpg.py:707-821          MADDPG._learn_individual (critic TD target, NaN
                                                  rules, MSE loss and its gradient)
  * agilerl/hpo/mutation.py:311-453, 515-827      Mutations.mutation / rl_hyperparam_mutation /
                                                  parameter_mutation (+ RLParameter /
                                                  HyperparameterConfig, algorithms/core/registry.py)
  * agilerl/modules/custom_components.py:38-131   NoisyLinear (init / noise draw order, forwards)
  * agilerl/networks/custom_modules.py:127-162    DuelingDistributionalMLP.forward (q / probs / log)

Usage:  python tests/golden/gen_golden.py  [--ref /root/reference]
"""

from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import types

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- #
# import stubs                                                                #
# --------------------------------------------------------------------------- #
class _StubMeta(type):
    """Placeholder classes answer any class attribute (enum members, ...)."""

    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return f"<stub {cls.__name__}.{name}>"

    def __getitem__(cls, item):  # generic annotations (ModuleDict[EvolvableModule])
        return cls


class _StubModule(types.ModuleType):
    """Module whose every attribute is a fresh placeholder class."""

    def __getattr__(self, name):  # noqa: D401
        if name.startswith("__"):
            raise AttributeError(name)
        cls = _StubMeta(name, (), {"__init__": lambda self, *a, **k: None})
        setattr(self, name, cls)
        return cls


def _stub(name: str) -> types.ModuleType:
    mod = _StubModule(name)
    mod.__path__ = []  # behave like a package
    sys.modules[name] = mod
    return mod


def _install_stubs() -> None:
    for name in [
        "gymnasium",
        "gymnasium.spaces",
        "tensordict",
        "tensordict.nn",
        "pettingzoo",
        "agilerl",
        "agilerl.typing",
        "agilerl.protocols",
        "agilerl.utils",
        "agilerl.utils.algo_utils",
        "agilerl.algorithms",
        "agilerl.algorithms.core",
        "agilerl.algorithms.core.base",
        "agilerl.algorithms.core.registry",
        "agilerl.modules",
        "agilerl.modules.base",
        "agilerl.modules.configs",
        "agilerl.modules.custom_components",
        "agilerl.networks",
        "agilerl.networks.value_networks",
        "agilerl.networks.q_networks",
        "agilerl.wrappers",
        "agilerl.wrappers.make_evolvable",
        "agilerl.components",
        "agilerl.algorithms.core.registry_stub",
        "agilerl.wrappers.agent",
        "fastrand",
    ]:
        _stub(name)
    sys.modules["gymnasium"].spaces = sys.modules["gymnasium.spaces"]


def _load(ref: str, modname: str, relpath: str):
    path = os.path.join(ref, relpath)
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------- #
# GAE                                                                         #
# --------------------------------------------------------------------------- #
def gen_gae(rb_mod, out: dict) -> None:
    RolloutBuffer = rb_mod.RolloutBuffer
    cases = [
        # (T, N, p_done, use_gae, gamma, lam, seed)
        (16, 128, 0.01, True, 0.99, 0.95, 0),   # config-2 shape (one agent)
        (64, 33, 0.05, True, 0.99, 0.95, 1),    # ragged N
        (1, 7, 0.5, True, 0.99, 0.95, 2),       # T == 1: only the bootstrap branch
        (40, 16, 0.3, True, 0.97, 0.9, 3),      # dense dones, other gamma/lambda
        (512, 128, 0.01, True, 0.99, 0.95, 4),  # long scan
        (32, 64, 0.05, False, 0.99, 0.95, 5),   # Monte-Carlo branch
        (24, 5, 1.0, True, 0.99, 0.95, 6),      # every step terminal
        (24, 5, 0.0, True, 0.99, 1.0, 7),       # no terminal, lambda 1
    ]
    for k, (T, N, pd, use_gae, gamma, lam, seed) in enumerate(cases):
        rng = np.random.default_rng(seed)
        r = rng.standard_normal((T, N)).astype(np.float32)
        v = rng.standard_normal((T, N)).astype(np.float32)
        d = rng.random((T, N)) < pd
        lv = rng.standard_normal(N).astype(np.float32)
        ld = rng.random(N) < pd
        rb = object.__new__(RolloutBuffer)
        rb.capacity, rb.num_envs, rb.full, rb.pos = T, N, True, T
        rb.use_gae, rb.gamma, rb.gae_lambda = use_gae, gamma, lam
        rb.buffer = {
            "rewards": torch.from_numpy(r.copy()),
            "dones": torch.from_numpy(d.copy()),
            "values": torch.from_numpy(v.copy()),
            "advantages": torch.zeros(T, N),
            "returns": torch.zeros(T, N),
        }
        rb.compute_returns_and_advantages(torch.from_numpy(lv), torch.from_numpy(ld))
        out[f"gae{k}"] = dict(
            rewards=r, values=v, dones=d.astype(np.uint8), last_value=lv,
            last_done=ld.astype(np.uint8), gamma=np.float64(gamma), lam=np.float64(lam),
            use_gae=np.int32(use_gae),
            advantages=rb.buffer["advantages"].numpy().copy(),
            returns=rb.buffer["returns"].numpy().copy(),
        )


# --------------------------------------------------------------------------- #
# segment tree + PER                                                          #
# --------------------------------------------------------------------------- #
def gen_segment_tree(st_mod, out: dict) -> None:
    Sum, Min = st_mod.SumSegmentTree, st_mod.MinSegmentTree
    rng = np.random.default_rng(11)
    cap = 64
    s, m = Sum(cap), Min(cap)
    idx = rng.integers(0, cap, 300)
    val = np.abs(rng.standard_normal(300)) + 1e-3
    for i, x in zip(idx, val):
        s[int(i)] = float(x)
        m[int(i)] = float(x)
    q = np.concatenate([rng.random(200) * s.sum(), [0.0, s.sum(), s.sum() * 0.5]])
    ret = np.array([s.retrieve(float(u)) for u in q], dtype=np.int64)
    ranges = [(0, 0), (3, 17), (0, 63), (10, 11), (5, -1), (31, 33)]
    sums = np.array([s.sum(a, b) for a, b in ranges])
    mins = np.array([m.min(a, b) for a, b in ranges])
    out["segtree"] = dict(
        cap=np.int64(cap), set_idx=idx.astype(np.int64), set_val=val,
        sum_tree=np.array(s.tree), min_tree=np.array(m.tree), queries=q,
        retrieve=ret, ranges=np.array(ranges, dtype=np.int64), range_sum=sums, range_min=mins,
    )


def _per_add(buf, n: int) -> None:
    """The priority half of PrioritizedReplayBuffer.add (replay_buffer.py:296-309);
    the TensorDict storage half is not needed for the tree."""
    for _ in range(n):
        buf._update_priority(buf.tree_ptr, buf.max_priority)
        buf.tree_ptr = (buf.tree_ptr + 1) % buf.max_size
    buf._size = min(buf._size + n, buf.max_size)


def gen_per(rp_mod, out: dict) -> None:
    PER = rp_mod.PrioritizedReplayBuffer
    cases = [
        # (max_size, n_add, B, beta, alpha, rounds, seed)
        (100, 60, 32, 0.4, 0.6, 3, 21),
        (1000, 1000, 64, 0.4, 0.6, 4, 22),     # full buffer, config-3 batch
        (5000, 7321, 64, 0.6, 0.6, 3, 23),     # wrapped ring, non-pow2 max_size
        (4096, 3000, 256, 0.4, 0.5, 2, 24),    # pow2 capacity, partial fill
    ]
    for k, (max_size, n_add, B, beta, alpha, rounds, seed) in enumerate(cases):
        torch.manual_seed(seed)
        rng = np.random.default_rng(seed)
        buf = PER(max_size, alpha=alpha)
        _per_add(buf, n_add)
        rec = {"max_size": np.int64(max_size), "n_add": np.int64(n_add), "B": np.int64(B),
               "beta": np.float64(beta), "alpha": np.float64(alpha), "seed": np.int64(seed),
               "rounds": np.int64(rounds)}
        # record the uniform stream the sampler consumes (global torch CPU generator)
        for rd in range(rounds):
            state = torch.get_rng_state()
            u = torch.rand(B).numpy().copy()
            torch.set_rng_state(state)
            idxs = buf._sample_proportional(B)
            w = buf._calculate_weights(idxs, beta)
            pri = (np.abs(rng.standard_normal(B)) * (0.1 if rd == 1 else 1.0)).astype(np.float32)
            if rd == 2:
                pri[: B // 4] = 1e-9  # hits the 1e-5 floor
            buf.update_priorities(idxs.unsqueeze(1), torch.from_numpy(pri))
            extra = 7 + 3 * rd
            _per_add(buf, extra)  # interleaved inserts at max priority
            rec[f"u{rd}"] = u
            rec[f"idx{rd}"] = idxs.numpy().astype(np.int64)
            rec[f"w{rd}"] = w.numpy().astype(np.float32)
            rec[f"pri{rd}"] = pri
            rec[f"extra{rd}"] = np.int64(extra)
            rec[f"sum_tree{rd}"] = np.array(buf.sum_tree.tree)
            rec[f"min_tree{rd}"] = np.array(buf.min_tree.tree)
            rec[f"max_priority{rd}"] = np.float64(buf.max_priority)
            rec[f"tree_ptr{rd}"] = np.int64(buf.tree_ptr)
            rec[f"size{rd}"] = np.int64(buf._size)
        out[f"per{k}"] = rec


# --------------------------------------------------------------------------- #
# PPO clipped-surrogate loss                                                  #
# --------------------------------------------------------------------------- #
class _FakeTD(dict):
    def is_empty(self):
        return len(self) == 0

    def get(self, key, default=None):
        return dict.get(self, key, default)

    def __getitem__(self, key):
        if isinstance(key, str):
            return dict.__getitem__(self, key)
        idx = torch.as_tensor(np.asarray(key))
        return _FakeTD({k: v[idx] for k, v in self.items()})


def gen_ppo(ppo_mod, spaces_mod, out: dict) -> None:
    PPO = ppo_mod.PPO
    cases = [
        # (S, batch, epochs, clip, vf, ent, seed)
        (2048, 128, 4, 0.2, 0.5, 0.01, 31),  # config-2 rollout
        (300, 64, 2, 0.1, 1.0, 0.05, 32),    # short last minibatch
    ]
    for k, (S, bs, E, clip, vf, ent, seed) in enumerate(cases):
        rng = np.random.default_rng(seed)
        old_logp = rng.uniform(-3, -0.05, S).astype(np.float32)
        # per-sample "network outputs" the fake evaluate_actions returns as leaves
        new_logp = (old_logp + rng.normal(0, 0.15, S)).astype(np.float32)
        adv = (rng.standard_normal(S) * 2 + 0.3).astype(np.float32)
        ret = rng.standard_normal(S).astype(np.float32)
        old_v = rng.standard_normal(S).astype(np.float32)
        new_v = (old_v + rng.normal(0, 0.3, S)).astype(np.float32)
        H = rng.uniform(0, np.log(4), S).astype(np.float32)

        P_logp = torch.tensor(new_logp, requires_grad=True)
        P_v = torch.tensor(new_v, requires_grad=True)
        P_H = torch.tensor(H, requires_grad=True)
        snaps: list = []

        class _Opt:
            def zero_grad(self):
                for p in (P_logp, P_v, P_H):
                    p.grad = None

            def step(self):
                snaps.append((P_logp.grad.clone(), P_v.grad.clone(), P_H.grad.clone()))

        class _Net:
            def parameters(self):
                return []

        class _RB:
            def size(self):
                return S

        fake = object.__new__(PPO)
        fake.batch_size, fake.update_epochs = bs, E
        fake.clip_coef, fake.vf_coef, fake.ent_coef = clip, vf, ent
        fake.target_kl, fake.accelerator, fake.max_grad_norm = None, None, 0.5
        fake.action_space = spaces_mod.Discrete()
        fake.optimizer, fake.actor, fake.critic = _Opt(), _Net(), _Net()
        fake.rollout_buffer = _RB()

        def _eval(obs, actions, hidden_state=None, action_mask=None):
            i = obs.long().view(-1)
            return P_logp[i], P_H[i], P_v[i]

        fake.evaluate_actions = _eval
        td = _FakeTD(
            observations=torch.arange(S, dtype=torch.float32).view(S, 1),
            actions=torch.zeros(S, 1),
            log_probs=torch.tensor(old_logp),
            advantages=torch.tensor(adv),
            returns=torch.tensor(ret),
            values=torch.tensor(old_v),
        )
        np.random.seed(seed)
        perm_state = np.random.get_state()
        mean_loss = PPO._learn_from_rollout_buffer_flat(fake, buffer_td_external=td)
        # replay the permutation stream the learner consumed
        np.random.set_state(perm_state)
        perms = []
        idx = np.arange(S)
        for _ in range(E):
            np.random.shuffle(idx)
            perms.append(idx.copy())
        n_mb = len(snaps)
        out[f"ppo{k}"] = dict(
            S=np.int64(S), batch=np.int64(bs), epochs=np.int64(E), clip=np.float64(clip),
            vf=np.float64(vf), ent=np.float64(ent), seed=np.int64(seed),
            old_logp=old_logp, new_logp=new_logp, adv=adv, ret=ret, old_v=old_v,
            new_v=new_v, H=H, adv_norm=td["advantages"].numpy().copy(),
            perms=np.stack(perms).astype(np.int64), mean_loss=np.float64(mean_loss),
            g_logp=np.stack([s[0].numpy() for s in snaps]),
            g_v=np.stack([s[1].numpy() for s in snaps]),
            g_H=np.stack([s[2].numpy() for s in snaps]),
            n_minibatches=np.int64(n_mb),
        )


# --------------------------------------------------------------------------- #
# DQN TD target                                                               #
# --------------------------------------------------------------------------- #
def gen_dqn(dqn_mod, out: dict) -> None:
    DQN = dqn_mod.DQN
    for k, (B, A, double, gamma, seed) in enumerate(
        [(128, 2, False, 0.99, 41), (64, 6, True, 0.97, 42), (33, 4, False, 0.9, 43)]
    ):
        rng = np.random.default_rng(seed)
        q_next_online = rng.standard_normal((B, A)).astype(np.float32)
        q_next_target = rng.standard_normal((B, A)).astype(np.float32)
        q_cur = rng.standard_normal((B, A)).astype(np.float32)
        r = rng.standard_normal((B, 1)).astype(np.float32)
        d = (rng.random((B, 1)) < 0.2).astype(np.float32)
        a = rng.integers(0, A, (B, 1)).astype(np.int64)
        obs_tag, next_tag = torch.zeros(B, 1), torch.ones(B, 1)
        Qc = torch.tensor(q_cur, requires_grad=True)
        rec: dict = {}

        class _Actor:
            def __call__(self, x):
                return Qc if float(x[0, 0]) == 0 else torch.tensor(q_next_online)

        class _Target:
            def __call__(self, x):
                return torch.tensor(q_next_target)

        class _Crit:
            def __call__(self, q_eval, y):
                rec["q_eval"], rec["y"] = q_eval.detach().clone(), y.detach().clone()
                return torch.nn.functional.mse_loss(q_eval, y)

        class _Opt:
            def zero_grad(self):
                Qc.grad = None

            def step(self):
                rec["g_q"] = Qc.grad.clone()

        fake = object.__new__(DQN)
        fake.double, fake.gamma, fake.accelerator = double, gamma, None
        fake.actor, fake.actor_target, fake.criterion, fake.optimizer = _Actor(), _Target(), _Crit(), _Opt()
        loss = DQN.update(fake, obs_tag, torch.tensor(a), torch.tensor(r), next_tag, torch.tensor(d))
        out[f"dqn{k}"] = dict(
            double=np.int32(double), gamma=np.float64(gamma), q_next_online=q_next_online,
            q_next_target=q_next_target, q_cur=q_cur, r=r, d=d, a=a,
            y=rec["y"].numpy(), q_eval=rec["q_eval"].numpy(), loss=np.float32(loss.item()),
            g_q=rec["g_q"].numpy(),
        )


# --------------------------------------------------------------------------- #
# Rainbow C51 projection                                                      #
# --------------------------------------------------------------------------- #
def gen_c51(rainbow_mod, out: dict) -> None:
    Rainbow = rainbow_mod.RainbowDQN
    cases = [
        # (B, A, Z, vmin, vmax, gamma, seed)
        (64, 6, 51, -200.0, 200.0, 0.99**4, 51),   # config 3 (n-step gamma)
        (64, 6, 51, -100.0, 100.0, 0.99, 52),      # create_population overrides
        (40, 4, 51, 0.0, 200.0, 0.99, 53),         # class defaults
        (17, 3, 11, -10.0, 10.0, 0.9, 54),         # small support, heavy clamping
    ]
    for k, (B, A, Z, vmin, vmax, gamma, seed) in enumerate(cases):
        rng = np.random.default_rng(seed)
        support = torch.linspace(vmin, vmax, Z)
        q_next = rng.standard_normal((B, A)).astype(np.float32)
        lt = torch.tensor(rng.standard_normal((B, A, Z)).astype(np.float32) * 2)
        tdist = torch.softmax(lt, dim=-1).clamp(min=1e-3).numpy()
        lc = torch.tensor(rng.standard_normal((B, A, Z)).astype(np.float32))
        logp_cur = torch.log_softmax(lc, dim=-1).numpy()
        scale = (vmax - vmin) * 0.3
        r = (rng.standard_normal((B, 1)) * scale).astype(np.float32)
        r[:3, 0] = [vmax * 5, vmin * 5, 0.0]  # clamp both ends
        d = (rng.random((B, 1)) < 0.2).astype(np.float32)
        a = rng.integers(0, A, (B, 1)).astype(np.int64)

        class _Actor:
            def __call__(self, x, q=True, log=False):
                if float(x.reshape(-1)[0]) == 1.0:  # next obs
                    return torch.tensor(q_next)
                return torch.tensor(logp_cur)

        class _Target:
            def __call__(self, x, q=True, log=False):
                return torch.tensor(tdist)

        fake = object.__new__(Rainbow)
        fake.actor, fake.actor_target = _Actor(), _Target()
        fake.batch_size, fake.num_atoms, fake.support = B, Z, support
        fake.v_min, fake.v_max = vmin, vmax
        fake.delta_z = (vmax - vmin) / (Z - 1)
        fake.device = "cpu"
        fake.preprocess_observation = lambda o: o
        loss = Rainbow._dqn_loss(
            fake, torch.zeros(B, 1), torch.tensor(a), torch.tensor(r), torch.ones(B, 1),
            torch.tensor(d), gamma,
        )
        out[f"c51_{k}"] = dict(
            B=np.int64(B), A=np.int64(A), Z=np.int64(Z), vmin=np.float64(vmin),
            vmax=np.float64(vmax), gamma=np.float64(gamma), support=support.numpy(),
            q_next=q_next, target_dist=tdist, logp_cur=logp_cur, r=r, d=d, a=a,
            loss=loss.numpy(),
        )


# --------------------------------------------------------------------------- #
# tournament selection                                                        #
# --------------------------------------------------------------------------- #
def gen_tournament(tour_mod, out: dict) -> None:
    TS = tour_mod.TournamentSelection

    class _Agent:
        def __init__(self, index, fitness):
            self.index, self.fitness, self.parent = index, fitness, index

        def clone(self, index=None, wrap=True):
            c = _Agent(self.index if index is None else index, list(self.fitness))
            c.parent = self.index
            return c

    for k, (P, tsize, elitism, eval_loop, seed) in enumerate(
        [(8, 2, True, 1, 61), (8, 3, False, 2, 62), (32, 2, True, 3, 63), (5, 4, True, 1, 64)]
    ):
        rng = np.random.default_rng(seed)
        fit = rng.standard_normal((P, 4)) * 50
        fit[1] = fit[0]  # a tie
        pop = [_Agent(i + 10 * k, list(fit[i])) for i in range(P)]
        ts = TS(tsize, elitism, P, eval_loop)
        ts.language_model = False
        np.random.seed(seed)
        elite, new_pop = ts.select(pop)
        out[f"tour{k}"] = dict(
            P=np.int64(P), tsize=np.int64(tsize), elitism=np.int32(elitism),
            eval_loop=np.int64(eval_loop), seed=np.int64(seed), fitness=fit,
            indices=np.array([a.index for a in pop], dtype=np.int64),
            elite_parent=np.int64(elite.parent),
            parents=np.array([a.parent for a in new_pop], dtype=np.int64),
            new_indices=np.array([a.index for a in new_pop], dtype=np.int64),
        )


# --------------------------------------------------------------------------- #
# PPO learn() end to end                                                      #
# --------------------------------------------------------------------------- #
def _flat_names(mods: dict) -> dict:
    """reference state-dict names -> tensors for the shared-encoder PPO:
    actor.encoder.model.*, actor.head_net.model.*, critic.head_net.model.*"""
    out = {}
    for pre, m in mods.items():
        for k, t in m.state_dict().items():
            out[pre + k] = t.detach().clone().numpy()
    return out


def gen_ppo_learn(ppo_mod, en_mod, tu_mod, dist_mod, spaces_mod, out: dict) -> None:
    """The reference's _learn_from_rollout_buffer_flat on a real network: the
    encoder / heads are the reference's create_mlp modules (encoder:
    output_layernorm, ReLU output; heads: output_vanish), evaluate_actions is
    the shared-encoder forward of ppo.py:487-491 with log_prob_discrete /
    entropy_discrete and apply_action_mask_discrete, and the optimizer is
    torch.optim.Adam over actor + critic parameters (what OptimizerWrapper
    builds).  Everything after evaluate_actions is the reference's own loop."""
    PPO = ppo_mod.PPO
    create_mlp = en_mod.create_mlp
    cases = [
        # (name, T, N, obs, A, enc, latent, actor, critic, batch, epochs, target_kl, masks, lr, seed)
        ("learn0", 16, 128, 8, 4, [64], 64, [64], [64], 128, 4, None, False, 1e-3, 71),  # config 2
        ("learn1", 15, 20, 4, 2, [64], 64, [64], [16], 64, 3, 0.004, True, 3e-3, 72),    # KL stop + masks
        ("learn2", 16, 128, 8, 4, [64], 64, [64], [64], 128, 4, None, False, 1e-3, 73),  # Adam step > 0
    ]
    carry = None
    for (name, T, N, D, A, enc, lat, ah, ch, bs, E, tkl, use_masks, lr, seed) in cases:
        torch.manual_seed(seed)
        encoder = create_mlp(D, lat, enc, output_vanish=False, output_activation="ReLU", layer_norm=True,
                             output_layernorm=True, name="encoder")
        actor_head = create_mlp(lat, A, ah, output_vanish=True, output_activation=None, layer_norm=True,
                                name="actor")
        critic_head = create_mlp(lat, 1, ch, output_vanish=True, output_activation=None, layer_norm=True,
                                 name="value")
        mods = {"actor.encoder.model.": encoder, "actor.head_net.model.": actor_head,
                "critic.head_net.model.": critic_head}
        if name == "learn2":  # continue learn0's agent (parameters + Adam state)
            with torch.no_grad():
                for pre, m in mods.items():
                    for k, t in m.state_dict().items():
                        t.copy_(torch.as_tensor(carry["state"][pre + k]))
        params = [p for m in mods.values() for p in m.parameters()]
        opt = torch.optim.Adam(params, lr=lr)
        if name == "learn2":
            names = [pre + k for pre, m in mods.items() for k, _ in m.named_parameters()]
            for n_, p_ in zip(names, params):
                opt.state[p_] = {"step": torch.tensor(float(carry["step"])),
                                 "exp_avg": torch.as_tensor(carry["exp_avg"][n_]).clone(),
                                 "exp_avg_sq": torch.as_tensor(carry["exp_avg_sq"][n_]).clone()}
        init = _flat_names(mods)
        rng = np.random.default_rng(seed)
        S = T * N
        obs = rng.standard_normal((S, D)).astype(np.float32)
        masks = None
        if use_masks:
            masks = rng.random((S, A)) < 0.7
            masks[np.arange(S), rng.integers(0, A, S)] = True  # at least one legal action
        with torch.no_grad():
            lat_t = encoder(torch.tensor(obs))
            logits = actor_head(lat_t)
            if masks is not None:
                logits = dist_mod.apply_action_mask_discrete(logits, torch.tensor(masks))
            probs = torch.softmax(logits, -1).numpy().astype(np.float64)
            probs /= probs.sum(1, keepdims=True)
            act = np.array([rng.choice(A, p=p) for p in probs], dtype=np.int64)
            old_logp = tu_mod.log_prob_discrete(logits, torch.tensor(act)).numpy()
            old_v = critic_head(lat_t).squeeze(-1).numpy()
        old_logp = (old_logp + rng.normal(0, 0.02, S)).astype(np.float32)
        old_v = (old_v + rng.normal(0, 0.1, S)).astype(np.float32)
        adv = (rng.standard_normal(S) * 1.5 + 0.2).astype(np.float32)
        ret = (old_v + rng.standard_normal(S)).astype(np.float32)

        class _Net:
            def __init__(self, ms):
                self.ms = ms

            def parameters(self):
                return [p for m in self.ms for p in m.parameters()]

        class _RB:
            def size(self):
                return S

        fake = object.__new__(PPO)
        fake.batch_size, fake.update_epochs = bs, E
        fake.clip_coef, fake.vf_coef, fake.ent_coef = 0.2, 0.5, 0.01
        fake.target_kl, fake.accelerator, fake.max_grad_norm = tkl, None, 0.5
        fake.action_space = spaces_mod.Discrete()
        fake.optimizer = opt
        fake.actor, fake.critic = _Net([encoder, actor_head]), _Net([critic_head])
        fake.rollout_buffer = _RB()
        kls_seen: list = []

        def _eval(obs, actions, hidden_state=None, action_mask=None):
            lat_ = encoder(obs)
            lg = actor_head(lat_)
            if action_mask is not None:
                lg = dist_mod.apply_action_mask_discrete(lg, action_mask)
            lp = tu_mod.log_prob_discrete(lg, actions)
            ent = tu_mod.entropy_discrete(lg)
            return lp, ent, critic_head(lat_).squeeze(-1)

        fake.evaluate_actions = _eval
        td = dict(observations=torch.tensor(obs), actions=torch.tensor(act).view(S, 1).float(),
                  log_probs=torch.tensor(old_logp), advantages=torch.tensor(adv), returns=torch.tensor(ret),
                  values=torch.tensor(old_v))
        if masks is not None:
            td["action_masks"] = torch.tensor(masks)
        td = _FakeTD(td)
        np.random.seed(seed)
        perm_state = np.random.get_state()
        mean_loss = PPO._learn_from_rollout_buffer_flat(fake, buffer_td_external=td)
        # replay the permutation stream the learner consumed (all E epochs drawn;
        # an early stop uses a prefix)
        np.random.set_state(perm_state)
        perms = []
        idx = np.arange(S)
        for _ in range(E):
            np.random.shuffle(idx)
            perms.append(idx.copy())
        final = _flat_names(mods)
        names = [pre + k for pre, m in mods.items() for k, _ in m.named_parameters()]
        m_out = {n_: opt.state[p_]["exp_avg"].numpy().copy() for n_, p_ in zip(names, params)}
        v_out = {n_: opt.state[p_]["exp_avg_sq"].numpy().copy() for n_, p_ in zip(names, params)}
        step = int(opt.state[params[0]]["step"])
        n_mb = -(-S // bs)
        rec = dict(T=np.int64(T), N=np.int64(N), obs_dim=np.int64(D), n_actions=np.int64(A),
                   enc=np.array(enc, np.int64), latent=np.int64(lat), actor_hidden=np.array(ah, np.int64),
                   critic_hidden=np.array(ch, np.int64), batch=np.int64(bs), epochs=np.int64(E),
                   target_kl=np.float64(-1.0 if tkl is None else tkl), lr=np.float64(lr), seed=np.int64(seed),
                   clip=np.float64(0.2), vf=np.float64(0.5), ent=np.float64(0.01), max_norm=np.float64(0.5),
                   obs=obs, actions=act, old_logp=old_logp, old_v=old_v, adv=adv, ret=ret,
                   perms=np.stack(perms).astype(np.int64), mean_loss=np.float64(mean_loss),
                   step_in=np.int64(0 if carry is None or name != "learn2" else carry["step"]),
                   step_out=np.int64(step), epochs_run=np.int64(step - (0 if name != "learn2" else carry["step"]))
                   // n_mb)
        if masks is not None:
            rec["masks"] = masks.astype(np.uint8)
        for n_, a_ in init.items():
            rec["init." + n_] = a_
            if name == "learn2":
                rec["init_m." + n_] = carry["exp_avg"].get(n_, np.zeros_like(a_))
                rec["init_v." + n_] = carry["exp_avg_sq"].get(n_, np.zeros_like(a_))
        for n_, a_ in final.items():
            rec["final." + n_] = a_
        for n_ in names:
            rec["m." + n_] = m_out[n_]
            rec["v." + n_] = v_out[n_]
        out[name] = rec
        if name == "learn0":
            carry = dict(state=final, exp_avg=m_out, exp_avg_sq=v_out, step=step)


# --------------------------------------------------------------------------- #
# n-step fold, multi-agent replay sampling, MADDPG critic target              #
# --------------------------------------------------------------------------- #
class _CloneTD(dict):
    def clone(self):
        return _CloneTD({k: v.clone() for k, v in self.items()})


def gen_nstep(rp_mod, out: dict) -> None:
    """MultiStepReplayBuffer._get_n_step_info on batched transitions (the
    reference's vectorised add: one TensorDict per env step)."""
    import collections

    MSB = rp_mod.MultiStepReplayBuffer
    cases = [
        # (n_step, num_envs, obs_dim, p_done, gamma, seed, done key)
        (3, 4, 3, 0.0, 0.99, 81, "done"),
        (4, 5, 2, 0.3, 0.99, 82, "done"),         # some env done -> early stop (any)
        (4, 16, 4, 0.05, 0.9, 83, "terminated"),
        (2, 1, 1, 0.5, 0.97, 84, "termination"),
    ]
    for k, (n, B, D, pd, gamma, seed, dkey) in enumerate(cases):
        rng = np.random.default_rng(seed)
        trs = []
        for _ in range(n):
            trs.append(_CloneTD(obs=torch.tensor(rng.standard_normal((B, D)), dtype=torch.float32),
                                reward=torch.tensor(rng.standard_normal((B, 1)) * 3, dtype=torch.float32),
                                next_obs=torch.tensor(rng.standard_normal((B, D)), dtype=torch.float32),
                                **{dkey: torch.tensor(rng.random((B, 1)) < pd, dtype=torch.float32)}))
        buf = object.__new__(MSB)
        buf.n_step, buf.gamma = n, gamma
        buf.n_step_buffer = collections.deque(trs, maxlen=n)
        buf.reward_key, buf.ns_key, buf.done_key = "reward", "next_obs", None
        buf.initialized = False
        res = buf._get_n_step_info()
        rec = dict(n_step=np.int64(n), gamma=np.float64(gamma), done_key=np.array(dkey))
        for i, t in enumerate(trs):
            for f, v in t.items():
                rec[f"in{i}.{'done' if f == dkey else f}"] = v.numpy()
        for f, v in res.items():
            rec[f"out.{'done' if f == dkey else f}"] = v.numpy()
        out[f"nstep{k}"] = rec


def gen_ma_replay(mar_mod, out: dict) -> None:
    """MultiAgentReplayBuffer: vectorised saves (ring wrap-around, binary
    fields with and without NaN), then random.seed + sample.  obs_to_tensor
    (agilerl/utils/algo_utils.py:746-773, an np.ndarray -> torch.as_tensor(
    ...).float()) is the only helper the sample path calls."""
    import random

    mar_mod.obs_to_tensor = lambda obs, device: torch.as_tensor(obs, device=device).float()
    MAR = mar_mod.MultiAgentReplayBuffer
    fields = ["obs", "action", "reward", "next_obs", "done"]
    agents = ["speaker_0", "listener_0"]
    dims = {"speaker_0": (3, 3), "listener_0": (11, 5)}
    for k, (mem, steps, n_envs, batch, seed) in enumerate([(50, 23, 4, 16, 3), (1000, 40, 8, 64, 4)]):
        rng = np.random.default_rng(seed)
        buf = MAR(mem, fields, agents, device="cpu")
        rec = dict(memory_size=np.int64(mem), steps=np.int64(steps), n_envs=np.int64(n_envs),
                   batch=np.int64(batch), seed=np.int64(seed))
        for t in range(steps):
            nan = t == steps - 1
            obs = {a: rng.standard_normal((n_envs, dims[a][0])).astype(np.float32) for a in agents}
            act = {a: rng.random((n_envs, dims[a][1])).astype(np.float32) for a in agents}
            rew = {a: rng.standard_normal(n_envs).astype(np.float32) for a in agents}
            nxt = {a: rng.standard_normal((n_envs, dims[a][0])).astype(np.float32) for a in agents}
            done = {a: (rng.random(n_envs) < 0.3) for a in agents}
            if nan:
                rew["listener_0"][0] = np.nan
                done["listener_0"] = done["listener_0"].astype(np.float32)
                done["listener_0"][0] = np.nan
            for f, d in zip(fields, (obs, act, rew, nxt, done)):
                for a in agents:
                    rec[f"save{t}.{f}.{a}"] = np.asarray(d[a])
            buf.save_to_memory(obs, act, rew, nxt, done, is_vectorised=True)
        for s in range(3):
            random.seed(100 * seed + s)
            sample = buf.sample(batch)
            for f, per in zip(fields, sample):
                for a in agents:
                    rec[f"sample{s}.{f}.{a}"] = per[a].numpy()
        out[f"marep{k}"] = rec


def gen_maddpg(maddpg_mod, out: dict) -> None:
    """MADDPG._learn_individual with stand-in critic / target / actor: the
    critic TD target y = r + (1 - d) * gamma * Q'(s', a') after the NaN rules
    (reward NaN -> 0, done NaN -> 1 then uint8), the MSE critic loss and its
    gradient dL/dQ (captured at the critic optimizer step)."""
    MADDPG = maddpg_mod.MADDPG
    for k, (B, gamma, seed) in enumerate([(64, 0.95, 91), (33, 0.99, 92), (1024, 0.9, 93)]):
        rng = np.random.default_rng(seed)
        q = rng.standard_normal((B, 1)).astype(np.float32)
        qn = rng.standard_normal((B, 1)).astype(np.float32)
        r = rng.standard_normal((B, 1)).astype(np.float32)
        d = (rng.random((B, 1)) < 0.2).astype(np.float32)
        r[rng.random(B) < 0.05] = np.nan
        d[rng.random(B) < 0.05] = np.nan
        Q = torch.tensor(q, requires_grad=True)
        rec: dict = {}

        class _Critic:
            def __call__(self, states, actions):
                return Q

        class _Target:
            def __call__(self, states, actions):
                return torch.tensor(qn)

        class _Actor:
            def __call__(self, x):
                return torch.zeros(B, 2)

        class _COpt:
            def zero_grad(self):
                Q.grad = None

            def step(self):
                rec["g_q"] = Q.grad.clone()

        class _AOpt:
            def zero_grad(self):
                pass

            def step(self):
                pass

        class _Crit:
            def __call__(self, q_eval, y):
                rec["y"] = y.detach().clone()
                return torch.nn.functional.mse_loss(q_eval, y)

        fake = object.__new__(MADDPG)
        fake.gamma, fake.accelerator, fake.agent_ids = gamma, None, ["a0"]
        fake.get_network_id = lambda agent_id: agent_id
        fake.actors, fake.critics, fake.critic_targets = {"a0": _Actor()}, {"a0": _Critic()}, {"a0": _Target()}
        fake.actor_optimizers, fake.critic_optimizers = {"a0": _AOpt()}, {"a0": _COpt()}
        fake.criterion = _Crit()
        _, closs = MADDPG._learn_individual(fake, "a0", torch.zeros(B, 2), torch.zeros(B, 2), {"a0": torch.zeros(B, 1)},
                                            {"a0": torch.zeros(B, 1)}, {"a0": torch.zeros(B, 2)},
                                            {"a0": torch.tensor(r)}, {"a0": torch.tensor(d)})
        out[f"maddpg{k}"] = dict(gamma=np.float64(gamma), q=q, q_next=qn, r=r, d=d, y=rec["y"].numpy(),
                                 critic_loss=np.float64(closs), g_q=rec["g_q"].numpy())


# --------------------------------------------------------------------------- #
# HPO mutations                                                               #
# --------------------------------------------------------------------------- #
class _MutNet(torch.nn.Module):
    """A policy with the reference's actor state-dict names (encoder.model.*,
    head_net.model.*) whose 2-D weights parameter_mutation perturbs."""

    def __init__(self, D, A, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        enc = torch.nn.Sequential()
        enc.add_module("encoder_linear_layer_1", torch.nn.Linear(D, 64))
        enc.add_module("encoder_layer_norm_1", torch.nn.LayerNorm(64))
        enc.add_module("encoder_linear_layer_output", torch.nn.Linear(64, 64))
        head = torch.nn.Sequential()
        head.add_module("actor_linear_layer_1", torch.nn.Linear(64, 64))
        head.add_module("actor_layer_norm_1", torch.nn.LayerNorm(64))
        head.add_module("actor_linear_layer_output", torch.nn.Linear(64, A))
        self.encoder, self.head_net = torch.nn.Module(), torch.nn.Module()
        self.encoder.model, self.head_net.model = enc, head
        with torch.no_grad():
            for p_ in self.parameters():
                p_.copy_(torch.randn(p_.shape, generator=g) * 0.3)


def gen_mutation(mut_mod, reg_mod, out: dict) -> None:
    """Mutations.mutation over a small fake population for several
    generations: the choices drawn, the RL-hyperparameter values (shared
    HyperparameterConfig, torch-drawn sample / grow-or-shrink), and the
    parameter-mutated policy weights."""
    RLParameter, HPC = reg_mod.RLParameter, reg_mod.HyperparameterConfig
    cases = [
        # (P, no, arch, params, act, rl_hp, mutate_elite, seed, generations)
        (4, 0.4, 0.0, 0.2, 0.0, 0.2, True, 42, 6),    # ppo.yaml-like (architecture / activation off)
        (8, 0.0, 0.0, 0.5, 0.0, 0.5, False, 7, 5),    # no elite mutation
    ]
    for k, (P, no, arch, par, act, rlhp, mut_elite, seed, G) in enumerate(cases):
        hp = HPC(lr=RLParameter(min=1e-4, max=1e-2), batch_size=RLParameter(min=8, max=1024, dtype=int),
                 ent_coef=RLParameter(min=0.001, max=0.1), update_epochs=RLParameter(min=1, max=10, dtype=int))

        class _OptCfg:
            lr = "lr"

        class _Registry:
            def __init__(self):
                self.hp_config = hp  # shared, as create_population hands it to every agent
                self.optimizers = [_OptCfg()]
                self.groups = []

            def policy(self, return_group=False):
                grp = types.SimpleNamespace(eval_network="actor", shared_networks=None)
                return grp if return_group else "actor"

        class _Agent:
            def __init__(self, i):
                self.index, self.lr, self.batch_size, self.ent_coef, self.update_epochs = i, 1e-3, 128, 0.01, 4
                self.registry = _Registry()
                self.actor = _MutNet(8, 4, 1000 * k + i)
                self.mut, self.reinits = None, 0

            def get_lr_names(self):
                return ["lr"]

            def reinit_optimizers(self, optimizer=None):
                self.reinits += 1

            def mutation_hook(self):
                pass

        pop = [_Agent(i) for i in range(P)]
        init_w = {f"a{i}.{n}": t.detach().clone().numpy() for i, a in enumerate(pop)
                  for n, t in a.actor.state_dict().items()}
        m = mut_mod.Mutations(no_mutation=no, architecture=arch, new_layer_prob=0.2, parameters=par,
                              activation=act, rl_hp=rlhp, mutation_sd=0.1, mutate_elite=mut_elite,
                              rand_seed=seed, device="cpu")
        muts, hps = [], []
        for _ in range(G):
            pop = m.mutation(pop)
            muts.append([str(a.mut) for a in pop])
            hps.append([[a.lr, a.batch_size, a.ent_coef, a.update_epochs, a.reinits] for a in pop])
        rec = dict(P=np.int64(P), probs=np.array([no, arch, par, act, rlhp], np.float64),
                   mutate_elite=np.int32(mut_elite), seed=np.int64(seed), generations=np.int64(G),
                   muts=np.array(muts), hps=np.array(hps, np.float64))
        for n, v in init_w.items():
            rec["init." + n] = v
        for i, a in enumerate(pop):
            for n, t in a.actor.state_dict().items():
                rec[f"final.a{i}.{n}"] = t.detach().numpy().copy()
        out[f"mut{k}"] = rec


# --------------------------------------------------------------------------- #
def gen_dueling(ref: str, en, out: dict) -> None:
    """NoisyLinear (agilerl/modules/custom_components.py:38-131) and the
    DuelingDistributionalMLP head forward (agilerl/networks/custom_modules.py:
    127-162) on noisy create_mlp streams (utils/evolvable_networks.py:527-644),
    run by the reference's own code: seeded construction (parameter / noise
    draw order), train / eval forwards, a re-drawn noise sample, and the head's
    q / probability / log-probability outputs."""
    cc = _load(ref, "agilerl.modules.custom_components", "agilerl/modules/custom_components.py")
    for name in ("NoisyLinear", "GumbelSoftmax", "NewGELU"):  # evolvable_networks bound the stubs at import
        if hasattr(cc, name):
            setattr(en, name, getattr(cc, name))
    _stub("agilerl.modules.mlp")
    cm = _load(ref, "agilerl.networks.custom_modules", "agilerl/networks/custom_modules.py")
    # NoisyLinear alone
    torch.manual_seed(5)
    nl = cc.NoisyLinear(12, 7, std_init=0.4)
    init = {k: v.detach().clone().numpy() for k, v in nl.state_dict().items()}
    x = torch.randn(9, 12)
    y_train = nl(x).detach().numpy()
    nl.eval()
    y_eval = nl(x).detach().numpy()
    nl.train()
    torch.manual_seed(9)
    nl.reset_noise()
    out["noisy0"] = dict(x=x.numpy(), y_train=y_train, y_eval=y_eval, w_eps2=nl.weight_epsilon.numpy().copy(),
                         b_eps2=nl.bias_epsilon.numpy().copy(),
                         **{f"init.{k}": v for k, v in init.items()})
    # the dueling distributional head (Rainbow's q_networks.py:208-230 head: noisy, LayerNorm, vanish)
    for k, (L, H, A, Z, vmin, vmax, seed) in enumerate([(32, [16], 6, 51, -10.0, 10.0, 21),
                                                         (20, [24, 24], 3, 11, -200.0, 200.0, 22)]):
        torch.manual_seed(seed)
        kw = dict(input_size=L, hidden_size=list(H), output_vanish=True, output_activation=None, noisy=True,
                  init_layers=False, layer_norm=True, activation="ReLU", noise_std=0.5)
        value = en.create_mlp(output_size=Z, name="value", **kw)
        adv = en.create_mlp(output_size=A * Z, name="advantage", **kw)
        head = object.__new__(cm.DuelingDistributionalMLP)
        head.model, head.advantage_net = value, adv
        head.num_atoms, head.num_actions = Z, A
        head.support = torch.linspace(vmin, vmax, Z)
        x = torch.randn(13, L)
        fwd = cm.DuelingDistributionalMLP.forward
        rec = dict(x=x.numpy(), support=head.support.numpy(), dims=np.array([L, A, Z], np.int64),
                   hidden=np.array(H, np.int64),
                   q=fwd(head, x).detach().numpy(), probs=fwd(head, x, q=False).detach().numpy(),
                   logp=fwd(head, x, log=True).detach().numpy())
        for pre, m in (("model.", value), ("advantage_net.", adv)):
            for kk, v in m.state_dict().items():
                rec[f"sd.{pre}{kk}"] = v.detach().clone().numpy()
        out[f"dueling{k}"] = rec


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", nargs="*", default=None, help="write only these fixture groups")
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(args.ref, "agilerl")):
        print("reference checkout not present; nothing generated")
        return
    torch.set_num_threads(1)
    _install_stubs()
    ref = args.ref
    st = _load(ref, "agilerl.components.segment_tree", "agilerl/components/segment_tree.py")
    rp = _load(ref, "agilerl.components.replay_buffer", "agilerl/components/replay_buffer.py")
    rb = _load(ref, "agilerl.components.rollout_buffer", "agilerl/components/rollout_buffer.py")
    ppo = _load(ref, "agilerl.algorithms.ppo", "agilerl/algorithms/ppo.py")
    dqn = _load(ref, "agilerl.algorithms.dqn", "agilerl/algorithms/dqn.py")
    rainbow = _load(ref, "agilerl.algorithms.dqn_rainbow", "agilerl/algorithms/dqn_rainbow.py")
    tour = _load(ref, "agilerl.hpo.tournament", "agilerl/hpo/tournament.py")
    tu = _load(ref, "agilerl.utils.torch_utils", "agilerl/utils/torch_utils.py")
    en = _load(ref, "agilerl.utils.evolvable_networks", "agilerl/utils/evolvable_networks.py")
    dist_mod = _load(ref, "agilerl.networks.distributions", "agilerl/networks/distributions.py")
    reg = _load(ref, "agilerl.algorithms.core.registry", "agilerl/algorithms/core/registry.py")
    mut = _load(ref, "agilerl.hpo.mutation", "agilerl/hpo/mutation.py")
    mar = _load(ref, "agilerl.components.multi_agent_replay_buffer",
                "agilerl/components/multi_agent_replay_buffer.py")
    maddpg = _load(ref, "agilerl.algorithms.maddpg", "agilerl/algorithms/maddpg.py")

    groups: dict[str, dict] = {}
    gen_gae(rb, groups)
    gen_segment_tree(st, groups)
    gen_per(rp, groups)
    gen_ppo(ppo, sys.modules["gymnasium.spaces"], groups)
    gen_dqn(dqn, groups)
    gen_c51(rainbow, groups)
    gen_tournament(tour, groups)
    gen_ppo_learn(ppo, en, tu, dist_mod, sys.modules["gymnasium.spaces"], groups)
    gen_mutation(mut, reg, groups)
    gen_nstep(rp, groups)
    gen_ma_replay(mar, groups)
    gen_maddpg(maddpg, groups)
    gen_dueling(ref, en, groups)

    if args.only:
        groups = {k: v for k, v in groups.items() if k in set(args.only)}
        old = json.load(open(os.path.join(HERE, "META.json")))
        groups_all = sorted(set(old.get("groups", [])) | set(groups))
    else:
        groups_all = sorted(groups)
    prev = json.load(open(os.path.join(HERE, "META.json"))) if os.path.exists(os.path.join(HERE, "META.json")) else {}
    meta = {
        **{k: v for k, v in prev.items() if k == "arch_fixtures"},  # gen_arch_golden.py's record
        "generator": "tests/golden/gen_golden.py",
        "torch": torch.__version__,
        "numpy": np.__version__,
        "python": sys.version.split()[0],
        "reference_pins": {"torch": "2.9.0 (pyproject.toml:34)", "numpy": ">=2 (pyproject.toml:22)"},
        "groups": groups_all,
    }
    for name, rec in groups.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    with open(os.path.join(HERE, "META.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(groups), "fixtures")


if __name__ == "__main__":
    main()
