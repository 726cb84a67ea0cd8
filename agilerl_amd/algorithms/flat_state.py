"""One agent's learner state in flat device buffers, for the per-agent DQN /
RainbowDQN ``learn`` (dqn.py:326-358, dqn_rainbow.py:369-501).

The reference ends every update with clip_grad_norm_ over the actor's
parameters (Rainbow: 10.0), torch.optim.Adam, and a Polyak soft update that
walks the parameter tensors one by one.  On the GPU each of those is a
string of small launches per parameter tensor (28 tensors for the config-3
network), and the per-agent update is bound by launch overhead, not by the
GPU.  Here the agent's online parameters, target parameters, gradients and
Adam moments live in flat ``[n]`` buffers, with the modules' parameters and
the optimizer's state tensors as views of them, so the tail of the update is
one gradient gather, one agx_clip_adam (norm clip fused with Adam, the same
kernel as the population learner) and one agx_polyak over the whole network.

The torch optimizer stays the source of truth for everything outside
``learn``: its ``exp_avg`` / ``exp_avg_sq`` are the flat moments' views and
every parameter's ``step`` tensor is advanced per update (one foreach add), so
state_dict / checkpoints / clones read current values (and a torch
optimizer step taken outside ``learn`` updates the same views; the device
step count follows it).  Anything that
replaces the modules, the optimizer or its state (mutation, clone, checkpoint
load) invalidates the flat state; the next ``learn`` adopts the new tensors
(current values copied in)."""

from __future__ import annotations

import torch

from .. import _lib


def _plain_adam(opt) -> bool:
    if not isinstance(opt, torch.optim.Adam) or len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    # fused Adam keeps its 'step' tensors on the device; the flat state swaps
    # in CPU step tensors, which a later torch step would then mix with device ones
    return not (g.get("amsgrad") or g.get("maximize") or g.get("weight_decay", 0.0) or g.get("capturable")
                or g.get("differentiable") or g.get("fused"))


class FlatLearnState:
    """Flat online / target / gradient / Adam buffers of one agent."""

    def __init__(self, actor, target, opt):
        self.actor, self.target, self.opt = actor, target, opt
        self.params = list(actor.parameters())
        self.tparams = list(target.parameters())
        if len(self.params) != len(self.tparams) or any(p.shape != q.shape for p, q in
                                                        zip(self.params, self.tparams)):
            raise ValueError("flat learner state: online and target networks differ in shape")
        dev = self.params[0].device
        sizes = [p.numel() for p in self.params]
        self.n = n = sum(sizes)
        # online and target parameters as the two rows of one [2, n] buffer: a
        # tensor's online and target copies sit n elements apart, so the
        # no-grad forwards on s' take both networks in one grouped launch
        # (pair_view, dqn.py)
        self.pair = torch.empty(2, n, dtype=torch.float32, device=dev)
        self.prm, self.tgt = self.pair[0], self.pair[1]
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        step = 0
        for p in self.params:
            st = opt.state.get(p)
            if st and "step" in st:
                step = int(st["step"])
                break
        self.step_ts = [torch.tensor(float(step)) for _ in self.params]  # the torch Adam "step" of each
        self.host_step = step
        self.steps = torch.full((1,), step, dtype=torch.int64, device=dev)
        off = 0
        with torch.no_grad():
            for p, q, k, st_t in zip(self.params, self.tparams, sizes, self.step_ts):
                shape = p.shape
                v = self.prm[off:off + k].view(shape)
                v.copy_(p.data)
                p.data = v
                tv = self.tgt[off:off + k].view(shape)
                tv.copy_(q.data)
                q.data = tv
                st = opt.state.get(p) or {}
                mv, vv = self.m[off:off + k].view(shape), self.v[off:off + k].view(shape)
                if "exp_avg" in st:
                    mv.copy_(st["exp_avg"])
                    vv.copy_(st["exp_avg_sq"])
                opt.state[p] = {"step": st_t, "exp_avg": mv, "exp_avg_sq": vv}
                off += k
        self.offs = {}
        off = 0
        for p, k in zip(self.params, sizes):
            self.offs[id(p)] = (off, k)
            off += k
        self.ptrs = [p.data_ptr() for p in self.params]
        self.tptrs = [q.data_ptr() for q in self.tparams]
        self.mptrs = [opt.state[p]["exp_avg"].data_ptr() for p in self.params]
        self.lr = float(opt.param_groups[0]["lr"])
        self.lr_dev = torch.full((1,), self.lr, dtype=torch.float32, device=dev)
        self.offsets = torch.tensor([0, n], dtype=torch.int64)
        lib = _lib.load()
        self.workspace = torch.empty(max(16, lib.agx_adam_workspace_bytes(1, n)), dtype=torch.uint8, device=dev)

    def pair_view(self, p: torch.Tensor) -> torch.Tensor:
        """[2, *p.shape]: online parameter p and its target copy, one view."""
        off, k = self.offs[id(p)]
        return self.pair[:, off:off + k].view(2, *p.shape)

    def valid(self, actor, target, opt) -> bool:
        if actor is not self.actor or target is not self.target or opt is not self.opt or not _plain_adam(opt):
            return False
        ps = list(actor.parameters())
        if len(ps) != len(self.params):
            return False
        state = opt.state
        for p, q, ptr, mptr, st_t in zip(ps, self.params, self.ptrs, self.mptrs, self.step_ts):
            if p is not q or p.data_ptr() != ptr:
                return False
            st = state.get(p)
            if st is None or st.get("step") is not st_t or st["exp_avg"].data_ptr() != mptr:
                return False
        return all(q.data_ptr() == ptr for q, ptr in zip(target.parameters(), self.tptrs))

    def step(self, max_norm: float) -> bool:
        """Gather the gradients, clip (max_norm > 0) + Adam in one launch.
        The clipped gradients stay in the flat buffer; ``.grad`` keeps the
        unclipped ones, which nothing reads before the next zero_grad.
        False (nothing done) when a parameter has no gradient: torch's Adam
        skips such a parameter, so the caller steps the torch optimizer."""
        if any(p.grad is None for p in self.params):
            return False
        self.sync()
        self.launch(max_norm)
        self.advance()
        return True

    # step() in three parts, for a captured update (learn_graph.py): the host
    # bookkeeping runs around every replay, only launch() is in the graph
    def sync(self) -> None:
        """Host -> device: a mutated learning rate, and the Adam step count when
        the torch optimizer stepped these parameters itself."""
        g = self.opt.param_groups[0]
        lr = float(g["lr"])
        if lr != self.lr:
            self.lr = lr
            self.lr_dev.fill_(lr)
        t = int(self.step_ts[0])
        if t != self.host_step:  # the torch optimizer stepped these parameters itself
            self.steps.fill_(t)
            self.host_step = t

    def launch(self, max_norm: float) -> None:
        """The device work: gradient gather + agx_clip_adam (its step count and
        learning rate read from device memory)."""
        torch.cat([p.grad.reshape(-1) for p in self.params], out=self.grad)
        g = self.opt.param_groups[0]
        b1, b2 = g["betas"]
        _lib.call("agx_clip_adam", self.prm.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                  1, self.n, self.offsets.data_ptr(), 1, float(max_norm), self.lr_dev.data_ptr(), float(b1),
                  float(b2), float(g["eps"]), self.steps.data_ptr(), None, self.workspace.data_ptr(), _lib.stream())

    def advance(self) -> None:
        """The torch optimizer's step tensors follow the device count."""
        torch._foreach_add_(self.step_ts, 1.0)
        self.host_step += 1

    def polyak(self, tau: float) -> None:
        _lib.call("agx_polyak", self.tgt.data_ptr(), self.prm.data_ptr(), self.n, float(tau), _lib.stream())


def flat_state(agent) -> FlatLearnState | None:
    """The agent's valid flat state (adopting its current tensors when the
    modules / optimizer changed), or None where it does not apply (CPU, an
    optimizer other than plain single-group Adam)."""
    actor, target, opt = agent.actor, agent.actor_target, agent.optimizer
    if agent.device.type != "cuda" or not _plain_adam(opt):
        return None
    # rows of a live RainbowPopulationLearner: it owns the tensors (a learner
    # that was released, or tensors the agent has since replaced, do not count)
    owned = agent.__dict__.get("_pop_rows")
    if owned is not None:
        learner, ptrs = owned[0](), owned[1]
        if learner is not None and tuple(p.data_ptr() for p in actor.parameters()) == ptrs:
            return None
        agent.__dict__.pop("_pop_rows", None)
    fs = agent.__dict__.get("_flat")
    if fs is not None and fs.valid(actor, target, opt):
        return fs
    fs = FlatLearnState(actor, target, opt)
    agent.__dict__["_flat"] = fs
    return fs
