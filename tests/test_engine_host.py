"""Host logic of the population engine's multi-group training loop (CPU, no
GPU): PopulationEngine._train_paced_together with stand-in runners whose
launches start after a number of polls.  Every group runs all its
iterations in order, each rollout's steps are released before they are
waited for, a launch that has not started is never waited for, and an
exception releases every in-flight launch with the abort word before any
is drained."""

import pytest
import torch

from agilerl_amd.population.engine import PopulationEngine

ABORT = 0xFFFFFFFF


class _Lib:
    def __init__(self, log):
        self.log = log

    def agx_host_signal(self, ctl, seq):
        self.log.append(("signal", ctl, seq))


class _Ctx:
    def __init__(self, lib, ctl):
        self.lib, self.ctl, self.t, self.loss = lib, ctl, 0, torch.zeros(1)


class _Pop:
    def __init__(self, T):
        self.T = T

    def prepare_learn(self):
        pass


class _Runner:
    """A group's runner: its launch 'starts' `delay` polls after it was begun."""

    def __init__(self, name, T, delay, log, lib, fail_at=None):
        self.name, self.T, self.delay, self.log, self.lib, self.fail_at = name, T, delay, log, lib, fail_at
        self._paced_before = True
        self.iterations = 0
        self.polls = 0
        self.released = -1
        self.aborted = False

    def begin_iteration(self):
        self.iterations += 1
        self.polls = 0
        self.released = -1
        self.log.append(("begin", self.name, self.iterations))
        return _Ctx(self.lib, self.name)

    def launch_running(self):
        self.polls += 1
        return self.polls > self.delay

    def pace_release(self, c):
        assert self.polls > self.delay, "released a launch that has not started"
        self.released = c.t
        self.log.append(("release", self.name, c.t))

    def pace_wait_step(self, c):
        assert self.released == c.t, "waited for a step that was not released"
        if self.fail_at is not None and (self.iterations, c.t) == self.fail_at:
            raise RuntimeError("env step failed")
        self.log.append(("step", self.name, c.t))
        c.t += 1

    def end_iteration(self, c):
        assert c.t == self.T
        self.log.append(("end", self.name, self.iterations))
        return c.loss

    def abort_iteration(self, c):
        self.aborted = True
        self.log.append(("abort", self.name))


class _Group:
    def __init__(self, runner):
        self.runner, self.pop = runner, _Pop(runner.T)


def _engine(runners):
    eng = PopulationEngine.__new__(PopulationEngine)
    eng.groups = [_Group(r) for r in runners]
    return eng


@pytest.mark.parametrize("delays", [(0, 0, 0), (3, 0, 7), (5, 5, 1)])
def test_groups_paced_together_run_every_iteration_in_order(delays):
    log = []
    lib = _Lib(log)
    runners = [_Runner(n, T, d, log, lib) for n, T, d in zip("abc", (4, 2, 3), delays)]
    eng = _engine(runners)
    left = [3, 5, 2]
    pending = [[] for _ in runners]
    eng._train_paced_together(list(left), [None] * 3, pending, None)
    for r, n_it, got in zip(runners, left, pending):
        assert r.iterations == n_it and len(got) == n_it
        steps = [e for e in log if e[0] == "step" and e[1] == r.name]
        assert [s[2] for s in steps] == list(range(r.T)) * n_it  # each iteration's steps, in order
        ends = [e[2] for e in log if e[0] == "end" and e[1] == r.name]
        assert ends == list(range(1, n_it + 1))
    # the groups' steps interleave (paced together), not one group after another
    names = [e[1] for e in log if e[0] == "step"]
    assert sum(x != y for x, y in zip(names, names[1:])) > len(runners) - 1


def test_an_exception_releases_every_launch_before_draining():
    log = []
    lib = _Lib(log)
    runners = [_Runner("a", 10, 0, log, lib), _Runner("b", 4, 2, log, lib, fail_at=(1, 1)),
               _Runner("c", 3, 50, log, lib)]
    eng = _engine(runners)
    with pytest.raises(RuntimeError, match="env step failed"):
        eng._train_paced_together([2, 2, 2], [None] * 3, [[], [], []], None)
    first_abort = next(i for i, e in enumerate(log) if e[0] == "abort")
    signalled = {e[1] for e in log[:first_abort] if e[0] == "signal" and e[2] == ABORT}
    assert signalled == {"a", "b", "c"}  # every in-flight launch, the unstarted one included
    assert all(r.aborted for r in runners)


class _PermPop:
    perm_source = "numpy"

    def __init__(self, P, S, E):
        self.P, self.S, self.update_epochs = P, S, E
        self.block = None

    def discard_prefetch(self):
        pass

    def set_generation_perms(self, block):
        self.block = block


class _PermGroup:
    def __init__(self, slots, S, E, learn_step):
        self.slots, self.learn_step = slots, learn_step
        self.pop = _PermPop(len(slots), S, E)


@pytest.mark.parametrize("rank", [0, 1])
def test_generation_perms_follow_the_reference_shuffle_order(rank):
    """draw_generation_perms batches consecutive same-shape agents into one
    native draw; the rows must equal the reference's loop (global agent after
    global agent, each learn a fresh arange(S) shuffled E times in place,
    agilerl/algorithms/ppo.py:836-842) with the global stream left where that
    loop leaves it."""
    import numpy as np

    # global plan over 2 ranks x 3 agents: (S, E, learn_step); a run of equal
    # shapes crosses the rank boundary, one agent has a mutated learn_step
    gplan = [(8, 2, 4), (8, 2, 4), (8, 2, 4), (8, 2, 4), (12, 3, 4), (4, 2, 2)]
    evo = 8
    eng = PopulationEngine.__new__(PopulationEngine)
    eng.rank, eng.P, eng.world = rank, 3, 2
    eng.global_plan = gplan
    local = gplan[3 * rank:3 * rank + 3]
    # groups: one per distinct shape on this rank, slots in order
    groups = {}
    for j, x in enumerate(local):
        groups.setdefault(x, []).append(j)
    eng.groups = [_PermGroup(slots, S, E, ls) for (S, E, ls), slots in groups.items()]
    np.random.seed(99)
    eng.draw_generation_perms(evo)
    after = np.random.get_state(legacy=True)[2]

    np.random.seed(99)
    want = {}
    for gid, (S, E, ls) in enumerate(gplan):
        K = max(1, -(evo // -ls))
        rows = []
        for _ in range(K):
            idx = np.arange(S)
            learn = []
            for _ in range(E):
                np.random.shuffle(idx)
                learn.append(idx.copy())
            rows.append(learn)
        want[gid] = rows
    assert np.random.get_state(legacy=True)[2] == after
    for g in eng.groups:
        for r, slot in enumerate(g.slots):
            for k, learn in enumerate(want[3 * rank + slot]):
                for e, row in enumerate(learn):
                    assert np.array_equal(g.pop.block[k, e, r], row)
