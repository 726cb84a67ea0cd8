"""Per-round timing of the groups' paced-together rollouts
(PopulationEngine._train_paced_together): 8 agents x 128 envs split into 4
groups by learn_step; for every host round, how many rollouts it paced and
how long each wait (release -> all workgroups done) took by its position in
the round (diagnostic)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import agilerl_amd  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402
from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.engine import PopulationEngine  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population import runner as R  # noqa: E402

P, N = 8, 128
G = int(os.environ.get("GROUPS", 4))
pop = PPOPopulation(ActorCriticSpec(obs_dim=8, n_actions=4), P, N, learn_step=2048, batch_size=128,
                    update_epochs=4, device="cuda", seeds=list(range(P)))
envs = [SyntheticVecEnv(N, seed=10 + j) for j in range(P)]
views = [type("V", (), {"learn_step": 2048})() for _ in range(P)]
eng = PopulationEngine(pop, views, StackedVecEnv(envs))
states = eng.local_states()
for j in range(P):
    states[j].learn_step = [2048, 1024, 512, 256][j % G] if G > 1 else 2048
eng.regroup(states)
print("groups", len(eng.groups), "paced together", eng._paced_together())
lib = _lib.load()
log = []
orig_rel, orig_wait = R.PopulationRunner.pace_release, R.PopulationRunner.pace_wait_step
orig_wait_fn = lib.agx_host_wait


def rel(self, c):
    log.append(("rel", id(self), time.perf_counter()))
    return orig_rel(self, c)


class W:
    def __call__(self, *a):
        t0 = time.perf_counter()
        rc = orig_wait_fn(*a)
        log.append(("wait", None, time.perf_counter() - t0))
        return rc


orig_begin, orig_end, orig_run = (R.PopulationRunner.begin_iteration, R.PopulationRunner.end_iteration,
                                  R.PopulationRunner.launch_running)
ev = collections.defaultdict(list)


def begin(self):
    ev[id(self)].append(["b", time.perf_counter(), None, None, self.pop.T, self.pop.S])
    return orig_begin(self)


def running(self):
    r = orig_run(self)
    if r and ev[id(self)] and ev[id(self)][-1][2] is None:
        ev[id(self)][-1][2] = time.perf_counter()
    return r


def end(self, c):
    if ev[id(self)]:
        ev[id(self)][-1][3] = time.perf_counter()
    return orig_end(self, c)


for _ in range(2):
    eng.train(2 * 2048)
torch.cuda.synchronize()
R.PopulationRunner.pace_release = rel
lib.agx_host_wait = W()
R.PopulationRunner.begin_iteration, R.PopulationRunner.end_iteration, R.PopulationRunner.launch_running = \
    begin, end, running
t0 = time.perf_counter()
eng.train(4 * 2048)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
R.PopulationRunner.pace_release = orig_rel
lib.agx_host_wait = orig_wait_fn
# rounds: a run of releases then the waits
rounds, cur = [], None
for kind, who, v in log:
    if kind == "rel":
        if cur is None or cur["waits"]:
            cur = {"n": 0, "waits": []}
            rounds.append(cur)
        cur["n"] += 1
    else:
        cur["waits"].append(v)
bypos = collections.defaultdict(list)
for r in rounds:
    for i, w in enumerate(r["waits"]):
        bypos[(r["n"], i)].append(w)
print(f"train(4 x 2048 steps) {dt * 1e3:.1f} ms, {len(rounds)} rounds")
for key in sorted(bypos):
    v = np.array(bypos[key]) * 1e6
    print(f"rounds pacing {key[0]} rollouts, wait #{key[1]}: n={len(v)} median {np.median(v):.1f} us, p90 {np.percentile(v, 90):.1f}")

# per group: each iteration's begin -> launch running (waits on the group's own
# previous learner + launch latency) and running -> end (pacing the T steps)
for k, its in ev.items():
    its = [x for x in its if x[2] is not None and x[3] is not None]
    if not its:
        continue
    w = np.array([x[2] - x[1] for x in its]) * 1e6
    p = np.array([x[3] - x[2] for x in its]) * 1e6
    gap = np.array([its[i + 1][1] - its[i][3] for i in range(len(its) - 1)] or [0]) * 1e6
    print(f"group T={its[0][4]} S={its[0][5]}: {len(its)} iterations, begin->running median {np.median(w):.0f} us, "
          f"pacing median {np.median(p):.0f} us, end->next begin median {np.median(gap):.0f} us, "
          f"span {1e3 * (its[-1][3] - its[0][1]):.1f} ms")
