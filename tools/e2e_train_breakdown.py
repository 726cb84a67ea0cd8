"""Where the end-to-end leg's train phase goes on the host: time inside
runner.iteration (of which pacing the persistent rollout, and waiting in it
for the rollout's first step), the generation's shuffle draw, and the final
sync (losses / error words).  Architecture mutations off, 3 generations
(diagnostic; wraps the functions, no change to the path)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py"]
os.environ.setdefault("AGX_BENCH_E2E_LONG", "0")
os.environ.setdefault("AGX_BENCH_E2E_NO_ARCH_ONLY", "1")
import bench  # noqa: E402
from agilerl_amd.population import engine as E  # noqa: E402
from agilerl_amd.population import runner as R  # noqa: E402
from agilerl_amd.population import ppo_pop as PP  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[key] += time.perf_counter() - t
            cnt[key] += 1
    setattr(obj, name, g)


wrap(R.PopulationRunner, "iteration", "iteration")
wrap(R.PopulationRunner, "_pace_persistent", "pace")
wrap(R.PopulationRunner, "_launch_persistent", "launch_rollout")
wrap(PP.PPOPopulation, "learn", "learn_enqueue")
wrap(PP.PPOPopulation, "finish_rollout", "finish_rollout")
wrap(PP.PPOPopulation, "prefetch_permutations", "prefetch_perms")
wrap(PP.PPOPopulation, "prepare_learn", "prepare_learn")
wrap(PP.PPOPopulation, "check_errors", "check_errors")
wrap(E.PopulationEngine, "train", "train")
wrap(E.PopulationEngine, "draw_generation_perms", "draw_perms")
wrap(E.PopulationEngine, "evaluate", "evaluate")
wrap(E.PopulationEngine, "_train_paced_together", "paced_together")
wrap(R.PopulationRunner, "begin_iteration", "begin_iteration")
wrap(R.PopulationRunner, "end_iteration", "end_iteration")
wrap(R.PopulationRunner, "pace_wait_step", "pace_wait_step")
wrap(R.PopulationRunner, "_env_step", "env_step")
wrap(R.PopulationRunner, "_finish_persistent", "finish_persistent")
wrap(R.PopulationRunner, "_mark_stats", "mark_stats")
wrap(R.PopulationRunner, "launch_running", "launch_running")
wrap(R.PopulationRunner, "pace_release", "pace_release")

if __name__ == "__main__":
    out = bench.train_on_policy_leg(generations=3)
    gens = 4 + 1  # warm-up run (1 generation) + 3 timed, counted together
    print({k: out[k]["ms_per_generation"] for k in out if isinstance(out[k], dict)}, file=sys.stderr)
    for k in sorted(acc, key=lambda k: -acc[k]):
        print(f"{k:16s} {acc[k] / 4 * 1e3:8.2f} ms per generation  ({cnt[k]} calls, "
              f"{acc[k] / max(cnt[k], 1) * 1e6:8.1f} us each)")
