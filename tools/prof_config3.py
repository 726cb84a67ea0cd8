"""Profile target: bench.config3_leg (population-batched Rainbow learner)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(bench.config3_leg(iters=int(os.environ.get("ITERS", 5))))
