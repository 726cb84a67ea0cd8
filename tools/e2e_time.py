"""Time bench.py's end-to-end train_on_policy leg alone (diagnostic)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py"]
import bench  # noqa: E402

if __name__ == "__main__":
    g = int(os.environ.get("GENS", 2))
    print(json.dumps(bench.train_on_policy_leg(generations=g)), flush=True)
