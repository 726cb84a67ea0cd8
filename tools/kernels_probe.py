"""Time bench.py's §8d kernel set (PER sample/update, C51, TD target) alone.

    python tools/kernels_probe.py            # prints the kernels JSON
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    peak = float(sys.argv[1]) if len(sys.argv) > 1 else 6422.0
    print(json.dumps(bench.kernels_leg(peak), indent=1))
