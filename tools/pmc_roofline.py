"""The bench roofline workload alone (1 GAE + 4 loss launches x 3 reps), for
the rocprofv3 --pmc passes:

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o roof -- python tools/pmc_roofline.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o roof -- python tools/pmc_roofline.py
  python tools/pmc_summarize.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/r1_pmc_traffic.json
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

run_gae, run_loss, S = bench.roofline_workload()
for _ in range(3):
    run_gae()
    for _ in range(bench.ROOF_E):
        run_loss()
torch.cuda.synchronize()
print("done", S)
