"""Per-launch HBM bytes of agx_c51_project_loss (c51_dma_kernel) from the
FETCH_SIZE / WRITE_SIZE passes of tools/c51_pmc.py (B = 2^20, A = 6, Z = 51):
  python tools/pmc_c51_summary.py gpurun_out/c51_fetch gpurun_out/c51_write [rows]
``rows``: the selected-rows form (agx_c51_project_loss_rows over
tools/prof_c51_rows.py: two contiguous [B][Z] rows, r, d in; loss out).
Same gfx950 correction as tools/pmc_summarize.py (2 x FETCH_SIZE)."""
import csv
import glob
import json
import os
import sys


ROWS = len(sys.argv) > 3 and sys.argv[3] == "rows"
TAG = "c51_dma_kernel<51, true, true>" if ROWS else "c51_dma_kernel<51, true, false>"


def vals(d, counter):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter and TAG in row["Kernel_Name"]:
                out.append(float(row["Counter_Value"]))
    if not out:
        raise SystemExit(f"no c51_dma_kernel {counter} rows under {d}")
    return sum(out) / len(out), len(out)


B, A, Z = 1 << 20, 6, 51
fetch, nf = vals(sys.argv[1], "FETCH_SIZE")
write, nw = vals(sys.argv[2], "WRITE_SIZE")
read_alg = B * (2 * Z * 4 + 4 + 4) if ROWS else B * (A * 4 + 2 * Z * 4 + 8 + 4 + 4)  # (q row,) two Z-rows, (a,) r, d
write_alg = B * 4  # loss
out = {
    "kernel": (f"{TAG} (agx_c51_project_loss_rows, B=2^20, Z=51, proj=None)" if ROWS
               else f"{TAG} (agx_c51_project_loss, B=2^20, A=6, Z=51, proj=None)"),
    "launches": {"fetch": nf, "write": nw},
    "fetch_kb": fetch, "write_kb": write,
    "read_bytes": 2 * fetch * 1024, "write_bytes": write * 1024,
    "read_bytes_per_row": 2 * fetch * 1024 / B, "write_bytes_per_row": write * 1024 / B,
    "algorithmic_read_per_row": read_alg / B, "algorithmic_write_per_row": write_alg / B,
    "traffic_over_algorithmic": (2 * fetch + write) * 1024 / (read_alg + write_alg),
}
print(json.dumps(out, indent=1))
