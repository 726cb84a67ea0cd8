"""Per-launch HBM bytes of the roofline kernels from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; KB units).  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE taken as is."""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            key = "gae" if "gae_kernel" in name else "loss" if "ppo_loss" in name else None
            if key:
                vals.setdefault(key, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
write, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
S = 8 * 1024 * 8192
out = {
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of tools/pmc_roofline.py on MI355X",
    "correction": "bytes = 2 x FETCH_SIZE (gfx950 counts 64 B per 128 B read request) + WRITE_SIZE; KB x 1024",
    "launches": {"fetch": nf, "write": nw},
    "gae_fetch_kb": fetch["gae"], "gae_write_kb": write["gae"],
    "loss_fetch_kb": fetch["loss"], "loss_write_kb": write["loss"],
    "gae_bytes": (2 * fetch["gae"] + write["gae"]) * 1024,
    "loss_bytes": (2 * fetch["loss"] + write["loss"]) * 1024,
    "gae_algorithmic_bytes": 17 * S,
    "loss_algorithmic_bytes": 40 * S,
}
out["gae_traffic_over_algorithmic"] = out["gae_bytes"] / out["gae_algorithmic_bytes"]
out["loss_traffic_over_algorithmic"] = out["loss_bytes"] / out["loss_algorithmic_bytes"]
print(json.dumps(out, indent=1))
