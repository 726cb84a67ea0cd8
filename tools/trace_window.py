"""Kernel statistics (the rocprofv3 --stats columns) of one timed window of a
kernel trace, between marker launches (agx_debug_stream's stream_kernel<1>,
tools/prof_config3.py): window k = the kernels between markers 2k and 2k + 1
(k = 0: the batched loop, 1: the per-agent loop).  Writes CSV to stdout and
the agx:: share of the window's kernel time to stderr; SEQ=n also lists the
window's first n kernels in launch order (name, duration) on stderr."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
which = {"batched": 0, "per_agent": 1}.get(sys.argv[2] if len(sys.argv) > 2 else "per_agent", 1)
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, (_, _, n) in enumerate(ks) if "stream_kernel<1>" in n]
if len(marks) < 2 * which + 2:
    sys.exit(f"trace_window: {len(marks)} markers, window {which} needs {2 * which + 2}")
a, b = marks[2 * which], marks[2 * which + 1]
win = ks[a + 1:b]
agg = collections.defaultdict(list)
for s, e, n in win:
    agg[n].append(e - s)
tot = sum(sum(v) for v in agg.values())
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    w.writerow([n, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v)])
agx = sum(sum(v) for n, v in agg.items() if "agx::" in n)
span = win[-1][1] - win[0][0] if win else 0
print(f"window {sys.argv[2] if len(sys.argv) > 2 else 'per_agent'}: {len(win)} kernels, {tot / 1e6:.2f} ms kernel time "
      f"over a {span / 1e6:.2f} ms span; agx:: kernels {agx / 1e6:.2f} ms = {100.0 * agx / max(tot, 1):.1f} %",
      file=sys.stderr)
import os  # noqa: E402

for s_, e_, n_ in win[:int(os.environ.get("SEQ", "0"))]:
    print(f"{(e_ - s_) / 1e3:8.1f} us  {n_[:100]}", file=sys.stderr)
