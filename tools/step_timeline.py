"""Timeline of the headline step (bench.py population leg: 8 agents x 128
envs, T = 16, one group) from a rocprofv3 kernel trace: per iteration the
persistent rollout kernel, the GAE / gather kernels and the learner, and the
device-idle gaps between them (diagnostic):

  rocprofv3 --kernel-trace --output-format csv -d DIR -o st -- python bench.py --steps 20 --warmup 3 \\
      --no-cpu --no-config5 --no-config3 --no-train-on-policy --no-roofline
  python tools/step_timeline.py DIR/.../st_kernel_trace.csv"""
import csv
import statistics as S
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
roll = [i for i, k in enumerate(ks) if "ppo_rollout_persistent_kernel" in k[2]]
seg = {"rollout": [], "rollout->learn start": [], "learn": [], "learn end->next rollout start": [], "period": []}
for a, b in zip(roll, roll[1:]):
    r = ks[a]
    lrn = [k for k in ks[a + 1:b] if "ppo_learn_kernel" in k[2]]
    if len(lrn) != 1:
        continue
    L = lrn[0]
    seg["rollout"].append(r[1] - r[0])
    seg["rollout->learn start"].append(L[0] - r[1])
    seg["learn"].append(L[1] - L[0])
    seg["learn end->next rollout start"].append(ks[b][0] - L[1])
    seg["period"].append(ks[b][0] - r[0])
for k, v in seg.items():
    if v:
        print(f"{k:32s} median {S.median(v) / 1e3:8.1f} us  (n={len(v)}, min {min(v) / 1e3:.1f}, max {max(v) / 1e3:.1f})")
