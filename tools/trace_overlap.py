"""Summarise a rocprofv3 kernel trace of the end-to-end leg: per kernel family
the count and total time, and how much of the learners' time overlaps another
learner (a different queue / stream) — the groups' learns should run side by
side on the device."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""),
      r.get("Stream_Id", "")) for r in rows]
k.sort()
tot = collections.defaultdict(lambda: [0, 0])
for s, e, n, q, st in k:
    key = n.split("(")[0][-60:]
    tot[key][0] += 1
    tot[key][1] += e - s
for key, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:15]:
    print(f"{t / 1e6:9.2f} ms {c:6d}  {key}")
learn = [(s, e, q, st) for s, e, n, q, st in k if "learn" in n and "gather" not in n]
ov = 0
for i, (s, e, q, st) in enumerate(learn):
    for s2, e2, q2, st2 in learn[i + 1:]:
        if s2 >= e:
            break
        ov += min(e, e2) - s2
span = (k[-1][1] - k[0][0]) if k else 0
print(f"learn kernels {len(learn)}, total {sum(e - s for s, e, _, _ in learn) / 1e6:.2f} ms, pairwise overlap "
      f"{ov / 1e6:.2f} ms, trace span {span / 1e6:.1f} ms; queues {sorted({q for _, _, q, _ in learn})}, "
      f"streams {sorted({st for _, _, _, st in learn})}")
# per queue: kernel-busy time, the persistent rollouts' share, and the idle gaps
byq = collections.defaultdict(list)
for s, e, n, q, st in k:
    byq[q].append((s, e, n))
for q in sorted(byq):
    ks = byq[q]
    busy = sum(e - s for s, e, _ in ks)
    roll = sum(e - s for s, e, n in ks if "persistent" in n)
    lrn = sum(e - s for s, e, n in ks if "learn" in n and "gather" not in n)
    gaps = sorted(ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1))
    big = sum(g for g in gaps if g > 20000)
    print(f"queue {q}: {len(ks)} kernels, busy {busy / 1e6:.1f} ms (rollout {roll / 1e6:.1f}, learn {lrn / 1e6:.1f}), "
          f"span {(ks[-1][1] - ks[0][0]) / 1e6:.1f} ms, gaps > 20 us {big / 1e6:.1f} ms")
