# Instruction mix of the partnered runtime-shape learner (graph_stamps.py's mutated shape, one
# learn()): per-wave VALU / SALU / memory instruction counts.  One --pmc pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_F32 --output-format csv -d gpurun_out/pmc_ginst -o run -- python3 tools/graph_stamps.py > gpurun_out/pmc_ginst.log 2>&1
echo "rc=$?"
f=$(find gpurun_out/pmc_ginst -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "graph_part" in k:
        w = v["SQ_WAVES"]
        print(k, {c: round(x / w) for c, x in v.items()}, "waves", w)
PY
