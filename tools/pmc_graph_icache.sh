# Instruction-fetch counters of the partnered runtime-shape learner (graph_once.py, 3 learn() calls):
# is its code footprint thrashing the instruction cache?  One --pmc pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_gicache -o run -- python3 tools/graph_once.py > gpurun_out/pmc_gicache.log 2>&1
echo "rc=$?"
f=$(find gpurun_out/pmc_gicache -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "graph" in k:
        print(k, dict(v))
PY
