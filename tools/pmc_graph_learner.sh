# PMC passes on the runtime-shape learner's few-row form (graph_once.py: 3 learn() calls at the
# config-2 shape; separate passes, --kernel-trace only), summarised per wave.
set -e
export TMPDIR=/tmp
P=/tmp/agx_prof_g
mkdir -p gpurun_out $P
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $P/g1 -o g -- python tools/graph_once.py > gpurun_out/pmc_g1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $P/g2 -o g -- python tools/graph_once.py > gpurun_out/pmc_g2.log 2>&1
python - <<'PY'
import csv, glob, collections
for d in ("/tmp/agx_prof_g/g1", "/tmp/agx_prof_g/g2"):
    acc = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "graph_part_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc.get("SQ_WAVES", 1.0) or 1.0
    for k, v in sorted(acc.items()):
        print(f"{k:28s} {v:16.0f}  per wave {v / w:12.1f}")
PY
