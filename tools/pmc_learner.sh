# PMC passes on the fused learner (separate passes, --kernel-trace only; see MI355X_MICROARCH rocprofv3 notes)
set -e
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d gpurun_out/pmc_l1 -o l -- python tools/learn_only.py > gpurun_out/pmc_l1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_l2 -o l -- python tools/learn_only.py > gpurun_out/pmc_l2.log 2>&1
python - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc_l1", "gpurun_out/pmc_l2"):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "ppo_learn_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(k, v[-1])
PY
