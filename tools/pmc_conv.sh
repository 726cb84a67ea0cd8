# PMC passes on one conv layer's kernels (tools/conv_bench.py, LAYER=$L; separate --pmc passes, --kernel-trace only)
set -e
export TMPDIR=/tmp
L=${L:-1}
D=${D:-gpurun_out/pmc_conv}
mkdir -p $D
LAYER=$L timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d /tmp/pmc_c1 -o c -- python tools/conv_bench.py > $D/p1.log 2>&1
LAYER=$L timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d /tmp/pmc_c2 -o c -- python tools/conv_bench.py > $D/p2.log 2>&1
LAYER=$L timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d /tmp/pmc_c3 -o c -- python tools/conv_bench.py > $D/p3.log 2>&1
python - <<'PY' > $D/summary.txt
import csv, glob, collections
for d in ("/tmp/pmc_c1", "/tmp/pmc_c2", "/tmp/pmc_c3"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "igemm_kernel" in n:
                key = n.split("(")[0].replace("void agx::conv::igemm_kernel", "")
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, cs in sorted(acc.items()):
        print(key, {k: round(sum(v) / len(v)) for k, v in sorted(cs.items())})
PY
cat $D/summary.txt
