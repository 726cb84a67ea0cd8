# Instruction-fetch counters of the fused learner (learn_time.py): is the
# kernel's code footprint thrashing the instruction cache?
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1
cd $GRAFT_REPO_ROOT
grep -o -E "SQC_[A-Z_]*ICACHE[A-Z_]*|SQ_[A-Z_]*INST[A-Z_]*|SQ_IFETCH[A-Z_]*" gpurun_out/pmc_list.txt | sort -u > gpurun_out/pmc_inst_names.txt
cat gpurun_out/pmc_inst_names.txt | head -40
REPS=10 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_icache -o run -- python3 tools/learn_time.py > gpurun_out/pmc_icache.log 2>&1
echo "rc=$?"
find gpurun_out/pmc_icache -name "*counter_collection*" | head -3
