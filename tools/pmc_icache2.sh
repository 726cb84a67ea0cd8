# i-cache hit/miss counters of the fused learner alone (learn_time.py); one --pmc pass
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=10 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_icache -o run -- python3 tools/learn_time.py > gpurun_out/pmc_icache.log 2>&1
echo "rc=$?"
