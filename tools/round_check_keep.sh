# Round check, then keep only the summaries that go to profiles/ (gpurun copies back <= 64 MiB)
set -o pipefail
R=${R:-r3}
R=$R bash tools/gpu_round_check.sh > gpurun_out/round_check.log 2>&1
rc=$?
# the learner's SQ counters and learn() time at P = 8 / 4 / 2 / 1
if [ $rc -eq 0 ]; then
  bash tools/learner_pmc_r3.sh > gpurun_out/learner_pmc_run.log 2>&1 && bash tools/learn_time_sweep.sh >> gpurun_out/learner_pmc_run.log 2>&1
  rc=$?
fi
mkdir -p gpurun_keep
cp gpurun_out/learner_pmc.txt gpurun_keep/${R}_learner_pmc.txt 2>/dev/null
cp gpurun_out/learn_sweep.log gpurun_keep/${R}_learn_sweep.log 2>/dev/null
cp gpurun_out/learner_pmc_run.log gpurun_keep/ 2>/dev/null
cp gpurun_out/round_check.log gpurun_out/pytest_gpu.log gpurun_out/bench_full.json gpurun_out/bench_full.err gpurun_keep/ 2>/dev/null
cp gpurun_out/${R}_*.json gpurun_keep/ 2>/dev/null
find gpurun_out/prof_$R -name "*kernel_stats.csv" -exec cp {} gpurun_keep/${R}_kernel_stats.csv \; 2>/dev/null
find gpurun_out/prof_c3_$R -name "*kernel_stats.csv" -exec cp {} gpurun_keep/${R}_config3_kernel_stats.csv \; 2>/dev/null
rm -rf gpurun_out/*
mv gpurun_keep gpurun_out/keep
echo rc=$rc
exit $rc
