# Learner evidence (R=r6 bash tools/gpu_learner_evidence.sh): fused learner learn() sweep (P = 8, 4, 2, 1) and PMC passes, the
# runtime-shape learner's PMC passes, phase stamps and graph_bench, the evaluation step latency.
set -o pipefail
export TMPDIR=/tmp
R=${R:-r6}
mkdir -p gpurun_out
bash tools/learn_time_sweep.sh > gpurun_out/${R}_learn_sweep.log 2>&1 || { tail -5 gpurun_out/${R}_learn_sweep.log; exit 1; }
cat gpurun_out/${R}_learn_sweep.log
bash tools/pmc_learner.sh > gpurun_out/${R}_learner_pmc.txt 2>&1 || { tail -5 gpurun_out/${R}_learner_pmc.txt; exit 1; }
rm -rf gpurun_out/pmc_l1 gpurun_out/pmc_l2
tail -20 gpurun_out/${R}_learner_pmc.txt
bash tools/pmc_graph_learner.sh > gpurun_out/${R}_graph_learner_pmc.txt 2>&1 || { tail -5 gpurun_out/${R}_graph_learner_pmc.txt; exit 1; }
cat gpurun_out/${R}_graph_learner_pmc.txt
timeout -k 10 120 python -u tools/graph_stamps.py 2>&1 | grep -v amdgpu.ids > gpurun_out/${R}_graph_stamps.log || exit 1
timeout -k 10 200 python -u tools/graph_bench.py > gpurun_out/${R}_graph_bench.json 2> gpurun_out/graph_bench.err || exit 1
cat gpurun_out/${R}_graph_bench.json
bash tools/gpu_eval_latency.sh > gpurun_out/${R}_eval_latency.log 2>&1 || exit 1
grep -v Warning gpurun_out/${R}_eval_latency.log | grep -v "^  " 
