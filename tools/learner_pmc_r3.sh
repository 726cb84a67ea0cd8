# Round-3 learner evidence: the two SQ PMC passes of tools/pmc_learner.sh
# (summarised into gpurun_out/learner_pmc.txt) and learn() wall time at P = 8 and P = 1.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_learner.sh > gpurun_out/learner_pmc_raw.txt 2>&1 || { tail -20 gpurun_out/learner_pmc_raw.txt; exit 1; }
python tools/pmc_learner_summary.py gpurun_out/learner_pmc_raw.txt > gpurun_out/learner_pmc.txt || exit 1
timeout -k 10 120 python -u tools/learn_time.py > gpurun_out/learn_time.log 2>&1 || { tail -5 gpurun_out/learn_time.log; exit 1; }
P=1 timeout -k 10 120 python -u tools/learn_time.py >> gpurun_out/learn_time.log 2>&1 || { tail -5 gpurun_out/learn_time.log; exit 1; }
cat gpurun_out/learner_pmc.txt gpurun_out/learn_time.log
