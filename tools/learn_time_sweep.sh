# learn() wall time at P = 8, 4, 2, 1 agents (the strong-scaling shards of the 8-agent population)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/learn_sweep.log
for P in 8 4 2 1; do
  P=$P timeout -k 10 120 python -u tools/learn_time.py >> gpurun_out/learn_sweep.log 2>&1 || { tail -5 gpurun_out/learn_sweep.log; exit 1; }
done
grep learn gpurun_out/learn_sweep.log
