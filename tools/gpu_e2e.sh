# Partnered graph learner phase stamps, then the end-to-end train_on_policy leg (3 and 10 generations).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_stamps.py > gpurun_out/graph_stamps.log 2>&1 || { tail -5 gpurun_out/graph_stamps.log; exit 1; }
cat gpurun_out/graph_stamps.log
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 600 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
