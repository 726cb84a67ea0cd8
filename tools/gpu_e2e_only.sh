# The end-to-end train_on_policy leg (3 generations + the 10-generation run) with its phase breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 600 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
grep "train_on_policy" gpurun_out/e2e.err
cat gpurun_out/e2e.json
