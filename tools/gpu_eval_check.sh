# Evaluation / guard checks on the GPU box: population + learner + dynamic-shape tests, then the
# end-to-end train_on_policy leg with its per-phase breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_population_gpu.py tests/test_learner_parity_gpu.py tests/test_dynamic_shapes_gpu.py -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_eval.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_eval.log
[ $rc -eq 0 ] || exit $rc
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 400 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
