# Runtime-shape kernels + population engine: graph-learner / dynamic-shape / population GPU tests
# (few-row forms on), then the end-to-end leg with its phase breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_graph_learner_gpu.py tests/test_dynamic_shapes_gpu.py tests/test_population_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_graph.log
[ $rc -eq 0 ] || exit $rc
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 600 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
grep "train_on_policy" gpurun_out/e2e.err
