# Runtime-shape learner / persistent-rollout checks on the GPU box: population, graph-learner and
# dynamic-shape tests, graph_bench (rows per partner 16 and 8, one workgroup per agent), then the
# end-to-end leg.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_population_gpu.py tests/test_graph_learner_gpu.py tests/test_dynamic_shapes_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_graph.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/graph_bench.py > gpurun_out/graph_bench.json 2> gpurun_out/graph_bench.err || { tail -5 gpurun_out/graph_bench.err; exit 1; }
AGX_GRAPH_ROWS=8 timeout -k 10 200 python -u tools/graph_bench.py > gpurun_out/graph_bench_r8.json 2>> gpurun_out/graph_bench.err || { tail -5 gpurun_out/graph_bench.err; exit 1; }
cat gpurun_out/graph_bench.json gpurun_out/graph_bench_r8.json
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 600 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
