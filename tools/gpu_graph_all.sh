# Runtime-shape kernels: population, graph-learner and dynamic-shape GPU tests (few-row forms on,
# then off), the learner's phase stamps and graph_bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_graph_learner_gpu.py tests/test_dynamic_shapes_gpu.py tests/test_population_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_graph.log
[ $rc -eq 0 ] || exit $rc
AGX_GRAPH_FEW=0 timeout -k 10 600 python -u -m pytest tests/test_graph_learner_gpu.py tests/test_dynamic_shapes_gpu.py tests/test_population_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_graph_g.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_graph_g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/graph_stamps.py 2>&1 | grep -v amdgpu.ids > gpurun_out/graph_stamps.log || exit 1
cat gpurun_out/graph_stamps.log
timeout -k 10 200 python -u tools/graph_bench.py > gpurun_out/graph_bench.json 2> gpurun_out/graph_bench.err || { tail -5 gpurun_out/graph_bench.err; exit 1; }
cat gpurun_out/graph_bench.json
