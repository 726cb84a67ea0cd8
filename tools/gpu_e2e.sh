# Population GPU tests, partnered graph learner phase stamps (whole, then with each phase of the
# gradient pass skipped: AGX_GRAPH_DEBUG 1 forward GEMMs, 2 dW, 4 dX, 8 row passes + loss), then the
# end-to-end train_on_policy leg (3 and 10 generations).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_population_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_pop.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_pop.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/graph_stamps.log
for d in 0 1 2 4 8; do
  echo "== AGX_GRAPH_DEBUG=$d" >> gpurun_out/graph_stamps.log
  AGX_GRAPH_DEBUG=$d timeout -k 10 120 python -u tools/graph_stamps.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/graph_stamps.log || exit 1
done
cat gpurun_out/graph_stamps.log
GENS=3 AGX_BENCH_E2E_LONG=${LONG:-10} timeout -k 10 600 python -u tools/e2e_time.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
grep "train_on_policy" gpurun_out/e2e.err
cat gpurun_out/e2e.json
