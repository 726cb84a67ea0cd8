# LDS-resident evaluation weights: population / dynamic-shape GPU tests (TESTS=1), then the
# evaluation step latency with the weights in LDS and from L2 (AGX_EVAL_WLDS=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_population_gpu.py tests/test_dynamic_shapes_gpu.py tests/test_dropin_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_eval.log 2>&1
  rc=$?
  tail -8 gpurun_out/pytest_eval.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/eval_latency.log
for w in 1 0; do
  for m in 0 1; do
    echo "AGX_EVAL_WLDS=$w MUTATED=$m" >> gpurun_out/eval_latency.log
    AGX_EVAL_WLDS=$w MUTATED=$m timeout -k 10 120 python -u -W ignore tools/eval_latency.py >> gpurun_out/eval_latency.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/eval_latency.log
