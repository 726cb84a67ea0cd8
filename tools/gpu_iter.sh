# One GPU iteration: the whole -m gpu suite (all failures listed), then a
# short bench.  Usage (from the repo root): bash tools/gpu_iter.sh [pytest args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_quick.log 2>&1 || { tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -c 1500 gpurun_out/bench_quick.log
exit $rc
