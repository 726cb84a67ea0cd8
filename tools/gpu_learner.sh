# Learner iteration on the GPU box: learner parity tests, phase stamps, learn() time.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_learner_parity_gpu.py tests/test_population_gpu.py -m gpu -q -x -rf --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_learner.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_learner.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/learn_stamps.py > gpurun_out/stamps.log 2>&1 || { tail -5 gpurun_out/stamps.log; exit 1; }
timeout -k 10 120 python -u tools/learn_time.py >> gpurun_out/stamps.log 2>&1 || { tail -5 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
