# Evaluation-launch step latency (tools/eval_latency.py), compiled shape then a mutated one.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/eval_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/eval_latency.log || exit 1
MUTATED=1 timeout -k 10 120 python -u tools/eval_latency.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/eval_latency.log || exit 1
