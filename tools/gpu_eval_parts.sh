# Evaluation step latency with the population in 2, 3, 4 and 8 parts (AGX_EVAL_PARTS).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/eval_parts.log
for n in 2 3 4 8; do
  echo "== parts $n" >> gpurun_out/eval_parts.log
  AGX_EVAL_PARTS=$n timeout -k 10 120 python -u tools/eval_latency.py 2>&1 | grep "pass:" >> gpurun_out/eval_parts.log || exit 1
done
cat gpurun_out/eval_parts.log
