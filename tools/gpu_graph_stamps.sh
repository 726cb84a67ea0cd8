# Partnered runtime-shape learner: per-layer phase stamps (graph_stamps.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_stamps.py > gpurun_out/graph_stamps.log 2>&1 || { tail -20 gpurun_out/graph_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_stamps.log
