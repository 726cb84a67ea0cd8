# cProfile of the end-to-end leg (host hot spots), then the runtime-shape learner's phase stamps and graph_bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GENS=3 timeout -k 10 600 python -u tools/e2e_profile.py > gpurun_out/e2e_profile.txt 2> gpurun_out/e2e_profile.err || { tail -20 gpurun_out/e2e_profile.err; exit 1; }
grep "train_on_policy" gpurun_out/e2e_profile.err
timeout -k 10 120 python -u tools/graph_stamps.py 2>&1 | grep -v amdgpu.ids > gpurun_out/graph_stamps.log || exit 1
head -12 gpurun_out/graph_stamps.log
timeout -k 10 200 python -u tools/graph_bench.py > gpurun_out/graph_bench.json 2> gpurun_out/graph_bench.err || { tail -5 gpurun_out/graph_bench.err; exit 1; }
cat gpurun_out/graph_bench.json
