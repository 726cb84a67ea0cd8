set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py tests/test_image_ppo_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cnn.log 2>&1 || { tail -20 gpurun_out/cnn.log; exit 1; }
tail -1 gpurun_out/cnn.log
timeout -k 10 300 python -u tools/config5_time.py 10 2>&1 | grep ms/iter
git_stashed=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o c5 -- python tools/config5_time.py 5 > gpurun_out/c5prof.log 2>&1
