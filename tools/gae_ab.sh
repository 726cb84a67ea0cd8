# GAE tiled vs column form: parity tests, then the bench roofline leg with each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_components_gpu.py -k "gae or rollout_buffer" -x -q --timeout 200 --timeout-method thread > gpurun_out/gae_tests.log 2>&1 || { tail -20 gpurun_out/gae_tests.log; exit 1; }
tail -1 gpurun_out/gae_tests.log
for tile in 1 0 1 0; do
  AGX_GAE_TILE=$tile timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-config5 2>&1 | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read())['roofline'];print('tile', $tile, d['gae_ms'], d['gae_gbs'], d['loss_ms'], d['frac'], d['frac_of_measured'])"
done
