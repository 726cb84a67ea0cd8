set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python -u tools/learn_time.py 2>&1 | grep mean | sed "s/^/new: /"
  AGX_LIB=ab/libagx_prev.so timeout -k 10 120 python -u tools/learn_time.py 2>&1 | grep mean | sed "s/^/prev: /"
done
for r in 32 16 32 16; do
  AGX_ROLLOUT_ROWS=$r timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --no-config5 --no-roofline 2>&1 | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rows $r', d['ms_per_step'])"
done
