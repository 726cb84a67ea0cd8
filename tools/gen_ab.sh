set -o pipefail
for v in 1 0 1 0; do
  AGX_ROWS_GATHER=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu --no-config5 --no-roofline 2>&1 | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('rows_gather', $v, d['ms_per_step'])"
done
