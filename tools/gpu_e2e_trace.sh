# Kernel trace of the end-to-end leg (architecture mutations off, 3 generations): do the groups'
# learners overlap on the device?  Summarised by tools/trace_overlap.py.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && AGX_BENCH_E2E_NO_ARCH_ONLY=1 AGX_BENCH_E2E_LONG=0 GENS=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/e2e_time.py > $GRAFT_REPO_ROOT/gpurun_out/kt.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 gpurun_out/kt.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/kt -name "*kernel_trace.csv" | head -1)
python3 tools/trace_overlap.py "$f"
