# Round-end measurement sequence (run from the repo root on the GPU box):
#   R=r6 bash tools/gpu_round_check.sh
# GPU tests, the default bench line, a kernel trace of the bench, and the
# separate FETCH_SIZE / WRITE_SIZE passes over the roofline workload and over
# the C51 kernel.  rocprofv3 writes under /tmp/agx_prof (its traces are large);
# the summaries land in gpurun_out/ (copy them to profiles/).
set -o pipefail
export TMPDIR=/tmp
R=${R:-r6}
P=/tmp/agx_prof
mkdir -p gpurun_out $P
if [ -z "$SKIP_TESTS" ]; then  # SKIP_TESTS=1: the GPU tests ran in a call of their own
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${R}_pytest_gpu.log
fi
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
tail -c 400 gpurun_out/${R}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/prof -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu --no-config5 --no-config3 --no-train-on-policy > gpurun_out/prof_$R.log 2>&1 || { tail -20 gpurun_out/prof_$R.log; exit 1; }
cp $(find $P/prof -name "*kernel_stats.csv" | head -1) gpurun_out/${R}_kernel_stats.csv || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o roof -- python tools/pmc_roofline.py > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o roof -- python tools/pmc_roofline.py > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/c51_fetch -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_fetch.log 2>&1 || { tail -20 gpurun_out/c51_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/c51_write -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_write.log 2>&1 || { tail -20 gpurun_out/c51_write.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/c51r_fetch -o c51 -- python tools/prof_c51_rows.py > gpurun_out/c51r_fetch.log 2>&1 || { tail -20 gpurun_out/c51r_fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/c51r_write -o c51 -- python tools/prof_c51_rows.py > gpurun_out/c51r_write.log 2>&1 || { tail -20 gpurun_out/c51r_write.log; exit 1; }
python tools/pmc_summarize.py $P/pmc_fetch $P/pmc_write > gpurun_out/${R}_pmc_traffic.json || exit 1
python tools/pmc_c51_summary.py $P/c51_fetch $P/c51_write > gpurun_out/${R}_c51_pmc_traffic.json || exit 1
python tools/pmc_c51_summary.py $P/c51r_fetch $P/c51r_write rows > gpurun_out/${R}_c51_rows_pmc_traffic.json || exit 1
# config 3: the timed per-agent loop alone (between the marker launches of tools/prof_config3.py)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/prof_c3 -o c3 -- python tools/prof_config3.py > gpurun_out/prof_c3_$R.log 2>&1 || { tail -20 gpurun_out/prof_c3_$R.log; exit 1; }
python tools/trace_window.py $(find $P/prof_c3 -name "*kernel_trace.csv" | head -1) per_agent > gpurun_out/${R}_config3_kernel_stats.csv 2> gpurun_out/${R}_config3_window.txt || exit 1
cat gpurun_out/${R}_config3_window.txt
echo ALLOK
