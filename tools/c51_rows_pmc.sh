# FETCH / WRITE passes (one counter set per run) + kernel trace of agx_c51_project_loss_rows
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c51r_fetch -o c51 -- python3 tools/prof_c51_rows.py > gpurun_out/c51r_fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c51r_write -o c51 -- python3 tools/prof_c51_rows.py > gpurun_out/c51r_write.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c51r_kt -o c51 -- python3 tools/prof_c51_rows.py > gpurun_out/c51r_kt.log 2>&1 &&
python3 tools/pmc_c51_summary.py gpurun_out/c51r_fetch gpurun_out/c51r_write rows > gpurun_out/c51r_summary.json
echo rc=$?
