set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/c51_sq -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_sq.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c51_fetch -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c51_kt -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_kt.log 2>&1 &&
C51_DONE_P=0 timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c51_kt0 -o c51 -- python tools/c51_pmc.py > gpurun_out/c51_kt0.log 2>&1
echo rc=$?
