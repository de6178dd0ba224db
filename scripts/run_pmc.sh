set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt -o kt --output-format csv -- $B > gpurun_out/pmc/kt.log 2>&1
rc=$?; echo "kt rc=$rc" > gpurun_out/pmc/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/sq -o sq --output-format csv -- $B > gpurun_out/pmc/sq.log 2>&1
rc=$?; echo "sq rc=$rc" >> gpurun_out/pmc/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc" >> gpurun_out/pmc/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- $B > gpurun_out/pmc/write.log 2>&1
rc=$?; echo "write rc=$rc" >> gpurun_out/pmc/steps.log
exit $rc
