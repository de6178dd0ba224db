set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
ARGS="2 filter_init {\"key\":\"timeout\"} 1000000 3"
for lib in libfsg libfsg_exp1; do
  export FSG_LIB=$PWD/fluvio_amd/_lib/$lib.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/exp/kt_$lib -o kt --output-format csv -- python3 tools_exp.py 2 filter_init '{"key":"timeout"}' 1000000 3 > gpurun_out/exp/kt_$lib.log 2>&1
  rc=$?; echo "$lib kt rc=$rc" >> gpurun_out/exp/steps.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/exp/sq_$lib -o sq --output-format csv -- python3 tools_exp.py 2 filter_init '{"key":"timeout"}' 1000000 3 > gpurun_out/exp/sq_$lib.log 2>&1
  rc=$?; echo "$lib sq rc=$rc" >> gpurun_out/exp/steps.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
