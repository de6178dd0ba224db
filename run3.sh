set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/steps.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python tools_stamps.py 2 filter_init '{"key": "timeout"}' 1000000 > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/steps.log
exit $rc
