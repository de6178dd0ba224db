set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/steps.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/steps.log"
