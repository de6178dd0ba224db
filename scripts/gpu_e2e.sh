#!/bin/bash
# GPU-box run: the full GPU suite, then the headline bench line with the
# C-ABI end-to-end leg, and the one-record latency line.  usage: scripts/gpu_e2e.sh tag
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
step tests $?
timeout -k 10 300 python -u bench.py --workload c2-substring --only --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_c2.log" 2>&1
step bench_c2 $?
timeout -k 10 300 python -u bench.py --workload f3-one-record --only --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_f3.log" 2>&1
step bench_f3 $?
timeout -k 10 300 python -u tests/perf_decompress.py > "$O/perf_decompress.log" 2>&1
step perf_decompress $?
exit 0
