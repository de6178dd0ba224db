#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "crc or kat or random_parity" > "$O/gpu_tests.log" 2>&1
step tests $?
for WL in c2-substring c2-json; do
  timeout -k 10 300 python -u bench.py --workload $WL --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_$WL.log" 2>&1
  step "bench_$WL" $?
done
exit 0
