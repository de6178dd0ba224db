#!/bin/bash
# Round-3 pass: focused GPU tests (-k), then bench workloads given as further
# arguments (each with --only), every GPU step under its own limit.
#   usage: scripts/gpu_r03c.sh tag "pytest -k expr" [workload ...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
K=$2
shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$O/gpu_tests.log" 2>&1
  step tests $?
fi
for WL in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$O/bench_$WL.log" 2>&1
  step "bench_$WL" $?
done
exit 0
