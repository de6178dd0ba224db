#!/bin/bash
# Quick GPU-box pass: parity tests, then one bench line per workload (no profiler).
#   usage: scripts/gpu_quick.sh tag "wl1 wl2 ..." [tests]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
WLS=$2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ -n "${3:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
  step tests $?
fi
for WL in $WLS; do
  timeout -k 10 300 python -u bench.py --workload "$WL" --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_$WL.log" 2>&1
  step "bench_$WL" $?
done
exit 0
