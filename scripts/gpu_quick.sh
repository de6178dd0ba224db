#!/bin/bash
# One GPU-box pass for iteration: selected parity tests (-k EXPR), then
# single-workload bench lines.  Each GPU step has its own time limit; the
# script stops at the first failing step.
#   usage: scripts/gpu_quick.sh tag "pytest -k expr" "wl1 wl2 ..."
set -u
cd "$GRAFT_REPO_ROOT"
TAG=$1
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "$2" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "$2" > "$O/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
for w in $3; do
  timeout -k 10 240 python -u bench.py --workload "$w" --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    --detail "$O/d_$w.json" > "$O/bench_$w.log" 2>&1
  rc=$?; echo "bench_$w rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
