#!/bin/bash
# Quick GPU pass: parity tests (optional) + one bench line.  usage: gpu_quick.sh tag [workload] [skip-tests]
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p "$O"
WL=${2:-c2-substring}
if [ -z "${3:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo tests failed; tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -2 "$O/gpu_tests.log"
fi
timeout -k 10 300 python -u bench.py --workload "$WL" --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
