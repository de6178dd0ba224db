#!/bin/bash
# GPU-box pass: parity tests, then the default bench line (headline + every
# workload, CPU baselines on the box's cores) exactly as the driver runs it.
#   usage: scripts/gpu_bench_full.sh tag
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
step tests $?
timeout -k 10 900 python -u bench.py > "$O/bench_full.log" 2>&1
step bench_full $?
exit 0
