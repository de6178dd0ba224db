#!/bin/bash
# parity subset + an A/B of one env switch on the headline: kernel traces with and without it
#   usage: scripts/gpu_ab.sh tag ENV_VAR "pytest -k expr"
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$3" > "$O/t.log" 2>&1 || exit $?
B="python3 $GRAFT_REPO_ROOT/bench.py --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/new" -o kt -- $B > "$O/new.log" 2>&1 || exit $?
env "$2=1" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/old" -o kt -- $B > "$O/old.log" 2>&1
