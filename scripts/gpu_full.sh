#!/bin/bash
# One GPU-box pass: parity tests, bench (with CPU baseline), rocprofv3 kernel
# stats of the same bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE)
# for the roofline `traffic` figure.  Every GPU step has its own time limit and
# the script stops at the first failing step.
#   usage: scripts/gpu_full.sh [tag] [workload] [skip-tests]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}
WL=${2:-c2-substring}
SKIP=${3:-}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ -z "$SKIP" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
  step tests $?
fi
timeout -k 10 300 python -u bench.py --workload "$WL" --steps 10 --warmup 2 > "$O/bench.log" 2>&1
step bench $?
B="python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B > "$O/kt.log" 2>&1
step kt $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o fetch --output-format csv -- $B > "$O/fetch.log" 2>&1
step fetch $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o write --output-format csv -- $B > "$O/write.log" 2>&1
step write $?
exit 0
