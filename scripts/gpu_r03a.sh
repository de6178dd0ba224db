#!/bin/bash
# Round-3 iteration pass: focused parity tests (-k filter), then the headline
# bench with the register-resident path and with FSG_NO_FLAT=1, then kernel
# stats of the headline.  Each GPU step has its own limit; stop at the first failure.
#   usage: scripts/gpu_r03a.sh tag "pytest -k expr"
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
K=${2:-flat}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$O/gpu_tests.log" 2>&1
step tests $?
timeout -k 10 300 python -u bench.py --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_flat.log" 2>&1
step bench_flat $?
FSG_NO_FLAT=1 timeout -k 10 300 python -u bench.py --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_lean.log" 2>&1
step bench_lean $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$O/kt.log" 2>&1
step kt $?
exit 0
