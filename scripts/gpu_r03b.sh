#!/bin/bash
# Round-3 iteration pass: focused parity tests (-k), then the headline bench with
# the default library and with each variant library under fluvio_amd/_lib_exp/*,
# then kernel stats of the headline.  Each GPU step has its own limit.
#   usage: scripts/gpu_r03b.sh tag "pytest -k expr" [workload]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
K=${2:-flat}
WL=${3:-c2-substring}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$O/gpu_tests.log" 2>&1
  step tests $?
fi
B="--workload $WL --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u bench.py $B > "$O/bench_default.log" 2>&1
step bench_default $?
for d in fluvio_amd/_lib_exp/*/; do
  v=$(basename "$d")
  [ -f "$d/libfsg.so" ] || continue
  FSG_LIB="$GRAFT_REPO_ROOT/$d/libfsg.so" timeout -k 10 300 python -u bench.py $B > "$O/bench_$v.log" 2>&1
  step "bench_$v" $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$O/kt.log" 2>&1
step kt $?
exit 0
