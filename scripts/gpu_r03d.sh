#!/bin/bash
# Round-3: the default bench line (as the driver runs it), then per-workload
# kernel stats for the workloads given as arguments.  Each GPU step has its own limit.
#   usage: scripts/gpu_r03d.sh tag [workload ...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 600 python -u bench.py > "$O/bench_full.log" 2>&1
step bench_full $?
cd /tmp
for WL in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$WL" -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$O/kt_$WL.log" 2>&1
  step "kt_$WL" $?
done
exit 0
