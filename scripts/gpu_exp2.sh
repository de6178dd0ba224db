#!/bin/bash
# GPU-box experiment: the k_write_lean toggle on the 1 KB-record workloads, and f3.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
step() { echo "$1 rc=$2" >> "$O/steps.log"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
timeout -k 10 300 python -u bench.py --workload f3-one-record --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_f3.log" 2>&1
step f3 $?
for WL in c2-substring c3-filter-map c2-json; do
  FSG_WRITE_LEAN=1 timeout -k 10 300 python -u bench.py --workload $WL --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$O/bench_${WL}_wlean.log" 2>&1
  step "wlean_$WL" $?
done
exit 0
