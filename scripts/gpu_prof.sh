#!/bin/bash
# One GPU-box pass: (optional) parity tests, the default bench line (headline +
# workloads), then per workload a single-workload bench line, rocprofv3 kernel
# stats, PMC FETCH/WRITE passes and one SQ pass.  Every GPU step has its own
# time limit; the script stops at the first failing step.
#   usage: scripts/gpu_prof.sh tag "wl1 wl2 ..." [tests] [full]
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
if [ -n "${4:-}" ]; then
  timeout -k 10 900 python -u bench.py --detail "$O/bench_detail.json" > "$O/bench_full.log" 2>&1
  step bench_full $?
fi
for WL in $WLS; do
  timeout -k 10 300 python -u bench.py --workload "$WL" --only --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_$WL.log" 2>&1
  step "bench_$WL" $?
  B="python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$WL" -o kt -- $B > "$O/kt_$WL.log" 2>&1
  step "kt_$WL" $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$WL" -o fetch --output-format csv -- $B > "$O/fetch_$WL.log" 2>&1
  step "fetch_$WL" $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$WL" -o write --output-format csv -- $B > "$O/write_$WL.log" 2>&1
  step "write_$WL" $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d "$O/sq_$WL" -o sq --output-format csv -- $B > "$O/sq_$WL.log" 2>&1
  step "sq_$WL" $?
  cd "$GRAFT_REPO_ROOT"
done
exit 0
