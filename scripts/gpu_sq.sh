#!/bin/bash
# One SQ counter pass (+ kernel trace) per workload: gpu_sq.sh tag "wl1 wl2"
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
for WL in $2; do
  B="python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --detail $O/d_$WL.json"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$WL" -o kt -- $B > "$O/kt_$WL.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU -d "$O/sq_$WL" -o sq --output-format csv -- $B > "$O/sq_$WL.log" 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT"
done
