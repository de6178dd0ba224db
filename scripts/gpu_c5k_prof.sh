#!/bin/bash
# c5-keyed-agg kernel trace + one SQ pass (k_aggj_order_group's per-record cost)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
B="python3 $GRAFT_REPO_ROOT/bench.py --workload c5-keyed-agg --only --steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B > "$O/kt.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS -d "$O/sq" -o sq --output-format csv -- $B > "$O/sq.log" 2>&1
