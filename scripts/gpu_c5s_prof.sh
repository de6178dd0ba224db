#!/bin/bash
# c5-agg-sum kernel trace: where a step's time goes (kernels vs host gaps)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
B="python3 $GRAFT_REPO_ROOT/bench.py --workload c5-agg-sum --only --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B > "$O/kt.log" 2>&1
