#!/bin/bash
# kernel stats (rocprofv3 --kernel-trace --stats) of one bench workload, optionally
# with an environment assignment for the bench process
#   usage: scripts/gpu_kt.sh tag workload [VAR=value]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
WL=$2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
[ $# -ge 3 ] && export "$3"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$O/kt.log" 2>&1
echo "kt rc=$?" >> "$O/steps.log"
