#!/bin/bash
# HIP runtime API trace + kernel trace of one single-workload bench run: gpu_rt.sh tag workload [steps]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
B="python3 $GRAFT_REPO_ROOT/bench.py --workload $2 --only --steps ${3:-5} --warmup 1 --no-cpu-baseline --no-e2e --detail $O/d_$2.json"
cd /tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d "$O/rt_$2" -o rt -- $B > "$O/rt_$2.log" 2>&1
