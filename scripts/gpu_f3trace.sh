#!/bin/bash
# GPU-box: HIP API + kernel trace of the one-record process() path.  usage: scripts/gpu_f3trace.sh tag
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$O/prof" -o f3 -- python3 bench.py --workload f3-one-record --only --steps 1 --warmup 0 --no-cpu-baseline > "$O/bench_f3.log" 2>&1
echo "rc=$?" >> "$O/steps.log"
exit 0
