#!/bin/bash
# kernel trace + stats of one bench invocation: gpu_kt.sh OUT_NAME [bench args...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" > "$O/kt.log" 2>&1
