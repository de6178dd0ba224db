#!/bin/bash
# FETCH_SIZE calibration (scripts/fetch_calib.hip, prebuilt into tools_bin/)
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o fetch --output-format csv -- "$GRAFT_REPO_ROOT/tools_bin/fetch_calib" > "$O/fetch.log" 2>&1
echo "fetch rc=$?" >> "$O/steps.log"
