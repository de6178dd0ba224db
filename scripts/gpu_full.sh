#!/bin/bash
# the driver's default bench (all workloads, CPU baselines), then its kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
