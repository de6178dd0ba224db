#!/bin/bash
# GPU-box pass: a subset of the parity tests selected by -k (plus the smoke).
#   usage: scripts/gpu_tests_k.sh tag "k-expression"
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$2" > "$O/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc" >> "$O/steps.log"
exit $rc
