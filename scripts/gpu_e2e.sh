#!/bin/bash
# pipelined process_batch: its parity tests, then the c2 line with the e2e figure
#   usage: scripts/gpu_e2e.sh tag [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "${2:-pipelined}" > "$O/tests.log" 2>&1
rc=$?; echo "tests rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c2-substring --only --steps 10 --warmup 2 --no-cpu-baseline \
  --detail "$O/d_c2.json" > "$O/bench_c2.log" 2>&1
rc=$?; echo "bench rc=$rc" >> "$O/steps.log"; exit $rc
