#!/bin/bash
# f3: process() parity tests, the one-record bench and its kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "process or ingest or one_record" > $O/t.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload f3-one-record --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/f3.json 2> $O/f3.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_f3 -o kt -- python3 bench.py --workload f3-one-record --only --steps 1 --warmup 0 --no-cpu-baseline > $O/kt_f3.log 2>&1
