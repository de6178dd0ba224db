#!/bin/bash
# c5k: keyed / aggregate-json parity tests, then the c5-keyed-agg bench and its kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "aggj or aggregate_json or keyed or group" > $O/t.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5-keyed-agg --only --steps 3 --warmup 1 --no-cpu-baseline > $O/c5k.json 2> $O/c5k.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload c5-keyed-agg --only --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1
