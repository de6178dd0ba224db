#!/bin/bash
# C4 (array_map) check: the array parity tests, the c4 bench line, a kernel-trace profile
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "array" > $O/t.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload c4-array-map --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/c4.json 2> $O/c4.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload c4-array-map --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt.log 2>&1
