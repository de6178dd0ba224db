#!/bin/bash
# c1: regex parity tests, then the c1-regex bench line and its kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "regex or lean" > $O/t.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload c1-regex --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/c1.json 2> $O/c1.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload c1-regex --only --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt.log 2>&1
