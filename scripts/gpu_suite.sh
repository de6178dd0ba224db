#!/bin/bash
# the whole GPU parity suite, then the f3 and headline bench lines
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1 || exit $?
for W in f3-one-record c2-substring c4-array-map c5-keyed-agg; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
