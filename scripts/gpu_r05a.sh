#!/bin/bash
# round 5, first GPU pass: the whole GPU suite, then bench lines for the
# changed measurement paths (C5 step roofline, order_ms, fetch step)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1 || exit $?
for W in c2-substring c5-agg-sum c5-keyed-agg; do
  timeout -k 10 300 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
