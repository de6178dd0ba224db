#!/bin/bash
# JSON lean path: filter_json / projection parity tests, then the c2-json and c3 bench lines
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "json or project or lean or c3" > $O/t.log 2>&1 || exit $?
for W in c2-json c3-filter-map; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
