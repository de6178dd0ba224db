#!/bin/bash
# round-4 check: GPU parity suite, then c2-substring / c2-json / c3 benches and the c5 pair
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1 || exit $?
for W in c2-substring c2-json c3-filter-map; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
bash scripts/gpu_c5k_prof.sh $1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5-agg-sum --only --steps 3 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
