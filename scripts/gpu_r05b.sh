#!/bin/bash
# GPU suite, lean workload lines, then per-phase clocks of an FSG_LEAN_TIMING build (box only)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1 || exit $?
for W in ${2:-c2-substring c1-regex c2-json c3-filter-map}; do
  timeout -k 10 300 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
[ -n "${3:-}" ] || exit 0
make -B -C fluvio_amd/csrc -j16 EXTRA=-DFSG_LEAN_TIMING > $O/make.log 2>&1 || exit $?
for W in ${2:-c2-substring c1-regex c2-json}; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/$W.out 2> $O/$W.perr || exit $?
done
