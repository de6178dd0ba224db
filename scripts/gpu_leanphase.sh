#!/bin/bash
# experiment: k_eval_lean per-phase clock sums (a build with FSG_LEAN_TIMING made on the box only)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
make -B -C fluvio_amd/csrc -j16 EXTRA=-DFSG_LEAN_TIMING > $O/make.log 2>&1 || exit $?
for W in ${2:-c1-regex c2-json c2-substring}; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/$W.out 2> $O/$W.err || exit $?
done
