#!/bin/bash
# experiment: the lean kernel built as committed vs with EXTRA=$2 (made on the box), c2-substring / c1 / fetch lines
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
for V in base alt; do
  if [ $V = alt ]; then make -B -C fluvio_amd/csrc -j16 EXTRA="$2" > $O/make.log 2>&1 || exit $?; fi
  for W in ${3:-c2-substring c1-regex}; do
    timeout -k 10 200 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$V-$W.json 2> $O/$V-$W.err || exit $?
  done
done
