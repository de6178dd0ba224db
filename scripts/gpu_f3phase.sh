#!/bin/bash
# experiment: k_one phase timestamps (a build with FSG_ONE_TIMING made on the box only)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
make -B -C fluvio_amd/csrc -j16 EXTRA=-DFSG_ONE_TIMING > $O/make.log 2>&1 || exit $?
grep -q "s_store" fluvio_amd/csrc/*.s 2>/dev/null && exit 3
timeout -k 10 200 python -u bench.py --workload f3-one-record --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/f3.json 2> $O/f3.err
