#!/bin/bash
# A/B of an env-selected kernel variant: the GPU suite, then the headline
# bench with the default build and with env $2=1, then a kernel trace
#   usage: scripts/gpu_ab.sh OUT ENVVAR [workload]
set -e
o=gpurun_out/$1
V=$2
W=${3:-c2-substring}
mkdir -p $o
B="python -u bench.py --only --no-cpu-baseline --no-e2e --workload $W"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/t.log 2>&1
timeout -k 10 200 $B > $o/a.json
env $V=1 timeout -k 10 200 $B > $o/b.json
timeout -k 10 200 $B > $o/c.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --only --no-cpu-baseline --no-e2e --workload $W --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/$o/kt.log 2>&1
