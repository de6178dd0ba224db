#!/bin/bash
# c5-agg-sum under host-thread and hardware-queue settings: gpu_c5ab.sh OUT
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --workload c5-agg-sum --only --no-cpu-baseline --no-e2e --steps 10 --warmup 2 --detail $o/q$q.json > $o/q$q.log 2>&1 || exit 1
done
