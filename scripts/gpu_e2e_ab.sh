#!/bin/bash
# e2e (pipelined process_batch) A/B: scripts/gpu_e2e_ab.sh tag "chunk:upthreads ..." (bytes, FSG_PIPE_UP)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p "$O"
for cu in $2; do
  c=${cu%%:*}; u=${cu##*:}
  FSG_PIPE_CHUNK=$c FSG_PIPE_UP=$u timeout -k 10 300 python -u bench.py --workload c2-substring --only --steps 3 \
    --warmup 1 --no-cpu-baseline --detail "$O/d_${c}_$u.json" > "$O/b_${c}_$u.log" 2>&1
  rc=$?; echo "chunk $cu rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
