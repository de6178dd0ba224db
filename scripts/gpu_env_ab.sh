#!/bin/bash
# A/B of one environment knob on single-workload bench lines:
#   scripts/gpu_env_ab.sh tag VAR "v1 v2 ..." "wl1 wl2 ..." [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; VAR=$2; VALS=$3; WLS=$4
mkdir -p "$O"
if [ -n "${5:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "$5" > "$O/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && exit $rc
fi
for w in $WLS; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 240 python -u bench.py --workload "$w" --only --steps 10 --warmup 2 --no-cpu-baseline \
      --no-e2e --detail "$O/d_${w}_$v.json" > "$O/b_${w}_$v.log" 2>&1
    rc=$?; echo "$w $v rc=$rc" >> "$O/steps.log"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
