#!/bin/bash
# flat-path tests first, the GPU suite, lean workload lines (+ c2 with the flat path off), one PMC pass
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "flat" > $O/tflat.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1 || exit $?
for W in c2-substring c1-regex c2-json c3-filter-map; do
  timeout -k 10 300 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
FSG_WRITE_LDS=1 timeout -k 10 300 python -u bench.py --workload c2-substring --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/c2-noflat.json 2> $O/c2-noflat.err || exit $?
B="python3 $GRAFT_REPO_ROOT/bench.py --workload c2-substring --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B > "$O/kt.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$O/ic" -o ic --output-format csv -- $B > "$O/ic.log" 2>&1
echo "ic rc=$?" >> $O/steps.log
