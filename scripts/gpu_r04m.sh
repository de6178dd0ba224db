#!/bin/bash
# round-4 check: array / process() parity, then the c4, f3 and headline benches and a c4 kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "array or process or ingest or one_record or crc or reframe or max_bytes or filter" > $O/t.log 2>&1 || exit $?
for W in c4-array-map f3-one-record c2-substring; do
  timeout -k 10 200 python -u bench.py --workload $W --only --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$W.json 2> $O/$W.err || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload c4-array-map --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt.log 2>&1
