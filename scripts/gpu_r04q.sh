#!/bin/bash
# round-4 profiles: kernel traces of the headline, c4, f3 and c5k benches; decompression timing
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for W in c2-substring c4-array-map c2-json c1-regex; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$W -o kt -- python3 bench.py --workload $W --only --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/kt_$W.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_f3 -o kt -- python3 bench.py --workload f3-one-record --only --steps 1 --warmup 0 --no-cpu-baseline > $O/kt_f3.log 2>&1 || exit $?
timeout -k 10 300 python3 tests/perf_decompress.py > $O/perf_decompress.json 2> $O/perf_decompress.err
