#!/bin/bash
# A/B of libfsg.so builds: the in-tree build (tests + bench) against older
# builds kept side by side (FSG_LIB selects the library), bench lines
# alternating.  usage: scripts/gpu_lib_ab.sh OUT DIR1 [DIR2 ...] (dirs under fluvio_amd/)
set -e
o=gpurun_out/$1; shift
mkdir -p $o
B="python -u bench.py --only --no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $o/t.log 2>&1
timeout -k 10 200 $B > $o/base.json
for d in "$@"; do
  FSG_LIB=$PWD/fluvio_amd/$d/libfsg.so timeout -k 10 200 $B > $o/$d.json
done
timeout -k 10 200 $B > $o/base2.json
