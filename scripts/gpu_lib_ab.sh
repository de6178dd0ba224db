#!/bin/bash
# A/B of libfsg.so builds that differ by a compile-time constant: the headline
# bench line per build (FSG_LIB selects the library), plus the flat-path tests
# on each variant.  usage: scripts/gpu_lib_ab.sh OUT DIR1 [DIR2 ...] (dirs under fluvio_amd/)
set -e
o=gpurun_out/$1; shift
mkdir -p $o
B="python -u bench.py --only --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > $o/base.json
for d in "$@"; do
  FSG_LIB=$PWD/fluvio_amd/$d/libfsg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "flat or substring or filter_init or random" > $o/t_$d.log 2>&1
  FSG_LIB=$PWD/fluvio_amd/$d/libfsg.so timeout -k 10 200 $B > $o/$d.json
done
timeout -k 10 200 $B > $o/base2.json
