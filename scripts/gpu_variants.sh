#!/bin/bash
# A/B of libfsg.so variants built side by side (scripts/build_variant.sh):
# single-workload bench lines, in-tree build first and last.
#   usage: scripts/gpu_variants.sh OUT "wl1 wl2" DIR1 [DIR2 ...]   (dirs under fluvio_amd/)
set -u
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wls=$2; shift 2
mkdir -p $o
for w in $wls; do
  B="python -u bench.py --workload $w --only --no-cpu-baseline --no-e2e --steps 10 --warmup 2"
  timeout -k 10 200 $B --detail $o/base_$w.json > $o/base_$w.log 2>&1 || exit 1
  for d in "$@"; do
    FSG_LIB=$PWD/fluvio_amd/$d/libfsg.so timeout -k 10 200 $B --detail $o/${d}_$w.json > $o/${d}_$w.log 2>&1 || exit 1
  done
done
exit 0
