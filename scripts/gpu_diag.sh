#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o kt -- python3 $R/scripts/diag_lean.py 1000000 > $R/$O/kt.log 2>&1 || exit $?
for C in substr json; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/$O/sq_$C -o sq --output-format csv -- python3 $R/scripts/diag_lean.py 1000000 $C > $R/$O/sq_$C.log 2>&1 || exit $?
done
