#!/bin/bash
# SQ counters of the aggregate-json order walk (one c5-keyed-agg step)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/p1 -o p1 -- python3 bench.py --workload c5-keyed-agg --only --steps 1 --warmup 0 --no-cpu-baseline > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC --output-format csv -d $O/p2 -o p2 -- python3 bench.py --workload c5-keyed-agg --only --steps 1 --warmup 0 --no-cpu-baseline > $O/p2.log 2>&1
