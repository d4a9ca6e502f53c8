#!/bin/bash
# SQ counters of the C2 inflate launch for library variants (issue vs wait,
# instruction mix, LDS conflicts), one counter pass per rocprofv3 run.
# Usage: VARIANTS="default expmin" TAG=x bash scripts/pmc_lane3.sh -> gpurun_out/sq_<TAG>/
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C2="--steps 2 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame"
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=$ROOT/beast_amd/libbeast_pmd.so; else L=$ROOT/beast_amd/libbeast_pmd_$v.so; fi
  export BPMD_LIB=$L
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --output-format csv -d $OUT/$v -o p1 -- python3 $ROOT/bench.py $C2 > /dev/null 2> $OUT/$v.p1.err || exit 2
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
    --output-format csv -d $OUT/$v -o p2 -- python3 $ROOT/bench.py $C2 > /dev/null 2> $OUT/$v.p2.err || exit 3
done
python3 $ROOT/scripts/sq_summary.py $OUT
