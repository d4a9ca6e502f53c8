# SQ counters of the C2 lane-kernel launch for both lane designs (A/B):
# instruction mix and issue vs wait.  -> gpurun_out/sq_lane/<design>_p{1,2}
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/sq_lane
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for d in ${DESIGNS:-1 2}; do
  BPMD_LANE=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --output-format csv -d $OUT -o d${d}_p1 -- python3 $ROOT/scripts/ab_lane.py > $OUT/d${d}_p1.log 2>&1 || exit 2
  BPMD_LANE=$d timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_SMEM \
    --output-format csv -d $OUT -o d${d}_p2 -- python3 $ROOT/scripts/ab_lane.py > $OUT/d${d}_p2.log 2>&1 || exit 3
done
python3 $ROOT/scripts/sq_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
