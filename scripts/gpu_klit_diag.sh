# KLIT 4 vs 2: per-role loop counters (prof builds) and SQ instruction/wait counters (product builds)
set -o pipefail
OUT=gpurun_out/klit; mkdir -p $OUT
for v in prof profk2; do
  BPMD_LIB=beast_amd/libbeast_pmd_$v.so timeout -k 10 200 python -u scripts/diag_lane3.py > $OUT/diag_$v.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in default klit2; do
  if [ $v = default ]; then L=$GRAFT_REPO_ROOT/beast_amd/libbeast_pmd.so; else L=$GRAFT_REPO_ROOT/beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sq_$v -o p1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/p1_$v.err || exit 2
  BPMD_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES \
    --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sq_$v -o p2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame > /dev/null 2> $GRAFT_REPO_ROOT/$OUT/p2_$v.err || exit 3
done
cd $GRAFT_REPO_ROOT
for v in default klit2; do echo "== $v"; python scripts/sq_summary.py $OUT/sq_$v; done > $OUT/sq_summary.txt
tail -n +1 $OUT/diag_*.txt $OUT/sq_summary.txt
