# SQ counters (issue vs wait breakdown, instruction mix, LDS conflicts) for
# the bench workload's kernels, one counter pass per rocprofv3 run.
# Usage: TAG=r01 bash scripts/pmc_sq.sh     -> gpurun_out/sq_<TAG>/
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p $OUT
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --output-format csv -d $OUT -o p1 -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > /dev/null 2> $OUT/p1.err || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES \
  --output-format csv -d $OUT -o p2 -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > /dev/null 2> $OUT/p2.err || exit 3
echo done
