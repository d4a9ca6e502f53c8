# Kernel-trace statistics and HBM traffic counters for the bench workload.
# Writes summaries under gpurun_out/prof_<tag>/ (copy the ones to keep into
# profiles/).  Usage: TAG=r01 bash scripts/profile.sh
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/prof_$TAG
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --no-mixed"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace \
  -- python3 $ROOT/bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/err.log || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mixed > /dev/null 2>> $OUT/err.log || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mixed > /dev/null 2>> $OUT/err.log || exit 4
python3 $ROOT/scripts/pmc_summary.py $(find $OUT -name 'fetch_counter_collection.csv') \
  $(find $OUT -name 'write_counter_collection.csv') > $OUT/pmc.csv || exit 5
cp $(find $OUT -name 'trace_kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
echo done
