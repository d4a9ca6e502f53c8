# Kernel-trace statistics and HBM traffic counters for the bench workload.
# Writes CSV summaries under gpurun_out/prof_<tag>/ (copy the ones to keep
# into profiles/).  Usage: TAG=r01 bash scripts/profile.sh
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
mkdir -p $ROOT/gpurun_out
python -c "import __graft_entry__ as g; g.build()" > $ROOT/gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o trace \
  -- python3 $ROOT/bench.py $BENCH_ARGS > $ROOT/gpurun_out/prof_$TAG.bench.json 2> $ROOT/gpurun_out/prof_$TAG.err || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o fetch \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $ROOT/gpurun_out/prof_$TAG.err || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o write \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $ROOT/gpurun_out/prof_$TAG.err || exit 4
echo done
