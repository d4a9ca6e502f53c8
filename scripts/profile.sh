# rocprofv3 evidence for bench.py's roofline fields, C2 workload only:
#   kernel trace + stats of the C2 bench      -> <tag>_c2_kernel_stats.csv
#   FETCH_SIZE / WRITE_SIZE passes (separate) -> <tag>_c2_pmc.csv
#   FETCH_SIZE over a known 2 GiB read        -> <tag>_fetch_calib.csv
# Writes under gpurun_out/prof_<tag>/ (copy into profiles/ to keep).
# Usage: TAG=r02 bash scripts/profile.sh
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/prof_$TAG
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-deflate --no-frame"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace \
  -- python3 $ROOT/bench.py $C2 > $OUT/bench.json 2> $OUT/err.log || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame \
  > /dev/null 2>> $OUT/err.log || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write \
  -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame \
  > /dev/null 2>> $OUT/err.log || exit 4
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o calib \
  -- python3 $ROOT/scripts/calib_fetch.py > /dev/null 2>> $OUT/err.log || exit 5
python3 $ROOT/scripts/pmc_summary.py $(find $OUT -name 'fetch_counter_collection.csv') \
  $(find $OUT -name 'write_counter_collection.csv') > $OUT/c2_pmc.csv || exit 6
python3 $ROOT/scripts/fetch_calib_summary.py $(find $OUT -name 'calib_counter_collection.csv') \
  > $OUT/fetch_calib.csv || exit 7
cp $(find $OUT -name "trace_kernel_stats.csv" | head -1) $OUT/c2_kernel_stats.csv
python3 $ROOT/scripts/kernel_summary.py $(find $OUT -name "trace_kernel_trace.csv" | head -1) > $OUT/c2_kernels.csv || exit 8
echo done
