# rocprofv3 evidence for every timed op of bench.py besides C2 (scripts/profile.sh):
# for each leg/op of scripts/leg_profile.py
#   --kernel-trace --stats          -> <tag>_<leg>_<op>_kernels.csv (median of warm launches)
#   FETCH_SIZE, WRITE_SIZE (passes) -> <tag>_<leg>_<op>_pmc.csv
# Writes under gpurun_out/prof_<tag>/ (copy into profiles/ to keep).
# Usage: TAG=r03c bash scripts/profile_legs.sh [leg:op ...]
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
LIST=${@:-c3:deflate c4_l6:deflate c4_l6:inflate c5_l1:deflate c5_l1:inflate c5_l6:deflate c5_l6:inflate}
for lo in $LIST; do
  leg=${lo%%:*}; op=${lo##*:}; n=${leg}_${op}
  echo "== $n"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o trace \
    -- python3 $ROOT/scripts/leg_profile.py --leg $leg --op $op --steps 5 >> $OUT/log.txt 2>> $OUT/err.log || exit 2
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$n -o fetch \
    -- python3 $ROOT/scripts/leg_profile.py --leg $leg --op $op --steps 3 >> $OUT/log.txt 2>> $OUT/err.log || exit 3
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$n -o write \
    -- python3 $ROOT/scripts/leg_profile.py --leg $leg --op $op --steps 3 >> $OUT/log.txt 2>> $OUT/err.log || exit 4
  python3 $ROOT/scripts/kernel_summary.py $(find $OUT/$n -name 'trace_kernel_trace.csv' | head -1) > $OUT/${n}_kernels.csv || exit 5
  cp $(find $OUT/$n -name 'trace_kernel_stats.csv' | head -1) $OUT/${n}_kernel_stats.csv
  python3 $ROOT/scripts/pmc_summary.py $(find $OUT/$n -name 'fetch_counter_collection.csv') \
    $(find $OUT/$n -name 'write_counter_collection.csv') > $OUT/${n}_pmc.csv || exit 6
done
echo done
