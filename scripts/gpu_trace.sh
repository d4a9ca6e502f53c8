#!/bin/bash
# kernel trace only (no PMC passes) of leg_profile legs: gpurun_out/prof_<TAG>/<leg>_<op>_kernels.csv
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lo in "$@"; do
  leg=${lo%%:*}; op=${lo##*:}; n=${leg}_${op}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o trace \
    -- python3 $ROOT/scripts/leg_profile.py --leg $leg --op $op --steps 5 >> $OUT/log.txt 2>> $OUT/err.log || exit 2
  python3 $ROOT/scripts/kernel_summary.py $(find $OUT/$n -name 'trace_kernel_trace.csv' | head -1) > $OUT/${n}_kernels.csv || exit 5
  echo "== $n"; python3 -c "
import csv,sys
for x in csv.DictReader(open('$OUT/${n}_kernels.csv')):
    print(f\"{x['kernel'][:60]:60s} {x['calls']:>4} {int(x['median_ns_warm'])/1e6:9.3f} ms\")"
done
cat $OUT/log.txt
