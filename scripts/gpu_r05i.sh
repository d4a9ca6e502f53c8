#!/bin/bash
# round 5: per-stream facade latency breakdown (host times + kernel trace)
set -o pipefail
TAG=${TAG:-r05i}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python -u scripts/facade_latency.py 256 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
cat $OUT/lat.log | grep facade
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o t \
    -- python3 $GRAFT_REPO_ROOT/scripts/facade_latency.py 256 > /dev/null 2>&1) || exit 2
python3 scripts/kernel_summary.py $(find $OUT/prof -name "t_kernel_trace.csv" | head -1) > $OUT/kernels.csv || exit 3
head -20 $OUT/kernels.csv
