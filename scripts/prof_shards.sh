#!/bin/bash
# kernel traces of one 8-way shard of C4 and of C5 (inflate), current build:
# TAG=r04x bash scripts/prof_shards.sh  -> gpurun_out/prof_shards_TAG/<which>_{kernels,kernel_stats}.csv
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_shards_$TAG
mkdir -p $OUT
for w in ${WHICH:-c4:s8 c5:s8}; do
  n=${w/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o trace \
    -- python3 $R/scripts/diag_shards.py --child $w > $OUT/${n}_log.txt 2> $OUT/${n}_err.log || { tail -5 $OUT/${n}_err.log; exit 2; }
  cat $OUT/${n}_log.txt
  python3 $R/scripts/kernel_summary.py $(find $OUT/$n -name 'trace_kernel_trace.csv' | head -1) > $OUT/${n}_kernels.csv || exit 3
  cp $(find $OUT/$n -name 'trace_kernel_stats.csv' | head -1) $OUT/${n}_kernel_stats.csv
  head -16 $OUT/${n}_kernels.csv | cut -c1-150
done
