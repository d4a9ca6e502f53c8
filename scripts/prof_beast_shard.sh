#!/bin/bash
# kernel trace of one shard of C5 Beast payloads (scripts/diag_beast_shard.py):
# TAG=r06k LEVEL=1 PARTS=8 bash scripts/prof_beast_shard.sh -> gpurun_out/prof_bshard_TAG/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-r06}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_bshard_$TAG
mkdir -p $OUT
n=${LEG:-c5}_l${LEVEL:-1}_p${PARTS:-8}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o trace \
  -- python3 $R/scripts/diag_beast_shard.py ${LEG:-c5} ${LEVEL:-1} ${PARTS:-8} 3 > $OUT/${n}_log.txt 2> $OUT/${n}_err.log || { tail -5 $OUT/${n}_err.log; exit 2; }
cat $OUT/${n}_log.txt
python3 $R/scripts/kernel_summary.py $(find $OUT/$n -name 'trace_kernel_trace.csv' | head -1) > $OUT/${n}_kernels.csv || exit 3
head -20 $OUT/${n}_kernels.csv | cut -c1-160
