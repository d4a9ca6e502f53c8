#!/bin/bash
# round 5: Beast-payload shards -- kernel split and scan counters; e2e rate
set -o pipefail
TAG=${TAG:-r05d}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
for cfg in "c5 1 8" "c4 6 4" "c4 6 8"; do
  set -- $cfg
  timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 3 > $OUT/diag_$1_$2_$3.log 2>&1 || { tail $OUT/diag_$1_$2_$3.log; exit 1; }
  cat $OUT/diag_$1_$2_$3.log
  BPMD_LIB=beast_amd/libbeast_pmd_bpdiag.so timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 2 > $OUT/bpdiag_$1_$2_$3.log 2>&1 || exit 2
  tail -1 $OUT/bpdiag_$1_$2_$3.log
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1_$2_$3 -o t \
    -- python3 $ROOT/scripts/diag_beast_shard.py $1 $2 $3 3 > /dev/null 2>&1) || exit 3
  python3 scripts/kernel_summary.py $(find $OUT/prof_$1_$2_$3 -name "t_kernel_trace.csv" | head -1) > $OUT/kernels_$1_$2_$3.csv || exit 4
  head -20 $OUT/kernels_$1_$2_$3.csv
done
timeout -k 10 300 python -u scripts/e2e.py > $OUT/e2e.json 2> $OUT/e2e.err || { tail $OUT/e2e.err; exit 5; }
cat $OUT/e2e.json
