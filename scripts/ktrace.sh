#!/bin/bash
# rocprofv3 kernel trace + stats of the C2-only bench for one library
# variant: TAG=x [BPMD_LIB=...] bash scripts/ktrace.sh -> gpurun_out/kt_<TAG>/stats.csv
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/kt_${TAG:-run}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace \
  -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact \
  > $OUT/bench.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 2; }
f=$(find $OUT -name 'trace_kernel_stats.csv' | head -1)
cp $f $OUT/stats.csv
python3 -c "
import csv,sys
for r in csv.DictReader(open('$OUT/stats.csv')):
    n=r['Name'].split('(')[0][-60:]
    print(f\"{n:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:10.1f}\")
"
