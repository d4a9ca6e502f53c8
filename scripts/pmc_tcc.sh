#!/bin/bash
# L2 (TCC) and L1 (TCP) counters of the inflate lane kernel on C2 and on the
# whole C4 batch, one rocprofv3 pass per counter group (each within the
# per-pass block limits: <= 4 TCC, <= 4 TCP).
# Usage: TAG=r06a bash scripts/pmc_tcc.sh  -> gpurun_out/tcc_<TAG>/{c2,c4}_tcc.csv
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
OUT=$ROOT/gpurun_out/tcc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=("TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
        "TCC_READ_sum TCC_WRITE_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum")
for w in c2 c4; do
  if [ $w = c2 ]; then
    CMD="python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact"
  else
    CMD="python3 $ROOT/scripts/leg_profile.py --leg c4_l6 --op inflate --steps 2"
  fi
  files=()
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d $OUT/$w -o p$i -- $CMD > /dev/null 2>> $OUT/err.log || { tail -5 $OUT/err.log; exit 2; }
    files+=($(find $OUT/$w -name "p${i}_counter_collection.csv" | head -1))
  done
  python3 $ROOT/scripts/pmc_summary.py "${files[@]}" > $OUT/${w}_tcc.csv || exit 3
  python3 - $OUT/${w}_tcc.csv <<'EOF'
import csv, sys, collections, statistics
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "inflate_lane3" in r["kernel"]:
        acc[r["counter"]].append(float(r["value_kB"]))
for c, v in sorted(acc.items()):
    print(sys.argv[1].split("/")[-1], "inflate_lane3_kernel", c, "median over", len(v), "launches:", statistics.median(v))
EOF
done
echo done
