#!/bin/bash
# round 5: region size (BPMD_BP_SEGS segments per lane) on Beast and own shards
set -o pipefail
TAG=${TAG:-r05h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for segs in 1 2 4; do
  export BPMD_BP_SEGS=$segs
  for cfg in "c4 6 8" "c4 6 4" "c5 1 8"; do
    set -- $cfg
    timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 3 > $OUT/beast_${segs}_$1_$2_$3.log 2>&1 || { tail $OUT/beast_${segs}_$1_$2_$3.log; exit 1; }
    echo "segs $segs beast $(sed -n 2p $OUT/beast_${segs}_$1_$2_$3.log | cut -c1-40) | $(tail -1 $OUT/beast_${segs}_$1_$2_$3.log | cut -c1-110)"
    timeout -k 10 200 python -u scripts/diag_own_shard.py $1 $2 $3 3 > $OUT/own_${segs}_$1_$2_$3.log 2>&1 || { tail $OUT/own_${segs}_$1_$2_$3.log; exit 2; }
    echo "segs $segs own   $(sed -n 2p $OUT/own_${segs}_$1_$2_$3.log | cut -c1-40) | $(tail -1 $OUT/own_${segs}_$1_$2_$3.log | cut -c1-110)"
  done
done
