#!/bin/bash
# deflate: chain-step budget per parse lane (C4/C5 rate and size), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
for round in 1 2; do
for v in default cb192 cb160 cb128; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh r05v_${v}_$round 400 \
    "{k: (v['deflate_value'], round(v['ratio_rank_local'] / {'c4_l6': 0.2857, 'c5_l1': 0.9856, 'c5_l6': 0.9700}[k], 4), v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-virtual-shards --no-beast-payloads || exit 1
done
done
