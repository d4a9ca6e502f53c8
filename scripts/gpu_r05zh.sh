#!/bin/bash
# C4 deflate: history / chain-cap trade after the multi-candidate parse (rate and size vs Beast)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zh}
for v in default h2048c64 h4096c32 h4096c16; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_${v} 500 \
    "{k: (v['deflate_value'], round(v['ratio_rank_local'] / {'c4_l6': 0.2857, 'c5_l1': 0.9856, 'c5_l6': 0.9700}[k], 4), v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-virtual-shards --no-beast-payloads || exit 2
done
