#!/bin/bash
# A/B of library variants on the mixed legs (C4 / C5): deflate, inflate of
# this library's and of a Beast peer's payloads, projected 8-way speed-ups.
# Usage: TAG=x VARIANTS="r5 default" LEGS=c5_l1,c5_l6 ROUNDS=1 bash scripts/ab_legs.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-1}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_legs_${v}_$r 600 \
      "'$v', {k: (x['deflate'], x['inflate'], x['inflate_beast'], x.get('x_projected',{}).get('8'), x.get('shard8_ms_max')) for k, x in d['north_star'].items() if k in ('c4_l6', 'c5_l1', 'c5_l6')}, d['parity_ok']" \
      --steps 3 --warmup 1 --no-cpu-baseline --no-deflate --no-frame --no-exact --legs ${LEGS:-c5_l1,c5_l6} || exit 1
  done
done
