#!/bin/bash
# stored block before the stripped sync header: A/B on the shards (own and Beast payloads)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zs}
for round in 1 2; do
for v in default ts0; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_${v}_$round 900 \
    "{k: (v['inflate_value'], v['inflate_beast_value'], {n: (max(y['inflate_shard_ms']), max(y['inflate_beast_shard_ms'])) for n, y in v['virtual_shards'].items()}) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate || exit 2
done
done
