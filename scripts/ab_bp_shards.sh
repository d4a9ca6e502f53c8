# block-parallel 8-way projection A/B of library variants: LEGS=c5_l1,c5_l6 VARIANTS="a b" bash scripts/ab_bp_shards.sh
cd $GRAFT_REPO_ROOT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh abs_$v 500 \
    "'$v', {k: (v['inflate_value'], {n: (s['inflate_shard_ms'] if 'inflate_shard_ms' in s else None, s['inflate_projected_speedup']) for n, s in v['virtual_shards'].items()}, v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --legs ${LEGS:-c5_l1,c5_l6} || exit 1
done
