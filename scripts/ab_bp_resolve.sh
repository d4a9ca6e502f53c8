# A/B of the block-parallel resolve with / without loads ahead (BPMD_BP_RESOLVE_PF) on the mixed legs
# (the switch was removed with the rejected change: profiles/r04zzc_bp_resolve_loads_ahead_rejected.log)
cd $GRAFT_REPO_ROOT
E="{k: (v['inflate_value'], {n: (s.get('inflate_shard_ms'), s['inflate_projected_speedup']) for n, s in v['virtual_shards'].items()}, v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}"
for r in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    BPMD_BP_RESOLVE_PF=$v bash scripts/run_bench.sh rpf_${v}_$r 400 "'$v', $E" \
      --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --legs ${LEGS:-c4_l6,c5_l1} || exit 1
  done
done
