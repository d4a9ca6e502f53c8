# block-parallel segments per lane (BPMD_BP_SEGS) x long-payload split (BPMD_LONG_SHARE_PCT) sweep on the mixed legs
cd $GRAFT_REPO_ROOT
E="{k: (v['inflate_value'], {n: (s.get('inflate_shard_ms'), s['inflate_projected_speedup']) for n, s in v['virtual_shards'].items()}, v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}"
for sg in ${SEGS:-3 4 6}; do
  for sh in ${SHARES:-75 100 125}; do
    BPMD_BP_SEGS=$sg BPMD_LONG_SHARE_PCT=$sh bash scripts/run_bench.sh ss_${sg}_${sh} 400 "'segs $sg share $sh', $E" \
      --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --legs ${LEGS:-c4_l6} || exit 1
  done
done
