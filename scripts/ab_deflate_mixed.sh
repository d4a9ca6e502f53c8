# C4/C5 deflate A/B of library variants (whole batches): rate and C4 size vs Beast (ratio 0.2855)
cd $GRAFT_REPO_ROOT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh abm_$v 400 \
    "'$v', {k: (v['deflate_value'], v['inflate_value'], round(v['ratio_rank_local'] / (0.2855 if k == 'c4_l6' else 1), 4), v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-virtual-shards || exit 1
done
