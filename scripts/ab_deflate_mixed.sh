# C4/C5 deflate A/B of library variants (whole batches): rate and C4 size vs Beast (ratio 0.2855)
cd $GRAFT_REPO_ROOT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-virtual-shards 2>>gpurun_out/ab_mixed.err \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['mixed']; print('$v', {k: (v['deflate_value'], v['inflate_value'], round(v['ratio_rank_local'] / (0.2855 if k == 'c4_l6' else 1), 4), v['roundtrip_ok']) for k, v in m.items() if isinstance(v, dict)})" || exit 1
done
