# interleaved C3 deflate A/B of chain-cap variants: rate and size vs Beast
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-frame --no-exact 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['deflate']; print('$v', 'deflate', x['deflate_value'], 'size', round(x['ratio'] / 0.3409, 4), 'rt', x['roundtrip_ok'], 'inflate', d['value'])" || exit 1
  done
done
