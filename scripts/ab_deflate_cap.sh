# interleaved C3 deflate A/B of chain-cap variants: rate and size vs Beast
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L bash scripts/run_bench.sh abd_${v}_$r 300 \
      "'$v', 'deflate', d['deflate']['deflate_value'], 'size', round(d['deflate']['ratio'] / 0.3409, 4), 'rt', d['deflate']['roundtrip_ok'], 'inflate', d['value']" \
      --steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-frame --no-exact || exit 1
  done
done
