# interleaved C2 A/B of library variants (inflate only): VARIANTS="a b" ROUNDS=2 bash scripts/ab_inflate.sh
cd $GRAFT_REPO_ROOT
for r in $(seq ${ROUNDS:-2}); do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L bash scripts/run_bench.sh abi_${v}_$r 200 "'$v', d['value'], d['roofline']['kernel_ms'], d['parity_ok']" \
      --steps 20 --warmup 3 --no-cpu-baseline --no-deflate --no-mixed --no-frame || exit 1
  done
done
