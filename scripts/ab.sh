# A/B of library variants on the C2 bench (device-resident inflate + deflate);
# usage: VARIANTS="old r4t2" bash scripts/ab.sh   ("" = default library)
cd $GRAFT_REPO_ROOT
for v in $VARIANTS default; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh ab_$v 200 \
    "'inflate', d['value'], d['roofline']['kernel_ms'], d['parity_ok'], '| deflate', d.get('deflate',{}).get('deflate_value'), d.get('deflate',{}).get('roundtrip_ok')" \
    --steps 10 --warmup 2 --no-cpu-baseline ${AB_ARGS} || exit 1
done
