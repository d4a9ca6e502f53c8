# A/B of library variants on the C2 bench (device-resident inflate + deflate);
# usage: VARIANTS="old r4t2" bash scripts/ab.sh   ("" = default library)
cd $GRAFT_REPO_ROOT
for v in $VARIANTS default; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  echo "== $v"
  BPMD_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${AB_ARGS} 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); x=d.get('deflate',{}); print('inflate', d['value'], d['roofline']['kernel_ms'], d['parity_ok'], '| deflate', x.get('deflate_value'), x.get('roundtrip_ok'))" || exit 1
done
