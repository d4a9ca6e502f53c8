#!/bin/bash
# C1: parse segment floor of history chunks 32 (default) / 24 / 16 -- latency and wire bytes
# (ws_echo links beast_amd/libbeast_pmd.so itself, so each variant is copied over it in this scratch tree)
set -o pipefail
mkdir -p gpurun_out
T=r05zzs
O=gpurun_out/${T}_ab.log
: > $O
cp beast_amd/libbeast_pmd.so /tmp/base_pmd.so
for r in 1 2; do
  for v in base h24 h16; do
    if [ $v = base ]; then cp /tmp/base_pmd.so beast_amd/libbeast_pmd.so; else cp beast_amd/libbeast_pmd_$v.so beast_amd/libbeast_pmd.so; fi
    echo "== round $r $v" >> $O
    timeout -k 10 120 python scripts/facade_latency.py 256 >> $O 2>&1 || { echo "lat failed"; tail $O; exit 1; }
    timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread >> $O 2>&1 || { echo "c1 failed"; tail $O; exit 2; }
  done
done
cp /tmp/base_pmd.so beast_amd/libbeast_pmd.so
grep -E "==|facade per|C1 echo" $O
