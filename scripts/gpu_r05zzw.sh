#!/bin/bash
# C1 with and without hdr_par, interleaved (ws_echo inherits BPMD_ZSTREAM_HPAR)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05zzw_c1_hpar_ab.log
: > $O
for r in 1 2 3; do
  for hp in 1 0; do
    echo "== round $r hpar $hp" >> $O
    BPMD_ZSTREAM_HPAR=$hp timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread >> $O 2>&1 || { echo "c1 failed"; tail $O; exit 1; }
  done
done
grep -E "==|C1 echo" $O
