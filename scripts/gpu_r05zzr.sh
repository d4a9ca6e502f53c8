#!/bin/bash
# facade: polling the stream vs hipStreamSynchronize, interleaved; then C1 both ways
set -o pipefail
mkdir -p gpurun_out
T=r05zzr
O=gpurun_out/${T}_lat.log
: > $O
for r in 1 2 3; do
  for sp in 1 0; do
    echo "== round $r spin $sp" >> $O
    BPMD_STREAM_SPIN=$sp timeout -k 10 120 python scripts/facade_latency.py 256 >> $O 2>&1 || { echo "lat failed"; tail $O; exit 1; }
  done
done
for sp in 1 0; do
  echo "== C1 spin $sp" >> $O
  BPMD_STREAM_SPIN=$sp timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread >> $O 2>&1 || { echo "c1 failed"; tail $O; exit 2; }
done
grep -E "==|facade per|C1 echo" $O
