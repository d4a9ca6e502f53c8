#!/bin/bash
# N2 harness (tests/cpp/batch_streams.cpp) at several thread counts and sizes,
# GPU (batcher off, then on) and Beast's CPU codec:
# TAG=r06m bash scripts/n2_sweep.sh -> gpurun_out/<TAG>_n2_sweep.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_n2_sweep.log
python - <<'PY' || exit 2
from tests.test_facade import _build, _build_cpu_echo
_build("batch_streams"); _build_cpu_echo("batch_streams")
PY
: > $OUT
for size in ${SIZES:-1024 16384}; do
  for t in ${THREADS:-1 8 64}; do
    echo "== threads $t size $size" | tee -a $OUT
    timeout -k 10 200 tests/cpp/_build/batch_streams $t ${MSGS:-24} $size >> $OUT 2>&1 || { tail -3 $OUT; exit 3; }
    timeout -k 10 100 tests/cpp/_build/batch_streams_cpu $t ${MSGS:-24} $size >> $OUT 2>&1 || exit 4
  done
done
grep -v "^==" $OUT | grep -v amdgpu.ids
