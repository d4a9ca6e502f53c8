#!/bin/bash
# kernel + HIP API trace of the N2 harness (tests/cpp/batch_streams.cpp):
# TAG=r06o T=64 SIZE=1024 bash scripts/prof_n2.sh -> gpurun_out/prof_n2_TAG/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-r06}
cd $R && python - <<'PY' || exit 2
from tests.test_facade import _build
_build("batch_streams")
PY
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_n2_$TAG
mkdir -p $OUT
BATCH_STREAMS_ONLY_BATCHED=${ONLY_BATCHED:-0} timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $OUT/run -o trace \
  -- $R/tests/cpp/_build/batch_streams ${T:-64} ${MSGS:-24} ${SIZE:-1024} > $OUT/log.txt 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 3; }
cat $OUT/log.txt
for f in kernel_stats hip_api_stats; do
  p=$(find $OUT/run -name "trace_${f}.csv" | head -1)
  [ -n "$p" ] && cp $p $OUT/${f}.csv && echo "-- $f" && head -14 $OUT/${f}.csv | cut -c1-200
done
exit 0
