#!/bin/bash
# One bench.py run that can never fail silently: stdout (the JSON line) goes
# to gpurun_out/<tag>.json, stderr to <tag>.err, and the exit status and the
# stderr tail are printed next to a one-line summary (or the failure).
# Usage: scripts/run_bench.sh TAG TIMEOUT_S SUMMARY_PY [bench args...]
#   SUMMARY_PY: a python expression over d (the parsed line), e.g. "d['value']"
#   BPMD_LIB in the environment selects a library variant.
set -o pipefail
tag=$1; to=$2; expr=$3; shift 3
mkdir -p gpurun_out
timeout -k 10 "$to" python -u bench.py "$@" > gpurun_out/$tag.json 2> gpurun_out/$tag.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/$tag.err
if [ $rc -ne 0 ] || [ ! -s gpurun_out/$tag.json ]; then
  echo "$tag FAILED rc=$rc (124/137: time limit; 134/139: abort/segfault); stderr tail:"
  tail -8 gpurun_out/$tag.err | sed 's/^/    /'
  exit $(( rc == 0 ? 1 : rc ))
fi
python -c "import json,sys; d=json.load(open('gpurun_out/$tag.json')); print('$tag', $expr)" || exit 1
