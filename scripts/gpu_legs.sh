#!/bin/bash
# per-leg rocprof evidence (scripts/profile_legs.sh) + the 8-way shard legs;
# TAG names the output directory gpurun_out/prof_<TAG>
set -o pipefail
TAG=${TAG:-r03u}
TAG=$TAG bash scripts/profile_legs.sh ${@} || exit 1
cat gpurun_out/prof_$TAG/log.txt
for f in gpurun_out/prof_$TAG/*_kernels.csv; do echo "== $f"; cat $f; done
