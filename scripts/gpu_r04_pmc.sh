#!/bin/bash
# C2 inflate counters of the current build: SQ issue/wait mix (pmc_lane3.sh)
# and FETCH_SIZE / WRITE_SIZE (separate passes), into gpurun_out/
set -o pipefail
TAG=${TAG:-r04o}
R=$PWD
TAG=$TAG bash scripts/pmc_lane3.sh > gpurun_out/${TAG}_sq.txt 2>&1 || { cat gpurun_out/${TAG}_sq.txt; exit 1; }
cat gpurun_out/${TAG}_sq.txt
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C2="--steps 3 --warmup 1 --no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch -- python3 $R/bench.py $C2 > /dev/null 2> $OUT/err.log || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write -- python3 $R/bench.py $C2 > /dev/null 2>> $OUT/err.log || exit 3
python3 $R/scripts/pmc_summary.py $(find $OUT -name 'fetch_counter_collection.csv') $(find $OUT -name 'write_counter_collection.csv') > $OUT/c2_pmc.csv || exit 4
cat $OUT/c2_pmc.csv
