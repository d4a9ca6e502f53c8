cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in "binary 16384 65536 gpu 1" "json 9216 40960 gpu 6" "binary 4096 65536 beast 1" "json 4096 40960 beast 6"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bp2/$tag -o bp -- python3 $R/scripts/diag_bp.py case $c bp > $R/gpurun_out/prof_bp2_$tag.log 2>&1 || exit 3
done
echo done
