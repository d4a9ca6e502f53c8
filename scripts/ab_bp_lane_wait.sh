# A/B of the side-stream ordering switches on the mixed legs' block-parallel path:
# (the switches were removed with the rejected change: profiles/r04zzc_bp_lane_wait_prio_rejected.log)
#   base, BPMD_BP_LANE_WAIT=1, BPMD_BP_SIDE_PRIO=1, both; two rounds interleaved
cd $GRAFT_REPO_ROOT
E="{k: (v['inflate_value'], {n: (s.get('inflate_shard_ms'), s['inflate_projected_speedup']) for n, s in v['virtual_shards'].items()}, v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}"
for r in 1 2; do
  for v in base wait prio both; do
    case $v in
      base) W=0; P=0;; wait) W=1; P=0;; prio) W=0; P=1;; both) W=1; P=1;;
    esac
    BPMD_BP_LANE_WAIT=$W BPMD_BP_SIDE_PRIO=$P bash scripts/run_bench.sh lw_${v}_$r 400 "'$v', $E" \
      --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --legs ${LEGS:-c4_l6} || exit 1
  done
done
