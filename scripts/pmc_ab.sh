# FETCH_SIZE / WRITE_SIZE per inflate launch for library variants (ab_lane.py
# runs the default library first, then each variant, 9 launches each).
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmcab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $OUT -o $c -- python3 $ROOT/scripts/ab_lane.py > $OUT/$c.log 2>&1 || exit 2
done
python3 - <<'PY'
import csv, glob, collections
for c in ["FETCH_SIZE", "WRITE_SIZE"]:
    f = glob.glob(f"/root/repo/gpurun_out/pmcab/**/{c}_counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "lane" in r["Kernel_Name"]]
    vals = collections.defaultdict(float)
    for r in rows: vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    ks = sorted(vals)
    print(c, [round(vals[k] / 1024, 1) for k in ks], "MB (raw counter / 1024)")
PY
