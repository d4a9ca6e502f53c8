"""Per-kernel launch statistics from a rocprofv3 --kernel-trace CSV
(<out>_kernel_trace.csv): calls, the median duration with the first (cold)
launch of each kernel excluded, mean, min and max, in ns.  Torch's own setup
and check kernels are dropped.

    python scripts/kernel_summary.py gpurun_out/prof_TAG/.../x_kernel_trace.csv > profiles/TAG_leg_kernels.csv
"""
import csv
import statistics
import sys


def main():
    per = {}
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "at::native" in name or "rocclr" in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per.setdefault(short, []).append((int(r["Start_Timestamp"]), d))
    w = csv.writer(sys.stdout, lineterminator="\n")   # kernel names hold commas: quoted
    w.writerow(["kernel", "calls", "median_ns_warm", "mean_ns_all", "min_ns", "max_ns", "first_ns"])
    for k, v in sorted(per.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        ds = [d for _, d in v]
        warm = ds[1:] if len(ds) > 1 else ds
        w.writerow([k, len(ds), int(statistics.median(warm)), int(statistics.mean(ds)), min(ds), max(ds), ds[0]])


if __name__ == "__main__":
    main()
