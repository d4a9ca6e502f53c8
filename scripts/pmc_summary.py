"""Condenses rocprofv3 --pmc CSV output (FETCH_SIZE / WRITE_SIZE passes) into
profiles/rNN_*_pmc.csv rows: kernel, dispatch, counter, value_kB.

    python scripts/pmc_summary.py gpurun_out/prof_TAG/fetch_counter_collection.csv \
        gpurun_out/prof_TAG/write_counter_collection.csv > profiles/rNN_x_pmc.csv
"""
import csv
import sys


def main():
    w = csv.writer(sys.stdout, lineterminator="\n")   # kernel names hold commas: quoted
    w.writerow(["kernel", "dispatch", "counter", "value_kB"])
    for path in sys.argv[1:]:
        acc = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                # this engine's kernels and the library kernels it launches
                # (hipCUB sort / scan); not torch's setup and check kernels
                if "at::native" in name or "rocclr" in name:
                    continue
                short = name.split("(")[0]
                key = (short, r["Dispatch_Id"], r["Counter_Name"])
                acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
        for (k, d, c), v in sorted(acc.items(), key=lambda x: int(x[0][1])):
            w.writerow([k, d, c, f"{v:.6f}"])


if __name__ == "__main__":
    main()
