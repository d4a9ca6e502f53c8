"""Per-design averages of the SQ counters collected by scripts/pmc_lane3.sh
for the lane inflate kernel (one C2 launch = 64 Ki messages)."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        acc = collections.defaultdict(float)
        disp = set()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "inflate_lane" not in r["Kernel_Name"]:
                    continue
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        if not disp:
            continue
        k = len(disp)
        print(os.path.relpath(f, root), f"{k} launches")
        for c, v in sorted(acc.items()):
            print(f"  {c:24s} {v / k:16.0f}")


if __name__ == "__main__":
    main()
