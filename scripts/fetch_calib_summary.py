"""Turns the rocprofv3 FETCH_SIZE pass over scripts/calib_fetch.py into
profiles/<tag>_fetch_calib.csv: for each access pattern, the known bytes per
launch (2 GiB) divided by the counted bytes (FETCH_SIZE KiB x 1024).

    python scripts/fetch_calib_summary.py gpurun_out/prof_TAG/calib_counter_collection.csv
"""
import csv
import sys

KNOWN = 2 << 30


def main():
    per = {}
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            if "diag_read_kernel" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"]) * 1024
    ds = sorted(per)
    if len(ds) != 4:
        raise SystemExit(f"expected 4 calibration dispatches, got {len(ds)}")
    print("pattern,known_bytes,counted_bytes,bytes_per_counted_byte")
    for name, pair in (("coalesced_16B", ds[:2]), ("lane_slots", ds[2:])):
        counted = sorted(per[d] for d in pair)[-1]
        print(f"{name},{KNOWN},{int(counted)},{KNOWN / counted:.4f}")


if __name__ == "__main__":
    main()
