"""Per-kernel average of rocprofv3 --pmc counters (run_counter_collection.csv files)."""
import collections
import csv
import sys


def main(paths, match="attn"):
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in rows:
            full = r["Kernel_Name"].rsplit("(", 1)[0]
            if match not in full:
                continue
            k = full[full.find(match):][:70] + f" grid={r['Grid_Size']}"
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k, v in agg.items():
            nd = len(disp[k])
            vals = ", ".join(f"{c}={x / nd:.4g}" for c, x in sorted(v.items()))
            print(f"{k} [{nd}]: {vals}")


if __name__ == "__main__":
    main(sys.argv[1:])
