"""Per-kernel table from rocprofv3 --pmc passes (run_counter_collection.csv per pass dir).

usage: python tools/pmc_summary.py <pass_dir> [<pass_dir> ...]
FETCH_SIZE / WRITE_SIZE are KB per dispatch; durations come from the counter rows'
timestamps (profiled runs: clocks differ from unprofiled ones, see MI355X_MICROARCH.md)."""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"smpk::\(anonymous namespace\)::(\w+)(<[^()]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    if name.startswith("Cijk") or "Cijk" in name[:20]:
        return name[:40]
    return name.split("(")[0][:60]


def main(dirs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            k = short(r["Kernel_Name"])
            if "smpk" not in r["Kernel_Name"] and "Cijk" not in r["Kernel_Name"]:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    counters = sorted({c for k in vals for c in vals[k]})
    print("| kernel | dispatches | avg us (profiled) | " + " | ".join(counters) + " | derived |")
    print("|---|---|---|" + "---|" * len(counters) + "---|")
    for k in sorted(vals):
        us = sorted(durs[k])[len(durs[k]) // 2]
        row = [k, str(max(len(v) for v in vals[k].values())), f"{us:.1f}"]
        avg = {c: sum(vals[k][c]) / len(vals[k][c]) for c in vals[k]}
        for c in counters:
            row.append(f"{avg[c]:.4g}" if c in avg else "")
        derived = []
        if "FETCH_SIZE" in avg:
            derived.append(f"read {avg['FETCH_SIZE'] * 1024 / (us * 1e-6) / 1e12:.2f} TB/s")
        if "WRITE_SIZE" in avg:
            derived.append(f"write {avg['WRITE_SIZE'] * 1024 / (us * 1e-6) / 1e12:.2f} TB/s")
        if "SQ_INSTS_MFMA" in avg and avg.get("SQ_INSTS_MFMA"):
            derived.append(f"VALU/MFMA {avg.get('SQ_INSTS_VALU', 0) / avg['SQ_INSTS_MFMA']:.2f}")
        if "GRBM_GUI_ACTIVE" in avg:
            derived.append(f"clock {avg['GRBM_GUI_ACTIVE'] / 8 / (us * 1e-6) / 1e9:.2f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            derived.append(f"MFMA busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.1%}")
        row.append(", ".join(derived))
        print("| " + " | ".join(row) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
