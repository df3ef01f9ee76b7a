"""Per-kernel markdown table from rocprofv3 passes: `--stats` dir (time) + `--pmc` dirs
(run_counter_collection.csv each), averaged per dispatch.  FETCH_SIZE / WRITE_SIZE are KB;
'read'/'write' TB/s use the kernel-trace average duration.

'clock' = GRBM_GUI_ACTIVE / 8 XCDs / kernel-trace duration.  GRBM_GUI_ACTIVE counts the whole
counter-collection window of the dispatch, which carries a fixed ~0.25-0.35 M cycles (all XCDs)
of setup even for a 5 us kernel, and the duration comes from a different pass.  The ratio is
therefore only printed where that window is < 10 % of the count (GRBM_GUI_ACTIVE >= 3.5 M, i.e.
kernels of roughly >= 180 us); shorter kernels show no clock rather than a 4-6 GHz artefact."""
import collections
import csv
import glob
import os
import re
import sys


GRBM_MIN = 3.5e6  # counter-window setup (~0.35 M cycles) below 10 %


def main(stats_dir, pmc_dirs, pattern="smpk"):
    rx = re.compile(pattern)
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(stats_dir, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if rx.search(n):
                dur[short(n)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                if not rx.search(r["Kernel_Name"]):
                    continue
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
            for (disp, c), v in per.items():
                ctr[names[disp]][c].append(v)
    cols = sorted({c for k in ctr.values() for c in k})
    print("| kernel | calls | avg us | " + " | ".join(cols) + " | derived |")
    print("|---|---|---|" + "---|" * len(cols) + "---|")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        us = sum(dur[k]) / len(dur[k])
        vals = {c: sum(ctr[k][c]) / len(ctr[k][c]) for c in cols if ctr[k].get(c)}
        der = []
        if "FETCH_SIZE" in vals and us > 0:
            der.append(f"read {vals['FETCH_SIZE'] * 1024 / us / 1e6:.2f} TB/s")
        if "WRITE_SIZE" in vals and us > 0:
            der.append(f"write {vals['WRITE_SIZE'] * 1024 / us / 1e6:.2f} TB/s")
        if vals.get("GRBM_GUI_ACTIVE", 0.0) >= GRBM_MIN and us > 0:
            der.append(f"clock {vals['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f} GHz")
        if vals.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in vals:
            der.append(f"wait/wave {vals['SQ_WAIT_ANY'] / vals['SQ_WAVE_CYCLES']:.2f}")
        print(f"| {k} | {len(dur[k])} | {us:.1f} | " + " | ".join(f"{vals[c]:.4g}" if c in vals else "" for c in cols)
              + " | " + ", ".join(der) + " |")


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("smpk::", "")
    n = n.split("(")[0]
    return n.replace("void ", "")[:80]


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:-1] if len(sys.argv) > 3 else sys.argv[2:], sys.argv[-1] if len(sys.argv) > 3 else "smpk")
