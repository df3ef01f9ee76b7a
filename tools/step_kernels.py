"""Steady-state per-kernel table of the last full step in a rocprofv3 kernel trace (step
boundaries: the LM-head cross-entropy forward kernel); weight-gradient kernels split by grid."""
import collections
import csv
import sys

if sys.argv[1].endswith(".db"):  # rocprofv3's default rocpd SQLite output
    import sqlite3

    db = sqlite3.connect(sys.argv[1])
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Grid_Size_X": gx, "Workgroup_Size_X": wx}
            for n, s, e, gx, wx in db.execute("select name, start, end, grid_x, workgroup_x from kernels")]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "xent_fwd" in r["Kernel_Name"]]
last = rows[idx[-2]:idx[-1]]
t0, t1 = int(last[0]["Start_Timestamp"]), int(rows[idx[-1]]["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0.0, 0])
for r in last:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"]
    if "wgrad_glds" in k or "Cijk" in k:
        k = k[:48] + f" grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}"
    agg[k[:95]][0] += d
    agg[k[:95]][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"step {(t1 - t0) / 1e6:.1f} ms wall, {tot / 1e3:.1f} ms kernels")
for k, v in sorted(agg.items(), key=lambda x: -x[1][0])[:40]:
    print(f"{v[0] / 1e3:8.2f} ms {v[1]:4d} {v[0] / v[1]:8.1f} us  {k}")

# concurrency: busy union of the step (wall - union = idle gaps) and, per side-stream kernel
# family, how much of its time ran beside another kernel
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in last)
union, cs, ce = 0, None, None
for s, e, _ in iv:
    if cs is None or s > ce:
        if cs is not None:
            union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
if cs is not None:
    union += ce - cs
print(f"busy union {union / 1e6:.1f} ms, idle gaps {(t1 - t0 - union) / 1e6:.1f} ms, "
      f"overlapped kernel time {(tot * 1e3 - union) / 1e6:.1f} ms")
for fam in ("keep_bits", "oneshot", "device_copy"):
    mine = [(s, e) for s, e, n in iv if fam in n]
    if not mine:
        continue
    others = [(s, e) for s, e, n in iv if fam not in n]
    ov = 0
    for s, e in mine:
        for os_, oe in others:
            if oe > s and os_ < e:
                ov += min(e, oe) - max(s, os_)
    dur = sum(e - s for s, e in mine)
    print(f"{fam}: {dur / 1e6:.2f} ms, {100.0 * ov / max(dur, 1):.0f} % of it beside other kernels")
