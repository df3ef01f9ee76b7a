"""GPU busy fraction per step from a rocprofv3 kernel trace: union of kernel intervals vs the
wall span between consecutive step markers (the LM-head cross-entropy forward kernel, one per
step on the stage that owns the loss; `--marker` overrides)."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="xent_fwd")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
for s, e in zip(marks, marks[1:]):
    seg = rows[s:e]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[e]["Start_Timestamp"])
    busy, cur_s, cur_e = 0, None, None
    for r in seg:
        b, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_e is None or b > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = b, en
        else:
            cur_e = max(cur_e, en)
    busy += cur_e - cur_s
    print(f"step span {(t1 - t0) / 1e6:.1f} ms, kernels busy {busy / 1e6:.1f} ms ({100 * busy / (t1 - t0):.1f} %), "
          f"{len(seg)} kernels")
