"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel ms/step table (markdown)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"Kernel time per step: {tot / 1e6 / steps:.1f} ms ({steps:g} profiled steps)\n")
print("| ms/step | % | calls/step | avg us | kernel |")
print("|---|---|---|---|---|")
for r in rows[:top]:
    print(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | {float(r['Percentage']):.1f} | "
          f"{int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:90]}` |")
