"""Merge per-rank SMP_TIMELINE_FILE traces into one Chrome/Perfetto trace (pid = rank) and
print, for one step, each rank's task order (F = forward, B = backward, per microbatch).

usage: python tools/merge_timelines.py OUT.json STEP rank0.json rank1.json ...
"""
import json
import sys


def load(path):
    d = json.load(open(path))
    return d["traceEvents"] if isinstance(d, dict) else d


def main():
    out, step, paths = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    merged = []
    t0 = min(e["ts"] for p in paths for e in load(p) if "ts" in e)
    lines = []
    for rank, p in enumerate(paths):
        ev = load(p)
        merged.append({"name": "process_name", "ph": "M", "pid": rank, "args": {"name": f"pp_rank {rank}"}})
        for e in ev:
            e = dict(e)
            e["pid"] = rank
            if "ts" in e:
                e["ts"] = round(e["ts"] - t0, 3)
            merged.append(e)
        seq = []
        for e in sorted((e for e in ev if e.get("ph") == "X" and e.get("args", {}).get("step") == step),
                        key=lambda e: e["ts"]):
            kind = e["name"].split()[0]
            if kind in ("FWD", "BWD"):
                seq.append(f"{kind[0]}{e['args']['mb']}")
        lines.append(f"rank {rank}: " + " ".join(seq))
    json.dump({"traceEvents": merged, "displayTimeUnit": "ms"}, open(out, "w"))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
