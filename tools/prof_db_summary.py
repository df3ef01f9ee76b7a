"""Per-kernel summary of a rocprofv3 rocpd SQLite output (<name>_results.db): calls, mean / min
duration, VGPR / scratch of each kernel, sorted by total time.  usage: prof_db_summary.py db [n]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows = c.execute("select name, count(*), avg(duration), min(duration), max(vgpr_count), max(scratch_size) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
for name, cnt, avg, mn, vg, scr in rows[:n]:
    short = name[name.find("attn_"):] if "attn_" in name else name
    print(f"{cnt:5d} avg {avg / 1e3:8.1f} min {mn / 1e3:8.1f} us vgpr {vg} scratch {scr}  {short[:90]}")
