"""Per-kernel duration stats from a rocprofv3 SQLite result (rocpd): python tools/rocpd_stats.py run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration) from kernels group by name "
                 "order by sum(duration) desc").fetchall()
print("name,calls,avg_us,min_us,max_us")
for name, n, avg, mn, mx in rows:
    print(f"{name[:90]},{n},{avg / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f}")
# gaps between consecutive kernels on the same queue (launch-to-launch idle time)
ks = c.execute("select name, start, end from kernels order by start").fetchall()
gaps = {}
for (n0, s0, e0), (n1, s1, e1) in zip(ks, ks[1:]):
    key = (n0[:40], n1[:40])
    gaps.setdefault(key, []).append((s1 - e0) / 1e3)
print("gap_from,gap_to,count,median_us")
for (a, b), v in sorted(gaps.items()):
    v.sort()
    print(f"{a},{b},{len(v)},{v[len(v) // 2]:.2f}")
