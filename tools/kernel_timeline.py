"""Kernel busy/idle time and per-kernel totals of one rocprofv3 --kernel-trace run
(the rocpd SQLite output), for the dispatches after the largest gap (the timed
render after a warm-up).  usage: python tools/kernel_timeline.py RUN_results.db"""
import sqlite3, sys, collections
db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
tabs = [r[0] for r in cur.execute("select name from sqlite_master where type in ('table','view')")]
kd = [t for t in tabs if 'kernel_dispatch' in t and 'rocpd_kernel_dispatch' in t][0]
cols = [r[1] for r in cur.execute(f"pragma table_info({kd})")]
ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
kcols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
rows = cur.execute(f"select d.start, d.end, s.kernel_name from {kd} d join {ks} s on d.kernel_id = s.id order by d.start").fetchall()
# timed render = after the warm-up: split at the largest gap
gaps = [(rows[i+1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
t0 = rows[0][0]
big = sorted(gaps)[-3:]
print('n dispatches', len(rows), 'largest gaps (us)', [(g / 1e3, i) for g, i in big])
# take the dispatches after the largest gap
cut = max(big)[1] + 1
R = rows[cut:]
span = (R[-1][1] - R[0][0]) / 1e6
busy = collections.Counter(); cnt = collections.Counter()
for s, e, n in R:
    k = n.split('(')[0].split('<')[0].replace('void ', '').replace('surfdev::', '')
    busy[k] += (e - s) / 1e6; cnt[k] += 1
tot = sum(busy.values())
print(f'span {span:.1f} ms, kernel busy {tot:.1f} ms, idle {span - tot:.1f} ms over {len(R)} dispatches ({(span - tot) / len(R) * 1e3:.1f} us per dispatch)')
for k, v in busy.most_common():
    print(f'  {k:20s} {v:8.2f} ms  {cnt[k]:5d}  avg {v / cnt[k] * 1e3:8.1f} us')
