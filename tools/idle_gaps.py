"""GPU idle time of one rocprofv3 --kernel-trace run (rocpd SQLite output): the
union of all kernel intervals after the largest gap (the timed render after a
warm-up), the time no kernel runs, and the gaps by size -- e.g. the host's
poll between graph replays.  usage: python tools/idle_gaps.py RUN_results.db"""
import sqlite3, sys, collections
db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
tabs = [r[0] for r in cur.execute("select name from sqlite_master where type in ('table','view')")]
kd = [t for t in tabs if 'kernel_dispatch' in t and 'rocpd_kernel_dispatch' in t][0]
ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
rows = cur.execute(f"select d.start, d.end, s.kernel_name from {kd} d join {ks} s on d.kernel_id = s.id order by d.start").fetchall()
gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
cut = max(gaps)[1] + 1
R = rows[cut:]
name = lambda n: n.split('(')[0].split('<')[0].replace('void ', '').replace('surfdev::', '')
idle, hist, big = 0, collections.Counter(), []
end, prev = R[0][1], R[0]
for r in R[1:]:
    if r[0] > end:
        g = (r[0] - end) / 1e3
        idle += g
        b = '<2' if g < 2 else '2-10' if g < 10 else '10-50' if g < 50 else '50-200' if g < 200 else '>=200'
        hist[b] += g
        big.append((g, name(prev[2]), name(r[2])))
    if r[1] > end:
        end, prev = r[1], r
span = (end - R[0][0]) / 1e6
print(f'{len(R)} dispatches, span {span:.2f} ms, GPU idle {idle / 1e3:.2f} ms ({100 * idle / 1e3 / span:.1f} %)')
for b in ('<2', '2-10', '10-50', '50-200', '>=200'):
    print(f'  gaps {b:>6s} us: {hist[b] / 1e3:7.2f} ms')
by = collections.defaultdict(lambda: [0, 0.0])
for g, a, b in big:
    if g >= 10:
        by[(a, b)][0] += 1; by[(a, b)][1] += g
for (a, b), (n, t) in sorted(by.items(), key=lambda x: -x[1][1])[:10]:
    print(f'  {a:>14s} -> {b:<14s} {n:5d} gaps >= 10 us, {t / 1e3:7.2f} ms')
