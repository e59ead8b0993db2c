"""Per-phase cost of one rocprofv3 --kernel-trace run (rocpd SQLite output): the
dispatches after the largest gap (the timed render after a warm-up) cut into
phases at each k_extend launch; per phase its span (k_extend start to the next
one's), the busy time of each kernel and the idle time between them.  Prints
the median phase, the phases grouped by span, and the drain.
usage: python tools/phase_costs.py RUN_results.db [--all]"""
import collections
import re
import sqlite3
import statistics
import sys

db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
tabs = [r[0] for r in cur.execute("select name from sqlite_master where type in ('table','view')")]
kd = [t for t in tabs if 'kernel_dispatch' in t and 'rocpd_kernel_dispatch' in t][0]
ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
rows = cur.execute(f"select d.start, d.end, s.kernel_name from {kd} d join {ks} s on d.kernel_id = s.id order by d.start").fetchall()
gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
R = rows[max(gaps)[1] + 1:]
def name(n):
    m = re.match(r'_ZN7surfdev(\d+)', n)           # mangled: _ZN7surfdev<len><name>...
    if m:
        return n[m.end():m.end() + int(m.group(1))]
    return n.split('(')[0].split('<')[0].replace('void ', '').replace('surfdev::', '')
R = [(s, e, name(n)) for s, e, n in R]
starts = [i for i, r in enumerate(R) if r[2] == 'k_extend']
phases = []
for a, b in zip(starts, starts[1:] + [len(R)]):
    seg = R[a:b]
    t0, t1 = seg[0][0], (R[b][0] if b < len(R) else max(e for _, e, _ in seg))
    busy = collections.Counter()
    for s, e, n in seg:
        busy[n] += (e - s) / 1e3
    # idle: time in [t0, t1) covered by no kernel
    iv = sorted((s, e) for s, e, _ in seg)
    covered, end = 0, t0
    for s, e in iv:
        s, e = max(s, end), min(e, t1)
        if e > s:
            covered += e - s
            end = e
    phases.append({'span': (t1 - t0) / 1e3, 'idle': (t1 - t0 - covered) / 1e3, 'busy': busy, 'n': len(seg)})
tail = [r for r in R[:starts[0]]] if starts else []
spans = [p['span'] for p in phases]
print(f'{len(R)} dispatches, {len(phases)} phases, render span {(R[-1][1] - R[0][0]) / 1e6:.2f} ms')
if phases:
    med = sorted(phases, key=lambda p: p['span'])[len(phases) // 2]
    print(f"median phase {med['span']:.1f} us (idle {med['idle']:.1f} us, {med['n']} dispatches): " +
          ', '.join(f'{k} {v:.1f}' for k, v in med['busy'].most_common()))
    for lo, hi in ((0, 300), (300, 600), (600, 1000), (1000, 2000), (2000, 1e12)):
        sel = [p for p in phases if lo <= p['span'] < hi]
        if not sel:
            continue
        tot = collections.Counter()
        for p in sel:
            tot.update(p['busy'])
        print(f"  span {lo}-{hi} us: {len(sel)} phases, {sum(p['span'] for p in sel) / 1e3:.2f} ms, idle "
              f"{sum(p['idle'] for p in sel) / 1e3:.2f} ms; per phase " +
              ', '.join(f'{k} {v / len(sel):.1f}' for k, v in tot.most_common(6)))
    print(f'  sum of phase spans {sum(spans) / 1e3:.2f} ms, median {statistics.median(spans):.1f} us')
if '--all' in sys.argv:
    for i, p in enumerate(phases):
        print(i, f"{p['span']:.1f}", f"idle {p['idle']:.1f}", ' '.join(f'{k}:{v:.1f}' for k, v in sorted(p['busy'].items())))
