import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n_upd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('%10s %7s %9s %9s %6s  %s' % ('us/update', 'calls', 'avg_us', 'tot_us', 'pct', 'kernel'))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    t = float(r['TotalDurationNs'])
    print('%10.2f %7d %9.2f %9.1f %5.1f%%  %s' % (t / 1e3 / n_upd, int(r['Calls']), float(r['AverageNs']) / 1e3, t / 1e3,
                                               100 * t / tot, r['Name'][:100]))
print('total kernel time per update: %.1f us' % (tot / 1e3 / n_upd))
