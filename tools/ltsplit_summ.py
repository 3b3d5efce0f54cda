import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print('columns', list(rows[0].keys()))
zcol = [k for k in rows[0] if 'Grid' in k and 'Z' in k.upper()]
print('zcol', zcol)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    if 'lt_bsgs' not in r['Kernel_Name']: continue
    z = r[zcol[0]] if zcol else '?'
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[z][0] += 1; agg[z][1] += d
for z, (n, us) in sorted(agg.items()):
    print(f'grid z {z}: {n} dispatches, {us:.1f} us total, {us / n:.1f} us avg')
