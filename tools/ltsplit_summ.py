"""Summarise an ORION_LT_SPLIT=1 kernel trace: lt_bsgs dispatches grouped by
their grid depth (limbs per launch: 1 = limb 0 (q0), K = the P limbs, the rest
= the middle Q limbs).  Usage: python tools/ltsplit_summ.py <rocprofv3 dir>"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    if 'lt_bsgs' not in r['Kernel_Name']:
        continue
    z = int(r['Grid_Size_Z'])
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[z][0] += 1
    agg[z][1] += d
for z, (n, us) in sorted(agg.items()):
    print(f'limbs per launch {z}: {n} dispatches, {us:.1f} us total, {us / n:.1f} us avg, {us / n / z:.1f} us per limb')
