#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter collections: tools/pmc_kernels.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(f)):
            k = re.sub(r'^void\s+', '', row['Kernel_Name']).split('(')[0]
            acc[k][row['Counter_Name']].append(float(row['Counter_Value']))
names = sorted({c for k in acc for c in acc[k]})
for k in sorted(acc, key=lambda k: -sum(acc[k].get('SQ_WAVE_CYCLES', [0]))):
    if not acc[k].get('SQ_WAVE_CYCLES'):
        continue
    avg = {c: sum(v) / len(v) for c, v in acc[k].items()}
    wc = avg.get('SQ_WAVE_CYCLES', 1) or 1
    line = f'{k[:34]:34s}'
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
              'SQ_ACTIVE_INST_VMEM', 'SQ_WAIT_INST_LDS'):
        if c in avg:
            line += f' {c[3:][:14]}={avg[c] / wc:5.2f}'
    for c in ('SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_LDS_IDX_ACTIVE', 'SQ_LDS_BANK_CONFLICT',
              'SQ_INSTS_MFMA', 'SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_WAVES'):
        if c in avg:
            line += f' {c[3:][:12]}={avg[c]:.3g}'
    print(line)
