#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc collections (top kernels by name filter):
tools/pmc_all.py DIR [DIR ...]  (env PMC_FILTER: comma-separated substrings of kernel names)"""
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
filt = [x for x in os.environ.get('PMC_FILTER', '').split(',') if x]
for k in sorted(acc):
    if filt and not any(f in k for f in filt):
        continue
    print(k)
    for c in sorted(acc[k]):
        v = acc[k][c]
        print('    %-32s %14.4g  (n=%d)' % (c, sum(v) / len(v), len(v)))
