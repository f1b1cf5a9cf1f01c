#!/usr/bin/env python3
"""Summarise rocprofv3 output of one profiling round into JSON.

  tools/pmc_summarize.py OUTDIR > summary.json

OUTDIR holds `trace/` (--kernel-trace --stats), `pmc_fetch/` (--pmc FETCH_SIZE) and
`pmc_write/` (--pmc WRITE_SIZE), each collected in its own rocprofv3 pass because the two
counters do not fit one pass on gfx950.  HBM bytes per launch follow
/opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r'^void\s+', '', name.strip())
    name = name.split('(')[0]
    return name.split('<')[0].strip()


def variant(name):
    name = re.sub(r'^void\s+', '', name.strip())
    return name.split('(')[0].strip()


def read_counters(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get('Counter_Name') != counter:
                    continue
                acc[variant(row['Kernel_Name'])].append(float(row['Counter_Value']))
    return acc


def read_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out[variant(row['Name'])] = dict(calls=int(row['Calls']), avg_us=float(row['AverageNs']) / 1e3,
                                                 total_us=float(row['TotalDurationNs']) / 1e3,
                                                 pct=float(row['Percentage']))
    return out


def main(outdir):
    fetch = read_counters(os.path.join(outdir, 'pmc_fetch'), 'FETCH_SIZE')
    write = read_counters(os.path.join(outdir, 'pmc_write'), 'WRITE_SIZE')
    stats = read_stats(os.path.join(outdir, 'trace'))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fa = sum(f) / len(f) if f else None
        wa = sum(w) / len(w) if w else None
        hbm = None if fa is None or wa is None else (2.0 * fa + wa) * 1024.0
        kernels[k] = dict(launches_fetch=len(f), launches_write=len(w), fetch_kib_avg=fa, write_kib_avg=wa,
                          hbm_bytes_per_launch=hbm, trace=stats.get(k))
    by_short = collections.defaultdict(list)
    for k, v in kernels.items():
        if v['hbm_bytes_per_launch'] is not None:
            by_short[short(k)].append(v)
    agg = {}
    for s, vs in by_short.items():
        n = sum(v['launches_fetch'] for v in vs)
        agg[s] = sum(v['hbm_bytes_per_launch'] * v['launches_fetch'] for v in vs) / max(n, 1)
    json.dump(dict(method='(2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 per launch; separate rocprofv3 --pmc passes',
                   hbm_bytes_per_launch=agg, kernels=kernels, stats=stats), sys.stdout, indent=1)


if __name__ == '__main__':
    main(sys.argv[1])
