#!/usr/bin/env python3
"""Per-queue kernel gaps of a rocprofv3 --kernel-trace CSV (start of a kernel minus the end of the
previous kernel on the same HW queue), summarised per (previous kernel -> kernel) pair over the
last `--tail` dispatches.  Used to price the kernel boundaries of the rollout stream.

usage: python tools/kgaps.py gpurun_out/ktrace/kt_kernel_trace.csv [--tail 20000]"""
import argparse
import collections
import csv


def short(name):
    name = name.split('(')[0]
    return name.split('<')[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--tail', type=int, default=20000)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    rows = rows[-a.tail:]
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r['Queue_Id']].append(r)
    for q, rs in sorted(byq.items()):
        pairs = collections.defaultdict(list)
        durs = collections.defaultdict(list)
        busy = 0
        for p, r in zip(rs, rs[1:]):
            g = int(r['Start_Timestamp']) - int(p['End_Timestamp'])
            pairs[(short(p['Kernel_Name']), short(r['Kernel_Name']))].append(g / 1e3)
        for r in rs:
            d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            durs[short(r['Kernel_Name'])].append(d)
            busy += d
        span = (int(rs[-1]['End_Timestamp']) - int(rs[0]['Start_Timestamp'])) / 1e3
        print(f'queue {q}: {len(rs)} kernels over {span:.0f} us, busy {busy:.0f} us ({busy / max(span, 1e-9):.1%})')
        for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            v.sort()
            print(f'    {k:42s} n={len(v):6d} median {v[len(v) // 2]:7.2f} us')
        for (p, k), v in sorted(pairs.items(), key=lambda kv: -len(kv[1])):
            if len(v) < 50:
                continue
            v.sort()
            print(f'  gap {p:28s} -> {k:28s} n={len(v):6d} median {v[len(v) // 2]:6.2f} us  p10 {v[len(v) // 10]:6.2f}')


if __name__ == '__main__':
    main()
