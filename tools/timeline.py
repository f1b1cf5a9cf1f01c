#!/usr/bin/env python3
"""Iteration timeline from a rocprofv3 kernel trace: tools/timeline.py <kernel_trace.csv> [anchor] [n]

Splits the trace into engine iterations at each launch of the anchor kernel (default k_prep_fwd,
one per iteration), then prints, for the last n iterations averaged, every kernel's start
offset from the iteration start, its duration and its stream (queue), plus per-stream busy time,
so the critical path of the overlapped rollout / backward streams can be read off.
"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r'\(.*', '', name)
    return name.replace('void ', '')[:44]


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else 'k_prep_fwd'
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        nm = r.get('Kernel_Name') or r.get('Name')
        t0, t1 = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        q = r.get('Stream_Id') or r.get('Queue_Id')
        ks.append((t0, t1, short(nm), q))
    ks.sort()
    starts = [k[0] for k in ks if k[2].startswith(anchor)]
    if len(starts) < n + 2:
        n = len(starts) - 2
    its = list(zip(starts[-n - 1:-1], starts[-n:]))
    per = collections.defaultdict(list)     # (name, slot) -> [(off, dur, q)]
    busy = collections.defaultdict(float)
    lens = []
    for a, b in its:
        lens.append(b - a)
        slot = collections.Counter()
        for t0, t1, nm, q in ks:
            if a <= t0 < b:
                i = slot[nm]
                slot[nm] += 1
                per[(nm, i)].append((t0 - a, t1 - t0, q))
                busy[q] += (t1 - t0) / len(its)
    L = sum(lens) / len(lens)
    print('iterations %d, mean length %.1f us (min %.1f max %.1f)' % (len(its), L / 1e3, min(lens) / 1e3,
                                                                     max(lens) / 1e3))
    order = sorted(per, key=lambda k: sum(x[0] for x in per[k]) / len(per[k]))
    print('%-46s %5s %9s %9s %9s' % ('kernel', 'queue', 'start us', 'dur us', 'end us'))
    for k in order:
        v = per[k]
        off = sum(x[0] for x in v) / len(v) / 1e3
        dur = sum(x[1] for x in v) / len(v) / 1e3
        q = collections.Counter(x[2] for x in v).most_common(1)[0][0]
        print('%-46s %5s %9.1f %9.1f %9.1f  (%d)' % ('%s#%d' % k, q, off, dur, off + dur, len(v)))
    for q, b in sorted(busy.items()):
        print('queue %s busy %.1f us per iteration (%.0f%%)' % (q, b / 1e3, 100 * b / L))


if __name__ == '__main__':
    main()
