"""Per-kernel and per-copy-direction stats (count, total/avg/min/max us) from a rocprofv3 SQLite
output (rocpd *.db): python3 tools/rocpd_summary.py run_results.db > summary.csv"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
print('kind,name,calls,total_us,avg_us,min_us,max_us,avg_bytes,GB_per_s')
q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) from kernels "
     "group by name order by sum(duration) desc")
for name, n, tot, avg, mn, mx in c.execute(q):
    short = name.split('(')[0].replace(',', ';')
    print(f'kernel,{short},{n},{tot / 1e3:.1f},{avg / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f},,')
q = ("select src_agent_type || '->' || dst_agent_type, count(*), sum(duration), avg(duration), min(duration), "
     "max(duration), avg(size), sum(size) from memory_copies group by 1 order by sum(duration) desc")
for d, n, tot, avg, mn, mx, sz, stot in c.execute(q):
    print(f'copy,{d},{n},{tot / 1e3:.1f},{avg / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f},{sz:.0f},{stot / tot:.2f}')
