#!/usr/bin/env python3
"""Copy one profiling round (gpurun_out/prof_TAG from tools/profile_round.sh) into profiles/:
  profiles/roundR_TAG_bench.json (R from $A3C_ROUND, default 2), _kernel_stats.csv, _pmc_summary.json, and refresh
  profiles/pmc_hbm_bytes.json (read by bench.py for roofline.traffic)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rnd = 'round' + os.environ.get('A3C_ROUND', '2')
src = os.path.join(ROOT, 'gpurun_out', 'prof_' + tag)
dst = os.path.join(ROOT, 'profiles')
shutil.copy(os.path.join(src, 'bench.json'), os.path.join(dst, f'{rnd}_{tag}_bench.json'))
shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'), os.path.join(dst, f'{rnd}_{tag}_kernel_stats.csv'))
d = json.load(open(os.path.join(src, 'summary.json')))
json.dump(d, open(os.path.join(dst, f'{rnd}_{tag}_pmc_summary.json'), 'w'), indent=1)
out = dict(method=d['method'],
           source=f'profiles/{rnd}_{tag}_pmc_summary.json (tools/profile_round.sh {tag}: rocprofv3 --pmc FETCH_SIZE '
                  'and --pmc WRITE_SIZE passes of bench.py --steps 10, separate runs)',
           hbm_bytes_per_launch={k: round(v) for k, v in d['hbm_bytes_per_launch'].items()})
# an M2 round (tag ending in m2, bench.py --frames84) feeds the M2 bench line's roofline.traffic
json.dump(out, open(os.path.join(dst, 'pmc_hbm_bytes_m2.json' if tag.endswith('m2') else 'pmc_hbm_bytes.json'), 'w'),
          indent=1)
print(json.dumps(out['hbm_bytes_per_launch'], indent=1))
