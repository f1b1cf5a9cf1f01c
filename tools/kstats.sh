#!/bin/bash
# rocprofv3 kernel stats of a short bench run: tools/kstats.sh TAG [bench args]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
O=gpurun_out/ks_$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-kernel-timing --min-seconds 0 "$@" > $O/bench.json 2> $O/err.log || exit 1
f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print('%-60s %6s %9.2f us %5.1f%%' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
grep -o '"value": [0-9.]*' $O/bench.json
