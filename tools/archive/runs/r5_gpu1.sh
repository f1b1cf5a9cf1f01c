#!/bin/bash
# round 5, call 1: i8 MFMA layout probe, parity of the MFMA screen + new features, A/B vs the VALU screen
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g1; mkdir -p $O /tmp/pb
#/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/archive/probes/mfma_i8_layout.hip -o /tmp/pb/l 2>/dev/null || exit 1
#timeout -k 5 30 /tmp/pb/l > $O/layout.txt || { cat $O/layout.txt; exit 1; }
#cat $O/layout.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "matches_oracle or double_q or screen or preprocess or bench_shape" > $O/pytest1.log 2>&1
rc=$?; tail -3 $O/pytest1.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest1.log | head -30; exit $rc; }
for rep in 1 2 3; do
  for L in "" "async-rl-tensorflow_amd/lib/var/svalu/liba3c_hip.so" "async-rl-tensorflow_amd/lib/var/r5a/liba3c_hip.so"; do
    A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 200 > $O/ab.json 2>$O/ab.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/ab.json'));r=d['roofline']
print('${L:-mfma}', d['value'], 'frac', r['frac'], 'live_us', r['avg_us'], 'iso_us', r['isolated_us'], d['kernels']['k_head_screen_conv12'].get('live_us_by_step'))"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 > $O/bench20.json 2>$O/bench20.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench20.json'));print('steps20', d['value'], d['timing']['windows'], d['timing']['timed_seconds'], d['roofline']['frac'])"
bash tools/kstats.sh r5g1 || exit 1
