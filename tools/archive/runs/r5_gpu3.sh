#!/bin/bash
# round 5, call 3: backward-GEMM traffic knobs (knobs build) on M1 + PMC bytes of the GEMMs
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g3; mkdir -p $O
A3C_LIB=async-rl-tensorflow_amd/lib/var/cbp/liba3c_hip.so timeout -k 10 200 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
K=async-rl-tensorflow_amd/lib/var/knobs/liba3c_hip.so
for rep in 1 2 3; do
  for cfg in "X=0" "A3C_WKS_XCD=1" "A3C_GEMM_XCD=1" "A3C_L2BITS=1" "A3C_WKS_XCD=1 A3C_GEMM_XCD=1 A3C_L2BITS=1"; do
    env A3C_LIB=$K $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 200 > $O/ab.json 2>$O/ab.err || exit 1
    python3 -c "import json;d=json.load(open('$O/ab.json'));print('$cfg', d['value'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for cfg in "X=0" "A3C_WKS_XCD=1 A3C_GEMM_XCD=1 A3C_L2BITS=1"; do
  tag=$(echo $cfg | tr ' =' '__')
  env A3C_LIB=$K A3C_WAIT_VALUE=0 $cfg timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f_$tag -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing --min-seconds 0 > $O/f_$tag.log 2>&1 || exit 1
  env A3C_LIB=$K A3C_WAIT_VALUE=0 $cfg timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w_$tag -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing --min-seconds 0 > $O/w_$tag.log 2>&1 || exit 1
  mkdir -p $O/s_$tag && ln -sfn ../f_$tag $O/s_$tag/pmc_fetch && ln -sfn ../w_$tag $O/s_$tag/pmc_write && mkdir -p $O/s_$tag/trace
  python3 tools/pmc_summarize.py $O/s_$tag > $O/pmc_$tag.json || exit 1
  python3 - $O/pmc_$tag.json "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {n: round(v['hbm_bytes_per_launch'] / 1e6, 1) for n, v in d['kernels'].items()
                    if v['hbm_bytes_per_launch'] and ('gemm' in n or 'screen' in n or 'conv_bwd' in n or 'fc_part' in n)})
PY
done
