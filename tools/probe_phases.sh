#!/bin/bash
# Phase probes on the GPU box: conv backward phases (CB_PHASES build), fused head+screen+conv12
# phases (HS_TIMES build), then the default bench line.  Output under gpurun_out/probe/.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/probe; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
echo "[probe] cb_phases" && \
A3C_LIB=$V/cbp/liba3c_hip.so timeout -k 10 180 python3 -u tools/cb_phases.py > $O/cb.txt 2>&1 && cat $O/cb.txt && \
echo "[probe] hs_phases overlap" && \
A3C_LIB=$V/hst/liba3c_hip.so HS_KER=5 HS_OVERLAP=1 timeout -k 10 180 python3 -u tools/hs_phases.py > $O/hs1.txt 2>&1 && cat $O/hs1.txt && \
echo "[probe] bench" && \
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench.json 2> $O/bench.err && cat $O/bench.json
