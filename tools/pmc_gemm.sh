#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
O=gpurun_out/pmcg; mkdir -p $O
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing --min-seconds 0 --update sync"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1 || exit 1
PMC_FILTER=k_gemm,k_fc_fwd,k_conv_bwd,k_head_screen,k_conv12 python3 tools/pmc_all.py $O/p1 $O/p2
