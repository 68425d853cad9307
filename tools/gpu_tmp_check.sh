#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
args="default=base reference=base:2 wconst=ab/lib_r6_wconst.so:2 wrconst=ab/lib_r6_wrconst.so:2 nochains=ab/lib_r6_c_nochains.so:2"
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 7 $args 2>&1 | grep -v amdgpu.ids
BUDGET_TAG=r6w BUDGET_VARIANTS="$args" BUDGET_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" timeout -k 10 300 tools/gpu_budget.sh 2>&1 | tail -8
