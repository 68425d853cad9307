#!/bin/bash
# Inside the reference-order MFCC's chains (profiles/r06_chain_cost.txt section 3): launch times and PMC instruction counts
# of the CHAIN kernel with its weight loads (chain_wconst) and weight + power-row loads (chain_wconst+chain_rconst) replaced
# by constants, and with the chains skipped (chain_none): tools/ablate.py builds copied to ab/lib_r6_{wconst,wrconst,
# c_nochains}.so (outputs wrong by design). Needs those builds in ab/.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
args="default=base reference=base:2 wconst=ab/lib_r6_wconst.so:2 wrconst=ab/lib_r6_wrconst.so:2 nochains=ab/lib_r6_c_nochains.so:2"
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 7 $args 2>&1 | grep -v amdgpu.ids
BUDGET_TAG=r6w BUDGET_VARIANTS="$args" BUDGET_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" timeout -k 10 300 tools/gpu_budget.sh 2>&1 | tail -8
