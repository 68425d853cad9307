#!/bin/bash
# Dynamic instruction budget by ablation (tools/pmc_budget.py): one process runs every variant
# library in ab/ (tools/ablate.py builds copied there), one rocprofv3 --pmc pass per counter set.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/${BUDGET_TAG:-budget}
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
V="${BUDGET_VARIANTS:-BASE=base}"
if [ -n "$BUDGET_SETS" ]; then IFS='|' read -ra SETS <<< "$BUDGET_SETS"; else
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_SALU"
      "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU")
fi
i=0
for s in "${SETS[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $s --kernel-trace --output-format csv -d $O/set$i -o run -- python3 $R/tools/pmc_budget.py $V > $O/set$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 $O/set$i.log; exit 1; }
  i=$((i+1))
done
names=$(for v in $V; do echo -n "${v%%=*} "; done)
python3 $R/tools/pmc_budget.py --report $O $names | tee $O/budget.txt
