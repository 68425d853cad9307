#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/shares6 && mkdir -p $O && cd $R
for r in 1 2; do for v in eq base; do
  L=$R/abl/libabl_$v.so; [ $v = base ] && L=$R/meyda_amd/libmeyda_gpu.so
  MEYDA_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-path --no-pmc --no-every-output > $O/b_$v.log 2>&1 || { tail $O/b_$v.log; exit 1; }
  tail -1 $O/b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'alone', round(r['step_event_ms']['launch_alone_median_ms'],4))"
done; done
for v in eq base; do
  L=$R/abl/libabl_$v.so; [ $v = base ] && L=$R/meyda_amd/libmeyda_gpu.so
  MEYDA_AMD_LIB=$L timeout -k 10 200 python tools/configs_bench.py C5 C3 > $O/c_$v.log 2>&1 || exit 1
  echo "== $v"; grep '^{' $O/c_$v.log | python3 -c "
import sys,json
for l in sys.stdin:
    c=json.loads(l); print(c['config'], 'alone', round(c['kernel_ms'],4), 'piped', round(c['pipelined_ms'],4))"
done
