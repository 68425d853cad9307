#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/b2 && mkdir -p $O && cd $R
for a in "--steps 10 --warmup 2" "--steps 20 --warmup 5" ""; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-host-path --no-pmc --no-every-output > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$a', round(d['value']/1e6,1), round(d['ms_per_step'],4), r['step_event_ms'])"
done
