#!/bin/bash
# Launch overlap of consecutive steps (tools/step_overlap.py) with the persistent grid at its default size (1,024 workgroups
# at N = 1024) and capped to 768 and 512 (MGX_GRID_CAP): profiles/r06_step_overlap.txt, run 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
for cap in 0 768 512; do
  echo "== MGX_GRID_CAP=$cap"
  if [ $cap = 0 ]; then timeout -k 10 200 python tools/step_overlap.py --rounds 3 2>&1 | grep -v amdgpu.ids | tail -9
  else MGX_GRID_CAP=$cap timeout -k 10 200 python tools/step_overlap.py --rounds 3 2>&1 | grep -v amdgpu.ids | tail -9; fi || exit 1
done
