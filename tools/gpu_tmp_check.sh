#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for cap in 0 768 512; do
  echo "== MGX_GRID_CAP=$cap"
  if [ $cap = 0 ]; then timeout -k 10 200 python tools/step_overlap.py --rounds 3 2>&1 | grep -v amdgpu.ids | tail -9
  else MGX_GRID_CAP=$cap timeout -k 10 200 python tools/step_overlap.py --rounds 3 2>&1 | grep -v amdgpu.ids | tail -9; fi || exit 1
done
