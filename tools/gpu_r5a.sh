#!/bin/bash
# Round 5: the run-time schedule A/B (outputs checked bit for bit), the GPU suite, the two-rank
# rehearsal with the IPC gather, the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
echo "[r5a] dyn A/B"
DYN="1:2 1:4 2:1 2:2" timeout -k 10 300 python -u tools/dyn_ab.py 1024 2048 512 > $O/dyn_ab.log 2>&1 || { tail -30 $O/dyn_ab.log; exit 1; }
grep -v amdgpu.ids $O/dyn_ab.log
echo "[r5a] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
echo "[r5a] dist rehearsal"
timeout -k 10 900 bash tools/gpu_dist_rehearsal.sh > $O/dist.log 2>&1 || { tail -30 $O/dist.log; exit 1; }
cat $O/dist.log
echo "[r5a] bench"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic']); print(json.dumps(d['roofline_fp64'])); print(json.dumps(d['cpu_baseline'].get('all_cores'))); print(json.dumps(d['c4'].get('mfcc_exact'))); print(json.dumps(d['c5'].get('mfcc_exact'))); print('c5', d['c5']['kernel_ms'], d['c5']['roofline_frac']); print(json.dumps(d.get('latency'))[:1500])"
