#!/bin/bash
# Round 5: reference-order MFCC with two chain streams per lane (tree) vs one (ab/lib_chk1.so), outputs
# compared bit for bit; the GPU suite; the two-rank rehearsal with the IPC gather; the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b; mkdir -p $O
echo "[r5b] chains A/B"
for n in 1024 2048; do
  timeout -k 10 240 python -u tools/ab_libs.py --n $n --rounds 7 --compare default=base chainK2=base:2 chainK1=ab/lib_chk1.so:2 > $O/chain_$n.log 2>&1 || { tail -30 $O/chain_$n.log; exit 1; }
  grep -v amdgpu.ids $O/chain_$n.log | tail -8
done
timeout -k 10 240 python -u tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare c4=base c4K2=base:2 c4K1=ab/lib_chk1.so:2 > $O/chain_c4.log 2>&1 || { tail -30 $O/chain_c4.log; exit 1; }
grep -v amdgpu.ids $O/chain_c4.log | tail -8
echo "[r5b] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
echo "[r5b] dist rehearsal"
timeout -k 10 900 bash tools/gpu_dist_rehearsal.sh > $O/dist.log 2>&1 || { tail -30 $O/dist.log; exit 1; }
cat $O/dist.log
echo "[r5b] bench"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic']); print(json.dumps(d['roofline_fp64'])); print(json.dumps(d['cpu_baseline'].get('all_cores'))); print(json.dumps(d['mfcc_exact'])); print(json.dumps(d['c4'].get('mfcc_exact'))); print(json.dumps(d['c5'].get('mfcc_exact'))); print('c5', d['c5']['kernel_ms'], d['c5']['roofline_frac']); print(json.dumps(d.get('latency'))[:1500])"
