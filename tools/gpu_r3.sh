#!/bin/bash
# Round-3 GPU check: parity suite, bench line (all secondaries), the --gpus guard and a
# two-rank torchrun rehearsal of the control plane (ranks sharing the box's one GPU).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/${R3_TAG:-r3}
mkdir -p $O && cd $R
echo "[r3] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
echo "[r3] bench"
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
echo "[r3] --gpus 2 on one GPU must fail"
timeout -k 10 120 python bench.py --gpus 2 > $O/gpus2.log 2>&1; echo "rc=$?"; cat $O/gpus2.log | tail -2
echo "[r3] torchrun rehearsal"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --allow-shared-gpu --steps 20 --warmup 5 > $O/torchrun2.log 2>&1 || { tail -30 $O/torchrun2.log; exit 1; }
tail -c 1500 $O/torchrun2.log
echo "[r3] done"
