#!/bin/bash
# The driver's multi-GPU command line, rehearsed on a one-GPU box with two ranks sharing the
# device: first without the RCCL gather (the torchrun / gloo control path), then with it
# (RCCL may refuse two ranks on one device; that outcome is reported, not retried).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/dist
mkdir -p $O && cd $R
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 2 --no-gather --allow-shared-gpu > $O/nogather.log 2>&1
rc=$?; tail -2 $O/nogather.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --steps 5 --warmup 2 > $O/gather.log 2>&1
rc=$?; echo "gather rc=$rc"; grep -E "metric|Error|error|refuse|duplicate|Duplicate" $O/gather.log | head -5 | cut -c1-600
exit 0
