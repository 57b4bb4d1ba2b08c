#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks share the card,
# gloo process group (RCCL refuses two ranks on one device). The driver runs the
# real N = 2/4/8 with nccl on a full node.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo > gpurun_out/multi.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/multi.log | tail -3 | cut -c1-600
grep '"gather"' gpurun_out/multi.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gather', d['gather'], 'value', d['value'], 'n_gpus', d['n_gpus'])"
exit $rc
