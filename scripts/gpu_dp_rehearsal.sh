#!/bin/bash
# Rehearse bench.py's N > 1 code path on a one-GPU box: 2 ranks, gloo, both on cuda:0, in-launch
# polls off (two processes share the card: SD_POLL=0).  The driver's own scaling runs use one GPU
# per rank over RCCL (nccl); this only checks that every multi-rank branch runs and aggregates.
set -eo pipefail
cd $GRAFT_REPO_ROOT
SD_POLL=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --stream-steps 3 \
  > gpurun_out/dp2.json 2> gpurun_out/dp2.err
python -c "import json; d=json.loads(open('gpurun_out/dp2.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','n_gpus','ms_per_step')}); print(d['strong_scaling']); print({k: d['stream'][k] for k in ('value','n_gpus','ms_per_step','exact')})"
