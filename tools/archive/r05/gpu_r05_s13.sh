#!/bin/bash
# r05 session 13: the N > 1 bench path rehearsed with 2 ranks on the one GPU
# (gloo instead of RCCL, every rank on cuda:0), as the driver launches it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s13
mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --rehearse-same-device --no-cpu --no-c3d > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench2.json'))
print({k: d[k] for k in ('metric','value','n_gpus','ms_per_step','scaling','config')})
print('update ms', d.get('ppo_update_ms'), 'allreduce ms', d.get('update_allreduce_ms'), 'train', d.get('train_env_steps_per_s'))"
echo ALLDONE
