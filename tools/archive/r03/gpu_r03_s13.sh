#!/bin/bash
# r03 session 13: full GPU suite + smoke on the current tree; the N>1 bench path rehearsed with 2 ranks on the one GPU (gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s13
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-same-device --no-cpu --no-c3d --steps 16 --warmup 4 > $O/rehearse2.json 2>$O/rehearse2.err || { tail -30 $O/rehearse2.err; exit 1; }
tail -c 1500 $O/rehearse2.json; echo
echo ALLDONE
