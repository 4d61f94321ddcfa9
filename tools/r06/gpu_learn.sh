#!/bin/bash
# round 6: the published learning curve with the torch autograd update (fused_update = 0), seed $1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/repro_learning.py --fused-update 0 --seed $1 --out gpurun_out/r06_learn_autograd_seed$1 > gpurun_out/r06_learn_autograd_seed$1.log 2>&1
rc=$?; tail -3 gpurun_out/r06_learn_autograd_seed$1.log; exit $rc
