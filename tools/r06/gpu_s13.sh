#!/bin/bash
# round 6 session 10: k_dense rows skipped past a group's longest chain, rows line-aligned
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > gpurun_out/r06_s13_bench.json 2> gpurun_out/r06_s13_bench.err || exit $?
bash tools/r06/gpu_prof.sh s13
