#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update --no-steady > gpurun_out/r06_exp_fullrows.json 2> gpurun_out/r06_exp_fullrows.err
