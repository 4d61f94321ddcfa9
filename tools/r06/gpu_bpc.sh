#!/bin/bash
# round 6: pipelined k_dense blocks per CU sweep (variant builds in _var6/)
set -o pipefail
mkdir -p gpurun_out
for b in 4 6 8; do
  RT_LIB_PATH=$PWD/_var6/librtenv_bpc$b.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > gpurun_out/r06_bpc$b.json 2> gpurun_out/r06_bpc$b.err || exit $?
done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > gpurun_out/r06_bpc5.json 2> gpurun_out/r06_bpc5.err
