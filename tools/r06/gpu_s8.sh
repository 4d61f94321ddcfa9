#!/bin/bash
# round 6 session 8: persistent lung stream with cross-item prefetch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_s8_bench.json 2> gpurun_out/r06_s8_bench.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_trainer.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_rollout.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s8_tests.log 2>&1 || { tail -5 gpurun_out/r06_s8_tests.log; exit 1; }
tail -2 gpurun_out/r06_s8_tests.log
timeout -k 10 300 python bench.py --gpus 2 --rehearse-same-device --steps 10 --warmup 4 --no-cpu --no-c3d --no-steady > gpurun_out/r06_s8_rehearse2.json 2> gpurun_out/r06_s8_rehearse2.err || exit $?
