#!/bin/bash
# round 6 session 14: the whole GPU suite + smoke + the driver's bench on the current tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s14_tests.log 2>&1 || { tail -20 gpurun_out/r06_s14_tests.log; exit 1; }
tail -2 gpurun_out/r06_s14_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_s14_smoke.log 2>&1 || { tail -5 gpurun_out/r06_s14_smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_s14_bench.json 2> gpurun_out/r06_s14_bench.err || exit $?
