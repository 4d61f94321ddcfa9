#!/bin/bash
# round 6 session 8: persistent lung stream with cross-item prefetch + its profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_s8_bench.json 2> gpurun_out/r06_s8_bench.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_trainer.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_rollout.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s8_tests.log 2>&1 || { tail -5 gpurun_out/r06_s8_tests.log; exit 1; }
tail -2 gpurun_out/r06_s8_tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_s8_prof -o kd -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_s8_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/r06_s8_pmc1 -o kd -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_s8_pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/r06_s8_pmc2 -o kd -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_s8_pmc2.log 2>&1 || exit $?
python3 tools/r06/summarize_prof.py gpurun_out/r06_s8_prof_summary.txt gpurun_out/r06_s8_prof gpurun_out/r06_s8_pmc1 gpurun_out/r06_s8_pmc2
mkdir -p gpurun_out/keep && cp gpurun_out/r06_s8_prof/*/*kernel_stats.csv gpurun_out/keep/ 2>/dev/null
rm -rf gpurun_out/r06_s8_prof gpurun_out/r06_s8_pmc1 gpurun_out/r06_s8_pmc2
