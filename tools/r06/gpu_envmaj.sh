#!/bin/bash
# round 6: timing-only k_dense variant reading whole contiguous 1-KiB rows (tools: RT_LUNG_PROBE)
set -o pipefail
mkdir -p gpurun_out
RT_LIB_PATH=$PWD/_var6/librtenv_envmaj.so GROUPS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_envmaj_prof -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_envmaj_prof.log 2>&1 || exit $?
RT_LIB_PATH=$PWD/_var6/librtenv_envmaj.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/r06_envmaj_pmc2 -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_envmaj_pmc2.log 2>&1 || exit $?
python3 tools/r06/summarize_prof.py gpurun_out/r06_envmaj_summary.txt gpurun_out/r06_envmaj_prof gpurun_out/r06_envmaj_pmc2
rm -rf gpurun_out/r06_envmaj_prof gpurun_out/r06_envmaj_pmc2
RT_LIB_PATH=$PWD/_var6/librtenv_envmaj.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > gpurun_out/r06_envmaj_bench.json 2> gpurun_out/r06_envmaj_bench.err
