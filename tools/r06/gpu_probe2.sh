#!/bin/bash
# round 6: timing-only k_dense variant reading whole contiguous 1-KiB rows (tools: RT_LUNG_PROBE)
set -o pipefail
mkdir -p gpurun_out
RT_LIB_PATH=$PWD/_var6/librtenv_probe2.so GROUPS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_probe2_prof -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_probe2_prof.log 2>&1 || exit $?
RT_LIB_PATH=$PWD/_var6/librtenv_probe2.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/r06_probe2_pmc2 -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > gpurun_out/r06_probe2_pmc2.log 2>&1 || exit $?
python3 tools/r06/summarize_prof.py gpurun_out/r06_probe2_summary.txt gpurun_out/r06_probe2_prof gpurun_out/r06_probe2_pmc2
rm -rf gpurun_out/r06_probe2_prof gpurun_out/r06_probe2_pmc2
