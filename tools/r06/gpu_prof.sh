#!/bin/bash
# round 6: profile the lung-stream kernel alone (kernel stats + two PMC passes), tag $1
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
O=gpurun_out/r06_${T}
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d ${O}_prof -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > ${O}_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_BUSY_CYCLES -d ${O}_pmc1 -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > ${O}_pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d ${O}_pmc2 -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > ${O}_pmc2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS TA_BUSY_avr TA_TA_BUSY_sum -d ${O}_pmc3 -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > ${O}_pmc3.log 2>&1 || true
python3 tools/r06/summarize_prof.py ${O}_prof_summary.txt ${O}_prof ${O}_pmc1 ${O}_pmc2 ${O}_pmc3
mkdir -p gpurun_out/keep && cp ${O}_prof/*kernel_stats.csv gpurun_out/keep/r06_${T}_kernel_stats.csv 2>/dev/null
rm -rf ${O}_prof ${O}_pmc1 ${O}_pmc2 ${O}_pmc3
