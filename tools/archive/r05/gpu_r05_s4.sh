#!/bin/bash
# r05 session 4: conv1's Winograd forward in 256-thread blocks now the
# default -- C3D PMC per stage on this tree, C3D + trainer gates; the HIP API
# timeline of the value window's head and tail (tools/call_cost_trace.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_vision.py > $O/pytest_c3d.log 2>&1 || { tail -40 $O/pytest_c3d.log; exit 1; }
tail -1 $O/pytest_c3d.log
export C3D_PMC_B=512
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1 || { tail -5 $O/*.log; exit 1; }
unset C3D_PMC_B
python3 tools/c3d_pmc_summary.py $O $O/c3d_pmc_b512.json > $O/c3d_pmc_b512.txt
cat $O/c3d_pmc_b512.txt
cp $O/c3d_pmc_b512.json profiles/r05/r05_c3d_pmc_b512.json
rm -rf $O/a $O/b $O/c $O/t
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages.txt 2> $O/stages.err || { tail -20 $O/stages.err; exit 1; }
grep -v "^{" $O/stages.txt
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/tr -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_tr.json 2> $O/bench_tr.err || { tail -20 $O/bench_tr.err; exit 1; }
python3 tools/call_cost_trace.py $O/tr 20 > $O/call_cost.txt; head -80 $O/call_cost.txt
rm -rf $O/tr
echo ALLDONE
