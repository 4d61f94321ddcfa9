# C3D stage kernels: instruction mix and stall counters (two separate --pmc passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3dpmc
export TMPDIR=/tmp C3D_PMC_B=${C3D_PMC_B:-64}
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d gpurun_out/c3dpmc/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > gpurun_out/c3dpmc/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d gpurun_out/c3dpmc/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > gpurun_out/c3dpmc/b.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/c3dpmc/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > gpurun_out/c3dpmc/c.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/c3dpmc/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > gpurun_out/c3dpmc/t.log 2>&1
echo EXIT $?
tail -3 gpurun_out/c3dpmc/a.log gpurun_out/c3dpmc/b.log
