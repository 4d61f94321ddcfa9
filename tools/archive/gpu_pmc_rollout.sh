# PMC passes over the persistent rollout kernel (one pass per counter group)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rpmc/trace -o run -- python3 tools/rollout_pmc_driver.py > gpurun_out/rpmc_trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/rpmc/p1 -o run --output-format csv -- python3 tools/rollout_pmc_driver.py > gpurun_out/rpmc_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/rpmc/p2 -o run --output-format csv -- python3 tools/rollout_pmc_driver.py > gpurun_out/rpmc_p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P3 -d gpurun_out/rpmc/p3 -o run --output-format csv -- python3 tools/rollout_pmc_driver.py > gpurun_out/rpmc_p3.log 2>&1
rc=$?
ls -R gpurun_out/rpmc | head -30
exit $rc
