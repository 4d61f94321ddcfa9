# PMC passes over k_ppo_grad_mfma (minibatch 32768): issue / wait / MFMA / LDS counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MBS=32768
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
timeout -k 10 200 python3 tools/bench_ppo_grad.py > gpurun_out/grad_bench.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/gpmc/p1 -o run --output-format csv -- python3 tools/bench_ppo_grad.py > gpurun_out/gpmc_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/gpmc/p2 -o run --output-format csv -- python3 tools/bench_ppo_grad.py > gpurun_out/gpmc_p2.log 2>&1
rc=$?
cat gpurun_out/grad_bench.log | tail -1; tail -3 gpurun_out/gpmc_p2.log
exit $rc
