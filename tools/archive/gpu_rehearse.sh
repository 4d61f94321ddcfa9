# trainer tests, the 1-GPU bench, and a 2-rank rehearsal of the N>1 bench path on one GPU (gloo)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tr.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_quick.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rehearse-same-device --no-cpu --steps 16 --warmup 4 > gpurun_out/bench_r2.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_tr.log; tail -1 gpurun_out/bench_quick.log | cut -c1-200; tail -1 gpurun_out/bench_r2.log | cut -c1-300
exit $rc
