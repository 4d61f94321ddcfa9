set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_fused_step.py tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_quick.log 2>&1
tail -8 gpurun_out/pytest_quick.log; tail -1 gpurun_out/bench_quick.log | cut -c1-400
exit $rc
