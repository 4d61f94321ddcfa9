set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_quick.log 2>&1 && \
bash tools/archive/gpu_dense_pmc.sh
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench_quick.log
exit $rc
