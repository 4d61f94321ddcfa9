# pipelined dense rollout: parity tests, the GPU suite, bench (2 groups vs 1), kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_rollout.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu --rollout-groups 1 > gpurun_out/bench_g1.log 2>&1 && \
export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_rollout.log; tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-600; tail -1 gpurun_out/bench_g1.log | cut -c1-400
