# pipelined dense rollout: k_dense and latency kernels on separate streams (RT_PIPE_DL=1),
# the latency stream at high priority (2), vs the per-group streams (0); parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dl
RT_PIPE_DL=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dl/pytest2.log 2>&1 || exit 1
RT_PIPE_DL=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dl/pytest1.log 2>&1 || exit 1
i=0
for v in 0 1 2 0 1 2; do
  i=$((i + 1))
  RT_PIPE_DL=$v timeout -k 10 120 python -u bench.py --no-cpu --no-update > gpurun_out/dl/b_${v}_r$i.log 2>&1 || exit 1
done
echo EXIT $?
