# pipelined dense rollout: policy block size / k_dense turn sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/pytest_rollout.log 2>&1 || exit 1
for cfg in "4 1" "8 1" "2 1" "16 1" "4 0" "8 0"; do
  set -- $cfg
  RT_PIPE_WPB=$1 RT_PIPE_SERIAL=$2 timeout -k 10 120 python -u bench.py --no-cpu --no-update > gpurun_out/sweep/b_$1_$2.log 2>&1 || exit 1
done
timeout -k 10 120 python -u bench.py --no-cpu --no-update --rollout-groups 1 > gpurun_out/sweep/b_g1.log 2>&1
echo EXIT $?
