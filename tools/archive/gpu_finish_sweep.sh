# pipelined dense rollout: k_finish waves per block (RT_FINISH_WPB), two passes; parity at 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fsweep
RT_FINISH_WPB=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fsweep/pytest.log 2>&1 || exit 1
i=0
for w in 4 2 1 4 2 1; do
  i=$((i + 1))
  RT_FINISH_WPB=$w timeout -k 10 120 python -u bench.py --no-cpu --no-update > gpurun_out/fsweep/b_${w}_r$i.log 2>&1 || exit 1
done
echo EXIT $?
