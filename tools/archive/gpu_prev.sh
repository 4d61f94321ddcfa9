# dense rollout with the previous step's finish fused into the policy kernel: parity + bench + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prev
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_fused_step.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prev/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/prev/bench.json 2> gpurun_out/prev/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prev/prof -o run -- python3 bench.py --no-cpu --no-update > gpurun_out/prev/prof_bench.json 2> gpurun_out/prev/prof.err
echo EXIT $?
tail -2 gpurun_out/prev/pytest.log
