set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02f
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02f/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_steady.py > gpurun_out/r02f/probe.log 2>&1
echo EXIT $?
tail -3 gpurun_out/r02f/tests.log; grep label gpurun_out/r02f/probe.log
