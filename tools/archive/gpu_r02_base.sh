# round-2 baseline on a fresh box: GPU suite + default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
echo EXIT $?
tail -2 gpurun_out/r02a/pytest_gpu.log; cat gpurun_out/r02a/bench.json | head -c 3000
