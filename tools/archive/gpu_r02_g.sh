set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02g/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02g/bench.json 2>gpurun_out/r02g/bench.err
echo EXIT $?
tail -3 gpurun_out/r02g/tests.log
