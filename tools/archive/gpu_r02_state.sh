# round-2 re-entry: full GPU suite + smoke + default bench + rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02t
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02t/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02t/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r02t/bench.json 2> gpurun_out/r02t/bench.err && \
cd /tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02t/prof -o run -- python3 bench.py --no-cpu > gpurun_out/r02t/prof.log 2>&1
rc=$?
echo EXIT $rc
tail -3 gpurun_out/r02t/pytest_gpu.log; tail -2 gpurun_out/r02t/smoke.log; tail -c 600 gpurun_out/r02t/bench.json
exit $rc
