# round-2 re-entry: full GPU suite + smoke + default bench + rocprofv3 kernel stats
set -o pipefail
OUT=${OUT:-r02u}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${OUT:-r02u}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${OUT:-r02u}/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT:-r02u}/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${OUT:-r02u}/bench.json 2> gpurun_out/${OUT:-r02u}/bench.err && \
cd /tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/evprof -o run -- python3 bench.py --no-cpu > gpurun_out/${OUT:-r02u}/prof.log 2>&1 && python tools/rocpd_stats.py /tmp/evprof/run_results.db gpurun_out/${OUT:-r02u}/kernel_stats.csv
rc=$?
echo EXIT $rc
tail -3 gpurun_out/${OUT:-r02u}/pytest_gpu.log; tail -2 gpurun_out/${OUT:-r02u}/smoke.log; tail -c 600 gpurun_out/${OUT:-r02u}/bench.json
exit $rc
