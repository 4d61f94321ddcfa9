# round-2 closing evidence: full GPU suite + smoke + default bench + rocprofv3 kernel stats + vision benches (64^3, 128^3)
set -o pipefail
OUT=${OUT:-r02f}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/evprof -o run -- python3 bench.py --no-cpu > gpurun_out/$OUT/prof.log 2>&1 && \
python tools/rocpd_stats.py /tmp/evprof/run_results.db gpurun_out/$OUT/kernel_stats.csv && \
timeout -k 10 400 python -u bench.py --vision --no-cpu > gpurun_out/$OUT/vision64.json 2> gpurun_out/$OUT/vision64.err && \
timeout -k 10 600 python -u bench.py --vision --grid 128 --no-cpu > gpurun_out/$OUT/vision128.json 2> gpurun_out/$OUT/vision128.err
rc=$?
echo EXIT $rc
tail -n 2 gpurun_out/$OUT/pytest_gpu.log; tail -n 1 gpurun_out/$OUT/smoke.log
exit $rc
