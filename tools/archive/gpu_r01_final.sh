# round-1 evidence: GPU suite, smoke, default bench, rocprofv3 kernel stats, k_dense PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin4
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin4/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin4/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/fin4/bench.json 2> gpurun_out/fin4/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin4/prof -o run -- python3 bench.py --no-cpu > gpurun_out/fin4/prof_bench.json 2> gpurun_out/fin4/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fin4/pmc_fetch -o run --output-format csv -- python3 bench.py --env-only --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/fin4/pmc_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/fin4/pmc_write -o run --output-format csv -- python3 bench.py --env-only --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/fin4/pmc_w.log 2>&1
echo EXIT $?
tail -2 gpurun_out/fin4/pytest_gpu.log; tail -1 gpurun_out/fin4/smoke.log
