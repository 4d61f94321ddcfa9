set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/spmc
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/spmc/kt -o run --output-format csv -- python3 tools/probe_steady_pmc.py > gpurun_out/spmc/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/spmc/f -o run --output-format csv -- python3 tools/probe_steady_pmc.py > gpurun_out/spmc/f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/spmc/w -o run --output-format csv -- python3 tools/probe_steady_pmc.py > gpurun_out/spmc/w.log 2>&1
echo EXIT $?
find gpurun_out/spmc -name "*.csv" | head
