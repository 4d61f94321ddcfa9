# HBM traffic of k_dense_persist (the pipelined rollout's dose stream, 2048 envs per launch):
# FETCH_SIZE / WRITE_SIZE in separate passes -> profiles/k_dense_persist_pmc.json (tools/parse_pmc.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ppmc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ppmc/fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/ppmc/f.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ppmc/write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/ppmc/w.log 2>&1
echo EXIT $?
