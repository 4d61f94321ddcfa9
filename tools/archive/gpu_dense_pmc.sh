# k_dense HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes) -> profiles/k_dense_pmc.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/dpmc/fetch -o run --output-format csv -- python3 bench.py --env-only --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/dpmc_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/dpmc/write -o run --output-format csv -- python3 bench.py --env-only --steps 20 --warmup 2 --no-cpu --no-update > gpurun_out/dpmc_w.log 2>&1
