# k_dense unroll / slice sweep (_variants/librtenv_d<unroll>_<slice>.so), env-only bench, two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dsweep
for pass in 1 2; do
  for f in _variants/librtenv_d*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 120 python -u bench.py --env-only --no-cpu --no-update --steps 64 > gpurun_out/dsweep/${v}_$pass.log 2>&1 || exit 1
  done
done
echo EXIT $?
