# C3D forward experiments: _variants/librtenv_c3d_*.so through tools/bench_c3d_kernels.py, two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3dexp
for pass in 1 2; do
  for f in _variants/librtenv_c3d_*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 200 python -u tools/bench_c3d_kernels.py > gpurun_out/c3dexp/${v}_$pass.log 2>&1 || exit 1
  done
done
for f in gpurun_out/c3dexp/*_2.log; do echo $f; tail -1 $f | cut -c1-400; done
