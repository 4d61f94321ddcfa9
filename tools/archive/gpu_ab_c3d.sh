# A/B of the C3D stage kernels (_variants/librtenv_c3d_*.so, two passes) + the C3D parity tests on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abc3d
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3d.py -x -q --timeout 200 --timeout-method thread > gpurun_out/abc3d/pytest.log 2>&1 || exit 1
for pass in 1 2; do
  for f in _variants/librtenv_c3d_*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 200 python -u tools/bench_c3d_kernels.py > gpurun_out/abc3d/${v}_$pass.log 2>&1 || exit 1
  done
done
echo EXIT $?
