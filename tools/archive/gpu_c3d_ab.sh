# C3D: parity tests on the in-tree build, then A/B of _variants/librtenv_c3d_*.so (tools/bench_c3d_kernels.py, 2 passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3dab
rm -f gpurun_out/c3dab/*
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3d.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c3dab/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/c3dab/pytest.log
[ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for f in _variants/librtenv_c3d_*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 200 python -u tools/bench_c3d_kernels.py ${C3D_B:-64} > gpurun_out/c3dab/${v}_$pass.log 2>&1 || exit 1
  done
done
python tools/c3d_ab_summary.py gpurun_out/c3dab
