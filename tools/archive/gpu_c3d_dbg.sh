set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3ddbg
for f in _variants/librtenv_dbg_*.so; do
  v=$(basename $f .so)
  RT_LIB_PATH=$f timeout -k 10 200 python -u -m pytest tests/test_gpu_c3d.py -v -k forward --timeout 100 --timeout-method thread > gpurun_out/c3ddbg/$v.log 2>&1
  echo "$v: $(grep -cE 'PASSED' gpurun_out/c3ddbg/$v.log) passed $(grep -cE 'FAILED' gpurun_out/c3ddbg/$v.log) failed"
  grep -E "Mismatched" gpurun_out/c3ddbg/$v.log | head -5
done
