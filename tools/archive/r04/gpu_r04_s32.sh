#!/bin/bash
# r04 session 32: Winograd data gradient at three blocks per CU (53 KB LDS
# share: one-row z chunks) vs two (variant dg53): C3D tests on the variant,
# stage times of both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s32
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_dg53.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1 || { tail -60 $O/pytest_c3d.log; exit 1; }
tail -2 $O/pytest_c3d.log
for v in prod dg53; do
  if [ $v = prod ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=_variants/librtenv_$v.so; fi
  timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/c3d_stages_$v.txt 2> $O/c3d_stages_$v.err || { tail -30 $O/c3d_stages_$v.err; exit 1; }
  echo "== $v"; grep -v "^{" $O/c3d_stages_$v.txt | grep "f32"
done
echo ALLDONE
