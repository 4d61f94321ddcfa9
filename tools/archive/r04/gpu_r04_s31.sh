#!/bin/bash
# r04 session 31: conv3 Winograd forward at 3 waves per SIMD
# (amdgpu_waves_per_eu): C3D tests + stage times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s31
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1 || { tail -60 $O/pytest_c3d.log; exit 1; }
tail -2 $O/pytest_c3d.log
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/c3d_stages.txt 2> $O/c3d_stages.err || { tail -30 $O/c3d_stages.err; exit 1; }
grep -v "^{" $O/c3d_stages.txt
echo ALLDONE
