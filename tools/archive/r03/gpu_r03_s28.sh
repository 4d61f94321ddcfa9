#!/bin/bash
# r03 session 28: bf16x3 conv1 -- C3D, frontend, vision and trainer GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s28
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_frontend.py tests/test_gpu_vision.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo ALLDONE
