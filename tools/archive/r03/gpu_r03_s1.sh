#!/bin/bash
# r03 session 1: the new / changed GPU tests (vision DP, binding, vision CLI, wide C3D)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_binding.py tests/test_gpu_dp.py tests/test_gpu_c3d.py \
  "tests/test_gpu_frontend.py::test_train_cli_vision_reference_grid" > gpurun_out/r03_s1_pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r03_s1_pytest.log
exit $rc
