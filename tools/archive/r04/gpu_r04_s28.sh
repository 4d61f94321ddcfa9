#!/bin/bash
# r04 session 28: vision tests incl. the render-from-store-rows parity test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s28
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_vision.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
echo ALLDONE
