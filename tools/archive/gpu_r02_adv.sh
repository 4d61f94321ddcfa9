# round-2: ADVICE fixes (LDS order, reseed, bitwise resume) + a short learning-run timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_trainer.py tests/test_gpu_frontend.py > gpurun_out/r02a/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/repro_learning.py --out gpurun_out/r02a/learn2m --total 2000000 > gpurun_out/r02a/learn2m.log 2>&1
rc=$?
echo EXIT $rc
grep -E "passed|failed|FAIL|Error" gpurun_out/r02a/tests.log | tail -8; tail -4 gpurun_out/r02a/learn2m.log
exit $rc
