# round-2: DP f64 test, beam list test, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "dp or beam_list" > gpurun_out/r02d/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err
echo EXIT $?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r02d/tests.log | tail -8; tail -5 gpurun_out/r02d/bench.err
