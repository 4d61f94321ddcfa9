# A/B of k_ppo_grad_mfma variants (_variants/librtenv_v*.so) + the update parity tests on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in v0 v2 v0 v2; do
  RT_LIB_PATH=_variants/librtenv_$v.so MBS=32768 timeout -k 10 120 python -u tools/bench_ppo_grad.py >> gpurun_out/ab/grad_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests -m gpu -k "ppo or update or grad or trainer" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
echo EXIT $?
cat gpurun_out/ab/grad_*.log; tail -2 gpurun_out/ab/pytest.log
