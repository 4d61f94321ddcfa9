# A/B of k_ppo_grad_mfma variants (_variants/librtenv_*.so, ABAB order) + the update parity tests on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/grad_*.log
for pass in 1 2; do
  for f in _variants/librtenv_*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f MBS=32768 timeout -k 10 120 python -u tools/bench_ppo_grad.py 2>/dev/null | sed "s/^/$v /" >> gpurun_out/ab/grad.log || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -k "ppo or update or grad or trainer" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
echo EXIT $?
cat gpurun_out/ab/grad.log; tail -2 gpurun_out/ab/pytest.log
