# kernel timeline of the PPO update (bench.py, update phase): durations and inter-kernel gaps
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-updprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/updprof -o run -- python3 bench.py --no-cpu --no-c3d --no-steady > $OUT/bench.json 2> $OUT/bench.err
rc=$?
python tools/rocpd_gaps.py /tmp/updprof/run_results.db k_ppo_grad_mfma k_ppo_reduce k_adam k_shuffle k_adv_partial k_adv_stats k_gae k_dense_persist k_step_policy k_finish | tee $OUT/gaps.txt
exit $rc
