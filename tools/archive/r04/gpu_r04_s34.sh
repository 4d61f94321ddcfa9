#!/bin/bash
# r04 session 34: PPO update -- W2 partials stored write-through (float4
# sc1) by k_ppo_grad_mfma, k_ppo_reduce_adam loads the Adam state before
# its arrival wait -- vs HEAD (updold): trainer/DP tests, three A/B runs of
# the bench's update timing, rocprofv3 kernel stats of the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s34
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trainer.py tests/test_gpu_dp.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for v in old new; do
  if [ $v = old ]; then export RT_LIB_PATH=_variants/librtenv_updold.so; else unset RT_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-steady > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', $rep, 'value', round(d['value']/1e6,3), 'upd f32 us', round(1000*d['ppo_update_ms'],2), 'bf16x3 us', round(1000*d['ppo_update_ms_bf16x3'],2), 'iter', round(d['train_env_steps_per_s']/1e6,3))"
done
done
unset RT_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 4 --warmup 2 --no-cpu --no-c3d --no-steady > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
grep -E "ppo|adam|reduce" $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo ALLDONE
