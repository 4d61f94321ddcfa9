#!/bin/bash
# r04 session 10: k_dense's reduction with few VALU ops per float4 (ballot
# popcount count, f32 partial sums) vs the previous build (b5u8): parity
# (rollout, headline doses.lung vs the oracle, parity), three A/B runs each;
# the incremental persistent rollout's phase timeline; the PPO update's
# phase timeline and a rocprofv3 kernel trace of the update
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for v in old new; do
  if [ $v = old ]; then export RT_LIB_PATH=_variants/librtenv_b5u8.so; else unset RT_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()}, 'iso', round(r['isolated']['kernel_ms'],4), 'incr', round(d['other_step_mode']['env_steps_per_s']/1e6,2))"
done
done
unset RT_LIB_PATH
timeout -k 10 300 python3 tools/trace_env.py --mode incremental --persistent --steps 24 > $O/trace_incr.json 2> $O/trace_incr.err || { tail -30 $O/trace_incr.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04_s10/trace_incr.json"))
print("incr", " ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}/{v['max']:.1f}" for k, v in d["phases_us"].items()))
print("   ", d.get("persistent"))
PY
timeout -k 10 300 python3 tools/trace_update.py > $O/trace_update.json 2> $O/trace_update.err || { tail -30 $O/trace_update.err; exit 1; }
cut -c1-1500 $O/trace_update.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 4 --warmup 2 --no-cpu --no-c3d --no-steady > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
grep -E "ppo|adam|reduce" $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo ALLDONE
