#!/bin/bash
# r04 session 21: k_finish_step again, with the parameter DMA issued before the finish
# and step (k_finish_step: finish of step t-1 + policy + march of step t):
# rollout parity, A/B vs the previous build (prev), three runs each, and the
# phase timeline (staggered)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s21
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_trainer.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for v in prev new; do
  if [ $v = prev ]; then export RT_LIB_PATH=_variants/librtenv_prev.so; else unset RT_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'timed', round(r['timed_pass_ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()}, 'iso', round(r['isolated']['kernel_ms'],4))"
done
done
unset RT_LIB_PATH
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --stagger --steps 24 --dump $O/stamps.npy > $O/trace_stagger.json 2> $O/trace_stagger.err || { tail -30 $O/trace_stagger.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04_s21/trace_stagger.json"))
print(" ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}/{v['max']:.1f}" for k, v in d["phases_us"].items()))
PY
echo ALLDONE
