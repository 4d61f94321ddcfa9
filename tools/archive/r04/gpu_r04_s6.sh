#!/bin/bash
# r04 session 6: policy parameters staged by LDS DMA, the finish's tumour
# gather with 4 voxels per lane in flight (lung bit packed in the voxel
# coordinates): env/rollout/policy/trainer parity, the pipelined-rollout phase
# timeline (staggered), and a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s6
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused_step.py tests/test_gpu_rollout.py tests/test_gpu_trainer.py tests/test_gpu_vision.py tests/test_gpu_binding.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --stagger --steps 24 > $O/trace_stagger.json 2> $O/trace_stagger.err || { tail -30 $O/trace_stagger.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04_s6/trace_stagger.json"))
print(" ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}/{v['max']:.1f}" for k, v in d["phases_us"].items()))
for k, v in d["kernel_span_us"].items():
    print("   ", k, {a: round(b, 1) for a, b in v.items()})
PY
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'timed', round(r['timed_pass_ms_per_step'],4), 'steady', round(d['steady_state']['ms_per_step'],4), 'kms', {k: round(v,4) for k,v in r['kernel_ms_all'].items()}, 'upd f32 us', round(d['ppo_update_ms']*1000,1), 'march', r.get('march',{}).get('frac'), 'incr', d['other_step_mode']['env_steps_per_s'])"
echo ALLDONE
