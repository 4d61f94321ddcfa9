#!/bin/bash
# r04 session 16: render gather (vision parity + trainer), configs[3] vision
# bench f32, and the incremental persistent rollout's raw stamps (straggler
# analysis: per-wave life vs block / tumour)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s16
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_vision.py tests/test_gpu_trainer.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python -c "
import json; d=json.load(open('$O/vision_f32.json'))
print('vision f32: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s; c3d train pass f32', round(d['c3d_mfma']['train_pass']['ms'],3), 'bf16x3', round(d['c3d_mfma']['bf16x3']['train_pass_ms'],3))"
timeout -k 10 300 python3 tools/trace_env.py --mode incremental --persistent --steps 24 --dump $O/stamps_incr.npy > $O/trace_incr.json 2> $O/trace_incr.err || { tail -30 $O/trace_incr.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04_s16/trace_incr.json"))
print("incr", " ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}/{v['max']:.1f}" for k, v in d["phases_us"].items()))
print("   ", d.get("persistent"))
PY
echo ALLDONE
