#!/bin/bash
# r03 session 16: k_ppo_grad_mfma phase timelines (f32, bf16x3) and the bf16x3 error report
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s16
mkdir -p $O
timeout -k 10 120 python -u tools/prec_report.py $O/prec.json || exit 1
for p in f32 bf16x3; do
  RT_PPO_PREC=$p timeout -k 10 120 python -u tools/trace_update.py > $O/trace_$p.json || exit 1
  python -c "import json; d=json.load(open('$O/trace_$p.json')); print('$p', {k: round(v['median'],2) for k, v in d['phases_us'].items()}, 'exit', [round(x,1) for x in d['exit_us']])"
done
