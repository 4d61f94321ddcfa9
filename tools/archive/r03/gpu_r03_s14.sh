#!/bin/bash
# r03 session 14: how MFMA-bound is k_ppo_grad_mfma's tile phase? timing-only variants with 1/2 and 1/4
# of the 64x64 products (RT_MF_DIV, wrong results), update A/B via bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s14
mkdir -p $O
for rep in 1 2; do for lib in base div2 div4; do
  export RT_LIB_PATH=$PWD/_variants/librtenv_$lib.so
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --steps 16 --warmup 4 > $O/u.json 2>$O/u.err || { tail $O/u.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/u.json').read().strip().splitlines()[-1]); print('$lib', round(d['ppo_update_ms']*1000,2), 'us/minibatch')"
done; done
