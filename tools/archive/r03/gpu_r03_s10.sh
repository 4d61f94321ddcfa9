#!/bin/bash
# r03 session 10: one-round-trip parameter staging in k_ppo_grad_mfma (tests + update A/B), then the C3D PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trainer.py tests/test_gpu_dp.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for lib in default oldstage; do
  if [ $lib = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_$lib.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --steps 16 --warmup 4 > $O/u.json 2>$O/u.err || { tail $O/u.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/u.json').read().strip().splitlines()[-1]); print('$lib', round(d['ppo_update_ms']*1000,2), 'us/minibatch', round(d['train_env_steps_per_s']/1e6,3), 'M train')"
done; done
unset RT_LIB_PATH
bash tools/gpu_r03_s9.sh
