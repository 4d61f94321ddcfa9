#!/bin/bash
# r04 session 9: k_dense_persist shape sweep at 5-8 blocks per CU x 2-8 float4 loads
# in flight per thread (the chain kernels wait behind the dose stream queue)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in b5u8 b5u4 b5u2 b6u4 b8u4 b8u2 b7u4; do
  RT_LIB_PATH=_variants/librtenv_$v.so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()}, 'iso', round(r['isolated']['kernel_ms'],4))"
done
done
echo ALLDONE
