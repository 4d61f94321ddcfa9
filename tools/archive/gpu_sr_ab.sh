# weight-gradient ring slot residue A/B: in-tree build (12) vs variants 16 / 8: parity + per-stage wgrad timing + vision bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-sr}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for pass in 1 2; do
  for v in 12 16 8; do
    if [ $v = 12 ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_sr$v.so; fi
    timeout -k 10 120 python tools/bench_c3d_kernels.py 64 > $OUT/k_${v}_p${pass}.json || exit 1
    python -c "import json,sys; d=json.loads(open('$OUT/k_${v}_p${pass}.json').read().strip().splitlines()[-1]); print('sr=$v', {k:round(v['wgrad_ms'],3) for k,v in d.items() if isinstance(v,dict)})"
  done
done
for v in 12 16; do
  if [ $v = 12 ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_sr$v.so; fi
  timeout -k 10 300 python -u bench.py --vision --no-cpu > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]); print('sr=$v vision', round(d['value']), 'update_ms', round(d['ppo_update_ms'],1))"
done
