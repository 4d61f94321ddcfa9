# groups=2 forward: z-shift ring kernel (default) vs the dense ring kernel (RT_C3D_ZS=0): parity, stage timing, vision bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-zs}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in 1 0; do RT_C3D_ZS=$v timeout -k 10 100 python tools/bench_grp.py || exit 1; RT_C3D_ZS=$v timeout -k 10 100 python tools/bench_grp.py --big || exit 1; done
for pass in 1 2; do
  for v in 1 0; do
    RT_C3D_ZS=$v timeout -k 10 300 python -u bench.py --vision --no-cpu > $OUT/b_z${v}_p${pass}.json 2> $OUT/b_z${v}_p${pass}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/b_z${v}_p${pass}.json').read().strip().splitlines()[-1]); c=d['roofline']['c3d_mfma']; print('zs=$v pass $pass vision', round(d['value']), 'update_ms', round(d['ppo_update_ms'],1), 'c3d fwd ms', round(c['forward_ms'],3), 'TF/s', round(c['achieved'],1))"
  done
done
