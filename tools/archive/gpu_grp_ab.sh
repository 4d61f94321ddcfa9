# grouped-stage forward: z-shift kernel (default) vs the dense ring kernel (RT_C3D_GRP=0): parity, then vision bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-grp}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error|assert" $OUT/pytest.log | head -30; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for pass in 1 2; do
  for v in 1 0; do
    RT_C3D_GRP=$v timeout -k 10 300 python -u bench.py --vision --no-cpu > $OUT/b_g${v}_p${pass}.json 2> $OUT/b_g${v}_p${pass}.err || exit 1
    python -c "
import json; d=json.loads(open('$OUT/b_g${v}_p${pass}.json').read().strip().splitlines()[-1]); c=d['roofline']['c3d_mfma']
st=c.get('stages',{})
print('grp=$v pass $pass vision', round(d['value']), 'update_ms', round(d['ppo_update_ms'],1), 'c3d fwd', round(c['forward_ms'],3) if 'forward_ms' in c else c, {k: (round(v.get('forward_ms',0),3), round(v.get('train_forward_ms',0),3)) for k,v in st.items()} if isinstance(st,dict) else '')"
  done
done
