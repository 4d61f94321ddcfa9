#!/bin/bash
# r03 session 40: transposed window reduction in the ring forward epilogue (RT_EPI_T): C3D tests, A/B timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s40
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_vision.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in epi1 epi0 epi1 epi0; do
  if [ $v = epi1 ]; then L=""; else L="$PWD/_variants/librtenv_$v.so"; fi
  RT_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-update --steps 8 --warmup 4 > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/b_$v.json'))['c3d_mfma']; s=d['stages']['conv1']; b=d['bf16x3']['stages']['conv1']
print('$v conv1 f32 fwd', round(s['forward_ms'],3), 'train', round(s['train_forward_ms'],3), '| bf16x3 fwd', round(b['forward_ms'],3), 'train', round(b['train_forward_ms'],3), '| train pass f32', round(d['train_pass']['ms'],3), 'bf16x3', round(d['bf16x3']['train_pass_ms'],3))"
done
echo ALLDONE
