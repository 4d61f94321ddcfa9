#!/bin/bash
# r05 session 24: the sparse weight gradient's window loop software-pipelined
# (wp: the next window's patch reads issued before this window's FMAs, two
# register sets, 3 waves per SIMD instead of 4) vs the in-tree loop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s24
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_wp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_wp.log 2>&1 || { tail -40 $O/pytest_wp.log; exit 1; }
tail -1 $O/pytest_wp.log
for i in 1 2; do
for v in base wp; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_${v}_$i.txt 2> $O/stages_${v}_$i.err || { tail -20 $O/stages_${v}_$i.err; exit 1; }
  echo "== $v $i"; grep -v "^{" $O/stages_${v}_$i.txt | grep "f32" | grep -v bf16
done
done
echo ALLDONE
