#!/bin/bash
# r05 session 19: the Winograd column sums as scalar adds instead of
# v_pk_add_f32 (in-tree source), with the SLP vectorizer off (scns) or on
# (base), against the committed source with SLP off (ns) and on (head)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s19
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_scns.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_configs.py > $O/pytest_scns.log 2>&1 || { tail -40 $O/pytest_scns.log; exit 1; }
tail -1 $O/pytest_scns.log
for i in 1 2; do
for v in head base ns scns; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_${v}_$i.txt 2> $O/stages_${v}_$i.err || { tail -20 $O/stages_${v}_$i.err; exit 1; }
  echo "== $v $i"; grep -v "^{" $O/stages_${v}_$i.txt | grep "f32" | grep -v bf16
done
done
echo ALLDONE
