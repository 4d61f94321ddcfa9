#!/bin/bash
# r05 session 21: timing-only builds (wrong results) that cut the Winograd
# forward's z-axis output-transform VALU by half (x1) or all of it (x2):
# does the forward speed up with fewer VALU per MFMA?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s21
mkdir -p $O
for i in 1 2; do
for v in base x1 x2; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_${v}_$i.txt 2> $O/stages_${v}_$i.err || { tail -20 $O/stages_${v}_$i.err; exit 1; }
  echo "== $v $i"; grep -v "^{" $O/stages_${v}_$i.txt | grep "f32" | grep -v bf16 | head -2
done
done
echo ALLDONE
