#!/bin/bash
# r05 session 17: Winograd forward with wave issue priority raised for the
# MFMA column phase and lowered for the input transform (p1 / p3 variant builds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s17
mkdir -p $O
for i in 1 2; do
for v in base p1 p3; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_${v}_$i.txt 2> $O/stages_${v}_$i.err || { tail -20 $O/stages_${v}_$i.err; exit 1; }
  echo "== $v $i"; grep -v "^{" $O/stages_${v}_$i.txt | grep "f32" | grep -v bf16
done
done
echo ALLDONE
