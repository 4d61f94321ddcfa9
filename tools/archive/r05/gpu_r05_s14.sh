#!/bin/bash
# r05 session 14: c3d.hip under the AMDGPU scheduler strategies (variant
# builds: silp = max-ilp, smem = max-memory-clause, sminreg =
# iterative-minreg) vs the default: C3D gates on each, stage times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s14
mkdir -p $O
for v in base silp smem sminreg; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_$v.txt 2> $O/stages_$v.err || { tail -20 $O/stages_$v.err; exit 1; }
  echo "== $v"; grep -v "^{" $O/stages_$v.txt | grep "f32"
done
for v in silp smem sminreg; do
  RT_LIB_PATH=_variants/librtenv_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_$v.log 2>&1; echo "$v pytest rc=$? $(tail -1 $O/pytest_$v.log)"
done
echo ALLDONE
