#!/bin/bash
# round 6: conv1's Winograd forward at 4 waves per SIMD (<= 128 VGPRs, ~20
# spilled; 4 blocks per CU, a quarter of the LDS each) with and without the
# batched patch reads, against the tree (3 waves per SIMD): C3D gates on c1w4,
# stage times alternated
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_c1w4
mkdir -p $O
RT_LIB_PATH=$PWD/_var6/librtenv_c1w4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c3d.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for t in cur c1w4 c1w4nb; do
    L=""; [ $t != cur ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 300 python tools/c3d_stage_times.py > $O/${t}_$i.txt 2> $O/${t}_$i.err || { tail $O/${t}_$i.err; exit 1; }
  done
done
for f in $O/cur_1.txt $O/c1w4_1.txt $O/c1w4nb_1.txt $O/cur_2.txt $O/c1w4_2.txt $O/c1w4nb_2.txt; do echo "== $f"; grep -E "f32     conv1|^f32 forward" $f; done
