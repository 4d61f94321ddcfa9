#!/bin/bash
# round 6: Winograd forward with the whole half's patch reads issued before
# the input transform (in-tree library) against the previous read order
# (_var6/librtenv_nob.so): C3D gates, stage times alternated
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_wino
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c3d.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python tools/c3d_stage_times.py > $O/batch_$i.txt 2> $O/batch_$i.err || { tail $O/batch_$i.err; exit 1; }
  RT_LIB_PATH=$PWD/_var6/librtenv_nob.so timeout -k 10 300 python tools/c3d_stage_times.py > $O/nob_$i.txt 2> $O/nob_$i.err || { tail $O/nob_$i.err; exit 1; }
done
for f in $O/batch_1.txt $O/nob_1.txt $O/batch_2.txt $O/nob_2.txt; do echo "== $f"; grep -v "^{" $f; done
