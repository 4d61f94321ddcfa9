#!/bin/bash
# r03 session 5: vision end to end (configs[3] 64^3 and the configs[4] share at 128^3) with the sparse weight gradient
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s5
mkdir -p $O
timeout -k 10 400 python -u bench.py --vision --no-cpu --steps 16 --warmup 4 > $O/vision64.json 2>$O/v64.err || { tail $O/v64.err; exit 1; }
tail -c 1200 $O/vision64.json; echo
timeout -k 10 600 python -u bench.py --vision --grid 128 --no-cpu --no-c3d --steps 8 --warmup 2 > $O/vision128.json 2>$O/v128.err || { tail $O/v128.err; exit 1; }
tail -c 1200 $O/vision128.json; echo
echo ALLDONE
