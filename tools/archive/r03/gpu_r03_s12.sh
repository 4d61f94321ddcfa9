#!/bin/bash
# r03 session 12: where a vision PPO minibatch goes (kernel trace of bench.py --vision, 64^3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s12
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-c3d --steps 8 --warmup 2 > $O/v64.json 2>$O/v64.err || { tail $O/v64.err; exit 1; }
head -30 $O/kt/run_kernel_stats.csv | cut -c1-180
find $O -name "*.db" -delete
echo ALLDONE
