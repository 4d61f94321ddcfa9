#!/bin/bash
# r03 session 20 (re-entry): full GPU suite + smoke + default bench + kernel-trace stats on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s20
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-steady --no-c3d > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
find $O/prof -name "*.db" -delete
echo ALLDONE
