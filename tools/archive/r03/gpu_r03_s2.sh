#!/bin/bash
# r03 session 2: remaining changed GPU tests; window/fixed-cost probe (+ kernel
# trace); steady-state trace of bench.py; the default bench line; k_dense_persist PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c3d.py "tests/test_gpu_frontend.py::test_train_cli_vision_reference_grid" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/probe_window.py > $O/window.jsonl 2>$O/window.err || { tail $O/window.err; exit 1; }
cat $O/window.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/wkt -o run --output-format csv -- python3 tools/probe_window.py > $O/window_kt.jsonl 2>$O/window_kt.err || { tail $O/window_kt.err; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bkt -o run --output-format csv -- python3 bench.py --no-cpu > $O/bench_kt.json 2>$O/bench_kt.err || { tail $O/bench_kt.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/dense_pmc_segments.py $O/pf $O/pw $O/k_dense_persist_pmc.json
python3 tools/steady_trace.py $O/wkt > $O/window_trace.jsonl
python3 tools/steady_trace.py $O/bkt > $O/bench_trace.jsonl
find $O -name "*.db" -delete
echo ALLDONE
