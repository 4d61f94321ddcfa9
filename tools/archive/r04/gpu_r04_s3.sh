#!/bin/bash
# r04 session 3: the Winograd conv1 forward (k_conv1_wino) and the cleanup
# build through the C3D stage tests, the extractor test (argmax-routed f64
# reference) and the rollout / trainer / DP / RCCL tests, the C3D stage
# timings, the first-window probe plain and under a rocprofv3 kernel trace,
# and a short bench (value on staggered phases, fused reduce+Adam update)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s3
mkdir -p $O
# test failures (rc 1) do not stop the session; a fault, abort or time limit does
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1
rc=$?; [ $rc -le 1 ] || { tail -60 $O/pytest_c3d.log; exit 1; }
grep -E "^(FAILED|E  )" $O/pytest_c3d.log | cut -c1-200 || true
tail -2 $O/pytest_c3d.log
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/c3d_stages.txt 2> $O/c3d_stages.err || { tail -30 $O/c3d_stages.err; exit 1; }
grep -v "^{" $O/c3d_stages.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_trainer.py tests/test_gpu_dp.py tests/test_gpu_rccl.py tests/test_gpu_headline.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/probe_first_window.py > $O/probe.jsonl 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
cut -c1-150 $O/probe.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 tools/probe_first_window.py > $O/probe_prof.jsonl 2> $O/probe_prof.err || { tail -20 $O/probe_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
rm -rf $O/prof
python3 tools/window_kernels.py $O/kernel_trace.csv > $O/windows.txt
grep "^window" $O/windows.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'timed', round(r['timed_pass_ms_per_step'],4), 'steady', round(d['steady_state']['ms_per_step'],4), 'upd f32 us', round(d['ppo_update_ms']*1000,1), 'bf16x3 us', round(d['ppo_update_ms_bf16x3']*1000,1), 'march', r.get('march',{}).get('frac'))"
echo ALLDONE
