#!/bin/bash
# r04 session 5: Winograd data gradient with batched window loads and two
# blocks per CU (C3D tests + stage times), the phase timeline of the
# pipelined dense rollout (traced build; lockstep and staggered phases), and
# the configs[3] vision bench f32 with a rocprofv3 kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1
rc=$?; [ $rc -le 1 ] || { tail -60 $O/pytest_c3d.log; exit 1; }
grep -E "^(FAILED|E  )" $O/pytest_c3d.log | cut -c1-200 || true
tail -2 $O/pytest_c3d.log
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/c3d_stages.txt 2> $O/c3d_stages.err || { tail -30 $O/c3d_stages.err; exit 1; }
grep -v "^{" $O/c3d_stages.txt
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --steps 24 > $O/trace_lockstep.json 2> $O/trace_lockstep.err || { tail -30 $O/trace_lockstep.err; exit 1; }
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --stagger --steps 24 > $O/trace_stagger.json 2> $O/trace_stagger.err || { tail -30 $O/trace_stagger.err; exit 1; }
python3 - <<'EOF'
import json
for n in ("lockstep", "stagger"):
    d = json.load(open(f"gpurun_out/r04_s5/trace_{n}.json"))
    print(n, " ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}/{v['max']:.1f}" for k, v in d["phases_us"].items()))
    for k, v in d["kernel_span_us"].items():
        print("   ", k, {a: round(b, 1) for a, b in v.items()})
EOF
timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python -c "
import json; d=json.load(open('$O/vision_f32.json'))
print('vision f32: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s; c3d train pass f32', round(d['c3d_mfma']['train_pass']['ms'],3), 'bf16x3', round(d['c3d_mfma']['bf16x3']['train_pass_ms'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-c3d > $O/vision_prof.json 2> $O/vision_prof.err || { tail -20 $O/vision_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/vision_kernel_stats.csv
rm -rf $O/prof
head -16 $O/vision_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
echo ALLDONE
