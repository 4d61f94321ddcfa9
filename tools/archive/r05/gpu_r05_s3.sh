#!/bin/bash
# r05 session 3: (a) conv1's Winograd forward in 256-thread blocks, 3 per CU
# (variant w256) vs the in-tree 512-thread block: C3D gates, stage times,
# vision f32 end to end; (b) a kernel + HIP API trace of the driver's bench
# command cut at the value window (tools/call_cost_trace.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trainer.py tests/test_gpu_parity.py -k "gae or shuffle or update_call or termination" > $O/pytest_upd.log 2>&1 || { tail -40 $O/pytest_upd.log; exit 1; }
tail -1 $O/pytest_upd.log
RT_LIB_PATH=_variants/librtenv_w256.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d_w256.log 2>&1 || { tail -40 $O/pytest_c3d_w256.log; exit 1; }
tail -1 $O/pytest_c3d_w256.log
for v in base w256; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v = w256 ] && L=_variants/librtenv_w256.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_$v.txt 2> $O/stages_$v.err || { tail -20 $O/stages_$v.err; exit 1; }
  grep -v "^{" $O/stages_$v.txt | head -8
done
for v in base w256; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v = w256 ] && L=_variants/librtenv_w256.so
  RT_LIB_PATH=$L timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_$v.json 2> $O/vision_$v.err || { tail -20 $O/vision_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/vision_$v.json'))
print('$v vision f32: rollout', round(d['value']), 'minibatch ms', round(d['ppo_update_ms'],2), 'iteration', round(d['train_env_steps_per_s']))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/tr -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_tr.json 2> $O/bench_tr.err || { tail -20 $O/bench_tr.err; exit 1; }
python3 tools/call_cost_trace.py $O/tr 20 | tee $O/call_cost.txt
f=$(find $O/tr -name "*kernel_trace.csv" | head -1); python3 - "$f" <<'PY' > $O/value_window_kernels.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
m = next(i for i, r in enumerate(rows) if "k_probe_stream" in r["Kernel_Name"])
t0 = int(rows[m]["Start_Timestamp"])
for r in rows[m: m + 125]:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:34]
    print(f"q{r['Queue_Id']:>3s} {n:34s} {(int(r['Start_Timestamp']) - t0) / 1e3:9.2f} {(int(r['End_Timestamp']) - t0) / 1e3:9.2f}")
PY
head -20 $O/value_window_kernels.txt; tail -8 $O/value_window_kernels.txt
rm -rf $O/tr
echo ALLDONE
