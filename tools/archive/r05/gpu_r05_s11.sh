#!/bin/bash
# r05 session 11 (evidence on the tree): the whole GPU suite, smoke, the
# driver's bench command plain (x2) and under rocprofv3 --kernel-trace --stats,
# k_dense_persist FETCH_SIZE / WRITE_SIZE (separate --pmc passes), the C3D PMC
# per stage (separate passes) + stage times, vision f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s11
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || { tail -30 $O/bench$i.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/dense_pmc_segments.py $O/pf $O/pw $O/k_dense_persist_pmc.json > /dev/null
rm -rf $O/pf $O/pw
export C3D_PMC_B=512
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1 || { tail -5 $O/*.log; exit 1; }
unset C3D_PMC_B
python3 tools/c3d_pmc_summary.py $O $O/c3d_pmc_b512.json > $O/c3d_pmc_b512.txt
cat $O/c3d_pmc_b512.txt
rm -rf $O/a $O/b $O/c $O/t
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages.txt 2> $O/stages.err || { tail -20 $O/stages.err; exit 1; }
grep -v "^{" $O/stages.txt
timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_s11"
for i in (1, 2):
    d = json.load(open(f"{O}/bench{i}.json")); r = d["roofline"]; s = d["steady_state"]
    print("bench", i, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", round(s["ms_per_step"], 4),
          "vs_value", round(s["vs_value"], 4), "frac", round(r["frac"], 3), "step_frac", round(r["step_frac_of_hbm"], 3),
          "upd f32 us", round(d["ppo_update_ms"] * 1000, 1), "train", round(d["train_env_steps_per_s"] / 1e6, 2),
          "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2), "incr frac", round(d["other_step_mode"]["roofline"]["frac"], 3),
          "cpu", d["cpu_baseline"].get("value"))
d = json.load(open(f"{O}/vision_f32.json"))
print("vision f32: rollout", round(d["value"]), "minibatch ms", round(d["ppo_update_ms"], 2), "iteration", round(d["train_env_steps_per_s"]))
PY
echo ALLDONE
