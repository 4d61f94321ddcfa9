#!/bin/bash
# r05 session 1: per-call precision (ABI 4), reduce+Adam occupancy check, new
# tests (staggered start vs oracle, update call == grad + adam, episode t);
# C3D PMC per stage on the current tree (bench's c3d_mfma reads it), then the
# whole GPU suite, smoke and the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s1
mkdir -p $O
export C3D_PMC_B=512
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1 || { tail -5 $O/*.log; exit 1; }
unset C3D_PMC_B
python3 tools/c3d_pmc_summary.py $O $O/c3d_pmc_b512.json > $O/c3d_pmc_b512.txt
cat $O/c3d_pmc_b512.txt
mkdir -p profiles/r05 && cp $O/c3d_pmc_b512.json profiles/r05/r05_c3d_pmc_b512.json
rm -rf $O/a $O/b $O/c $O/t
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED|^ERROR" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_s1"
d = json.load(open(f"{O}/bench.json")); r = d["roofline"]; s = d["steady_state"]; c = d["c3d_mfma"]
print("bench", round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", round(s["ms_per_step"], 4),
      "frac", round(r["frac"], 3), "step_frac", round(r["step_frac_of_hbm"], 3),
      "upd f32 us", round(d["ppo_update_ms"] * 1000, 1), "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2),
      "incr frac", round(d["other_step_mode"]["roofline"]["frac"], 3))
print("c3d fwd frac", round(c["forward"]["frac"], 3), "train frac", round(c["train_pass"]["frac"], 3), "train ms", round(c["train_pass"]["ms"], 3))
for k, v in c["stages"].items():
    print(k, {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items() if "frac" in kk or kk.endswith("_ms")},
          {kk: (vv["mfma_busy"], vv["count_matches_planner"], vv["busy_x_clock_over_2.4GHz"]) for kk, vv in v.items() if kk.endswith("_pmc")})
PY
echo ALLDONE
