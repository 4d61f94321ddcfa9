#!/bin/bash
# r04 session 14: Winograd forward patch reads as whole ds_read_b64 (64-bank rule) on the
# bank-model strides; planner unchanged: C3D tests, stage times, PMC b512, vision f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s14
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1 || { tail -60 $O/pytest_c3d.log; exit 1; }
tail -2 $O/pytest_c3d.log
timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/c3d_stages.txt 2> $O/c3d_stages.err || { tail -30 $O/c3d_stages.err; exit 1; }
grep -v "^{" $O/c3d_stages.txt
export C3D_PMC_B=512
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1 || { tail -5 $O/*.log; exit 1; }
unset C3D_PMC_B
python3 tools/c3d_pmc_summary.py $O $O/c3d_pmc_b512.json
python3 -c "
import json; d=json.load(open('$O/c3d_pmc_b512.json'))['kernels']
for k,v in d.items(): print(k[:50], 'lds_conflict_frac', round(v.get('lds_conflict_frac',0),3), 'lds_active', round(v.get('lds_active_frac',0),3))"
rm -rf $O/a $O/b $O/c $O/t
timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python -c "
import json; d=json.load(open('$O/vision_f32.json'))
print('vision f32: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s; c3d train pass f32', round(d['c3d_mfma']['train_pass']['ms'],3), 'bf16x3', round(d['c3d_mfma']['bf16x3']['train_pass_ms'],3))"
echo ALLDONE
