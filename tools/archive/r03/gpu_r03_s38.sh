#!/bin/bash
# r03 session 38: PMC of the C3D stage kernels with bf16x3 products (RT_CONV_PREC) (separate --pmc passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp C3D_PMC_B=256 PYTHONUNBUFFERED=1 RT_CONV_PREC=bf16x3
O=gpurun_out/r03_s38
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1
rc=$?
tail -2 $O/a.log $O/b.log $O/c.log
python3 tools/c3d_pmc_summary.py $O $O/summary.json > /dev/null; find $O -name "*.db" -delete
echo EXIT $rc
python3 -c "
import json; d=json.load(open(\"gpurun_out/r03_s38/summary.json\"))
for k,v in d.items():
    if isinstance(v, dict): print(k[:70], {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in list(v.items())[:12]})
"
