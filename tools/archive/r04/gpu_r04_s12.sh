#!/bin/bash
# r04 session 12: PMC of the C3D stage kernels at batch 512 (Winograd forward
# and data gradient, sparse weight gradient): instruction mix, LDS bank
# conflicts, MFMA busy (separate --pmc passes, then a kernel-trace pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp C3D_PMC_B=512
O=gpurun_out/r04_s12
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $O/a -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/b -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 -d $O/c -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/c.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 tools/c3d_pmc_driver.py > $O/t.log 2>&1 || { tail -5 $O/*.log; exit 1; }
python3 tools/c3d_pmc_summary.py $O $O/c3d_pmc_b512.json
rm -rf $O/a $O/b $O/c $O/t
echo ALLDONE
