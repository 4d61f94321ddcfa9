# round-2: reproduce the reference's learning curve (configs/default.yaml to 2.5e7 env steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02l
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/repro_learning.py --out gpurun_out/r02l/seed1 --total 25000000 > gpurun_out/r02l/seed1.log 2>&1
rc=$?
echo EXIT $rc
tail -3 gpurun_out/r02l/seed1.log
exit $rc
