# kernel trace of the vision bench (configs[3], 512 envs at 64^3): where the update time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-visprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --vision --no-cpu --steps 16 --warmup 4 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -c 400 $OUT/bench.json
exit $rc
