# kernel trace of the vision bench (configs[3], 512 envs at 64^3): where the update time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-visprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/visprof -o run -- python3 bench.py --vision --no-cpu --steps 16 --warmup 4 ${EXTRA} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
python tools/rocpd_stats.py /tmp/visprof/run_results.db $OUT/kernel_stats.csv
tail -c 400 $OUT/bench.json
exit $rc
