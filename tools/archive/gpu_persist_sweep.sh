# persistent k_dense (RT_DENSE_PERSIST blocks per CU) under the two-group pipeline:
# blocks per CU x policy block waves (RT_PIPE_WPB) x k_dense turns (RT_PIPE_SERIAL), repeated
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/psweep4
i=0
for cfg in "6 2 8 1" "5 2 8 1" "7 2 8 1" "6 2 16 1" "5 2 16 1" "6 2 8 1" "5 2 8 1" "7 2 8 1" "6 2 16 1" "5 2 16 1"; do
  set -- $cfg
  i=$((i + 1))
  RT_DENSE_PERSIST=$1 RT_PIPE_WPB=$3 RT_PIPE_SERIAL=$4 timeout -k 10 120 python -u bench.py --no-cpu --no-update --rollout-groups $2 > gpurun_out/psweep4/b_$1_$2_$3_$4_r$i.log 2>&1 || exit 1
done
echo EXIT $?
