set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/rowsab; mkdir -p $O
for i in 1 2; do
  N=6 ROUNDS=1 timeout -k 10 240 python3 tools/ppo_ab.py "" > $O/base_$i.log 2>&1; echo "base $(tail -1 $O/base_$i.log)"
  BGX_LIB=scratch/lib_rows3.so N=6 ROUNDS=1 timeout -k 10 240 python3 tools/ppo_ab.py "" > $O/rows3_$i.log 2>&1; echo "rows3 $(tail -1 $O/rows3_$i.log)"
done
