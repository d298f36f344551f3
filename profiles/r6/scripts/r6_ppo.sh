set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/ppo6; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo_fused.py tests/test_gpu_train.py > $O/tests.log 2>&1
tail -3 $O/tests.log
for i in 1 2; do
  BGX_LIB=scratch/lib_prev.so N=6 ROUNDS=1 timeout -k 10 240 python3 tools/ppo_ab.py "" > $O/prev_$i.log 2>&1; echo "prev $(tail -1 $O/prev_$i.log)"
  N=6 ROUNDS=1 timeout -k 10 240 python3 tools/ppo_ab.py "" > $O/new_$i.log 2>&1; echo "new  $(tail -1 $O/new_$i.log)"
done
