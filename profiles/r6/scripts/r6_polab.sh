set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/polab; mkdir -p $O
A="--steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0"
for i in 1 2 3; do
  BGX_LIB=scratch/lib_head.so timeout -k 10 200 python3 bench.py $A > $O/head_$i.log 2>&1; echo "head $(grep -o '"value": [0-9.]*' $O/head_$i.log | head -1)"
  timeout -k 10 200 python3 bench.py $A > $O/new_$i.log 2>&1; echo "new  $(grep -o '"value": [0-9.]*' $O/new_$i.log | head -1)"
done
