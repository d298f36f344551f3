set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/c3ab; mkdir -p $O
A="--steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0"
for i in 1 2; do
  for v in head not2 noboth; do
    if [ $v = head ]; then L=mlp-ppo-2ply-p3_amd/bgx/libbgx.so; else L=scratch/lib_$v.so; fi
    BGX_LIB=$L timeout -k 10 200 python3 bench.py $A > $O/${v}_$i.log 2>&1; echo "$v $(grep -o '"value": [0-9.]*' $O/${v}_$i.log | head -1)"
  done
done
