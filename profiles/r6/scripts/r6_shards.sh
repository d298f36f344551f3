set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/shards; mkdir -p $O
A="--steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0"
for i in 1 2; do
  for sh in 4 2 8 4; do
    timeout -k 10 200 python3 bench.py $A --shards $sh > $O/s${sh}_$i.log 2>&1; echo "shards $sh: $(grep -o '"value": [0-9.]*' $O/s${sh}_$i.log | head -1)"
  done
  timeout -k 10 200 python3 bench.py $A --fork-steps > $O/fork_$i.log 2>&1; echo "fork: $(grep -o '"value": [0-9.]*' $O/fork_$i.log | head -1)"
done
