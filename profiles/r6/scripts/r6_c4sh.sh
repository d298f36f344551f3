set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6/c4sh; mkdir -p $O
A="--steps 5 --warmup 1 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline --two-ply-batches 3"
for i in 1 2; do
  for sh in 4 8 2 4 6; do
    timeout -k 10 300 python3 bench.py $A --c4-shards $sh > $O/s${sh}_$i.log 2>&1; python3 -c "
import json; d=[l for l in open('$O/s${sh}_$i.log') if l.startswith('{\"metric')][-1]; d=json.loads(d); print('c4 shards $sh', round(d['two_ply']['root_decisions_per_s']/1e6,3), 'h128', round(d['two_ply_h128']['root_decisions_per_s']/1e6,3))"
  done
done
