#!/bin/bash
# C3 graph length 2 vs 4 at 4 linear shards, alternating runs, 20 and 1,000 steps.
O=gpurun_out/r4t
mkdir -p $O
export TMPDIR=/tmp
B="--warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); print('$1', round(d['value']/1e6,1))"; }
for r in 1 2 3; do for G in 2 4; do
  timeout -k 10 120 python bench.py --steps 20 --graph-steps $G $B > $O/g${G}_20.$r.log 2>&1 && v $O/g${G}_20.$r.log || exit 1
done; done
for r in 1 2; do for G in 2 4; do
  timeout -k 10 200 python bench.py --steps 1000 --graph-steps $G $B > $O/g${G}_1000.$r.log 2>&1 && v $O/g${G}_1000.$r.log || exit 1
done; done
