#!/bin/bash
# C2: forked vs linear env steps (one shard, HIP graph), after a C3 leg as in the default bench.
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
B="--steps 20 --warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 200 --mirror-steps 0 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); print('$1', round(d['one_ply_selfplay']['env_steps_per_s']/1e6,2))"; }
for r in 1 2; do
timeout -k 10 200 python bench.py $B > $O/fork$r.log 2>&1 && v $O/fork$r.log || exit 1
BGX_C2_LINEAR=1 timeout -k 10 200 python bench.py $B > $O/lin$r.log 2>&1 && v $O/lin$r.log || exit 1
done
