#!/bin/bash
# C2 as 1 / 2 / 4 linear shards, each replayed as its own HIP graph, after a C3 leg.
O=gpurun_out/r4r
mkdir -p $O
export TMPDIR=/tmp
B="--steps 20 --warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 200 --mirror-steps 0 --no-cpu-baseline"
for S in 1 2 4 1 2 4; do
timeout -k 10 200 python bench.py $B --c2-shards $S > $O/s$S.log 2>&1 || { tail -5 $O/s$S.log; exit 1; }
python -c "import json; l=[x for x in open('$O/s$S.log') if x.startswith('{')][-1]; d=json.loads(l)['one_ply_selfplay']; print('C2 shards $S', round(d['env_steps_per_s']/1e6,2), d['hip_graph'])"
done
