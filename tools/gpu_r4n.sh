#!/bin/bash
# host_mirror with 4 linear C3 shards: copies on per-shard copy streams vs on the shard's own stream.
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp
B="--steps 20 --warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 64 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); print('$1', round(d['value']/1e6,1), 'mirror', round(d['host_mirror']['env_steps_per_s']/1e6,1))"; }
for r in 1 2; do
timeout -k 10 200 python bench.py $B > $O/side$r.log 2>&1 && v $O/side$r.log || exit 1
BGX_MIRROR_OWN=1 timeout -k 10 200 python bench.py $B > $O/own$r.log 2>&1 && v $O/own$r.log || exit 1
BGX_MIRROR_OWN=1 timeout -k 10 200 python bench.py $B --shards 2 > $O/own2s$r.log 2>&1 && v $O/own2s$r.log || exit 1
timeout -k 10 200 python bench.py $B --shards 2 > $O/side2s$r.log 2>&1 && v $O/side2s$r.log || exit 1
done
