#!/bin/bash
# C3 shard count / graph length with linear (one-stream) env steps, 20 and 1,000 steps.
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
B="--warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); print('$1', round(d['value']/1e6,1))"; }
run() {
  local n=$1; shift
  timeout -k 10 200 env "$@" python bench.py $B $EXTRA > $O/$n.log 2>&1 && v $O/$n.log
}
for S in 4 8; do for G in 2 4; do
  EXTRA="--steps 20 --shards $S --graph-steps $G" run l${S}g${G}_20a BGX_STEP_LINEAR=1 || exit 1
  EXTRA="--steps 20 --shards $S --graph-steps $G" run l${S}g${G}_20b BGX_STEP_LINEAR=1 || exit 1
  EXTRA="--steps 1000 --shards $S --graph-steps $G" run l${S}g${G}_1000 BGX_STEP_LINEAR=1 || exit 1
done; done
EXTRA="--steps 20 --shards 4" run f4_20 BGX_X=1 || exit 1
EXTRA="--steps 1000 --shards 4" run f4_1000 BGX_X=1 || exit 1
EXTRA="--steps 20 --shards 2" run l2_20 BGX_STEP_LINEAR=1 || exit 1
