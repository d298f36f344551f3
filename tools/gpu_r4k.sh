#!/bin/bash
# A/B: the env step's light launch forked onto the engine's side stream (default) vs
# one stream (BGX_STEP_LINEAR=1: linear HIP graphs), C3 at 20 and 1,000 steps.
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
B="--warmup 5 --two-ply-batches 0 --horizon 0 --c2-steps 0 --mirror-steps 0 --no-cpu-baseline"
v() { python -c "import json; l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); print('$1', round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],4))"; }
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 $B > $O/fork20.$r.log 2>&1 && v $O/fork20.$r.log || exit 1
  BGX_STEP_LINEAR=1 timeout -k 10 120 python bench.py --steps 20 $B > $O/lin20.$r.log 2>&1 && v $O/lin20.$r.log || exit 1
done
timeout -k 10 200 python bench.py --steps 1000 $B > $O/fork1000.log 2>&1 && v $O/fork1000.log || exit 1
BGX_STEP_LINEAR=1 timeout -k 10 200 python bench.py --steps 1000 $B > $O/lin1000.log 2>&1 && v $O/lin1000.log || exit 1
BGX_STEP_LINEAR=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/th -o run -- python bench.py --steps 20 $B > $O/bh.log 2>&1 || exit 1
python tools/c3_window.py $O/th/run_kernel_trace.csv $O/bh.log 20
