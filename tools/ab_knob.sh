#!/bin/bash
# A/B of one env knob on C3 (rollout env steps/s): tools/ab_knob.sh VAR "v1 v2 .." [reps]
# after the GPU test files named in $AB_TESTS (if any)
set -e
mkdir -p gpurun_out
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $AB_TESTS > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for i in $(seq ${3:-2}); do
for v in $2; do
vv=$v; [ "$v" = default ] && vv=""
env $1=$vv timeout -k 10 200 python bench.py --steps 400 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > gpurun_out/abk_${v//\//_}.log 2>&1
python -c "import json;l=json.loads([x for x in open('gpurun_out/abk_${v//\//_}.log').read().splitlines() if x.startswith('{')][-1]);print('$1=$v',round(l['value']/1e6,1))"
done; done
