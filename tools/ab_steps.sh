#!/bin/bash
# A/B an env knob on the C3 bench (steps/s, ms/step, env-step ms): tools/ab_steps.sh VAR VAL1 VAL2 ...
V=$1; shift
for r in 1 2; do for c in "$@"; do
  env $V=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --horizon 0 --two-ply-batches 0 --c2-steps 0 \
    --no-cpu-baseline 2>&1 | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V=$c', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))" || exit 1
done; done
