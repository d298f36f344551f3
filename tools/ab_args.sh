#!/bin/bash
# C3-only bench per argument set ("--a x --b y"; "" = defaults).  Usage: tools/ab_args.sh ARGS...
for c in "$@"; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --two-ply-batches 0 --horizon 0 --no-cpu-baseline \
    --c2-steps 0 $c > gpurun_out/aba.log 2>&1 || exit 1
  python -c "import json; j=json.loads([l for l in open('gpurun_out/aba.log') if l.startswith('{')][-1]); print('${c:-default}', round(j['value']/1e6,2), 'M/s', round(j['ms_per_step'],4), 'ms/step', round(j['roofline']['kernel_ms'],4), 'ms env')" || exit 1
done
