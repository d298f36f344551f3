#!/bin/bash
# C3-only bench per env-var config ("K=V,K=V"; "" = defaults).  Usage: tools/ab_env_vars.sh CFG...
for c in "$@"; do
  ( for kv in ${c//,/ }; do export "$kv"; done
    timeout -k 10 200 python bench.py --steps 300 --warmup 5 --two-ply-batches 0 --horizon 0 --no-cpu-baseline \
      --c2-steps 0 > gpurun_out/abv.log 2>&1 || exit 1
    python -c "import json; j=json.loads([l for l in open('gpurun_out/abv.log') if l.startswith('{')][-1]); print('${c:-default}', round(j['value']/1e6,2), 'M/s', round(j['ms_per_step'],4), 'ms/step', round(j['roofline']['kernel_ms'],4), 'ms env')" ) || exit 1
done
