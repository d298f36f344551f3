#!/bin/bash
# A/B of library builds on one GPU box: for each LIB (path, or "default"), a C3-only
# bench line and the 2-ply experiment (defaults).  Usage: tools/ab_c3c4.sh LIB...
set -e
for L in "$@"; do
  if [ "$L" = default ]; then unset BGX_LIB; else export BGX_LIB=$L; fi
  T=$(basename $L .so)
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --two-ply-batches 0 --horizon 0 --no-cpu-baseline \
     --c2-steps 0 > gpurun_out/ab_$T.log 2>&1
  python -c "import json,sys; j=json.loads([l for l in open('gpurun_out/ab_$T.log') if l.startswith('{')][-1]); print('$T C3', round(j['value']/1e6,2), 'M/s', round(j['roofline']['kernel_ms'],4), 'ms env step')"
  timeout -k 10 200 python tools/exp_2ply.py "" 2>&1 | grep -v amdgpu.ids | sed "s/^/$T C4 /"
done
