#!/bin/bash
# A/B of 2-ply enumerator configs on one GPU box: for each BGX_2PLY_HEAVY value,
# one short bench (C3 5 steps + C4 2 batches).  Usage: tools/ab_2ply.sh CFG...
set -e
for c in "$@"; do
  BGX_2PLY_HEAVY=$c BGX_2PLY_DEBUG=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --horizon 0 \
    --no-cpu-baseline --two-ply-batches 2 > gpurun_out/ab2_$c.log 2>&1
  python - "$c" <<'PY'
import json, sys
c = sys.argv[1]
lines = open(f"gpurun_out/ab2_{c}.log").read().splitlines()
j = json.loads([l for l in lines if l.startswith("{")][-1])
dbg = [l for l in lines if l.startswith("[bgx 2-ply]")][-1]
print(c, round(j["two_ply"]["root_decisions_per_s"]), dbg)
PY
done
