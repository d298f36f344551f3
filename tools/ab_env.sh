#!/bin/bash
# A/B an env knob on the 2-ply bench: tools/ab_env.sh VAR VAL1 VAL2 ...
set -e
V=$1; shift
for c in "$@"; do
  env $V=$c BGX_2PLY_DEBUG=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --horizon 0 \
    --no-cpu-baseline --two-ply-batches 2 > gpurun_out/abe_$c.log 2>&1
  python - "$c" <<'PY'
import json, sys
c = sys.argv[1]
lines = open(f"gpurun_out/abe_{c}.log").read().splitlines()
j = json.loads([l for l in lines if l.startswith("{")][-1])["two_ply"]
print(c, round(j["root_decisions_per_s"]), round(j["enumeration_ms_per_batch"], 2), round(j["evaluation_ms_per_batch"], 2),
      j["roofline"]["achieved"])
PY
done
