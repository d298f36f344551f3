#!/bin/bash
# A/B whole env settings on the 2-ply bench: tools/ab_envs.sh "A=1 B=2" "A=3" ...
set -e
i=0
for c in "$@"; do
  i=$((i+1))
  env $c BGX_2PLY_DEBUG=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --horizon 0 \
    --no-cpu-baseline --two-ply-batches 2 --c2-steps 0 > gpurun_out/abs_$i.log 2>&1
  python - "$i" "$c" <<'PY'
import json, sys
i, c = sys.argv[1], sys.argv[2]
lines = open(f"gpurun_out/abs_{i}.log").read().splitlines()
j = json.loads([l for l in lines if l.startswith("{")][-1])["two_ply"]
print(c, "C4", round(j["root_decisions_per_s"]), round(j["enumeration_ms_per_batch"], 2), round(j["evaluation_ms_per_batch"], 2), "C3", round(json.loads([l for l in lines if l.startswith("{")][-1])["value"] / 1e6, 2))
PY
done
