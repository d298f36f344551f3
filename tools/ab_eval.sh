#!/bin/bash
# A/B of libbgx.so variants on C4 (2-ply at H = 40 and H = 128): one short bench per
# variant.  Usage: tools/ab_eval.sh NAME...   (build/libbgx_NAME.so, "default" = in-tree)
for n in "$@"; do
  if [ "$n" = default ]; then L=""; else L=build/libbgx_$n.so; fi
  BGX_LIB=$L timeout -k 10 300 python bench.py --steps 20 --horizon 0 --c2-steps 0 --no-cpu-baseline --mirror-steps 0 \
    > gpurun_out/abe_$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
l = json.loads([x for x in open(f"gpurun_out/abe_{n}.log").read().splitlines() if x.startswith("{")][-1])
print(n, "C3", round(l["value"] / 1e6, 1), *[(k, round(l[k]["root_decisions_per_s"]), round(l[k]["evaluation_ms_per_batch"], 2),
      round(l[k]["enumeration_ms_per_batch"], 2), round(l[k]["roofline"]["frac"], 3)) for k in ("two_ply", "two_ply_h128")])
PY
done
