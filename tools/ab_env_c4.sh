#!/bin/bash
# C4 A/B over env settings (2-ply at H = 40 and H = 128): tools/ab_env_c4.sh "" "BGX_2PLY_HGRID=1024 BGX_2PLY_LGRID=4096" ...
# ("" = defaults; each set run twice, interleaved)
mkdir -p gpurun_out
for rep in 1 2; do
  n=0
  for set in "$@"; do
    n=$((n + 1))
    env $set timeout -k 10 300 python bench.py --steps 20 --horizon 0 --c2-steps 0 --no-cpu-baseline --mirror-steps 0 \
      > gpurun_out/abc4_$n.log 2>&1 || { echo "[$set] failed"; tail -5 gpurun_out/abc4_$n.log; exit 1; }
    python - "$set" gpurun_out/abc4_$n.log <<'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[2]).read().splitlines() if x.startswith("{")][-1])
print(f"[{sys.argv[1]}]", *[(k, round(l[k]["root_decisions_per_s"] / 1e6, 3), round(l[k]["enumeration_ms_per_batch"], 2),
      round(l[k]["evaluation_ms_per_batch"], 2)) for k in ("two_ply", "two_ply_h128")])
PY
  done
done
