#!/bin/bash
# Kernel-time stats of the C3 rollout step alone: tools/prof_c3.sh TAG [VAR=VALUE ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
mkdir -p gpurun_out/c3_$tag
env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3_$tag -o c3 -- python3 bench.py --steps 200 --two-ply-batches 0 --c2-steps 0 --horizon 0 --no-cpu-baseline --mirror-steps 0 > gpurun_out/c3_$tag/bench.log 2>&1
f=$(find gpurun_out/c3_$tag -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.1f} us {float(r["Percentage"]):6.2f}%')
PY
