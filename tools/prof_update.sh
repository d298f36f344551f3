#!/bin/bash
# Kernel trace of PPO updates at the production batch (tools/ppo_time.py: one rollout of
# B = 65,536 x T = 32, then N updates): per-kernel stats + busy/idle of the last update.
# Usage: tools/prof_update.sh TAG   -> gpurun_out/TAG/...
set -e
TAG=$1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
N=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python tools/ppo_time.py > $OUT/run.log 2>&1
python - "$OUT" <<'PY'
import csv, sys, collections
out = sys.argv[1]
rows = list(csv.DictReader(open(out + "/trace/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# updates are separated by >= 50 ms idle gaps (tools/ppo_time.py): the last segment
cut = [i for i in range(1, len(rows)) if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 20_000_000]
last = rows[cut[-1]:] if cut else rows
busy, end = 0, int(last[0]["Start_Timestamp"])
for r in last:
    s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += max(0, e0 - max(s0, end))
    end = max(end, e0)
agg = collections.defaultdict(lambda: [0, 0])
for r in last:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-70:]
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
span = int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])
print(f"last update: span {span/1e6:.3f} ms, GPU busy {busy/1e6:.3f} ms, kernels {len(last)}")
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{t/1e3:10.1f} us  x{c:3d}  {t/c/1e3:8.1f} us/call  {n}")
# the largest idle gaps of the last update, with the kernels either side
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-60:]
gaps, end, prev = [], int(last[0]["End_Timestamp"]), last[0]
for r in last[1:]:
    s0 = int(r["Start_Timestamp"])
    if s0 > end:
        gaps.append((s0 - end, nm(prev), nm(r)))
    if int(r["End_Timestamp"]) > end:
        end, prev = int(r["End_Timestamp"]), r
gaps.sort(reverse=True)
print(f"idle gaps: {len(gaps)}, total {sum(g[0] for g in gaps)/1e6:.3f} ms; largest:")
for g, a, b in gaps[:20]:
    print(f"{g/1e3:9.1f} us  after {a}  before {b}")
PY
