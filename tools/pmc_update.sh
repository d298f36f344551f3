#!/bin/bash
# PMC passes over the PPO update kernels (tools/ppo_time.py, one rollout + N updates at
# B = 65,536 x T = 32): instruction mix and wave-time split per kernel.
# Usage: tools/pmc_update.sh TAG  -> gpurun_out/TAG/{u1,u2}
set -e
TAG=$1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
RE='k_ppo_gw1|k_ppo_gw2|k_ppo_rows|k_fc1_rec'
N=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "$RE" --output-format csv -d $OUT/u1 -o run -- python tools/ppo_time.py > $OUT/u1.log 2>&1
N=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$RE" --output-format csv -d $OUT/u2 -o run -- python tools/ppo_time.py > $OUT/u2.log 2>&1
python - "$OUT" <<'PY'
import csv, sys, collections, glob
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for p in ("u1", "u2"):
    f = glob.glob(f"{out}/{p}/*counter_collection.csv")[0]
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES": cnt[(p, n)] += 1
for n, c in agg.items():
    wc = c["SQ_WAVE_CYCLES"] / 2 or 1
    print(n, {k: round(v / 1e6, 2) for k, v in c.items() if k not in ("SQ_WAVE_CYCLES",)})
    print("   split: active %.2f wait_any %.2f wait_inst %.2f (lds %.2f) valu %.2f" % tuple(c[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU")))
PY
