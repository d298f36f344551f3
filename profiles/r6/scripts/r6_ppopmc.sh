set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6/ppopmc; mkdir -p $OUT
R='k_fc1_rec|k_ppo_rows|k_ppo_gw1$|k_ppo_gw2$|k_ppo_gw1\(|k_ppo_gw2\('
export N=1 ROUNDS=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$R" --output-format csv -d $OUT/p2 -o run -- python3 tools/ppo_ab.py "" > $OUT/p2.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$R" --output-format csv -d $OUT/p1 -o run -- python3 tools/ppo_ab.py "" > $OUT/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" --output-format csv -d $OUT/p3 -o run -- python3 tools/ppo_ab.py "" > $OUT/p3.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" --output-format csv -d $OUT/p4 -o run -- python3 tools/ppo_ab.py "" > $OUT/p4.log 2>&1
SQ_MIN_WAVES=100 python3 tools/sq_summary.py $OUT/p1 $OUT/p2 > $OUT/summary.txt
python3 - $OUT > $OUT/bytes.txt <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p3", "p4"):
    for f in glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-40:]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    print(k, {n: (len(v), round(sum(v) / len(v) / 1e6, 1)) for n, v in c.items()}, "(dispatches, mean KB... see unit note)")
PY
cat $OUT/summary.txt | head -80; cat $OUT/bytes.txt
