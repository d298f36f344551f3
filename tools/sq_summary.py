"""Per-kernel SQ counter summary (per wave) from rocprofv3 --pmc CSVs.
Usage: python tools/sq_summary.py DIR [DIR...]   (each DIR holds run_counter_collection.csv)"""
import csv, collections, sys, glob, os

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-60:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[k]["#" + r["Counter_Name"]] += 1
for k, c in agg.items():
    w = c.get("SQ_WAVES", 0)
    if not w or w < float(os.environ.get("SQ_MIN_WAVES", "1000")):
        continue
    print(k)
    for n in sorted(x for x in c if not x.startswith("#")):
        print("   %-24s total %.4g  per wave %.1f" % (n, c[n], c[n] / w * (c["#SQ_WAVES"] / c["#" + n])))
