import glob, json, re
for tag in ("new", "old"):
    vals = []
    for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.log")):
        for line in open(f):
            if line.startswith("{"):
                d = json.loads(line)
                vals.append((d["value"] / 1e6, d["ms_per_step"], d["roofline"]["kernel_ms"]))
    print(tag, " ".join("%.2fM/%.3fms/%.3fms" % v for v in vals))
