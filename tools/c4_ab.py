"""Print the C4 (2-ply) figures of bench.py JSON lines side by side: python tools/c4_ab.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f).read().splitlines() if x.startswith("{")]
    if not lines:
        print(f, "no bench line")
        continue
    d = json.loads(lines[-1])
    out = []
    for k in ("two_ply", "two_ply_h128"):
        if k in d:
            t = d[k]
            out.append(f"{k}: {t['root_decisions_per_s'] / 1e6:.3f}M roots/s enum {t['enumeration_ms_per_batch']:.2f} "
                       f"eval {t['evaluation_ms_per_batch']:.2f} ms frac {t['roofline']['frac']:.3f}")
    print(f, " | ".join(out))
