"""Summarize a tools/profile.sh run: per-kernel stats + HBM traffic per launch of
the dominant kernels.

FETCH_SIZE calibration (MI355X_MICROARCH.md §HBM: the guide's x2 correction is
for 16-B-per-lane streaming reads; "other access widths are uncalibrated:
calibrate on a known byte count in your own access pattern"):
tools/calib/fetch_calib.hip -> profiles/r2_fetch_calibration.json.  The env
step's access shapes -- a 64-B lane record read 1 B per lane, 4-/8-B scalar
reads, 4-/8-B and 64-B stores -- are each ONE 64-B EA request that FETCH_SIZE
tallies at 64 B, so the env-step kernels' bytes are (FETCH_SIZE + WRITE_SIZE)
x 1024, not doubled; the 2-ply evaluator's 16-B-per-lane pool stream keeps the
guide's doubling."""
import csv
import json
import os
import statistics
import sys

out, cmd = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
pmc_cmd = sys.argv[3] if len(sys.argv) > 3 else cmd
stats = list(csv.DictReader(open(os.path.join(out, "trace", "run_kernel_stats.csv"))))


def pmc(kind, counter):
    res = {}
    p = os.path.join(out, kind, "run_counter_collection.csv")
    if not os.path.exists(p):
        return res
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == counter:
            res.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return res


fetch, write = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
kernels = []
for s in stats:
    name = s["Name"]
    k = {"name": name, "calls": int(s["Calls"]), "avg_ns": float(s["AverageNs"]), "pct": float(s["Percentage"])}
    f = next((v for n, v in fetch.items() if n == name), None)
    w = next((v for n, v in write.items() if n == name), None)
    if f and w:
        k["FETCH_SIZE_KiB"] = statistics.mean(f)
        k["WRITE_SIZE_KiB"] = statistics.mean(w)
        k["hbm_bytes_per_launch"] = (k["FETCH_SIZE_KiB"] + k["WRITE_SIZE_KiB"]) * 1024   # calibrated, see top
    kernels.append(k)
# per-dispatch durations of the dominant kernels over the timed tail (last --steps launches)
tail = None
for tok in cmd.split():
    pass
args = cmd.split()
if "--steps" in args:
    tail = int(args[args.index("--steps") + 1])
trace = list(csv.DictReader(open(os.path.join(out, "trace", "run_kernel_trace.csv"))))
for k in kernels[:4]:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in trace if r["Kernel_Name"] == k["name"]]
    if tail and len(d) >= tail:
        k["avg_ns_timed_tail"] = statistics.mean(d[-tail:])
# the env step = every kernel bgx_step launches once per step (Philox split dispatch):
# both k_step launches, the dispatch-order sort, and the overflow tiers.  Their
# durations are averaged over the C3 (B = 65,536) dispatches only: the default bench
# also runs C2 at B = 4,096 with the same kernels, told apart by grid size.
STEP_KERNELS = ("k_step<0", "k_order_count", "k_order_scatter", "k_movegen_over<0")
env = {"kernels": [], "hbm_bytes_per_step": 0.0, "busy_ns_per_step": 0.0}
for k in kernels:
    short = k["name"].replace("(anonymous namespace)::", "").replace("void ", "")
    if any(short.startswith(p) for p in STEP_KERNELS):
        rows = [r for r in trace if r["Kernel_Name"] == k["name"]]
        gmax = max(int(r["Grid_Size_X"]) for r in rows)
        big = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if int(r["Grid_Size_X"]) * 4 >= gmax]
        if short.startswith("k_step<0"):
            k["avg_ns_c3"] = statistics.mean(big)
        env["kernels"].append({"name": short.split("(")[0], "avg_ns": k.get("avg_ns_c3", k["avg_ns"]),
                               "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch")})
        env["busy_ns_per_step"] += k.get("avg_ns_c3", k["avg_ns"])
        env["hbm_bytes_per_step"] += k.get("hbm_bytes_per_launch") or 0.0
# 2-ply evaluator (k_eval): MFMA busy cycles (SQ_VALU_MFMA_BUSY_CYCLES counts cycles,
# 32 per v_mfma_f32_32x32x16; MI355X_MICROARCH.md constants table) over 1024 SIMDs x
# the kernel's duration at 2.4 GHz, and its HBM read bytes (2 x FETCH_SIZE KiB)
ev = {}
mf = pmc("mfma", "SQ_VALU_MFMA_BUSY_CYCLES")
ef = pmc("efetch", "FETCH_SIZE")
ek = next((k for k in kernels if "k_eval" in k["name"]), None)
if ek and mf:
    busy = statistics.mean(next(iter(mf.values())))
    ev = {"kernel": ek["name"], "avg_ns": ek["avg_ns"], "mfma_busy_cycles": busy,
          "mfma_busy_frac_at_2p4GHz": busy / (1024 * ek["avg_ns"] * 2.4)}
    if ef:
        ev["hbm_read_bytes"] = 2 * statistics.mean(next(iter(ef.values()))) * 1024
summary = {"command": "python bench.py " + cmd, "pmc_command": "python bench.py " + pmc_cmd,
           "kernels": kernels[:20], "env_step": env, "two_ply_eval": ev}
json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k in kernels[:20]:
    print(f"{k['pct']:6.2f}% {k['avg_ns']/1e3:10.1f} us (tail {k.get('avg_ns_timed_tail', 0)/1e3:.1f}) "
          f"x{k['calls']:4d}  {k['name'][:70]}  {k.get('hbm_bytes_per_launch', 0)/1e6:.1f} MB")
