"""Summarize a tools/profile.sh run: per-kernel stats, HBM traffic per launch of
the env-step kernels, the env step's SQ instruction mix and wave-cycle split
(the issue-rate roofline), and every 2-ply evaluator k_eval<*> with its OWN
counter rows (MFMA busy, VALU, HBM read).

FETCH_SIZE calibration (MI355X_MICROARCH.md §HBM: the guide's x2 correction is
for 16-B-per-lane streaming reads; "other access widths are uncalibrated:
calibrate on a known byte count in your own access pattern"):
tools/calib/fetch_calib.hip -> profiles/r2_fetch_calibration.json.  The env
step's access shapes -- a 64-B lane record read 1 B per lane, 4-/8-B scalar
reads, 4-/8-B and 64-B stores -- are each ONE 64-B EA request that FETCH_SIZE
tallies at 64 B, so the env-step kernels' bytes are (FETCH_SIZE + WRITE_SIZE)
x 1024, not doubled; the 2-ply evaluator's 16-B-per-lane pool stream keeps the
guide's doubling.

Usage: python tools/summarize_profile.py OUT "bench args" "pmc bench args"
"""
import csv
import json
import os
import statistics
import sys

CLOCK_GHZ = 2.4          # MI355X peak engine clock (MI355X_MICROARCH.md chip table)
CUS, SIMDS = 256, 1024

out, cmd = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
pmc_cmd = sys.argv[3] if len(sys.argv) > 3 else cmd
stats = list(csv.DictReader(open(os.path.join(out, "trace", "run_kernel_stats.csv"))))


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def pmc_rows(kind):
    """{kernel name: {counter: [value per dispatch]}} of one --pmc pass."""
    res = {}
    p = os.path.join(out, kind, "run_counter_collection.csv")
    if not os.path.exists(p):
        return res
    for r in csv.DictReader(open(p)):
        d = res.setdefault(r["Kernel_Name"], {})
        d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return res


def pmc(kind, counter):
    return {n: v[counter] for n, v in pmc_rows(kind).items() if counter in v}


fetch, write = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
kernels = []
for s in stats:
    name = s["Name"]
    k = {"name": name, "calls": int(s["Calls"]), "avg_ns": float(s["AverageNs"]), "pct": float(s["Percentage"])}
    f, w = fetch.get(name), write.get(name)
    if f and w:
        k["FETCH_SIZE_KiB"] = statistics.mean(f)
        k["WRITE_SIZE_KiB"] = statistics.mean(w)
        k["hbm_bytes_per_launch"] = (k["FETCH_SIZE_KiB"] + k["WRITE_SIZE_KiB"]) * 1024   # calibrated, see top
    kernels.append(k)
args = cmd.split()
tail = int(args[args.index("--steps") + 1]) if "--steps" in args else None
trace = list(csv.DictReader(open(os.path.join(out, "trace", "run_kernel_trace.csv"))))
for k in kernels[:4]:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in trace if r["Kernel_Name"] == k["name"]]
    if tail and len(d) >= tail:
        k["avg_ns_timed_tail"] = statistics.mean(d[-tail:])

# ---------------------------------------------------------------- env step --
# the env step = every kernel bgx_step launches once per step (Philox split dispatch):
# both k_step launches, the dispatch-order sort, and the overflow tiers.  Durations are
# averaged over the C3 (B = 65,536) dispatches only: the default bench also runs C2 at
# B = 4,096 with the same kernels, told apart by grid size.
STEP_KERNELS = ("k_step<0", "k_order_count", "k_order_scatter", "k_movegen_over<0")
env = {"kernels": [], "hbm_bytes_per_step": 0.0, "busy_ns_per_step": 0.0}
for k in kernels:
    sh = short(k["name"])
    if any(sh.startswith(p) for p in STEP_KERNELS):
        rows = [r for r in trace if r["Kernel_Name"] == k["name"]]
        gmax = max(int(r["Grid_Size_X"]) for r in rows)
        big = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if int(r["Grid_Size_X"]) * 4 >= gmax]
        if sh.startswith("k_step<0"):
            k["avg_ns_c3"] = statistics.mean(big)
        env["kernels"].append({"name": sh, "avg_ns": k.get("avg_ns_c3", k["avg_ns"]),
                               "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch")})
        env["busy_ns_per_step"] += k.get("avg_ns_c3", k["avg_ns"])
        env["hbm_bytes_per_step"] += k.get("hbm_bytes_per_launch") or 0.0

# The C3 step's kernels over the timed window of a C3-only kernel trace (the "c3trace"
# pass: bench.py --steps K, C3 only): the timed replays are the K x shards policy
# dispatches before the 16 x shards eager steps that follow the timed region; each
# kernel's average launch duration over that window (the roofline's rocprof figure).
c3t = os.path.join(out, "c3trace", "run_kernel_trace.csv")
if os.path.exists(c3t):
    rows = sorted(csv.DictReader(open(c3t)), key=lambda r: int(r["Start_Timestamp"]))
    a3 = os.environ.get("C3TRACE_ARGS", "--steps 200").split()
    K3 = int(a3[a3.index("--steps") + 1])
    S3 = int(a3[a3.index("--shards") + 1]) if "--shards" in a3 else 4
    pol = [i for i, r in enumerate(rows) if "k_policy_act" in r["Kernel_Name"]]
    if len(pol) >= (16 + K3) * S3:
        lo, hi = pol[-(16 + K3) * S3], pol[-16 * S3]
        win = rows[lo:hi]
        per = {}
        for r in win:
            per.setdefault(short(r["Kernel_Name"]), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        t0 = int(win[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in win)
        env["timed_window"] = {"steps": K3, "shards": S3, "span_ms_per_step": (t1 - t0) / 1e6 / K3,
                               "kernels": {n: {"launches": len(d), "avg_us": statistics.mean(d) / 1e3}
                                           for n, d in sorted(per.items(), key=lambda x: -sum(x[1]))},
                               "command": "python bench.py " + " ".join(a3)}
        for k in env["kernels"]:
            w = env["timed_window"]["kernels"].get(k["name"])
            if w:
                k["avg_ns"] = w["avg_us"] * 1e3
                k["avg_source"] = "c3trace timed window"

# SQ passes of the C3 step alone ("sqi": instruction counts, "sqc": wave-cycle split).
# Both passes run the same command, so per-pass totals over all env-step dispatches /
# the lane-steps of that run give per-lane-step figures; the lane-steps are counted as
# k_order_count dispatches (one per shard step) x lanes per shard.
lanes_per_shard = None
if "--batch" in pmc_cmd.split():
    pa = pmc_cmd.split()
    lanes_per_shard = int(pa[pa.index("--batch") + 1]) // int(pa[pa.index("--shards") + 1] if "--shards" in pa else 4)
else:                                  # bench.py's defaults: 65,536 games as 4 shards (round 4)
    pa = pmc_cmd.split()
    lanes_per_shard = 65536 // int(pa[pa.index("--shards") + 1] if "--shards" in pa else 4)
sq = {}
for kind in ("sqi", "sqc"):
    rows = pmc_rows(kind)
    if not rows:
        continue
    shard_steps = len(next((v["SQ_WAVES"] for n, v in rows.items() if "k_order_count" in n), []))
    tot = {}
    for n, v in rows.items():
        if not any(short(n).startswith(p) for p in STEP_KERNELS):
            continue
        for c, vals in v.items():
            if c.startswith("SQ_") and c != "SQ_WAVES":
                tot[c] = tot.get(c, 0.0) + sum(vals)
    if shard_steps:
        sq[kind] = {"shard_steps": shard_steps, "per_lane_step": {c: t / (shard_steps * lanes_per_shard)
                                                                   for c, t in tot.items()}}
if sq:
    ins = sq.get("sqi", {}).get("per_lane_step", {})
    cyc = sq.get("sqc", {}).get("per_lane_step", {})
    env["sq"] = {"lanes_per_shard_step": lanes_per_shard, "instructions_per_lane_step": ins,
                 "quad_cycles_per_lane_step": cyc}
    if cyc.get("SQ_WAVE_CYCLES"):
        wc = cyc["SQ_WAVE_CYCLES"]
        env["sq"]["wave_time_split"] = {
            "active_any": cyc.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "wait_any (s_waitcnt / barrier: memory + LDS latency)": cyc.get("SQ_WAIT_ANY", 0) / wc,
            "wait_inst_any (issue stall)": cyc.get("SQ_WAIT_INST_ANY", 0) / wc,
            "wait_inst_lds (LDS issue stall, part of wait_inst_any)": cyc.get("SQ_WAIT_INST_LDS", 0) / wc,
            "active_valu": cyc.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "active_lds": cyc.get("SQ_ACTIVE_INST_LDS", 0) / wc}
    # issue-pipe capacities (cycles a unit is occupied per wave-instruction / units on the chip):
    # VALU wave64 = 2 cycles on a SIMD-32 (MI355X_MICROARCH.md "Wave scheduling"), 1,024 SIMDs;
    # SALU one instruction per cycle on each CU's single scalar unit (chip table "CU"), 256;
    # LDS one instruction issued per cycle per CU (a floor: wide accesses take more), 256;
    # SMEM / VMEM / branch one per cycle per CU each.
    if ins:
        env["sq"]["pipe_model"] = {"VALU": {"counter": "SQ_INSTS_VALU", "cycles_per_inst": 2, "units": SIMDS},
                                   "SALU": {"counter": "SQ_INSTS_SALU", "cycles_per_inst": 1, "units": CUS},
                                   "LDS": {"counter": "SQ_INSTS_LDS", "cycles_per_inst": 1, "units": CUS},
                                   "SMEM": {"counter": "SQ_INSTS_SMEM", "cycles_per_inst": 1, "units": CUS},
                                   "VMEM": {"counter": "SQ_INSTS_VMEM", "cycles_per_inst": 1, "units": CUS},
                                   "BRANCH": {"counter": "SQ_INSTS_BRANCH", "cycles_per_inst": 1, "units": CUS}}
        env["sq"]["clock_ghz"] = CLOCK_GHZ
        # unit-busy ns per shard step if that pipe alone bound the step
        env["sq"]["pipe_bound_ns_per_shard_step"] = {
            p: ins.get(m["counter"], 0.0) * lanes_per_shard * m["cycles_per_inst"] / m["units"] / CLOCK_GHZ
            for p, m in env["sq"]["pipe_model"].items()}

# ------------------------------------------------------------ 2-ply k_eval --
# every evaluator instantiation separately (k_eval<3> = H 40, k_eval<8> = H 128), each
# with its own counter rows: MFMA busy cycles (SQ_VALU_MFMA_BUSY_CYCLES counts cycles,
# 32 per v_mfma_f32_32x32x16; MI355X_MICROARCH.md constants table) over 1,024 SIMDs x
# its duration at 2.4 GHz; VALU instructions / active quad-cycles; HBM read bytes
# (2 x FETCH_SIZE KiB, the guide's 16-B streaming correction)
def wave_split(m):
    wc = statistics.mean(m["SQ_WAVE_CYCLES"]) if "SQ_WAVE_CYCLES" in m else 0
    if not wc:
        return None
    f = lambda c: statistics.mean(m[c]) / wc if c in m else None
    return {"active_any": f("SQ_ACTIVE_INST_ANY"), "wait_any (s_waitcnt / barrier)": f("SQ_WAIT_ANY"),
            "wait_inst_any (issue stall)": f("SQ_WAIT_INST_ANY"), "wait_inst_lds": f("SQ_WAIT_INST_LDS"),
            "active_lds": f("SQ_ACTIVE_INST_LDS"), "active_valu": f("SQ_ACTIVE_INST_VALU")}


mrows, erows = pmc_rows("mfma"), pmc_rows("efetch")
evals = []
for k in kernels:
    if not short(k["name"]).startswith("k_eval") or short(k["name"]).startswith("k_eval_rows"):
        continue
    e = {"kernel": short(k["name"]), "avg_ns": k["avg_ns"], "calls": k["calls"]}
    m = mrows.get(k["name"], {})
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        busy = statistics.mean(m["SQ_VALU_MFMA_BUSY_CYCLES"])
        e["mfma_busy_cycles"] = busy
        e["mfma_busy_frac_at_2p4GHz"] = busy / (SIMDS * k["avg_ns"] * CLOCK_GHZ)
    for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_MFMA", "SQ_WAVE_CYCLES", "SQ_WAVES",
              "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        if c in m:
            e[c] = statistics.mean(m[c])
    if "SQ_INSTS_MFMA" in m:      # the largest dispatch = one whole 65,536-root batch (one engine)
        e["SQ_INSTS_MFMA_max_dispatch"] = max(m["SQ_INSTS_MFMA"])
    if "SQ_INSTS_VALU" in e:      # VALU pipe busy (2 cycles per wave64 instruction, MFMA included)
        e["valu_issue_frac_at_2p4GHz"] = e["SQ_INSTS_VALU"] * 2 / (SIMDS * k["avg_ns"] * CLOCK_GHZ)
    f = erows.get(k["name"], {}).get("FETCH_SIZE")
    if f:
        e["hbm_read_bytes"] = 2 * statistics.mean(f) * 1024
    w2 = pmc_rows("eval2").get(k["name"], {})      # round 6: the evaluator's wave-time split
    if w2:
        e["wave_time_split"] = wave_split(w2)
    evals.append(e)

# ------------------------------------------------- C3 policy kernel (round 4) --
# k_policy_act on the C3 step (the pol1 / pol2 passes run the PMC command): per
# dispatch means of its counters; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1,024 SIMDs x
# its duration x 2.4 GHz); VALU issue = SQ_INSTS_VALU x 2 cycles / the same; the
# wave-time split from the quad-cycle counters (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
# = WAVE_CYCLES).  The duration is the kernel-trace average of its C3 dispatches.
def merged(kinds, pred):
    res = {}
    for kind in kinds:
        for n, v in pmc_rows(kind).items():
            if pred(short(n)):
                d = res.setdefault(short(n), {})
                for c, vals in v.items():
                    d.setdefault(c, vals)
    return res


policy = []
for name, m in merged(("pol1", "pol2"), lambda n: n.startswith("k_policy_act")).items():
    kk = next((k for k in kernels if short(k["name"]) == name), None)
    if not kk:
        continue
    rows = [r for r in trace if short(r["Kernel_Name"]) == name]
    gmax = max(int(r["Grid_Size_X"]) for r in rows)
    dur = statistics.mean([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
                           if int(r["Grid_Size_X"]) * 4 >= gmax])
    e = {"kernel": name, "avg_ns_c3": dur, "counters_per_dispatch": {c: statistics.mean(v) for c, v in m.items()}}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        e["mfma_busy_frac_at_2p4GHz"] = statistics.mean(m["SQ_VALU_MFMA_BUSY_CYCLES"]) / (SIMDS * dur * CLOCK_GHZ)
    if "SQ_INSTS_VALU" in m:
        e["valu_issue_frac_at_2p4GHz"] = statistics.mean(m["SQ_INSTS_VALU"]) * 2 / (SIMDS * dur * CLOCK_GHZ)
    e["wave_time_split"] = wave_split(m)
    policy.append(e)

# ------------------------------------------------ 2-ply enumerators (round 4) --
# per enumerator kernel: dispatch count, instruction totals and per-wave figures, the
# wave-time split (enum1 / enum2 passes, the 2-ply command), and the kernel-trace time
enums = []
for name, m in merged(("enum1", "enum2"), lambda n: n.startswith("k_enum")).items():
    kk = next((k for k in kernels if short(k["name"]) == name), None)
    e = {"kernel": name, "dispatches": len(next(iter(m.values()))),
         "totals": {c: sum(v) for c, v in m.items()},
         "avg_ns": kk["avg_ns"] if kk else None, "calls": kk["calls"] if kk else None,
         "wave_time_split": wave_split(m)}
    enums.append(e)

# per-pass, per-kernel counter totals and dispatch counts (the raw CSVs reduced, so the
# figures above can be recomputed from what is committed under profiles/)
with open(os.path.join(out, "pmc_totals.csv"), "w") as fo:
    fo.write("pass,kernel,counter,dispatches,total\n")
    for kind in ("fetch", "write", "sqi", "sqc", "mfma", "efetch", "eval2", "pol1", "pol2", "enum1", "enum2"):
        for n, v in pmc_rows(kind).items():
            for c, vals in v.items():
                fo.write(f"{kind},{short(n).replace(',', ';')},{c},{len(vals)},{sum(vals):.17g}\n")

summary = {"command": "python bench.py " + cmd, "pmc_command": "python bench.py " + pmc_cmd,
           "kernels": kernels[:24], "env_step": env, "two_ply_eval": evals, "policy": policy,
           "two_ply_enum": enums}
json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k in kernels[:24]:
    print(f"{k['pct']:6.2f}% {k['avg_ns']/1e3:10.1f} us (tail {k.get('avg_ns_timed_tail', 0)/1e3:.1f}) "
          f"x{k['calls']:4d}  {k['name'][:70]}  {k.get('hbm_bytes_per_launch', 0)/1e6:.1f} MB")
if "sq" in env:
    print(json.dumps(env["sq"], indent=1))
for e in evals + policy + enums:
    print(json.dumps(e))
