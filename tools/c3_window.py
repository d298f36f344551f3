"""The driver's short C3 window on the device clock: from a rocprofv3 kernel trace
of `bench.py --steps K` (C3 only), the timed replays' kernels are the K x shards
k_policy_act dispatches before the 16 x shards eager ones that follow the timed
region (bench.py: the roofline's event steps).  Prints the window's device span
(first kernel start to last kernel end), its busy union, the idle before the first
kernel after the previous one, and the per-step cadence, next to the bench line's
wall-clock ms_per_step.   Usage: tools/c3_window.py TRACE_CSV BENCH_LOG K [shards]"""
import csv
import json
import sys


def main():
    trace, log, K = sys.argv[1], sys.argv[2], int(sys.argv[3])
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    rows = list(csv.DictReader(open(trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    pol = [i for i, k in enumerate(ks) if "k_policy_act" in k[2]]
    eager = 16 * S
    first_pol = pol[-(eager + K * S)]
    first_eager_pol = pol[-eager]
    # the window: from the first timed policy dispatch to the kernel before the first eager one
    lo = first_pol
    hi = first_eager_pol - 1
    win = ks[lo:hi + 1]
    t0, t1 = win[0][0], max(k[1] for k in win)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    prev_end = max(k[1] for k in ks[:lo]) if lo else t0
    starts = [ks[i][0] for i in pol[-(eager + K * S):-eager]][::S]
    cad = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
    line = [x for x in open(log) if x.startswith("{")]
    d = json.loads(line[-1]) if line else {}
    out = {"kernels": len(win), "span_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6,
           "span_ms_per_step": (t1 - t0) / 1e6 / K, "idle_before_ms": (t0 - prev_end) / 1e6,
           "cadence_us_first": cad[:4], "cadence_us_last": cad[-4:],
           "cadence_us_mean": sum(cad) / max(len(cad), 1),
           "bench_ms_per_step": d.get("ms_per_step"), "bench_value_M": (d.get("value") or 0) / 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
