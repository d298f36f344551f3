"""GPU busy time vs wall time over a kernel trace (rocprofv3 --kernel-trace
*_kernel_trace.csv or its *_results.db): for the window spanning the last `--last` kernels (or
the whole trace) prints the union of kernel intervals, the wall span, and
the largest idle gaps with the kernels either side of them.

    python tools/trace_gaps.py gpurun_out/ppo/.../xxx_kernel_trace.csv --after k_encode_rec
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after", default=None, help="start the window at the last kernel whose name holds this")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    if a.trace.endswith(".db"):                     # rocprofv3's default SQLite output
        con = sqlite3.connect(a.trace)
        ks = sorted((int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels"))
    else:
        rows = list(csv.DictReader(open(a.trace)))
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if a.after:
        idx = [i for i, k in enumerate(ks) if a.after in k[2]]
        ks = ks[idx[-1]:] if idx else ks
    busy, gaps, cur_end, prev = 0, [], ks[0][0], None
    for s, e, n in ks:
        if s > cur_end:
            gaps.append((s - cur_end, prev, n))
        busy += max(0, e - max(s, cur_end))
        if e > cur_end:
            cur_end, prev = e, n
    span = cur_end - ks[0][0]
    print(f"kernels {len(ks)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
    by = {}
    for s, e, n in ks:
        by.setdefault(n[:90], [0, 0])
        by[n[:90]][0] += 1
        by[n[:90]][1] += e - s
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{c:6d} {t / 1e6:9.3f} ms  {n}")
    print("largest gaps:")
    for g, p, n in sorted(gaps, key=lambda x: -x[0])[:a.top]:
        print(f"  {g / 1e3:9.1f} us  after {str(p)[:60]}  before {n[:60]}")


if __name__ == "__main__":
    main()
