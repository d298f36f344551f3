"""Work split of the C4 reply enumerators (experiment; needs a BGX_COUNTERS build).

    python tools/enum_counters.py --build          # libbgx_cnt.so beside libbgx.so (CPU, hipcc)
    python tools/enum_counters.py [--age 180]      # on the GPU: one C4 batch, counters printed

Counters (csrc/bg_search.hip BG_CNT / BG_T1, s_memtime ticks are 100 MHz):
  1 rows entering nd_row, 3 rows sent to per-job walks at entry (bear-off possible / > 64
  first moves), 6 rows of nd_row_bar (replier on the bar), 8 their slow rolls, 4 slow
  rolls of nd_row's fast rows, 5 nd_row chunks, 13 two-steps emitted by nd_row, 9 ticks
  in nd_row (+ nd_row_bar), 10 ticks in the light enumerator's per-job walks, 11 those
  jobs, 12 ticks in the doubles enumerator's per-row job loops.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")
LIB = os.path.join(PKG, "bgx", "libbgx_cnt.so")
NAMES = {1: "nd_rows", 3: "nd_rows_rejected", 4: "slow_rolls_in_fast_rows", 5: "nd_chunks",
         6: "bar_rows", 8: "slow_rolls_in_bar_rows",
         13: "nd_two_steps_emitted", 9: "ticks_nd_row", 10: "ticks_light_per_job", 11: "light_per_job_jobs",
         12: "ticks_doubles_rows", 0: "ticks_doubles_table_walks", 2: "doubles_pure_walks", 14: "ticks_doubles_pure",
         7: "doubles_bar_jobs", 15: "ticks_doubles_bar",
         # bg_core.h's move-generator counters (+16)
         16: "core_doubles_calls", 17: "core_ticks_doubles", 18: "core_place_batches", 19: "core_depth2_fresh",
         21: "core_depth3_fresh", 22: "core_flat_leaves_calls", 23: "core_flat_leaves_children", 24: "core_commit_n",
         25: "core_ticks_doubles_to_got4", 26: "core_got4", 27: "core_ticks_push", 28: "core_ticks_probe",
         29: "core_ticks_place", 30: "core_depth2_children", 31: "core_depth3_children"}


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    with tempfile.TemporaryDirectory() as tmp:
        objs = []
        procs = []
        for s in G.HIP_SOURCES:
            o = os.path.join(tmp, s + ".o")
            objs.append(o)
            procs.append(subprocess.Popen(["hipcc"] + G.hipcc_flags(s) + ["-DBGX_COUNTERS", "-I" + os.path.join(ROOT, "include"), "-c",
                                                              os.path.join(PKG, "csrc", s), "-o", o]))
        if any(p.wait() for p in procs):
            raise SystemExit("hipcc failed")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs, check=True)
    print(LIB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--age", type=int, default=180)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=40)
    a = ap.parse_args()
    if a.build:
        return build()
    os.environ["BGX_LIB"] = LIB
    sys.path.insert(0, PKG)
    import torch
    import bgx
    from bgx import _lib
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, two_ply, two_ply_timings
    L = _lib.load()
    fn = L.bgx_debug_search_counters
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = PolicyNet().to(dev)
    net.pack()
    eng = bgx.Engine(batch=a.batch, max_moves=500, seed=77, dice="philox", auto_reset=True, device=dev)
    eng.reset(want_obs=False)
    for i in range(a.age):
        act, _, _ = net.act(eng, seed=5, step=i)
        eng.step(act, want_obs=False, want_info=False)
    torch.manual_seed(1)
    vh = ValueHead(PolicyNet(hidden_size=a.hidden).to(dev))
    two_ply(eng, vh)
    c = (ctypes.c_ulonglong * 32)()
    fn(ctypes.cast(c, ctypes.c_void_p))              # reset
    _, _, _, st = two_ply(eng, vh)
    te, tv = two_ply_timings(eng)
    fn(ctypes.cast(c, ctypes.c_void_p))
    out = {NAMES.get(i, f"c{i}"): int(c[i]) for i in range(32) if c[i]}
    out.update({"stats": st, "enumeration_ms": te, "evaluation_ms": tv, "age": a.age, "hidden": a.hidden})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
