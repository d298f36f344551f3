"""Diagnose the two-leaf-tiles-in-flight fault of the wide (H = 128) 2-ply evaluator
(experiment).  Runs the 48-root batch of
tests/test_gpu_search.py with the library at BGX_LIB (a -DBGX_WIDE_PAIR build), dumps
V per pool slot (BGX_2PLY_DUMP) and compares every valid leaf with an fp64 MLP on the
leaf's own encoding.  For each wrong leaf it tests simple explanations:
  * V of another leaf of the same 64-slot pair (the same column of the other tile, or
    another column): operands crossed between tiles / lanes;
  * the leaf's fp64 V with one replier point k-block, block 12 or the row part left out
    (an MFMA result read before it landed, or a stale accumulator);
and prints the slot positions within the pair.

    BGX_LIB=scratch/libbgx_pair.so python tools/pair_diag.py
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import bgx  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402
from bgx.search import ValueHead, two_ply  # noqa: E402


def main():
    mlp = dict(np.load(os.path.join(ROOT, "tests", "golden", "mlp.npz")))
    H = 128
    net = PolicyNet(hidden_size=H).cuda()
    pre = f"h{H}_"
    net.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in mlp.items()
                         if k.startswith(pre) and not k.endswith(("logits", "values"))})
    vh = ValueHead(net)
    B = 48
    eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(np.arange(500, 500 + B, dtype=np.uint32))
    eng.reset()
    rng = np.random.RandomState(2)
    for _ in range(25):
        nm = eng.n_moves().cpu().numpy()
        eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
    from test_gpu_search import _leaf_reference
    out = {}
    for trial in range(int(os.environ.get("TRIALS", "3"))):
        d = tempfile.mkdtemp()
        prefix = os.path.join(d, "d")
        from bgx._lib import debug_option
        debug_option("BGX_2PLY_DUMP", prefix)
        two_ply(eng, vh)
        debug_option("BGX_2PLY_DUMP", None)
        keys = np.fromfile(prefix + ".keys", np.uint32).reshape(-1, 4)
        tags = np.fromfile(prefix + ".tags", np.uint32)
        v = np.fromfile(prefix + ".v", np.float32)
        side = np.fromfile(prefix + ".side", np.uint32).reshape(-1, 4)
        ml = np.fromfile(prefix + ".ml", np.uint8)
        idx, vref = _leaf_reference(net, keys, tags, side, ml)
        err = np.abs(v[idx].astype(np.float64) - vref)
        bad = idx[err > 1e-6]
        ref_of = dict(zip(idx.tolist(), vref.tolist()))
        res = {"leaves": int(len(idx)), "bad": int(len(bad)),
               "slot_mod64_hist": np.bincount(bad % 64, minlength=64).tolist() if len(bad) else [],
               "max_err": float(err.max())}
        # explanations
        same_col_other_tile = other_leaf = 0
        for s in bad[:2000]:
            vb = float(v[s])
            pair = (s // 64) * 64
            cands = [ref_of.get(pair + k) for k in range(64) if pair + k != s]
            if ref_of.get(s ^ 32) is not None and abs(ref_of[s ^ 32] - vb) < 1e-6:
                same_col_other_tile += 1
            elif any(c is not None and abs(c - vb) < 1e-6 for c in cands):
                other_leaf += 1
        res["equals_same_column_other_tile"] = same_col_other_tile
        res["equals_another_leaf_of_pair"] = other_leaf
        res["examples"] = [{"slot": int(s), "v": float(v[s]), "ref": float(ref_of[int(s)])} for s in bad[:8]]
        out[f"trial{trial}"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
