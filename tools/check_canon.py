"""CPU check of the canonical sub-move order (bg_core.h canon_mask) for doubles.

Walks every doubles roll of many positions in the reference's DFS order with the
canonical pruning (a normal sub-move from a lower point after one from a higher
point is skipped; for PLAYER2 the chain bit a - d is kept only when the moved
checker is alone there) and NO dedup table or revisit memo, then checks
  * the max-length entries in walk order equal the oracle's ordered move list;
  * when no bear-off can occur within the walk (more than 3 checkers outside
    home or on the bar), every inserted afterstate is distinct -- the GPU walk
    then runs without a table.
Usage: python tools/check_canon.py [n_positions]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

HOME = [set(range(18, 24)), set(range(6))]


def gen(b, d, pl):
    """(normal source bits ascending, special) of get_moves_with_one_die."""
    own, opp = b[pl * 24:pl * 24 + 24], b[(1 - pl) * 24:(1 - pl) * 24 + 24]
    bar, off = b[48 + pl], b[50 + pl]
    if off == 15:
        return [], None
    if bar > 0:
        e = d - 1 if pl == 0 else 24 - d
        return ([], ("bar", e)) if opp[e] < 2 else ([], None)
    srcs = []
    for i in range(24):
        dst = i + d if pl == 0 else i - d
        if own[i] > 0 and 0 <= dst < 24 and opp[dst] < 2:
            srcs.append(i)
    special = None
    occ = [i for i in range(24) if own[i] > 0]
    if all(i in HOME[pl] for i in occ) and sum(own[i] for i in HOME[pl]) + off == 15:
        far = min(occ) if pl == 0 else max(occ)
        if (pl == 0 and far + d >= 24) or (pl == 1 and far - d < 0):
            special = ("off", far)
        else:
            e = 24 - d if pl == 0 else d - 1
            if e != far and own[e] > 0:
                special = ("off", e)
    return srcs, special


def apply(b, src, dst, pl):
    b = b.copy()
    o, p = pl * 24, (1 - pl) * 24
    if src == "bar":
        b[48 + pl] -= 1
    else:
        b[o + src] -= 1
    hit = 0
    if dst != "off":
        if b[p + dst] == 1:
            b[p + dst] = 0
            b[48 + 1 - pl] += 1
            hit = 1
        b[o + dst] += 1
    else:
        b[50 + pl] += 1
    return b, hit


def enc(src, dst, hit):
    s = 24 if src == "bar" else src
    t = 25 if dst == "off" else dst
    return s | (t << 5) | (hit << 10) | 0x8000


def children(b, d, pl, last, mirror=False, forbid=None):
    """(bit, src, dst) in DFS order, canonical after a sub-move with bit `last`.
    mirror (PLAYER2, set semantics only): bits <= last instead.
    forbid (PLAYER2 walks without bear-off, ordered): the points below an earlier
    sub-move's source that were occupied when it was made."""
    srcs, special = gen(b, d, pl)
    out = []
    for s in srcs:
        if forbid is not None:
            if (forbid >> s) & 1:
                continue
        elif last is not None and last < 24:
            if mirror:
                if s > last:
                    continue
            elif s < last:
                chain = pl == 1 and s == last - d and b[pl * 24 + s] == 1
                if not chain:
                    continue
        out.append((s, s, s + d if pl == 0 else s - d))
    if special is not None:
        kind, x = special
        out.append((31, "bar", x) if kind == "bar" else (31, x, "off"))
    return out


def walk(b0, d, pl, mirror=False, use_forbid=False):
    inserts = []          # (key bytes, encoded move, len) in walk order
    got4 = [False]

    def occ(b):
        return sum(1 << i for i in range(24) if b[pl * 24 + i] > 0)

    def rec(b, depth, last, code, forbid=0):
        kids = children(b, d, pl, last, mirror, forbid if use_forbid else None) if depth < 4 else []
        has_kids = bool(gen(b, d, pl)[0]) or gen(b, d, pl)[1] is not None
        if depth == 4 or (not has_kids and depth > 0):
            if depth == 4 or not got4[0]:
                inserts.append((b.tobytes(), code, depth))
            if depth == 4:
                got4[0] = True
            return
        for bit, s, t in kids:
            nb, hit = apply(b, s, t, pl)
            nf = forbid | (occ(b) & ((1 << bit) - 1)) if bit < 24 else forbid
            rec(nb, depth + 1, bit, code | (enc(s, t, hit) << (16 * depth)), nf)

    rec(b0, 0, None, 0)
    seen, out = set(), []
    for key, code, ln in inserts:
        if key in seen:
            continue
        seen.add(key)
        out.append((code, ln))
    mx = max((ln for _, ln in out), default=0)
    return [c for c, ln in out if ln == mx], inserts


def random_board(rng):
    x = np.zeros(52, np.int8)
    for p in (0, 1):
        left = 15
        if rng.rand() < 0.15:
            x[48 + p] = rng.randint(1, 3); left -= x[48 + p]
        if rng.rand() < 0.3:
            x[50 + p] = rng.randint(0, left); left -= x[50 + p]
        pts = list(range(18, 24)) if (p == 0 and rng.rand() < 0.3) else (
            list(range(6)) if (p == 1 and rng.rand() < 0.3) else list(range(24)))
        while left > 0:
            q = pts[rng.randint(len(pts))]
            if x[(1 - p) * 24 + q] > 0:
                pts = list(range(24))
                continue
            k = min(left, rng.randint(1, 4)); x[p * 24 + q] += k; left -= k
    return x


def check(n, seed=11):
    rng = np.random.RandomState(seed)
    checked = distinct_checked = 0
    for i in range(n):
        b = random_board(rng)
        pl = int(rng.randint(2))
        d = int(rng.randint(1, 7))
        ref, _ = O.movegen(b, pl, (d, d), cap=4096)
        got, inserts = walk(b, d, pl)
        assert [int(v) for v in ref] == got, (i, b.tolist(), pl, d)
        checked += 1
        outside = int(b[48 + pl]) + sum(int(b[pl * 24 + j]) for j in range(24) if j not in HOME[pl])
        if outside > 3:
            if pl == 0:
                keys = [k for k, _, _ in inserts]
                assert len(keys) == len(set(keys)), (i, b.tolist(), pl, d)
            else:
                # PLAYER2, ordered: the forbidden-point walk visits each state once,
                # first occurrences in the reference's order
                got_f, fins = walk(b, d, pl, use_forbid=True)
                keys = [k for k, _, _ in fins]
                assert len(keys) == len(set(keys)), ("forbid", i, b.tolist(), pl, d)
                assert [int(v) for v in ref] == got_f, ("forbid", i, b.tolist(), pl, d)
                # PLAYER2, set semantics (2-ply): the mirrored walk visits each
                # state once and yields the same set of afterstates
                _, mins = walk(b, d, pl, mirror=True)
                keys = [k for k, _, _ in mins]
                assert len(keys) == len(set(keys)), (i, b.tolist(), pl, d)
                mx = max(ln for _, _, ln in mins) if mins else 0
                want = set(O.apply_move(b, pl, int(v)).tobytes() for v in ref)
                assert set(k for k, _, ln in mins if ln == mx) == want, (i, b.tolist(), pl, d)
            distinct_checked += 1
    return checked, distinct_checked


if __name__ == "__main__":
    c, dc = check(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
    print(f"ok: {c} doubles positions equal the oracle; {dc} no-bear-off walks without a repeat")
