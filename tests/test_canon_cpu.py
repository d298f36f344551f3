"""The canonical sub-move order of the GPU move generator (bg_core.h canon_mask,
Gen::pure_walk / mirror), restated in Python and checked against the oracle on
random doubles positions: the walk's max-length entries equal the reference's
ordered list, and walks that cannot bear off visit every afterstate once (the
GPU runs them without a dedup table)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_canonical_doubles_walk():
    import check_canon
    checked, distinct = check_canon.check(1500, seed=5)
    assert checked == 1500 and distinct > 800
