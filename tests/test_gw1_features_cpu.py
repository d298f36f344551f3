"""bgx_ppo_gw1 builds its A operand (fc1 features of 8 rows, fp16, as autocast casts
them) in packed f16 arithmetic on t = 1024 + v: u = min(max(t A + B, 0), C)
(csrc/bg_ppo_fused.hip gw1_param / gw1_feats).  Every step is exact in f16, so the
result equals fp16 of the fp32 feature of immutable_board.py:171-212 for every byte
value a record can hold; off / 15 keeps the fp32 path.  Restated here in numpy."""
import numpy as np


def _params(f):
    """(byte, A, B, C, off) of feature f, as gw1_param."""
    if f < 196:
        p = 1 if f >= 98 else 0
        q = f - 98 * p
        if q < 96:
            k = q & 3
            if k < 3:
                return 24 * p + (q >> 2), 1.0, -1024.0 - k, 1.0, False
            return 24 * p + (q >> 2), 0.5, -513.5, 64.0, False
        if q == 96:
            return 48 + p, 0.5, -512.0, 64.0, False
        return 50 + p, 0.0, 0.0, 0.0, True
    if f < 198:
        return 52, (-1.0 if f == 196 else 1.0), (1025.0 if f == 196 else -1024.0), 1.0, False
    if f == 198:
        return 0, 0.0, 1.0, 1.0, False
    return 0, 0.0, 0.0, 0.0, False


def _reference(f, v):
    """fp32 feature value (board encoder semantics) of byte value v, then fp16."""
    v = np.float32(v)
    if f < 196:
        q = f % 98
        if q < 96:
            k = q & 3
            x = (v >= k + 1) * np.float32(1.0) if k < 3 else (np.float32((v - 3) / 2) if v >= 3 else np.float32(0))
        elif q == 96:
            x = v / np.float32(2.0)
        else:
            x = v * np.float32(1.0 / 15.0)
    elif f == 196:
        x = np.float32(1.0) - v
    elif f == 197:
        x = v
    elif f == 198:
        x = np.float32(1.0)
    else:
        x = np.float32(0.0)
    return np.float16(x)


def test_packed_f16_features_exact():
    for f in range(224):
        byte, A, B, C, off = _params(f)
        vals = range(0, 2) if byte == 52 else range(0, 16)
        for v in vals:
            if off:
                got = np.float16(np.float32(v) * np.float32(1.0 / 15.0))
            else:
                t = np.float16(1024 + v)
                prod = np.float16(t * np.float16(A))          # exact: A in {0, 1/2, 1, -1}
                assert float(prod) == float(t) * A
                u = np.float16(prod + np.float16(B))           # the fma's one rounding
                u = np.minimum(np.maximum(u, np.float16(0)), np.float16(C))
                got = u
            assert got == _reference(f, v), (f, v, got, _reference(f, v))
