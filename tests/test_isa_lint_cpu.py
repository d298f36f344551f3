"""The product library's gfx950 ISA carries no packed-FP32 instruction with an
op_sel modifier (tools/isa_lint.py).  Round 4's wrong 2-ply leaf
values came with `v_pk_fma_f32 ... op_sel:[0,1,0]` from LLVM's SLP vectorizer; this
guards every kernel of libbgx.so against that form coming back (a toolchain change, a
flag change, another source packing across tiles).  CPU only: llvm-objdump on the
built library."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_lint  # noqa: E402

LIB = os.path.join(ROOT, "mlp-ppo-2ply-p3_amd", "bgx", "libbgx.so")


def test_banned_pattern_matches_only_op_sel_forms():
    bad = "v_pk_fma_f32 v[80:81], v[130:131], v[236:237], v[80:81] op_sel:[0,1,0]// 0000000355F4: D3B05050"
    ok = "v_pk_fma_f32 v[80:81], v[82:83], v[240:241], v[80:81] op_sel_hi:[1,0,1]"
    assert isa_lint.BANNED.search(bad)
    assert isa_lint.BANNED.search("v_pk_mul_f32 v[0:1], v[0:1], v[2:3] op_sel:[1,0] op_sel_hi:[1,1]")
    assert not isa_lint.BANNED.search(ok)
    assert not isa_lint.BANNED.search("v_pk_fma_f16 v1, v1, s56, v198 op_sel:[0,1,0]")   # packed f16: other datapath


@pytest.mark.skipif(not os.path.exists(LIB), reason="libbgx.so not built")
def test_libbgx_has_no_op_sel_packed_fp32():
    objs = isa_lint.code_objects(LIB)
    assert len(objs) == 5, "one gfx950 code object per HIP source"
    banned, packed = isa_lint.lint(LIB)
    assert not banned, "\n".join(f"{k} +{j}: {ln}" for k, j, ln, _ in banned[:10])
    # the scan sees the packed-FP32 code that exists (the PPO kernels use the op_sel_hi form)
    assert sum(packed.values()) > 100
