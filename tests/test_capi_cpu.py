"""CPU-side checks of the drop-in boundary: libbgx.so loads (no GPU needed) and
exports every entry point include/bgx.h declares."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bgx.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(bgx_\w+)\s*\(", txt, re.M)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("bgx_engine_create", "bgx_step", "bgx_reset", "bgx_movegen", "bgx_encode"):
        assert s in syms


def test_library_exports_every_symbol():
    import bgx._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libbgx.so not built")
    lib = L.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    nm = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (bgx_\w+)", nm))
    assert set(declared_symbols()) <= exported
    assert set(L.SIGNATURES) == set(declared_symbols())


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "bgoracle" not in src, f


def test_library_built_from_these_sources():
    """Build provenance: the id compiled into libbgx.so equals the hash of the
    current csrc/ + include/ sources and flags (a stale library fails here)."""
    import __graft_entry__ as G
    import bgx._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libbgx.so not built")
    want = L.source_hash(G.flags_id())
    assert L.embedded_build_id() == want
    assert L.load().bgx_build_id().decode() == want


def test_oracle_under_asan():
    """The CPU oracle built with AddressSanitizer + UBSan (oracle/Makefile `asan`)
    plays 60 seeded random games (invalid actions, resets, match ends) and
    enumerates > 500-move positions with a small cap, checking checker
    conservation; any memory error or UB aborts."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    r = subprocess.run([os.path.join(ROOT, "oracle", "bgoracle_asan"), "60"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "asan ok" in r.stdout and "runtime error" not in r.stderr
