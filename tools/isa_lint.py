"""ISA lint for libbgx.so: extract every gfx950 code object from the library's
.hip_fatbin section (clang offload bundles), disassemble it with llvm-objdump and
report instruction forms that are banned from the product library.

Banned: packed-FP32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) carrying an
`op_sel:[...]` modifier, i.e. a low result that reads the HIGH dword of a source pair
(a broadcast).  Round 4's intermittent wrong 2-ply leaf values (columns 16-31 of the
first leaf tile, only at two waves per SIMD) came with exactly that form; the builds
without it are exact.  The `op_sel_hi` form (the default element
mapping) is allowed.

    python tools/isa_lint.py [LIB.so] [--dump DIR] [--context N]

Exit status 1 if a banned form is present.  tests/test_isa_lint_cpu.py runs it on the
built library."""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
BANNED = re.compile(r"\bv_pk_(fma|mul|add)_f32\b.*\bop_sel:\[")
PACKED_F32 = re.compile(r"\bv_pk_(fma|mul|add|mov)_f32\b")


def code_objects(lib: str) -> list[bytes]:
    """The amdgcn code objects of every offload bundle in LIB's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as tmp:
        fat = os.path.join(tmp, "fat.bin")
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib,
                        os.path.join(tmp, "stripped")], check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


def disassemble(obj: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(obj)
        f.flush()
        r = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn",
                            f.name], check=True, capture_output=True, text=True)
    return r.stdout


def kernels(asm: str):
    """Yield (symbol, [instruction lines]) for every function in a disassembly."""
    name, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name and line.strip():
            body.append(line.strip())
    if name:
        yield name, body


def demangle(names):
    import shutil
    tool = shutil.which("c++filt")
    if not tool or not names:
        return list(names)
    r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else list(names)


def lint(lib: str, dump: str | None = None, context: int = 0):
    """Returns (banned, packed): banned = [(kernel, index, line, context lines)],
    packed = {kernel: count of packed-FP32 instructions}."""
    banned, packed = [], {}
    for i, obj in enumerate(code_objects(lib)):
        asm = disassemble(obj)
        if dump:
            os.makedirs(dump, exist_ok=True)
            open(os.path.join(dump, f"co{i}.s"), "w").write(asm)
        for name, body in kernels(asm):
            k = sum(1 for ln in body if PACKED_F32.search(ln))
            if k:
                packed[name] = packed.get(name, 0) + k
            for j, ln in enumerate(body):
                if BANNED.search(ln):
                    banned.append((name, j, ln, body[max(0, j - context):j + 1]))
    return banned, packed


def main():
    args = sys.argv[1:]
    dump = context = None
    if "--dump" in args:
        i = args.index("--dump")
        dump = args[i + 1]
        del args[i:i + 2]
    if "--context" in args:
        i = args.index("--context")
        context = int(args[i + 1])
        del args[i:i + 2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = args[0] if args else os.path.join(root, "mlp-ppo-2ply-p3_amd", "bgx", "libbgx.so")
    banned, packed = lint(lib, dump, context or 0)
    names = sorted(packed)
    for n, d in zip(names, demangle(names)):
        print(f"packed-f32 {packed[n]:5d}  {d}")
    for name, j, ln, ctx in banned:
        print(f"BANNED {demangle([name])[0]} +{j}: {ln}")
        for c in ctx[:-1]:
            print(f"    {c}")
    print(f"{len(banned)} banned op_sel packed-FP32 instructions in {lib}")
    sys.exit(1 if banned else 0)


if __name__ == "__main__":
    main()
