"""Build libbgx.so variants for A/B runs on the GPU box (experiments; the product
library is __graft_entry__.build()'s):

    python tools/build_variant.py OUT.so -DNAME [...]      # every HIP source, extra defines
    python tools/build_variant.py OUT.so --agpr-form ...    # without -amdgpu-mfma-vgpr-form
    python tools/build_variant.py OUT.so --slp ...          # SLP vectorization in every source

then run e.g. `BGX_LIB=OUT.so python bench.py ...` beside the default build."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def main():
    out, extra = sys.argv[1], sys.argv[2:]
    agpr = "--agpr-form" in extra              # MFMA accumulators left to the compiler (AGPRs)
    slp = "--slp" in extra                     # SLP vectorization back on in every source
    extra = [f for f in extra if f not in ("--agpr-form", "--slp")]
    with tempfile.TemporaryDirectory() as tmp:
        objs, procs = [], []
        for s in G.HIP_SOURCES:
            flags = G.hipcc_flags(s)
            if agpr:
                i = flags.index("-amdgpu-mfma-vgpr-form")
                del flags[i - 1:i + 1]
            if slp:
                flags = [f for f in flags if f != "-fno-slp-vectorize"]
            flags += extra
            o = os.path.join(tmp, s + ".o")
            objs.append(o)
            procs.append(subprocess.Popen(["hipcc"] + flags + ["-I" + os.path.join(ROOT, "include"), "-c",
                                                              os.path.join(G.CSRC, s), "-o", o]))
        if any(p.wait() for p in procs):
            raise SystemExit("hipcc failed")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main()
