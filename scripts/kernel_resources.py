"""Per-kernel register / LDS / scratch usage of the built library (the gfx950 code object's
AMDGPU metadata notes), without running anything: a kernel with VGPRs > 128 at 512 threads fits
one workgroup per CU, <= 128 two.

usage: python3 scripts/kernel_resources.py [pattern ...]   (substrings of the mangled names)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("CVAE_LIB") or os.path.join(ROOT, "defensive-model-vae_amd", "cvae_amd", "libcvae_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(blob):
    """gfx950 ELF images inside the clang offload bundles of the shared library."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    for m in re.finditer(re.escape(magic), blob):
        p = m.start() + len(magic)
        n = struct.unpack_from("<Q", blob, p)[0]
        p += 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", blob, p)
            p += 24
            ident = blob[p:p + idlen].decode(errors="replace")
            p += idlen
            if "gfx950" in ident:
                out.append(blob[m.start() + off:m.start() + off + size])
    return out


def resources(lib=LIB, pats=()):
    """[{name, demangled, vgpr, sgpr, lds, scratch, wg}] of every kernel (whose mangled name contains
    one of `pats`, when given) in the library's gfx950 code objects."""
    blob = open(lib, "rb").read()
    out = []
    for co in code_objects(blob):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
        for k in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
            name = re.search(r"\.name:\s+(\S+)", k)
            if not name or (pats and not any(p in name.group(1) for p in pats)):
                continue
            g = lambda key: (re.search(rf"\.{key}:\s+(\S+)", k) or [None, "-1"])[1]  # noqa: E731
            dem = subprocess.run(["c++filt"], input=name.group(1), capture_output=True,
                                 text=True).stdout.strip()
            out.append({"name": name.group(1), "demangled": dem, "vgpr": int(g("vgpr_count")),
                        "sgpr": int(g("sgpr_count")), "lds": int(g("group_segment_fixed_size")),
                        "scratch": int(g("private_segment_fixed_size")), "wg": int(g("max_flat_workgroup_size"))})
    return out


def main():
    for r in resources(LIB, sys.argv[1:]):
        print(f"vgpr {r['vgpr']:>4} sgpr {r['sgpr']:>3} lds {r['lds']:>6} scratch {r['scratch']:>5} "
              f"wg {r['wg']:>4}  {r['demangled'][:150]}")


if __name__ == "__main__":
    main()
