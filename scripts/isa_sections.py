"""Static instruction mix of a straight-line chain kernel, section by section (VERDICT r04 Next #3:
attribute the wide fp8 chain's VALU to its sources).

The chain kernels are compile-time unrolled (sfor), so a section's static count is its dynamic count
per wave, up to the few runtime loops (`for e = tid; ...` tasks, `#pragma nounroll`) that the
counts flag.  In a CVAE_DIAG_STAMPS=2 build every bar()/sub() writes `s_memrealtime`; those split the
kernel's assembly into the sections scripts/diag_stamps.py names.

  hipcc --offload-arch=gfx950 -O3 ... -DCVAE_DIAG_STAMPS=2 --cuda-device-only -S -o k.s cvae_capi.hip
  python scripts/isa_sections.py k.s 'widechain_kernelINS_4ArchILi200ELi6ELi512ELi8ELi8ELb1ELb0ELb1E' [names]

names: "wfp8" (the SUB=1 DT=fp8 list of diag_stamps.py), "wbf16", "ring", or none (numbered).
"""
import re
import sys

NAMES = {
    "wfp8": (["pro:issue", "pro:transform", "pro:bar", "C0+copies", "E0 gemm", "E0 epi", "C1|E1"]
             + [f"E{i}" for i in range(2, 8)] + ["FC", "D0"] + [f"D{i}" for i in range(1, 7)]
             + ["D7+loss", "fixup", "D7b mx cvt", "D7b"] + [f"D{i}b" for i in range(6, 0, -1)]
             + ["D0b mx cvt", "D0b", "FCb mx cvt", "FCb gemm", "FCb epi"] + [f"E{i}b" for i in range(7, 1, -1)]
             + ["E1b|C1b", "partials"]),
    "wbf16": (["pro:issue", "pro:transform", "pro:bar", "C0+copies", "E0 gemm", "E0 epi", "C1|E1"]
              + [f"E{i}" for i in range(2, 8)] + ["FC", "D0"] + [f"D{i}" for i in range(1, 7)]
              + ["D7+loss", "fixup", "D7b"] + [f"D{i}b" for i in range(6, 0, -1)]
              + ["D0b", "FCb gemm", "FCb epi"] + [f"E{i}b" for i in range(7, 1, -1)] + ["E1b|C1b", "partials"]),
    "ring": ["pro:issue", "pro:transform", "pro:bar", "C0+copies", "E0 gemm", "E0 epi", "C1|E1", "E2", "E3",
             "FC", "reparam", "D0", "D1", "D2", "D3+loss", "fixup", "D3b", "D2b", "D1b", "D0b", "FCb gemm",
             "FCb epi", "E3b", "E2b", "E1b|C1b", "partials"],
}


def kernel_lines(path, pattern):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z_]\S*):(\s|$)", l)
        if start is None and m and pattern in m.group(1):
            start, name = i, m.group(1)
        elif start is not None and l.startswith(".Lfunc_end"):
            return name, lines[start + 1:i]
    raise SystemExit(f"no kernel matching {pattern!r} in {path}")


def classify(op):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vload"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "vstore"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op in ("s_waitcnt", "s_barrier", "s_nop", "s_memrealtime", "s_sleep", "s_setprio") or op.startswith("s_cbranch") \
            or op == "s_branch":
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, pattern = sys.argv[1], sys.argv[2]
    names = NAMES.get(sys.argv[3], []) if len(sys.argv) > 3 else []
    name, body = kernel_lines(path, pattern)
    secs, cur, branches = [], {}, 0
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or re.match(r"^\S+:(\s|$)", t):
            continue
        op = t.split()[0]
        if op == "s_memrealtime":
            secs.append((cur, branches))
            cur, branches = {}, 0
            continue
        c = classify(op)
        if c:
            cur[c] = cur.get(c, 0) + 1
            if op.startswith("s_cbranch") or op == "s_branch":
                branches += 1
    secs.append((cur, branches))
    print(name[:140])
    cols = ["valu", "mfma", "salu", "lds", "vload", "vstore", "smem", "ctl"]
    print(f"{'section':>14s} " + " ".join(f"{c:>6s}" for c in cols) + "  branches")
    tot = {c: 0 for c in cols}
    # section 0 is before the first stamp (the entry); sections between stamps i-1 and i are named i-1
    for i, (d, br) in enumerate(secs[1:]):
        nm = names[i] if i < len(names) else f"sec{i}"
        print(f"{nm:>14s} " + " ".join(f"{d.get(c, 0):6d}" for c in cols) + f"  {br}")
        for c in cols:
            tot[c] += d.get(c, 0)
    print(f"{'total':>14s} " + " ".join(f"{tot[c]:6d}" for c in cols))
    print(f"(entry before the first stamp: {secs[0][0]})")


if __name__ == "__main__":
    main()
