"""ISA audit of the render kernels (CPU only): the wide-buffer-store hazard behind round 2's
"stale path-state reads" (DESIGN.md §4 "path state").

A buffer store of more than 64 bits (dwordx3 / dwordx4) reads its data VGPRs over more than one
cycle; a VALU instruction that overwrites those VGPRs right after the store needs one wait state
in between, or the store writes the NEW value of the overwritten dwords.  LLVM's hazard
recognizer (GCNHazardRecognizer::createsVALUHazard) assumes the hazard does not exist when the
MUBUF store takes its soffset from an SGPR, so it inserts no wait state there -- but gfx950 has
it: a path-state record stored with `buffer_store_dwordx4 v[6:9], v102, s[12:15], s10 offen`
immediately followed by `v_sub_u32 v7, 0, v68` lost the high half of its z component (blue
channel NaN in 17 % of the pixels of a 4K 16-spp frame; the same kernel with 8-byte stores is
exact; tools/repro_pathstate.py, profiles/r03/pathstate_hazard.txt).

usage: python tools/isa_audit.py KERNEL.s   -> prints every hazard site, exit status 1 if any
"""
import re
import sys

STORE = re.compile(r"^\s*buffer_store_(dwordx3|dwordx4|b96|b128)\s+v\[(\d+):(\d+)\],\s*(\S+),\s*(s\[\d+:\d+\]),\s*(\S+)")
VALU_DST = re.compile(r"^\s*v_\w+\s+(?:v\[(\d+):(\d+)\]|v(\d+))")
FUNC = re.compile(r"^(_Z\w+):")


def instructions(lines):
    """(function, index, text) of every instruction (comments, directives and labels dropped)."""
    fn = None
    for i, raw in enumerate(lines):
        m = FUNC.match(raw)
        if m:
            fn = m.group(1)
            continue
        t = raw.split(";")[0].rstrip()
        s = t.strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        yield fn, i, s


def audit(text):
    ins = list(instructions(text.split("\n")))
    sites = []
    for k, (fn, i, s) in enumerate(ins[:-1]):
        m = STORE.match(s)
        if not m:
            continue
        soff = m.group(6)
        if not re.fullmatch(r"s\d+", soff):
            continue   # inline-constant soffset: LLVM inserts the wait state itself
        lo, hi = int(m.group(2)), int(m.group(3))
        nfn, j, nxt = ins[k + 1]
        d = VALU_DST.match(nxt)
        if not d or nfn != fn:
            continue
        dlo, dhi = (int(d.group(1)), int(d.group(2))) if d.group(1) else (int(d.group(3)), int(d.group(3)))
        if dlo <= hi and lo <= dhi:
            sites.append((fn, i + 1, s, nxt))
    return sites


if __name__ == "__main__":
    sites = audit(open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/rt_render.s").read())
    for fn, line, st, nxt in sites:
        print(f"{fn[:60]} line {line}: {st}  ->  {nxt}")
    print(f"{len(sites)} wide-store / VALU-overwrite hazard site(s)")
    sys.exit(1 if sites else 0)
