"""Static audit of s_waitcnt vmcnt coverage in a kernel's ISA (dev tool, CPU only).

For every vector-memory load of the kernel (buffer_/global_/flat_/scratch_load*), walks the
fall-through instruction stream to the first instruction that reads or overwrites one of the
load's destination VGPRs and checks that an `s_waitcnt vmcnt(k)` with k <= (vector-memory
operations issued after the load) lies in between -- i.e. that the hardware has returned the
loaded data before it is used.  Branch targets are followed too (depth-limited), so a use
reached through a jump is checked against the waits on that path.  Written to settle whether
the round-2 "stale path-state reads" could be a missing wait in the code the compiler emits
(DESIGN.md §4).  usage: python tools/waitcnt_audit.py /tmp/rt_render.s [kernel-substring]
"""
import re
import sys

VMEM = re.compile(r"^\s*(buffer|global|flat|scratch)_(load|store|atomic)\w*")
LOAD = re.compile(r"^\s*(buffer|global|flat|scratch)_load\w*\s+(v\[(\d+):(\d+)\]|v(\d+))")
WAIT = re.compile(r"s_waitcnt\s+(.*)")
VREG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.LBB[\w_]+):")
SMOV_CONST = re.compile(r"^\s*s_mov_b64\s+(s\[\d+:\d+\]),\s*(-1|0)\s*$")
SDEF = re.compile(r"^\s*s_\w+\s+(s\[\d+:\d+\]|s\d+|vcc)\b")
VCC_FROM = re.compile(r"^\s*s_(and|andn2)_b64\s+vcc,\s*exec,\s*(s\[\d+:\d+\])\s*$")
BRANCH = re.compile(r"^\s*s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)")


def regs(text):
    out = set()
    for a, b, c in VREG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = end = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\w*render_kernel\w*:", l) and sub in l:
            start = i
        elif start is not None and l.strip().startswith("s_endpgm"):
            end = i
            break
    body = []
    for l in lines[start:end + 1]:
        l = l.split(";")[0].rstrip()
        if l.strip():
            body.append(l)
    return body


def audit(body, max_depth=6):
    labels = {LABEL.match(l).group(1): i for i, l in enumerate(body) if LABEL.match(l)}
    problems, checked = [], 0

    # Known SGPR-pair flags along a path: the compiler lowers some if/else chains to a flag set with
    # s_mov_b64 s[a:b], -1 / 0 and a later "s_andn2_b64 vcc, exec, s[a:b]; s_cbranch_vccnz" -- a
    # branch whose outcome that flag decides.  Following only the feasible side keeps the audit from
    # reporting paths the hardware cannot take (e.g. skipping both the fp32 and the fp64 image store).
    def walk(i, dst, n_after, depth, seen, flags=None, vcc=None):
        flags = dict(flags or {})
        while i < len(body):
            l = body[i]
            key = (i, n_after, tuple(sorted(flags.items())), vcc)
            if key in seen:
                return
            seen.add(key)
            mc = SMOV_CONST.match(l)
            vf = VCC_FROM.match(l)
            if mc:
                flags[mc.group(1)] = int(mc.group(2))
            elif vf:
                f = flags.get(vf.group(2))
                # vcc = exec & s (and) or exec & ~s (andn2); exec is non-zero on a live path
                vcc = None if f is None else ((f != 0) if vf.group(1) == "and" else (f == 0))
            else:
                d = SDEF.match(l)
                if d and not l.lstrip().startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop")):
                    if d.group(1) == "vcc":
                        vcc = None
                    flags.pop(d.group(1), None)
            w = WAIT.search(l)
            if w:
                m = re.search(r"vmcnt\((\d+)\)", w.group(1))
                if m and int(m.group(1)) <= n_after:
                    return   # covered on this path
            if LABEL.match(l):
                i += 1
                continue
            op = l.split()[0]
            operands = l[len(l) - len(l.lstrip()) + len(op):]
            lm = LOAD.match(l)
            if lm:   # a later load into the same registers: vector-memory loads return in order, so
                     # it lands after this one and the earlier value is dead (a legal WAW)
                ldst = set(range(int(lm.group(3)), int(lm.group(4)) + 1)) if lm.group(3) else {int(lm.group(5))}
                addr = regs(operands.split(",", 1)[1]) if "," in operands else set()
                if ldst & dst and not (addr & dst):
                    return
            if dst & regs(operands) and not op.startswith("s_"):
                problems.append((i, l.strip(), n_after))
                return
            if VMEM.match(l):
                n_after += 1
            b = BRANCH.match(l)
            if b and b.group(1) in ("cbranch_vccnz", "cbranch_vccz") and vcc is not None:
                taken = vcc if b.group(1) == "cbranch_vccnz" else not vcc
                if taken:
                    if b.group(2) not in labels:
                        return
                    i = labels[b.group(2)] + 1
                    continue
                i += 1
                continue
            if b and depth < max_depth and b.group(2) in labels:
                walk(labels[b.group(2)] + 1, dst, n_after, depth + 1, seen, flags, vcc)
                if b.group(1) == "branch":
                    return
            if op == "s_endpgm":
                return
            i += 1

    for i, l in enumerate(body):
        m = LOAD.match(l)
        if not m:
            continue
        checked += 1
        dst = set(range(int(m.group(3)), int(m.group(4)) + 1)) if m.group(3) else {int(m.group(5))}
        walk(i + 1, dst, 0, 0, set())
    return checked, problems


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/rt_render.s"
    sub = sys.argv[2] if len(sys.argv) > 2 else "ILi4ELb0ELb0ELi8E"
    body = kernel_lines(path, sub)
    n, probs = audit(body)
    print(f"{sub}: {len(body)} instructions, {n} vector-memory loads checked, {len(probs)} uses without a covering vmcnt")
    sys.exit(1 if probs else 0)
    for i, l, k in probs[:20]:
        print(f"  line {i}: {l}   ({k} vmem ops issued after the load)")
