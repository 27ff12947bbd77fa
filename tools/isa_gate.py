"""Build gate: ISA hazard checks of the freshly built HIP kernels.

Run by blockframe-rs_amd/csrc/Makefile (and so by __graft_entry__.build())
on the gfx950 assembly listings of rs_kernels.hip and blake3_kernels.hip; a
finding fails the build, so a kernel that reaches the GPU box is always one
the checks accepted.  Two checks:

* in-flight asm-load registers (tools/inflight_check.py): no copy, spill,
  address or store-data use of a register whose inline-asm load has not been
  waited for (the round-1 GPU fault);
* VALU-written SGPR -> saddr VMEM within 5 wait states with no s_nop: the
  compiler's hazard recognizer does not look inside inline asm, and a stale
  base is an illegal address.

usage: python tools/isa_gate.py listing.s [listing.s ...]   (exit 1 on findings)
"""
import importlib.util
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _inflight():
    spec = importlib.util.spec_from_file_location("inflight_check",
                                                  os.path.join(HERE, "inflight_check.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _sgpr_dest(line):
    """SGPRs an instruction writes through its first operand (s7 or s[6:7]), else ()."""
    m = re.match(r"\s*([sv]_\w+)\s+s(?:(\d+)|\[(\d+):(\d+)\])\s*,", line)
    if not m:
        return ()
    if m.group(2) is not None:
        return (int(m.group(2)),)
    return tuple(range(int(m.group(3)), int(m.group(4)) + 1))


def sgpr_hazards(lines, window=6):
    """(line, VALU writer, VMEM) triples where a VALU instruction's SGPR result is
    still the value a saddr VMEM instruction reads, fewer than `window`
    instructions later with no s_nop between (an SMEM/SALU rewrite of the
    register in between ends the hazard)."""
    hits = []
    for i, l in enumerate(lines):
        m = re.search(r"global_(load|store)\w* .*?, s\[(\d+):(\d+)\]", l)
        if not m:
            continue
        lo, hi = int(m.group(2)), int(m.group(3))
        prev = [x for x in lines[max(0, i - 3 * window):i]
                if x.strip() and not x.strip().startswith((";", "."))][-window:]
        if any("s_nop" in x for x in prev):
            continue
        for r in range(lo, hi + 1):
            for w in reversed(prev):  # the most recent writer of s<r> decides
                if r in _sgpr_dest(w):
                    if w.strip().startswith("v_"):
                        hits.append((i, w.strip(), l.strip()))
                    break
    return hits


def gate(text):
    """Findings [(kernel, where, what)] of one listing."""
    ic = _inflight()
    out = []
    for name, body in ic.kernels(text):
        for k, t in ic.check(body):
            out.append((name, k, "in-flight asm-load register: " + t))
    for i, w, l in sgpr_hazards(text.split("\n")):
        out.append(("(listing)", i, f"VALU SGPR write '{w}' read by '{l}'"))
    return out


def main(paths):
    bad = 0
    for p in paths:
        findings = gate(open(p).read())
        for name, k, what in findings[:20]:
            print(f"ISA GATE {os.path.basename(p)}: {name[:80]} [{k}] {what}", file=sys.stderr)
        bad += len(findings)
    if bad:
        print(f"ISA GATE: {bad} finding(s); the kernels are not safe to run", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
