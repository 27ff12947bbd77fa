"""Static check: no instruction touches a VGPR whose inline-asm load is in flight.

The RS kernels issue their global loads from inline asm and wait for them
with a separate `s_waitcnt vmcnt(N)` asm (tools/../rs_kernels.hip).  The
compiler cannot see that an asm output register is written asynchronously:
if register allocation copies such a register (v_mov), reuses it, or spills
it before the wait, the kernel computes on garbage or -- when the register
is reused as an address -- faults the GPU.  This walks the control-flow
graph of every kernel in a gfx950 assembly listing, tracks the vector-memory
counter (every VMEM instruction counts; `s_waitcnt vmcnt(N)` retires all but
the newest N, in order), and reports copies / spills of a register of a
still-outstanding asm load and its use as a memory address or store source.

usage: python tools/inflight_check.py listing.s [kernel-substring]
"""
import re
import sys

VMEM = re.compile(r"^(global|buffer|scratch|flat)_\w+")
LABEL = re.compile(r"^(\.LBB\w+|_Z\w+):")
# Flagged: copies (register-allocator live-range splits) and spills of an
# in-flight register, and its use as a VMEM address or store source.  Plain
# arithmetic uses are not flagged: the analysis does not evaluate branch
# conditions, and the ring loops' CFG has paths that never execute on which
# the arithmetic would appear to read before its wait.
COPY = re.compile(r"^(v_mov_|v_accvgpr_|scratch_|v_cndmask)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
MAX_STATES = 64
MAX_VMCNT = 63  # the gfx9 counter saturates here: older ops are complete


def _vregs(text):
    regs = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            regs.add(int(m.group(3)))
        else:
            regs.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


def kernels(src):
    """(name, [lines]) per kernel function body."""
    lines = src.split("\n")
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\w+):", lines[i])
        if m and any(".type" in l and m.group(1) in l for l in lines[max(0, i - 6):i]):
            name = m.group(1)
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                j += 1
            yield name, lines[i + 1:j]
            i = j
        i += 1


def parse(body):
    """Instructions [(label_or_None, op, text, is_asm)], in order."""
    out, in_asm = [], False
    for raw in body:
        t = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if t == ";;#ASMSTART":
            in_asm = True
            continue
        if t == ";;#ASMEND":
            in_asm = False
            continue
        if not t:
            continue
        m = LABEL.match(t)
        if m:
            out.append((m.group(1), None, "", False))
            continue
        if t.startswith("."):
            continue
        op = t.split()[0]
        out.append((None, op, t, in_asm))
    return out


def check(body):
    ins = parse(body)
    labels = {lab: k for k, (lab, _, _, _) in enumerate(ins) if lab}
    # state: tuple of outstanding VMEM ops, oldest first; each = frozenset of
    # asm-load destination registers (empty for compiler-managed ops)
    seen, per_k = set(), {}
    work = [(0, ())]
    issues = set()
    while work:
        k, state = work.pop()
        while k < len(ins):
            key = (k, state)
            if key in seen:
                break
            seen.add(key)
            per_k[k] = per_k.get(k, 0) + 1
            if per_k[k] > MAX_STATES:
                issues.add((k, "analysis gave up: too many distinct counter states"))
                break
            lab, op, text, is_asm = ins[k]
            if lab:
                k += 1
                continue
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", text)
                if m:
                    n = int(m.group(1))
                    state = state[max(0, len(state) - n):]
                k += 1
                continue
            busy = set().union(*state) if state else set()
            if VMEM.match(op):
                ops = text.split(None, 1)[1] if " " in text else ""
                parts = [x.strip() for x in ops.split(",")]
                dst = _vregs(parts[0]) if "load" in op else set()
                srcs = set().union(*[_vregs(x) for x in (parts[1:] if "load" in op else parts)])
                if busy & srcs:  # an in-flight register as address / store data
                    issues.add((k, text))
                state = (state + ((frozenset(dst) if is_asm else frozenset()),))[-MAX_VMCNT:]
                k += 1
                continue
            if busy and COPY.match(op) and "_dpp" not in op and busy & _vregs(text):
                issues.add((k, text))
            if op in ("s_endpgm", "s_setpc_b64"):
                break
            if op == "s_branch":
                tgt = text.split()[1]
                k = labels.get(tgt, len(ins))
                continue
            if op.startswith("s_cbranch"):
                tgt = text.split()[1]
                if tgt in labels:
                    work.append((labels[tgt], state))
            k += 1
    return sorted(issues)


def main():
    src = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = 0
    for name, body in kernels(src):
        if pat not in name:
            continue
        issues = check(body)
        print(f"{name[:90]}: {len(issues)} in-flight register touches")
        for k, t in issues[:8]:
            print(f"    [{k}] {t}")
        bad += bool(issues)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
