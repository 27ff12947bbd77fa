"""Static ISA check of the product's HIP kernels (CPU: hipcc cross-compiles).

The RS kernel issues its global loads/stores from inline asm with a scalar
base (saddr).  gfx9-family hardware needs 5 wait states between a VALU write
of an SGPR (v_readfirstlane, v_readlane, ...) and a VMEM instruction reading
that SGPR; the compiler's hazard recognizer inserts them for its own
instructions but not inside inline asm.  A stale base is an illegal address,
i.e. a GPU fault.  This test keeps every saddr fed by SMEM/SALU only.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "blockframe-rs_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _isa(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                    "-S", "-I", CSRC, "-o", str(out), src], check=True, capture_output=True)
    return out.read_text().split("\n")


def _sgpr_dest(line):
    """SGPRs an instruction writes through its first operand (s7 or s[6:7]), else ()."""
    m = re.match(r"\s*([sv]_\w+)\s+s(?:(\d+)|\[(\d+):(\d+)\])\s*,", line)
    if not m:
        return ()
    if m.group(2) is not None:
        return (int(m.group(2)),)
    return tuple(range(int(m.group(3)), int(m.group(4)) + 1))


def _hazards(lines, window=6):
    """(line, VALU writer, VMEM) triples where a VALU instruction's SGPR result is
    still the value a saddr VMEM instruction reads, fewer than `window`
    instructions later with no s_nop between (an SMEM/SALU rewrite of the
    register in between ends the hazard)."""
    hits = []
    for i, l in enumerate(lines):
        m = re.search(r"global_(load|store)_dwordx\d+ .*?, s\[(\d+):(\d+)\]", l)
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


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["rs_kernels.hip", "blake3_kernels.hip"])
def test_no_valu_sgpr_to_vmem_hazard(src, tmp_path):
    lines = _isa(os.path.join(CSRC, src), tmp_path)
    assert any("global_" in l for l in lines)
    assert _hazards(lines) == []


def test_hazard_detector_flags_the_pattern():
    bad = ["\tv_readfirstlane_b32 s15, v33", "\tv_readfirstlane_b32 s14, v32",
           "\t;;#ASMSTART", "\tglobal_load_dwordx4 v[36:39], v40, s[14:15]"]
    assert len(_hazards(bad)) == 2
    ok = ["\ts_load_dwordx2 s[14:15], s[6:7], 0x0", "\ts_waitcnt lgkmcnt(0)",
          "\tglobal_load_dwordx4 v[36:39], v40, s[14:15]"]
    assert _hazards(ok) == []
    # the VALU result is only an SMEM address; the load overwrites the pair
    dead = ["\tv_readfirstlane_b32 s14, v36", "\tv_readfirstlane_b32 s15, v37",
            "\ts_load_dwordx2 s[14:15], s[14:15], 0x410", "\ts_waitcnt lgkmcnt(0)",
            "\tglobal_load_dwordx4 v[6:9], v38, s[14:15]"]
    assert _hazards(dead) == []


def _inflight():
    import importlib.util
    spec = importlib.util.spec_from_file_location("inflight_check",
                                                  os.path.join(ROOT, "tools", "inflight_check.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_copy_of_inflight_asm_load_registers(tmp_path):
    """The RS kernels' loads are inline asm waited for by a separate
    `s_waitcnt vmcnt` asm; a compiler copy, spill or address use of a
    destination register before its wait reads a stale value (a live-range
    split at a control-flow merge did exactly that in a first version of the
    streamed kernel, and a probe built the same way faulted the GPU).
    The traffic-only probe (variant 44) is checked too: a probe that faults
    costs a GPU box all the same."""
    ic = _inflight()
    src = "\n".join(_isa(os.path.join(CSRC, "rs_kernels.hip"), tmp_path))
    checked = 0
    for name, body in ic.kernels(src):
        checked += 1
        assert ic.check(body) == [], name
    assert checked >= 7  # ring kernel x 7 read orders / probe, tail kernel


def test_inflight_checker_flags_a_copy():
    ic = _inflight()
    body = ["\t;;#ASMSTART", "\tglobal_load_dwordx4 v[10:13], v2, s[4:5]", "\t;;#ASMEND",
            "\tv_mov_b64_e32 v[20:21], v[10:11]",
            "\t;;#ASMSTART", "\ts_waitcnt vmcnt(0)", "\t;;#ASMEND",
            "\tv_mov_b64_e32 v[22:23], v[12:13]", "\ts_endpgm"]
    assert [t for _, t in ic.check(body)] == ["v_mov_b64_e32 v[20:21], v[10:11]"]
    reuse = ["\t;;#ASMSTART", "\tglobal_load_dwordx4 v[10:13], v2, s[4:5]", "\t;;#ASMEND",
             "\tglobal_load_dwordx4 v[30:33], v11, s[4:5]", "\ts_endpgm"]
    assert len(ic.check(reuse)) == 1
