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


def _isa(src, tmp_path, defines=()):
    out = tmp_path / (os.path.basename(src) + "".join(defines) + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                    *[f"-D{d}" for d in defines], "-S", "-I", CSRC, "-o", str(out), src],
                   check=True, capture_output=True)
    return out.read_text().split("\n")


def _gate():
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_gate",
                                                  os.path.join(ROOT, "tools", "isa_gate.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _hazards(lines, window=6):
    return _gate().sgpr_hazards(lines, window)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,defines", [("rs_kernels.hip", ()),
                                         ("rs_kernels.hip", ("BFRS_AB_VARIANTS",)),
                                         ("blake3_kernels.hip", ())])
def test_no_valu_sgpr_to_vmem_hazard(src, defines, tmp_path):
    lines = _isa(os.path.join(CSRC, src), tmp_path, defines)
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
@pytest.mark.parametrize("defines,n_kernels", [((), 4), (("BFRS_AB_VARIANTS",), 20)])
def test_no_copy_of_inflight_asm_load_registers(tmp_path, defines, n_kernels):
    """The RS kernels' loads are inline asm waited for by a separate
    `s_waitcnt vmcnt` asm; a compiler copy, spill or address use of a
    destination register before its wait reads a stale value (a live-range
    split at a control-flow merge did exactly that in a first version of the
    streamed kernel, and a probe built the same way faulted the GPU).
    The product build carries 4 kernels (v76, the looped subfield and general
    rings, the tail kernel); the A/B build's variants and traffic-only probes
    are checked too: a probe that faults costs a GPU box all the same."""
    ic = _inflight()
    src = "\n".join(_isa(os.path.join(CSRC, "rs_kernels.hip"), tmp_path, defines))
    checked = 0
    for name, body in ic.kernels(src):
        checked += 1
        assert ic.check(body) == [], name
    if defines:
        assert checked >= n_kernels
    else:
        assert checked == n_kernels


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


BROKEN_KERNEL = r"""
#include <hip/hip_runtime.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void broken(const uint8_t *base, uint32_t *out) {
  u32x4 x;
  const uint32_t off = threadIdx.x * 16;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=&v"(x) : "v"(off), "s"(base) : "memory");
  uint32_t y;
  // uses a register of the load above as an address before any s_waitcnt
  asm volatile("global_load_dword %0, %1, %2" : "=&v"(y) : "v"(x.x), "s"(base) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(y), "+v"(x) :: "memory");
  out[threadIdx.x] = y + x.y;
}
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_build_gate_rejects_a_broken_kernel(tmp_path):
    """the gate build() runs (Makefile -> tools/isa_gate.py)
    fails on a kernel that uses an in-flight asm-load register as an address,
    and passes the product kernels."""
    import subprocess
    import sys
    src = tmp_path / "broken.hip"
    src.write_text(BROKEN_KERNEL)
    lst = tmp_path / "broken.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", str(src),
                    "-o", str(lst)], check=True, capture_output=True)
    gate = os.path.join(ROOT, "tools", "isa_gate.py")
    r = subprocess.run([sys.executable, gate, str(lst)], capture_output=True, text=True)
    assert r.returncode == 1 and "in-flight" in r.stderr, r.stderr
    ok = tmp_path / "blake3.s"
    ok.write_text("\n".join(_isa(os.path.join(CSRC, "blake3_kernels.hip"), tmp_path)))
    r = subprocess.run([sys.executable, gate, str(ok)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_makefile_runs_the_gate():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    assert "all: $(OUT) $(GATE)" in mk and "tools/isa_gate.py $(ISA)" in mk
