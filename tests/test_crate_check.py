"""CPU: tools/crate_check (the source-only Rust program that re-derives the
committed fixtures with reed-solomon-simd 3.1.0 wherever cargo exists) reads
exactly the fixture files and fields this repo commits, pins the crate
version BlockFrame links (reference Cargo.lock:1596-1605), calls the crate
API BlockFrame calls, and restates the KAT and the
synthetic workload bit for bit.  It cannot be compiled here (no Rust
toolchain), so these checks are textual plus a Python restatement of its
synthetic-bytes function."""
import json
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CC = os.path.join(ROOT, "tools", "crate_check")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _src():
    return open(os.path.join(CC, "src", "main.rs")).read()


def test_manifest_pins_the_reference_crate():
    toml = open(os.path.join(CC, "Cargo.toml")).read()
    assert re.search(r'^reed-solomon-simd = "=3\.1\.0"$', toml, re.M)
    assert "cffef0520d30fbd4151fb20e262947ae47fb0ab276a744a19b6398438105a072" in toml


def test_uses_the_crate_api_blockframe_calls():
    src = _src()
    for call in ("ReedSolomonEncoder::new(", ".add_original_shard(", ".encode()", ".recovery_iter()",
                 "ReedSolomonDecoder::new(", ".add_recovery_shard(", ".decode()",
                 ".restored_original("):
        assert call in src, call


def test_names_exactly_the_committed_fixture_files_and_fields():
    src = _src()
    files = set(re.findall(r'golden\("([a-z0-9_]+\.json)"\)', src))
    assert files == {"rs_small.json", "rs_r2.json", "rs_large.json"}
    for f in files:
        assert os.path.exists(os.path.join(GOLDEN, f)), f
    small = json.load(open(os.path.join(GOLDEN, "rs_small.json")))
    r2 = json.load(open(os.path.join(GOLDEN, "rs_r2.json")))
    large = json.load(open(os.path.join(GOLDEN, "rs_large.json")))
    case, dec = small["cases"][0], small["cases"][0]["decodes"][0]
    # every field the program indexes exists in the fixture it reads
    for key in re.findall(r'\bc\["([a-z_0-9]+)"\]', src) + re.findall(r'usize_of\(c, "([a-z_]+)"\)', src):
        assert key in case or key in r2["cases"][0], key
    for key in re.findall(r'\bd\["([a-z_]+)"\]', src):
        assert key in dec, key
    assert '["c2_128x32MiB"]' in src
    c2 = large["c2_128x32MiB"]
    for key in re.findall(r'\bg\["([a-z_0-9]+)"\]', src):
        assert key in c2 or key == "cases", key
    assert set(r2["cases"][0]["rates"]) == {"low", "high"}
    assert all(len(c["rates"]["low"]["recovery"]) == c["m"] for c in r2["cases"])


def test_kat_matches_survey_and_oracle(oracle):
    """The A.7 vector in the program = SURVEY.md Appendix A.7 = the oracle."""
    src = _src()
    hexes = re.findall(r'"([0-9a-f]{256})"', src)
    assert len(hexes) == 3
    survey = open(os.path.join(ROOT, "SURVEY.md")).read()
    for h in hexes:
        assert h in survey
    orig = [np.array([(i * 131 + b * 7 + 3) & 0xFF for b in range(128)], np.uint8) for i in range(30)]
    assert [r.tobytes().hex() for r in oracle.encode(orig, 3)] == hexes
    assert "af0a31fc6849a8c2d70bb02ba65bde41e81965a412e675ee1680d3c4516ccb12" in src


def test_synthetic_bytes_restated_exactly():
    """synth_segment in main.rs = blockframe-rs_amd/bfrs/synth.py."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
    from bfrs import synth
    src = _src()
    consts = {name: int(val.replace("_", ""), 16)
              for name, val in re.findall(r"const (G|M1|M2): u64 = 0x([0-9A-F_]+);", src)}
    assert consts == {"G": synth._G, "M1": synth._M1, "M2": synth._M2}
    assert "(seed << 44).wrapping_add(seg << 24)" in src

    def rust_restated(seed, seg, n):  # the Rust function, line by line
        mask = (1 << 64) - 1
        base = ((seed << 44) + (seg << 24)) & mask
        out = bytearray()
        for i in range((n + 7) // 8):
            z = ((base + i) * consts["G"]) & mask
            z = ((z ^ (z >> 30)) * consts["M1"]) & mask
            z = ((z ^ (z >> 27)) * consts["M2"]) & mask
            z ^= z >> 31
            out += z.to_bytes(8, "little")
        return bytes(out[:n])
    for seed, seg, n in ((0xB10C, 0, 4096), (0xB10C, 127, 1000), (1, 5, 77)):
        assert rust_restated(seed, seg, n) == synth.segment_np(seed, seg, n).tobytes()
