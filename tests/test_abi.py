"""CPU: the C-ABI library loads, exports exactly what include/bfrs.h declares,
and its host-side planner reproduces the oracle (no GPU compute here)."""
import itertools
import json
import os
import re

import numpy as np
import pytest
import torch

from gfnp import apply_matrix

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bfrs.h")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bfrs_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree(bfrs):
    assert declared_symbols() == sorted(bfrs.EXPORTS)


def test_library_exports_every_declared_symbol(bfrs):
    lib = bfrs.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    # nothing but the C-ABI is exported
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", bfrs.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = sorted(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert exported == declared_symbols()


def test_library_links_hip_not_oracle(bfrs):
    import subprocess
    out = subprocess.run(["ldd", bfrs.LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip64" in out
    assert "oracle" not in out


def test_abi_version_and_strerror(bfrs):
    L = bfrs.lib()
    assert L.bfrs_abi_version() == 1
    assert L.bfrs_strerror(bfrs.E_NOT_ENOUGH_SHARDS) == b"not enough shards"
    assert L.bfrs_strerror(bfrs.E_NOT_FOUND) == b"not found"
    # every code the header declares has its own text
    codes = re.findall(r"\b(BFRS_E_[A-Z_]+)\s*=\s*(-\d+)", open(HEADER).read())
    assert len(codes) == 17
    for name, val in codes:
        assert L.bfrs_strerror(int(val)) != b"unknown error", name


PRODUCT_KERNELS = {
    # v76: the unrolled SDWA-addressed GF(2^8)-subfield kernel (read groups of 64 tiles)
    "void bfrs::(anonymous namespace)::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)",
    # v75 / v73: the looped subfield and general GF(2^16) rings
    "void bfrs::(anonymous namespace)::gf_apply_ring_kernel<6, false, 16u, 1, 1, 1, 1>(bfrs::KernArgs)",
    "void bfrs::(anonymous namespace)::gf_apply_ring_kernel<6, false, 16u, 1, 1, 1, 0>(bfrs::KernArgs)",
    "bfrs::(anonymous namespace)::gf_tail_kernel(bfrs::KernArgs)",
    # device BLAKE3 (the Merkle re-verify of the read/repair path)
    # (3 tree levels inside a group; kernel 2's levels of <= 64 parents by
    # quads -- the lanes-only kernel 2 is in libbfrs_ab.so)
    "void bfrs::(anonymous namespace)::blake3_group_kernel<3u, 0u>(bfrs::HashMsg const*, "
    "unsigned int, unsigned int*, unsigned int*, unsigned int*)",
    "void bfrs::(anonymous namespace)::blake3_reduce_kernel<64u>(bfrs::HashReduce const*, "
    "unsigned int const*, unsigned int*, unsigned int*, unsigned int*)",
}


def test_product_code_object_carries_only_product_kernels(bfrs):
    """The A/B variant zoo and the traffic-only probes are not in libbfrs.so
    (they live in the measurement build libbfrs_ab.so, make ab)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import code_objects
    product = os.path.join(ROOT, "blockframe-rs_amd", "libbfrs.so")
    assert set(code_objects.kernels(product)) == PRODUCT_KERNELS
    ab = os.path.join(ROOT, "blockframe-rs_amd", "libbfrs_ab.so")
    if os.path.exists(ab):  # the measurement build carries more, never fewer
        assert PRODUCT_KERNELS < set(code_objects.kernels(ab))


PRODUCT_KNOBS = ["BFRS_CODEC_SLOTS", "BFRS_CODEC_STAGING", "BFRS_HOST_COPY_BUDGET",
                 "BFRS_KERNEL_VARIANT", "BFRS_PLAN_CACHE", "BFRS_PREFETCH_DEPTH"]


def _knob_strings(path):
    data = open(path, "rb").read()
    return sorted({m.decode() for m in re.findall(rb"BFRS_[A-Z0-9_]+", data)
                   if not m.startswith(b"BFRS_E_")})


def test_product_reads_only_the_documented_knobs():
    """libbfrs.so has one soak-proven configuration.  The
    only environment names in its binary are the six knobs include/bfrs.h
    documents; the concluded A/B knobs (knobs.hpp) live in libbfrs_ab.so."""
    product = os.path.join(ROOT, "blockframe-rs_amd", "libbfrs.so")
    assert _knob_strings(product) == PRODUCT_KNOBS
    doc = open(HEADER).read().split("#ifndef BFRS_H")[0]
    documented = sorted(set(re.findall(r"^ \*   (BFRS_[A-Z0-9_]+)", doc, flags=re.M)))
    assert documented == PRODUCT_KNOBS
    ab = os.path.join(ROOT, "blockframe-rs_amd", "libbfrs_ab.so")
    if os.path.exists(ab):
        assert set(PRODUCT_KNOBS) < set(_knob_strings(ab))


@pytest.mark.parametrize("value", ["44", "58", "77", "74", "abc", "76x", "-1"])
def test_unknown_kernel_variant_is_refused(bfrs, monkeypatch, value):
    """A stray BFRS_KERNEL_VARIANT never silently changes the product's kernel:
    anything but 76 / 75 / 73 fails bfrs_open with an error naming it."""
    if os.environ.get("BFRS_LIB", "libbfrs.so") != "libbfrs.so":
        pytest.skip("checks the product library")
    monkeypatch.setenv("BFRS_KERNEL_VARIANT", value)
    monkeypatch.setenv("BFRS_ALLOW_PROBE", "1")
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.Context(0)
    assert e.value.code == bfrs.E_INVALID_ARGUMENT
    assert "not built into this library" in str(e.value)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
@pytest.mark.parametrize("value", ["76", "75", "73", ""])
def test_product_kernel_variants_pass_the_check(bfrs, monkeypatch, value):
    monkeypatch.setenv("BFRS_KERNEL_VARIANT", value)
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.Context(0)
    assert e.value.code == bfrs.E_NO_DEVICE


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
def test_open_without_device_fails_loudly(bfrs):
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.Context(0)
    assert e.value.code == bfrs.E_NO_DEVICE


def test_default_rate_matches_oracle(bfrs, oracle):
    for k in range(1, 70):
        for m in (1, 2, 3, 4, 5, 8, 17):
            assert bfrs.use_high_rate(k, m) == oracle.use_high_rate(k, m), (k, m)


@pytest.mark.parametrize("k,m", [(30, 3), (8, 3), (20, 3), (1, 3), (2, 3), (3, 3), (4, 3),
                                 (16, 4), (10, 1), (65, 5)])
def test_encode_coefficients_match_oracle(bfrs, oracle, k, m):
    for i in range(k):
        unit = [np.zeros(64, np.uint8) for _ in range(k)]
        unit[i][0] = 1
        rec = oracle.encode(unit, m)
        for j in range(m):
            sym = int(rec[j][0]) | int(rec[j][32]) << 8
            assert bfrs.encode_coefficient(k, m, j, i) == sym, (j, i)


def test_planner_decode_matrices_reproduce_oracle(bfrs, gf_tables):
    """Applying bfrs_plan_decode's matrix (numpy, test-only) to the golden
    inputs gives the oracle's restored bytes, including the decodes whose
    recovery input was deliberately corrupted (pins the exact linear map)."""
    exp, log = gf_tables
    g = json.load(open(os.path.join(GOLDEN, "rs_small.json")))
    checked = 0
    for c in g["cases"]:
        k, m, n = c["k"], c["m"], c["shard_bytes"]
        if n % 64:
            continue
        orig = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in c["originals"]]
        for d in c["decodes"]:
            rec = [None if h is None else np.frombuffer(bytes.fromhex(h), np.uint8)
                   for h in d["recovery_used"]]
            op = [i not in d["erased"] for i in range(k)]
            rp = [r is not None for r in rec]
            mat = bfrs.plan_decode(k, m, op, rp)
            inputs = [r for r in rec if r is not None] + [orig[i] for i in range(k) if op[i]]
            outs = apply_matrix(mat, inputs, exp, log)
            missing = [i for i in range(k) if not op[i]]
            for i, a in zip(missing, outs):
                assert a.tobytes().hex() == d["restored"][str(i)], (k, m, d["erased"])
            checked += 1
    assert checked >= 30


@pytest.mark.parametrize("k,m", [(3, 5), (7, 5), (5, 9)])
def test_planner_lowrate_padding_round_trip(bfrs, oracle, gf_tables, k, m):
    """bfrs_plan_decode for LowRate shapes with zero-padded originals restores
    every pattern of m erasures (the pad is a known zero, not an erasure)."""
    exp, log = gf_tables
    rng = np.random.default_rng(k + 16 * m)
    data = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(k)]
    par = oracle.encode(data, m)
    for er in itertools.islice(itertools.combinations(range(k + m), m), 0, 25):
        op = [i not in er for i in range(k)]
        rp = [(k + j) not in er for j in range(m)]
        if all(op):
            continue
        mat = bfrs.plan_decode(k, m, op, rp)
        inputs = [par[j] for j in range(m) if rp[j]] + [data[i] for i in range(k) if op[i]]
        outs = apply_matrix(mat, inputs, exp, log)
        for i, a in zip([i for i in range(k) if not op[i]], outs):
            assert np.array_equal(a, data[i]), (k, m, er, i)


def test_archive_entry_points_reject_null_arguments(bfrs):
    """The pipeline entry points fail with BFRS_E_INVALID_ARGUMENT, never crash,
    on NULL handles/pointers (checked before any device work)."""
    import ctypes
    L = bfrs.lib()
    E = bfrs.E_INVALID_ARGUMENT
    buf = ctypes.create_string_buffer(256)
    rep = bfrs.RepairReport()
    out = ctypes.c_void_p()
    n = ctypes.c_size_t()
    assert L.bfrs_commit(None, b"/x", b"/y", 0, 0, buf, 256) == E
    assert L.bfrs_repair(None, b"/x", ctypes.byref(rep)) == E
    assert L.bfrs_health_check(None, b"/x", buf, 256, ctypes.byref(n)) == E
    assert L.bfrs_archive_open(None, b"/x", 4, 0, ctypes.byref(out)) == E
    assert L.bfrs_archive_size(None, None) == E
    assert L.bfrs_archive_read(None, 0, 0, None, ctypes.byref(n)) == E
    assert L.bfrs_archive_stats_get(None, None) == E
    assert L.bfrs_blake3_batch_dev(None, 1, None, None, None, None, None, None) == E
    assert L.bfrs_blake3_combine(None, 2, buf) == E
    assert L.bfrs_blake3_hex(None, 5, 1, buf) == E
    assert L.bfrs_merkle_root_hex(None, 1, buf) == E
    assert L.bfrs_manifest_check(None, 0, None, None, 0, None) == E
    L.bfrs_archive_close(None)  # no-op


def test_shard_pitch_layout_hint(bfrs):
    """bfrs_shard_pitch: small shards round to 256 B; >= 1 MiB shards get a
    pitch = 12 KiB (mod 64 KiB), never below the shard size."""
    assert bfrs.shard_pitch(0) == 0
    assert bfrs.shard_pitch(1) == 256
    assert bfrs.shard_pitch(8 << 10) == 8 << 10
    assert bfrs.shard_pitch(32 << 20) == (32 << 20) + 12288
    for s in [1 << 20, (1 << 20) + 1, 33554368, 25_000_000, 10**9 // 30]:
        p = bfrs.shard_pitch(s)
        assert s <= p < s + 65536 + 4096 and p % 65536 == 12288, (s, p)
    t = bfrs.empty_shards(3, 1 << 20, device="cpu")
    assert t.shape == (3, 1 << 20) and t.stride() == (bfrs.shard_pitch(1 << 20), 1)


def test_planner_random_shapes_match_oracle(bfrs, oracle, gf_tables):
    """Property check over random (k, m, erasure pattern, corrupted recovery):
    the planner's decode matrix (bfrs_plan_decode) applied on the CPU gives
    exactly the oracle decoder's bytes, and the planner's encode coefficients
    give the oracle's parity.  Covers both rates, padded LowRate shapes and
    multi-pass sizes (k > 64) that the fixed cases do not."""
    exp, log = gf_tables
    rng = np.random.default_rng(0xA11)
    shapes = [(int(rng.integers(1, 48)), int(rng.integers(1, 9))) for _ in range(24)]
    shapes += [(70, 3), (3, 6), (5, 9), (12, 12)]
    checked = 0
    for k, m in shapes:
        if not oracle.lib().oracle_supported(k, m):
            continue
        data = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(k)]
        par = oracle.encode(data, m)
        coef = [[bfrs.encode_coefficient(k, m, j, i) for i in range(k)] for j in range(m)]
        assert [a.tobytes() for a in apply_matrix(coef, data, exp, log)] == [p.tobytes() for p in par]
        for _ in range(3):
            e = int(rng.integers(1, min(k, m) + 1))
            lost = sorted(rng.choice(k + m, size=e, replace=False).tolist())
            op = [i not in lost for i in range(k)]
            rp = [(k + j) not in lost for j in range(m)]
            if all(op):
                continue
            rec = [par[j].copy() if rp[j] else None for j in range(m)]
            if any(rp) and rng.random() < 0.5:  # inconsistent input: pins the exact linear map
                j = next(j for j in range(m) if rp[j])
                rec[j][::3] ^= 0x77
            want = oracle.decode([data[i] if op[i] else None for i in range(k)], rec)
            mat = bfrs.plan_decode(k, m, op, rp)
            inputs = [rec[j] for j in range(m) if rp[j]] + [data[i] for i in range(k) if op[i]]
            got = apply_matrix(mat, inputs, exp, log)
            missing = [i for i in range(k) if not op[i]]
            for i, a in zip(missing, got):
                assert np.array_equal(a, want[i]), (k, m, lost, i)
            checked += 1
    assert checked >= 40


def test_binding_rejects_short_or_read_only_host_buffers():
    """The host-batch calls pass bare pointers: the Python binding refuses
    buffers shorter than shard_bytes and read-only outputs before any call."""
    import numpy as np
    import torch
    import bfrs
    chk = bfrs.Context._check_host_bufs
    ok = np.zeros(128, np.uint8)
    chk([ok, None, torch.zeros(128, dtype=torch.uint8)], 128, True, "t")
    with pytest.raises(ValueError, match="< shard_bytes"):
        chk([np.zeros(64, np.uint8)], 128, False, "t")
    with pytest.raises(ValueError, match="read-only"):
        chk([np.frombuffer(bytes(128), np.uint8)], 128, True, "t")
    with pytest.raises(ValueError, match="read-only"):
        chk([bytes(128)], 128, True, "t")
    chk([bytes(128)], 128, False, "t")  # inputs may be read-only
    with pytest.raises(ValueError, match="contiguous"):
        chk([torch.zeros(256, dtype=torch.uint8)[::2]], 128, False, "t")
    with pytest.raises(ValueError, match="read-only"):
        bfrs._out_nbytes(np.frombuffer(bytes(8), np.uint8))
