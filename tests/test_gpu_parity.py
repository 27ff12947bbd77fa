"""GPU parity: the HIP path through the C-ABI vs the oracle / golden fixtures.

Bit-exact for every byte (integer GF(2^16) work, no tolerance).  Small and
medium cases compare with the oracle directly; BASELINE config sizes compare
with committed SHA-256 digests (tests/golden/rs_large.json) and use
size-independent properties (encode -> erase -> decode round trip, BLAKE3 of
restored segments against the manifest-style hash of the original).
"""
import gc
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _small_cases():
    return json.load(open(os.path.join(GOLDEN, "rs_small.json")))["cases"]


def _np(h):
    return np.frombuffer(bytes.fromhex(h), np.uint8)


# ---------------------------------------------------------------- golden, host API
@pytest.mark.parametrize("case", _small_cases(), ids=lambda c: f"k{c['k']}m{c['m']}n{c['shard_bytes']}")
def test_host_encode_golden(ctx, case):
    orig = [_np(h) for h in case["originals"]]
    rec = ctx.encode(orig, case["m"])
    assert [r.tobytes().hex() for r in rec] == case["recovery"]


@pytest.mark.parametrize("case", _small_cases(), ids=lambda c: f"k{c['k']}m{c['m']}n{c['shard_bytes']}")
def test_host_decode_golden(ctx, case):
    k = case["k"]
    orig = [_np(h) for h in case["originals"]]
    for d in case["decodes"]:
        o = [None if i in d["erased"] else orig[i] for i in range(k)]
        r = [None if h is None else _np(h) for h in d["recovery_used"]]
        out = ctx.decode(o, r)
        assert {str(i): a.tobytes().hex() for i, a in out.items()} == d["restored"]


def test_r2_fixture_rate_invariant(ctx):
    """RS(3,3)/RS(4,3) (a 3- or 4-segment last tier-3 block): the product's
    parity equals the labelled LowRate AND HighRate fixture entries, which are
    identical (tests/test_oracle.py::test_rates_agree_in_the_default_rate_tie),
    and the 3-erasure decode restores the originals."""
    g = json.load(open(os.path.join(GOLDEN, "rs_r2.json")))
    for c in g["cases"]:
        orig = [_np(h) for h in c["originals"]]
        rec = [r.tobytes().hex() for r in ctx.encode(orig, c["m"])]
        assert rec == c["rates"]["low"]["recovery"] == c["rates"]["high"]["recovery"]
        o = [None if i in c["erased"] else orig[i] for i in range(c["k"])]
        out = ctx.decode(o, [_np(h) for h in rec])
        assert all(np.array_equal(out[i], orig[i]) for i in c["erased"])


# ---------------------------------------------------------------- device batch API vs oracle
def _dev_shards(arrs, dev="cuda"):
    return [torch.from_numpy(a.copy()).to(dev) for a in arrs]


@pytest.mark.parametrize("shard_bytes", [64, 8192, 1 << 20, (1 << 20) + 64 * 3, 65536 + 38])
def test_batch_encode_mixed_blocks_vs_oracle(ctx, oracle, shard_bytes):
    rng = np.random.default_rng(shard_bytes)
    ks = [30, 8, 1, 20, 2, 3]
    host = [[rng.integers(0, 256, shard_bytes, dtype=np.uint8) for _ in range(k)] for k in ks]
    d_orig = [t for blk in host for t in _dev_shards(blk)]
    d_rec = [torch.empty(shard_bytes, dtype=torch.uint8, device="cuda") for _ in range(3 * len(ks))]
    ctx.encode_batch_dev(ks, 3, shard_bytes, d_orig, d_rec)
    torch.cuda.synchronize()
    for b, blk in enumerate(host):
        want = oracle.encode(blk, 3)
        for j in range(3):
            got = d_rec[3 * b + j].cpu().numpy()
            assert np.array_equal(got, want[j]), (b, ks[b], j)


@pytest.mark.parametrize("byte", [0x00, 0xAB, 0xFF])
def test_constant_byte_segments_vs_oracle(ctx, oracle, byte):
    """SURVEY §8(d)'s constant-byte variant of the synthetic inputs
    (chunker/tests.rs:19-27 commits files of one repeated byte): RS(30,3) and
    RS(8,3) of constant segments at 1 MiB + 3 chunks, encode and a 3-erasure
    decode, against the oracle (a zero-skip or constant-folding shortcut in
    the kernel would show here)."""
    n = (1 << 20) + 64 * 3
    for k in (30, 8):
        segs = [np.full(n, byte, np.uint8) for _ in range(k)]
        want = oracle.encode(segs, 3)
        got = ctx.encode(segs, 3)
        assert all(np.array_equal(got[j], want[j]) for j in range(3)), (k, byte)
        er = [0, k // 2, k - 1]
        out = ctx.decode([None if i in er else segs[i] for i in range(k)], want)
        assert all(np.array_equal(out[i], segs[i]) for i in er), (k, byte)


def test_batch_decode_random_erasures_vs_oracle(ctx, oracle):
    rng = np.random.default_rng(7)
    n = 256 * 1024
    ks = [30, 30, 8, 20]
    host = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in ks]
    pars = [oracle.encode(blk, 3) for blk in host]
    d_orig, d_rec, d_out, erased = [], [], [], []
    for b, k in enumerate(ks):
        e = int(rng.integers(1, 4))
        # erase e data shards, and when e < 3 also drop a parity shard sometimes
        er = set(rng.choice(k, size=e, replace=False).tolist())
        drop_par = set() if e == 3 else {int(rng.integers(0, 3))}
        erased.append((er, drop_par))
        for i in range(k):
            d_orig.append(None if i in er else torch.from_numpy(host[b][i]).cuda())
            d_out.append(torch.empty(n, dtype=torch.uint8, device="cuda") if i in er else None)
        for j in range(3):
            d_rec.append(None if j in drop_par else torch.from_numpy(pars[b][j]).cuda())
    ctx.decode_batch_dev(ks, 3, n, d_orig, d_rec, d_out)
    torch.cuda.synchronize()
    off = 0
    for b, k in enumerate(ks):
        er, _ = erased[b]
        for i in range(k):
            if i in er:
                assert np.array_equal(d_out[off + i].cpu().numpy(), host[b][i]), (b, i)
        off += k


def test_every_k_1_to_30_one_batch(ctx, oracle):
    """One encode launch and one decode launch over 30 blocks with k = 1..30
    (every block shape BlockFrame's tier 3 can produce, odd k included: the
    unrotated padded passes), a ragged shard size, all against the oracle."""
    n = 3 * 8192 + 64 * 5 + 38
    ks = list(range(1, 31))
    rng = np.random.default_rng(130)
    host = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in ks]
    d_orig = [t for blk in host for t in _dev_shards(blk)]
    d_rec = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3 * len(ks))]
    ctx.encode_batch_dev(ks, 3, n, d_orig, d_rec)
    torch.cuda.synchronize()
    pars = []
    for b, blk in enumerate(host):
        want = oracle.encode(blk, 3)
        pars.append(want)
        for j in range(3):
            assert np.array_equal(d_rec[3 * b + j].cpu().numpy(), want[j]), (ks[b], j)
    dd_orig, d_out, erased = [], [], []
    for b, k in enumerate(ks):
        er = sorted(rng.choice(k, size=min(3, k), replace=False).tolist())
        erased.append(er)
        for i in range(k):
            dd_orig.append(None if i in er else d_orig[sum(ks[:b]) + i])
            d_out.append(torch.empty(n, dtype=torch.uint8, device="cuda") if i in er else None)
    ctx.decode_batch_dev(ks, 3, n, dd_orig, d_rec, d_out)
    torch.cuda.synchronize()
    off = 0
    for b, k in enumerate(ks):
        for i in erased[b]:
            assert np.array_equal(d_out[off + i].cpu().numpy(), host[b][i]), (k, i)
        off += k


def test_many_blocks_round_trip(ctx, oracle):
    """Enough blocks that every persistent workgroup of the phased/streamed
    kernels walks several super-tiles across passes with different tables
    (encode: k changes; decode: a different erasure pattern per block)."""
    n = 2 << 20
    ks = [30] * 10 + [8, 20, 4, 30, 12, 30, 6, 30]
    gen = torch.Generator(device="cuda").manual_seed(0xB10C)
    data = [torch.randint(0, 256, (k, n), dtype=torch.uint8, device="cuda", generator=gen) for k in ks]
    par = [torch.empty(3, n, dtype=torch.uint8, device="cuda") for _ in ks]
    ctx.encode_batch_dev(ks, 3, n, [d[i] for d in data for i in range(d.shape[0])],
                         [p[j] for p in par for j in range(3)])
    torch.cuda.synchronize()
    for b in (0, 10, 12, len(ks) - 1):  # parity vs the oracle on sampled blocks
        want = oracle.encode([data[b][i].cpu().numpy() for i in range(ks[b])], 3)
        for j in range(3):
            assert np.array_equal(par[b][j].cpu().numpy(), want[j]), (b, j)
    rng = np.random.default_rng(3)
    d_orig, d_out, erased = [], [], []
    for b, k in enumerate(ks):
        er = sorted(rng.choice(k, size=min(3, k), replace=False).tolist())
        erased.append(er)
        for i in range(k):
            d_orig.append(None if i in er else data[b][i])
            d_out.append(torch.empty(n, dtype=torch.uint8, device="cuda") if i in er else None)
    ctx.decode_batch_dev(ks, 3, n, d_orig, [p[j] for p in par for j in range(3)], d_out)
    torch.cuda.synchronize()
    off = 0
    for b, k in enumerate(ks):
        for i in erased[b]:
            assert torch.equal(d_out[off + i], data[b][i]), (b, i)
        off += k


def test_decode_inconsistent_input_matches_oracle(ctx, oracle):
    """Corrupted (non-codeword) input: restored bytes must equal the crate
    decoder's output, i.e. the same linear map, not just 'a' valid decode."""
    rng = np.random.default_rng(11)
    n = 4096
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    par = oracle.encode(data, 3)
    par[1] = par[1] ^ rng.integers(0, 256, n, dtype=np.uint8)
    o = [None if i in (4, 17) else data[i] for i in range(30)]
    want = oracle.decode(o, par)
    got = ctx.decode(o, par)
    for i in (4, 17):
        assert np.array_equal(got[i], want[i])


def test_large_code_multiphase(ctx, oracle):
    """k > 64 inputs (two accumulate phases) and m > 4 outputs (two output groups)."""
    rng = np.random.default_rng(5)
    for k, m, n in ((100, 6, 4096), (200, 3, 640)):
        d = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        want = oracle.encode(d, m)
        got = ctx.encode(d, m)
        assert all(np.array_equal(a, b) for a, b in zip(got, want)), (k, m)
        er = [1, 50, k - 1] + [2, 3, 4][: m - 3]
        o = [None if i in er else d[i] for i in range(k)]
        rest = ctx.decode(o, want)
        for i in er:
            assert np.array_equal(rest[i], d[i])


def test_device_path_limit_k1024(ctx, bfrs, oracle):
    """The device path's largest code (k = 1024, DESIGN §8: 16 accumulate
    phases of 64 inputs) against the oracle, and the documented refusal above it."""
    rng = np.random.default_rng(0x400)
    k, m, n = 1024, 3, 640
    d = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    want = oracle.encode(d, m, oracle.ENGINE_AVX2)
    got = ctx.encode(d, m)
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    er = [0, 511, 1023]
    o = [None if i in er else d[i] for i in range(k)]
    rest = ctx.decode(o, want)
    for i in er:
        assert np.array_equal(rest[i], d[i]), i
    with pytest.raises(bfrs.BfrsError) as e:
        ctx.encode(d + [d[0]], m)
    assert e.value.code == bfrs.E_UNSUPPORTED_SHARD_COUNT


def test_misaligned_device_pointer_rejected(ctx, bfrs):
    buf = torch.zeros(4096 + 16, dtype=torch.uint8, device="cuda")
    bad = buf.data_ptr() + 8
    outs = [torch.empty(4096, dtype=torch.uint8, device="cuda") for _ in range(3)]
    with pytest.raises(bfrs.BfrsError) as e:
        ctx.encode_batch_dev([1], 3, 4096, [bad], outs)
    assert e.value.code == bfrs.E_INVALID_ARGUMENT


# ---------------------------------------------------------------- host-memory batch (PCIe path)
@pytest.mark.parametrize("n", [64 * 150 + 38, (16 << 20) + 64 * 5 + 38])
def test_host_batch_pipeline_vs_oracle(ctx, oracle, n):
    """Streaming through HBM in 8 MiB column slabs must give the same bytes as
    one-shot: one slab with a folded tail chunk, and three slabs (two full,
    the third carrying 5 chunks plus the tail) rotating over the pipeline's
    streams.  (The slab width is fixed in libbfrs.so: round 4's sweep settled
    it)"""
    slab = n
    rng = np.random.default_rng(21)
    ks = [30, 8, 1, 20] if n < (1 << 20) else [30, 8, 1]
    host = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in ks]
    rec = [np.empty(n, np.uint8) for _ in range(3 * len(ks))]
    ctx.encode_host_batch(ks, 3, n, [a for blk in host for a in blk], rec)
    big = n > (1 << 20) and oracle.lib().oracle_have_avx2()  # the AVX2 engine for 16 MiB shards
    want = [oracle.encode(blk, 3, oracle.ENGINE_AVX2 if big else oracle.ENGINE_SCALAR)
            for blk in host]
    for b in range(len(ks)):
        for j in range(3):
            assert np.array_equal(rec[3 * b + j], want[b][j]), (slab, b, j)
    orig, out, er_all = [], [], []
    for b, k in enumerate(ks):
        er = set(range(min(3, k)))
        er_all.append(er)
        for i in range(k):
            orig.append(None if i in er else host[b][i])
            out.append(np.empty(n, np.uint8) if i in er else None)
    ctx.decode_host_batch(ks, 3, n, orig, rec, out)
    oi = 0
    for b, k in enumerate(ks):
        for i in er_all[b]:
            assert np.array_equal(out[oi + i], host[b][i]), (slab, b, i)
        oi += k


# ---------------------------------------------------------------- crate-API mirror
def test_streaming_encoder_decoder(ctx, bfrs, oracle):
    rng = np.random.default_rng(2)
    n = 64 * 100
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    enc = bfrs.ReedSolomonEncoder(ctx, 30, 3, n)
    for d in data:
        enc.add_original_shard(d)
    rec = list(enc.encode().recovery_iter())
    assert rec == [r.tobytes() for r in oracle.encode(data, 3)]
    assert [enc.recovery_view(j).tobytes() for j in range(3)] == rec
    with pytest.raises(bfrs.BfrsError) as e:
        enc.add_original_shard(data[0][:64])
    assert e.value.code == bfrs.E_DIFFERENT_SHARD_SIZE

    dec = bfrs.ReedSolomonDecoder(ctx, 30, 3, n)
    for i in range(30):
        if i not in (0, 9, 29):
            dec.add_original_shard(i, data[i])
    for j in range(3):
        dec.add_recovery_shard(j, rec[j])
    with pytest.raises(bfrs.BfrsError) as e:
        dec.add_recovery_shard(0, rec[0])
    assert e.value.code == bfrs.E_DUPLICATE_RECOVERY_SHARD_INDEX
    dec.decode()
    for i in (0, 9, 29):
        assert dec.restored_original(i) == data[i].tobytes()
    assert dec.restored_original(1) is None  # crate: Option::None for present shards


def test_codec_objects_share_one_context_across_threads(ctx, bfrs, oracle):
    """rayon workers share ONE context per device.  Encoders
    and decoders created concurrently on it (pooled codec slots, each with its
    own stream; plan cache under the context lock) give the oracle's bytes."""
    import threading
    rng = np.random.default_rng(11)
    n = 64 * 512 + 64
    blocks = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in (30, 8, 20, 30)]
    want = [[r.tobytes() for r in oracle.encode(b, 3)] for b in blocks]
    errors = []

    def worker(w):
        try:
            for rep in range(3):
                b = (w + rep) % len(blocks)
                data = blocks[b]
                enc = bfrs.ReedSolomonEncoder(ctx, len(data), 3, n)
                for d in data:
                    enc.add_original_shard(d)
                rec = list(enc.encode().recovery_iter())
                assert rec == want[b], (w, rep, b)
                del enc
                dec = bfrs.ReedSolomonDecoder(ctx, len(data), 3, n)
                lost = {(w + rep) % len(data), (w + rep + 1) % len(data)}
                for i, d in enumerate(data):
                    if i not in lost:
                        dec.add_original_shard(i, d)
                for j in range(3):
                    dec.add_recovery_shard(j, rec[j])
                dec.decode()
                for i in lost:
                    assert dec.restored_original(i) == data[i].tobytes(), (w, rep, i)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors


@pytest.mark.parametrize("staging", ["direct", "pinned"])
@pytest.mark.parametrize("slots", ["0", "1", "4"])
def test_codec_staging_slots_and_lifetimes(bfrs, oracle, monkeypatch, staging, slots):
    """Both staging modes of add_*_shard (BFRS_CODEC_STAGING) and any idle-slot
    count (BFRS_CODEC_SLOTS=0 keeps none: ADVICE r2) give the oracle's bytes
    through the objects and the wrappers; the caller's buffer is reusable as
    soon as add returns; objects outlive bfrs_close and are freed safely."""
    monkeypatch.setenv("BFRS_CODEC_STAGING", staging)
    monkeypatch.setenv("BFRS_CODEC_SLOTS", slots)
    c = bfrs.Context(0)
    rng = np.random.default_rng(21)
    n = 64 * 4096 + 64 * 3  # ragged against the 8 KiB tile
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    want = [r.tobytes() for r in oracle.encode(data, 3)]
    for rep in range(2):
        enc = bfrs.ReedSolomonEncoder(c, 30, 3, n)
        buf = np.empty(n, np.uint8)
        for d in data:
            buf[:] = d
            enc.add_original_shard(buf)  # the same buffer every time
        assert list(enc.encode().recovery_iter()) == want, rep
        del enc
    outs = [np.empty(n, np.uint8) for _ in range(3)]
    assert bfrs.Chunker(c).generate_parity_into(data, 30, 3, outs) == n
    assert [o.tobytes() for o in outs] == want
    par = [np.frombuffer(p, np.uint8) for p in want]
    slots_ = [None if i in (2, 17, 29) else data[i] for i in range(30)]
    for t in (2, 17, 29):
        assert bfrs.recover_segment_rs30_3(c, slots_, par, t) == data[t].tobytes()
    dec = bfrs.ReedSolomonDecoder(c, 30, 3, n)
    for i in range(30):
        if slots_[i] is not None:
            dec.add_original_shard(i, slots_[i])
    for j in range(3):
        dec.add_recovery_shard(j, par[j])
    dec.decode()
    assert dec.restored_view(17).tobytes() == data[17].tobytes()
    assert dec.restored_original(2) == data[2].tobytes()
    assert dec.restored_view(0) is None
    # a view outlives the Python name of its object: the encoder
    # stays alive through the view, so its slot is neither reused by the next
    # encoder nor freed (BFRS_CODEC_SLOTS=0), and the bytes stay the parity
    enc = bfrs.ReedSolomonEncoder(c, 30, 3, n)
    for d in data:
        enc.add_original_shard(d)
    view = enc.encode().recovery_view(1)
    rview = dec.restored_view(29)
    del enc
    gc.collect()
    other = bfrs.ReedSolomonEncoder(c, 30, 3, n)
    for d in data:
        other.add_original_shard(255 - d)
    other.encode()
    assert view.tobytes() == want[1] and rview.tobytes() == data[29].tobytes()
    del other, view, rview
    gc.collect()
    keep = bfrs.ReedSolomonEncoder(c, 8, 3, n)
    c.close()  # objects still alive: freeing them later is safe
    with pytest.raises(bfrs.BfrsError):
        keep.add_original_shard(data[0])  # but no other call on a closed context
    del dec, keep


def test_codec_argument_errors(ctx, bfrs):
    E = bfrs.BfrsError
    for args, code in (((30, 3, 0), bfrs.E_INVALID_SHARD_SIZE), ((30, 3, 63), bfrs.E_INVALID_SHARD_SIZE),
                       ((0, 3, 64), bfrs.E_UNSUPPORTED_SHARD_COUNT)):
        with pytest.raises(E) as e:
            bfrs.ReedSolomonEncoder(ctx, *args)
        assert e.value.code == code
    enc = bfrs.ReedSolomonEncoder(ctx, 2, 3, 64)
    enc.add_original_shard(np.zeros(64, np.uint8))
    with pytest.raises(E) as e:
        enc.encode()
    assert e.value.code == bfrs.E_TOO_FEW_ORIGINAL_SHARDS
    enc.add_original_shard(np.zeros(64, np.uint8))
    with pytest.raises(E) as e:
        enc.add_original_shard(np.zeros(64, np.uint8))
    assert e.value.code == bfrs.E_TOO_MANY_ORIGINAL_SHARDS
    dec = bfrs.ReedSolomonDecoder(ctx, 30, 3, 64)
    with pytest.raises(E) as e:
        dec.add_original_shard(30, np.zeros(64, np.uint8))
    assert e.value.code == bfrs.E_INVALID_ORIGINAL_SHARD_INDEX
    with pytest.raises(E) as e:
        dec.add_recovery_shard(3, np.zeros(64, np.uint8))
    assert e.value.code == bfrs.E_INVALID_RECOVERY_SHARD_INDEX
    dec.add_original_shard(0, np.zeros(64, np.uint8))
    with pytest.raises(E) as e:
        dec.decode()
    assert e.value.code == bfrs.E_NOT_ENOUGH_SHARDS


# ---------------------------------------------------------------- BlockFrame wrappers
def test_generate_parity_pads_like_reference(ctx, bfrs, oracle):
    """generate.rs:59-104: segments zero-padded to the longest one."""
    rng = np.random.default_rng(4)
    segs = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(7)] + \
           [rng.integers(0, 256, 1000, dtype=np.uint8)]
    par = bfrs.Chunker(ctx).generate_parity(segs, 8, 3)
    padded = [np.pad(s, (0, 4096 - s.size)) for s in segs]
    assert par == [r.tobytes() for r in oracle.encode(padded, 3)]
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.Chunker(ctx).generate_parity([], 0, 3)
    assert "No chunks provided" in str(e.value)


@pytest.mark.parametrize("staging", ["pinned", "direct"])
def test_crate_wrappers_at_shard_sizes_with_copy_remainders(bfrs, oracle, monkeypatch, staging):
    """Shard sizes that host_copy splits into parts with a remainder (12 MiB + 2
    into 3 parts, 32 MiB + 2 into 8): round 3 found its part size dropped the
    last bytes there (host_copy.cpp).  Through every wrapper that copies
    through pinned rows: generate_parity (k = 1: replication; k = 3 against
    the oracle), recover_segment_rs13 and recover_segment_rs30_3."""
    monkeypatch.setenv("BFRS_CODEC_STAGING", staging)
    c = bfrs.Context(0)
    try:
        rng = np.random.default_rng(12)
        for n in ((12 << 20) + 2, (32 << 20) + 2):
            one = rng.integers(0, 256, n, dtype=np.uint8)
            par = bfrs.Chunker(c).generate_parity([one], 1, 3)
            assert par == [one.tobytes()] * 3
            assert bfrs.recover_segment_rs13(c, par) == one.tobytes()
            three = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(3)]
            par3 = bfrs.Chunker(c).generate_parity(three, 3, 3)
            assert par3 == [r.tobytes() for r in oracle.encode(three, 3)]
        n = (12 << 20) + 2
        segs = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
        par30 = [np.frombuffer(p, np.uint8) for p in bfrs.Chunker(c).generate_parity(segs, 30, 3)]
        for target in (0, 17, 29):
            slots = [None if i in (target, 5, 23) else segs[i] for i in range(30)]
            got = bfrs.recover_segment_rs30_3(c, slots, par30, target)
            assert got == segs[target].tobytes()
    finally:
        c.close()


def test_config1_tier1_8MB_rs13(ctx, bfrs, oracle):
    """BASELINE config 1: single 8 MB file -> RS(1,3) (copies of the 64-padded
    data, generate.rs:26-57) and back through recover_segment_rs13."""
    from bfrs import synth
    for n in (8 * 1024 * 1024, 8_000_000, 8_000_002):
        data = synth.segment_np(1, 0, n)
        par = bfrs.Chunker(ctx).generate_parity_segmented(data)
        padded = (n + 63) // 64 * 64
        want = np.pad(data, (0, padded - n)).tobytes()
        assert par == [want] * 3
        assert par == [r.tobytes() for r in oracle.encode([np.frombuffer(want, np.uint8)], 3)]
        rec = bfrs.recover_segment_rs13(ctx, par, expected_size=n)
        assert rec == data.tobytes()
        assert oracle.blake3_hex(np.frombuffer(rec, np.uint8)) == oracle.blake3_hex(data)
    with pytest.raises(bfrs.BfrsError):  # empty file errors (src/chunker/tests.rs:181-194)
        bfrs.Chunker(ctx).generate_parity_segmented(b"")


def test_recovery_wrapper_errors_like_reference(ctx, bfrs):
    """src/filestore/recovery.rs:196-222."""
    p = [np.zeros(1024, np.uint8)] * 2
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.recover_segment_rs13(ctx, p)
    assert "Exactly 3 parity shards required" in str(e.value)
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.recover_segment_rs30_3(ctx, [None] * 30, [np.zeros(1024, np.uint8)] * 3, 0)
    assert "Too many missing segments" in str(e.value)
    with pytest.raises(bfrs.BfrsError) as e:
        bfrs.recover_segment_rs30_3(ctx, [None] * 29, [np.zeros(1024, np.uint8)] * 3, 0)
    assert "Exactly 30 segment slots required" in str(e.value)


def test_recover_segment_rs30_3_roundtrip(ctx, bfrs, oracle):
    rng = np.random.default_rng(9)
    n = 1 << 20
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    par = [np.frombuffer(p, np.uint8) for p in bfrs.Chunker(ctx).generate_parity(data, 30, 3)]
    slots = [None if i in (3, 14, 27) else data[i] for i in range(30)]
    for t in (3, 14, 27):
        got = bfrs.recover_segment_rs30_3(ctx, slots, par, t)
        assert got == data[t].tobytes()
    with pytest.raises(bfrs.BfrsError) as e:  # target present -> restored_original None
        bfrs.recover_segment_rs30_3(ctx, slots, par, 0)
    assert "Failed to restore target segment" in str(e.value)


def test_into_forms_match_wrappers(ctx, bfrs, oracle):
    """The caller-buffer forms bench.py's crate_api times: the same bytes as the
    wrappers (and the oracle), numpy or bytearray outputs, short buffers refused
    before the call."""
    rng = np.random.default_rng(10)
    n = 3 << 16
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    want = [r.tobytes() for r in oracle.encode(data, 3)]
    outs = [np.empty(n, np.uint8), bytearray(n), np.empty(n + 64, np.uint8)]
    assert bfrs.Chunker(ctx).generate_parity_into(data, 30, 3, outs) == n
    assert [bytes(o[:n]) for o in outs] == want
    with pytest.raises(ValueError):
        bfrs.Chunker(ctx).generate_parity_into(data, 30, 3, [np.empty(n - 2, np.uint8)] * 3)
    slots = [None if i == 11 else data[i] for i in range(30)]
    par = [np.frombuffer(p, np.uint8) for p in want]
    got = bytearray(n)
    assert bfrs.recover_segment_rs30_3_into(ctx, slots, par, 11, got) == n
    assert bytes(got) == data[11].tobytes()
    with pytest.raises(ValueError):
        bfrs.recover_segment_rs30_3_into(ctx, slots, par, 11, np.empty(n - 64, np.uint8))
    # an output that shares bytes with an input is refused before anything is
    # touched (out is first-touched while the inputs are staged)
    big = np.concatenate([data[0], data[1]])
    alias_slots = [big[:n], big[n:]] + slots[2:]
    par_w = [np.array(p) for p in par]
    for src, out in ((alias_slots, big[n // 2:n // 2 + n]), (slots, par_w[2])):
        keep = np.array(out)
        with pytest.raises(bfrs.BfrsError) as e:
            bfrs.recover_segment_rs30_3_into(ctx, src, par_w, 11, out)
        assert e.value.code == bfrs.E_INVALID_ARGUMENT and "overlaps" in str(e.value)
        assert np.array_equal(out, keep)
    assert bfrs.recover_segment_rs30_3_into(ctx, alias_slots, par_w, 11, got) == n
    assert bytes(got) == data[11].tobytes()


# ---------------------------------------------------------------- BASELINE config sizes
def _c2_workload(seed, nseg):
    from bfrs import synth
    shapes = synth.block_shapes(nseg)
    S = synth.SEGMENT_SIZE
    data = torch.empty(nseg, S, dtype=torch.uint8, device="cuda")
    for s in range(nseg):
        synth.fill_segment_torch(data[s], seed, s)
    return shapes, data


@pytest.mark.slow
def test_config2_encode_128x32MiB_golden(ctx):
    """BASELINE config 2: 4 x RS(30,3) + RS(8,3) at 32 MiB, bit-exact parity
    (SHA-256 per shard vs tests/golden/rs_large.json from the oracle)."""
    g = json.load(open(os.path.join(GOLDEN, "rs_large.json")))["c2_128x32MiB"]
    shapes, data = _c2_workload(g["seed"], g["segments"])
    S = g["segment_size"]
    rec = torch.empty(3 * len(shapes), S, dtype=torch.uint8, device="cuda")
    d_orig = [data[s] for s in range(g["segments"])]
    ctx.encode_batch_dev(shapes, 3, S, d_orig, [rec[i] for i in range(rec.shape[0])])
    torch.cuda.synchronize()
    for b in range(len(shapes)):
        for j in range(3):
            h = hashlib.sha256(rec[3 * b + j].cpu().numpy().tobytes()).hexdigest()
            assert h == g["parity_sha256"][b][j], (b, j)


@pytest.mark.slow
def test_config3_decode_3_erasures_128x32MiB(ctx, oracle):
    """BASELINE config 3: per block erase 3 random data shards (seed
    0xDEC0DE+block), restore on the GPU; restored == original bytes and BLAKE3
    (the manifest's per-segment hash, src/chunker/commit.rs:429) matches."""
    from bfrs import synth
    shapes, data = _c2_workload(0xB10C, 128)
    S = synth.SEGMENT_SIZE
    nb = len(shapes)
    rec = torch.empty(3 * nb, S, dtype=torch.uint8, device="cuda")
    d_orig = [data[s] for s in range(128)]
    ctx.encode_batch_dev(shapes, 3, S, d_orig, [rec[i] for i in range(3 * nb)])
    out = torch.empty(3 * nb, S, dtype=torch.uint8, device="cuda")
    dd_orig, dd_out, erased = [], [], []
    seg = 0
    for b, k in enumerate(shapes):
        er = sorted(np.random.default_rng(0xDEC0DE + b).choice(k, 3, replace=False).tolist())
        erased.append(er)
        for i in range(k):
            dd_orig.append(None if i in er else data[seg + i])
            dd_out.append(out[3 * b + er.index(i)] if i in er else None)
        seg += k
    ctx.decode_batch_dev(shapes, 3, S, dd_orig, [rec[i] for i in range(3 * nb)], dd_out)
    torch.cuda.synchronize()
    seg = 0
    for b, k in enumerate(shapes):
        for t, i in enumerate(erased[b]):
            assert torch.equal(out[3 * b + t], data[seg + i]), (b, i)
        seg += k
    # BLAKE3 re-verify of one restored segment against its original's hash
    b0 = out[0].cpu().numpy()
    assert oracle.blake3_hex(b0) == oracle.blake3_hex(data[erased[0][0]].cpu().numpy())


@pytest.mark.slow
@pytest.mark.parametrize("world", [8])
def test_config4_column_stripes_golden(ctx, bfrs, world):
    """BASELINE config 4 (10 GiB = 320 x 32 MiB, 10 x RS(30,3) + RS(20,3)) as the
    strong-scaled multi-GPU run splits it (bfrs.parallel.stripe_ranges): each
    of `world` simulated ranks encodes its 64-byte-aligned column stripe of
    every shard, in its own launch, into the same stripe of the parity.  The
    assembled parity must equal the golden SHA-256 of the unsplit oracle
    encode (tests/golden/rs_large.json): the partition needs no exchange."""
    from bfrs import parallel, synth
    g = json.load(open(os.path.join(GOLDEN, "rs_large.json")))["c4_320x32MiB"]
    S, nseg = g["segment_size"], g["segments"]
    shapes = synth.block_shapes(nseg)
    assert shapes == g["blocks"]
    data = bfrs.empty_shards(nseg, S)
    for s in range(nseg):
        synth.fill_segment_torch(data[s], g["seed"], s)
    rec = bfrs.empty_shards(3 * len(shapes), S)
    rec.fill_(0xA5)  # every byte must be overwritten by some stripe
    for lo, hi in parallel.stripe_ranges(S, world):
        ctx.encode_batch_dev(shapes, 3, hi - lo, [data[s][lo:hi] for s in range(nseg)],
                             [rec[i][lo:hi] for i in range(rec.shape[0])])
    torch.cuda.synchronize()
    for b in range(len(shapes)):
        for j in range(3):
            h = hashlib.sha256(rec[3 * b + j].cpu().numpy().tobytes()).hexdigest()
            assert h == g["parity_sha256"][b][j], (b, j)


def test_in_tree_library_is_the_one_loaded(bfrs):
    import ctypes.util  # noqa: F401
    maps = open("/proc/self/maps").read()
    assert bfrs.LIB_PATH in maps


@pytest.mark.parametrize("byte", [0x00, 0xAB, 0xFF])
def test_constant_byte_shards(ctx, oracle, byte):
    """Constant-byte input (mirrors src/chunker/tests.rs:19-27's constant-fill
    files): parity vs oracle, and a 3-erasure round trip."""
    n = 8192 + 64
    d = [np.full(n, byte, np.uint8) for _ in range(30)]
    want = oracle.encode(d, 3)
    got = ctx.encode(d, 3)
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    o = [None if i in (0, 15, 29) else d[i] for i in range(30)]
    rest = ctx.decode(o, want)
    for i in (0, 15, 29):
        assert np.array_equal(rest[i], d[i])


def test_random_shapes_host_api_vs_oracle(ctx, oracle):
    """Random (k, m), shard sizes with and without a tail chunk, random erasure
    patterns (some with a corrupted recovery shard): the HIP path through
    bfrs_encode / bfrs_decode gives the oracle's bytes.  Covers the looped
    kernels (k not in {30, 20, 8}), both rates and multi-pass codes."""
    rng = np.random.default_rng(0x5EED)
    shapes = [(int(rng.integers(1, 48)), int(rng.integers(1, 9))) for _ in range(16)]
    shapes += [(70, 3), (3, 6), (5, 9), (30, 3), (20, 3), (8, 3)]
    for k, m in shapes:
        if not oracle.lib().oracle_supported(k, m):
            continue
        n = int(rng.choice([64, 192, 4096 + 64, 8192 + 38, 130]))
        data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        want = oracle.encode(data, m)
        rec = ctx.encode(data, m)
        assert all(np.array_equal(a, b) for a, b in zip(rec, want)), (k, m, n)
        e = int(rng.integers(1, min(k, m) + 1))
        lost = sorted(rng.choice(k + m, size=e, replace=False).tolist())
        if all(i >= k for i in lost):
            lost[0] = 0
        r = [None if (k + j) in lost else want[j].copy() for j in range(m)]
        if any(x is not None for x in r) and rng.random() < 0.5:
            j = next(j for j in range(m) if r[j] is not None)
            r[j][::5] ^= 0x3C
        o = [None if i in lost else data[i] for i in range(k)]
        got = ctx.decode(o, r)
        ref = oracle.decode(o, r)
        assert sorted(got) == sorted(ref), (k, m, lost)
        for i in ref:
            assert np.array_equal(got[i], ref[i]), (k, m, n, lost, i)


def test_shards_larger_than_one_launch_window(ctx, oracle):
    """Shards past the 2 GiB launch window (runtime.cpp kMaxWindowBytes: the
    lane offsets are 32-bit) are processed in column windows: the
    parity across the window edge and in the tail chunk equals the oracle's
    on the same slices (the code acts per 64-byte chunk, so a chunk-aligned
    slice is a shard of its own), and an erased shard decodes back whole."""
    n = (2 << 30) + 4096 + 38  # two windows, the last one with a 38-byte tail chunk
    k = 2
    gen = torch.Generator(device="cuda").manual_seed(0x2B16)
    data = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=gen)
            for _ in range(k)]
    par = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
    ctx.encode_batch_dev([k], 3, n, data, par)
    torch.cuda.synchronize()
    edge = 2 << 30
    for lo, hi in ((0, 8192), (edge - 4096, edge + 4096), (n - 38 - 128, n)):
        want = oracle.encode([d[lo:hi].cpu().numpy() for d in data], 3)
        for j in range(3):
            assert np.array_equal(par[j][lo:hi].cpu().numpy(), want[j]), (lo, j)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.decode_batch_dev([k], 3, n, [None, data[1]], par, [out, None])
    torch.cuda.synchronize()
    assert torch.equal(out, data[0])
    del data, par, out
    torch.cuda.empty_cache()


def test_mixed_entry_points_share_one_context_across_threads(ctx, bfrs, oracle):
    """bfrs.h threading rule under a mixed load: host-API encodes/decodes (the
    context's slab pipeline), crate-shaped codec objects (pooled slots) and
    device-batch encodes on per-thread HIP streams, all at once on one
    context, each result checked against the oracle."""
    import threading
    rng = np.random.default_rng(0x7C)
    n = 64 * 1024 + 64
    blocks = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in (30, 8, 20, 5)]
    want = [oracle.encode(b, 3) for b in blocks]
    errors = []

    def host_api(w):
        for rep in range(3):
            b = (w + rep) % len(blocks)
            rec = ctx.encode(blocks[b], 3)
            assert all(np.array_equal(x, y) for x, y in zip(rec, want[b])), ("host", b)
            o = [None if i in (0, 2) else blocks[b][i] for i in range(len(blocks[b]))]
            out = ctx.decode(o, rec)
            assert np.array_equal(out[0], blocks[b][0]) and np.array_equal(out[2], blocks[b][2])

    def codec_objects(w):
        for rep in range(3):
            b = (w + rep) % len(blocks)
            enc = bfrs.ReedSolomonEncoder(ctx, len(blocks[b]), 3, n)
            for d in blocks[b]:
                enc.add_original_shard(d)
            assert list(enc.encode().recovery_iter()) == [r.tobytes() for r in want[b]], ("obj", b)

    def device_batch(w):
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            for rep in range(3):
                b = (w + rep) % len(blocks)
                d_in = [torch.from_numpy(x).to("cuda", non_blocking=False) for x in blocks[b]]
                d_out = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
                ctx.encode_batch_dev([len(blocks[b])], 3, n, d_in, d_out, stream=stream)
                stream.synchronize()
                for j in range(3):
                    assert np.array_equal(d_out[j].cpu().numpy(), want[b][j]), ("dev", b, j)

    def run(f, w):
        try:
            f(w)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(f"{f.__name__}[{w}]: {e!r}")

    ts = [threading.Thread(target=run, args=(f, w))
          for w in range(2) for f in (host_api, codec_objects, device_batch)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=180)
    assert not errors, errors


@pytest.mark.parametrize("staging", ["pinned", "direct"])
def test_generate_parity_slab_pipeline_vs_oracle(bfrs, oracle, monkeypatch, staging):
    """bfrs_generate_parity on a whole block of >= 16 MiB shards runs slab by
    slab (encoder_encode_slabs: ~8 MiB column slabs, each slab's kernel and
    D2H overlapping the next slab's copies); a short last segment is zero-
    padded (generate.rs:75-82) and a ragged shard size puts the tail in the
    last slab.  Every byte against the oracle; the direct staging takes the
    per-shard adds instead."""
    monkeypatch.setenv("BFRS_CODEC_STAGING", staging)
    c = bfrs.Context(0)
    rng = np.random.default_rng(77)
    for n, last in ((16 << 20, (5 << 20) + 3), ((24 << 20) + 38, (24 << 20) + 38)):
        segs = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(7)]
        segs.append(rng.integers(0, 256, last, dtype=np.uint8))
        padded = [np.pad(sg, (0, n - sg.size)) for sg in segs]
        want = [r.tobytes() for r in oracle.encode(padded, 3)]
        outs = [np.empty(n, np.uint8) for _ in range(3)]
        assert bfrs.Chunker(c).generate_parity_into(segs, 8, 3, outs) == n
        assert [o.tobytes() for o in outs] == want, (n, last)
        # the encoder the wrapper used went back to the pool: a later object on
        # the same slot starts clean
        enc = bfrs.ReedSolomonEncoder(c, 8, 3, n)
        for p in padded:
            enc.add_original_shard(p)
        assert list(enc.encode().recovery_iter()) == want
        del enc
    c.close()


def test_recover_rs30_3_slab_pipeline_vs_originals(bfrs, oracle):
    """recover_segment_rs30_3 on >= 16 MiB shards runs slab by slab
    (decoder_restore_slabs): 1, 2 and 3 erased segments with the target among
    them, a ragged shard size (tail in the last slab); the restored target
    equals the original.  A present target and a mismatched segment size still
    take the adds and give the reference's errors."""
    c = bfrs.Context(0)
    rng = np.random.default_rng(78)
    n = (16 << 20) + 64 * 3 + 2
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(30)]
    par = [np.frombuffer(p, np.uint8) for p in
           [r.tobytes() for r in oracle.encode(data, 3)]]
    for erased, target in (([7], 7), ([0, 29], 29), ([3, 14, 25], 14)):
        slots = [None if i in erased else data[i] for i in range(30)]
        out = np.empty(n, np.uint8)
        assert bfrs.recover_segment_rs30_3_into(c, slots, par, target, out) == n
        assert np.array_equal(out, data[target]), (erased, target)
    slots = [None if i == 5 else data[i] for i in range(30)]
    with pytest.raises(bfrs.BfrsError) as e:  # target present: restored_original is None
        bfrs.recover_segment_rs30_3_into(c, slots, par, 6, np.empty(n, np.uint8))
    assert "Failed to restore target segment" in str(e.value)
    short = list(slots)
    short[9] = data[9][:-2]
    with pytest.raises(bfrs.BfrsError) as e:  # the crate's DifferentShardSize
        bfrs.recover_segment_rs30_3_into(c, short, par, 5, np.empty(n, np.uint8))
    assert e.value.code == bfrs.E_DIFFERENT_SHARD_SIZE
    c.close()


def _c2_last_block_erasures():
    """bench.py's 3 erased indices of C2's last block, RS(8,3) (block 4)."""
    return sorted(np.random.default_rng(0xDEC0DE + 4).choice(8, 3, replace=False).tolist())


_MIB = (1 << 20) + 64 * 3


@pytest.mark.parametrize("k,m,erased,use,n", [
    (30, 3, [2, 11, 29], [0, 1, 2], 4096 + 64 * 3), (8, 3, [0, 7], [2, 1], 4096 + 64 * 3),
    (20, 3, [5], [1], 4096 + 64 * 3), (3, 5, [0, 1, 2], [0, 3, 4], 4096 + 64 * 3),
    (17, 6, [1, 4, 9, 16], [5, 0, 2, 3], 4096 + 64 * 3),
    # a BlockFrame-scale shard (1 MiB + 3 chunks: 4,099 chunks,
    # many launch tiles and workgroups) for RS(30,3) with 3 erasures, and the
    # RS(8,3) last block of C2 with the bench's own erasure pattern
    (30, 3, [4, 17, 23], [0, 1, 2], _MIB), (8, 3, _c2_last_block_erasures(), [0, 1, 2], _MIB)])
def test_product_follows_the_algebra(ctx, oracle, k, m, erased, use, n):
    """The HIP path against plain algebra rather than the oracle's transform
    (tests/test_rs_interpolation.py): encode = per-chunk Lagrange
    interpolation on the field points, decode from exactly k shards with a
    corrupted recovery shard = the linear system's unique solution."""
    import test_rs_interpolation as alg
    exp = np.array([oracle.gf_exp(i) for i in range(alg.ORDER)], np.int64)
    log = np.zeros(65536, np.int64)
    log[1:] = [oracle.gf_log(x) for x in range(1, 65536)]
    gf = (exp, log)
    rng = np.random.default_rng(31 * k + m + n)
    originals = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    rec = ctx.encode(originals, m)
    want = alg.interpolated_parity(gf, oracle, originals, m)
    assert all(np.array_equal(rec[j], want[j]) for j in range(m))
    rec = [r.copy() for r in rec]
    rec[use[0]][int(rng.integers(0, n))] ^= 0x3C
    out = ctx.decode([None if i in erased else originals[i] for i in range(k)],
                     [rec[j] if j in use else None for j in range(m)])
    coef = alg._coef_logs(gf, oracle, k, m)
    rhs = []
    for j in use:
        r = alg._symbols(rec[j])
        for i in range(k):
            if i not in erased:
                r = r ^ alg._mul(gf, coef[j, i], alg._symbols(originals[i]))
        rhs.append(r)
    x = alg._solve(gf, coef[np.ix_(use, erased)], np.stack(rhs))
    for a, i in enumerate(erased):
        assert np.array_equal(out[i], alg._bytes(x[a])), (k, m, i)


_SLAB_FAILURE_SCRIPT = r'''
import os, sys
import numpy as np
root = os.environ["BFRS_TEST_ROOT"]
sys.path.insert(0, os.path.join(root, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(root, "oracle"))
import bfrs, oracle
assert bfrs.LIB_PATH.endswith("libbfrs_ab.so"), bfrs.LIB_PATH
ctx = bfrs.Context(0)
rng = np.random.default_rng(0x51AB)
S = (16 << 20) + 64 * 3          # >= 16 MiB: the slab-pipelined wrappers, 2 slabs
segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(30)]
eng = oracle.ENGINE_AVX2 if oracle.lib().oracle_have_avx2() else oracle.ENGINE_SCALAR
want = oracle.encode(segs, 3, eng)
ch = bfrs.Chunker(ctx)
slots = [None if i == 7 else segs[i] for i in range(30)]
for fail in ("0", "1"):
    os.environ["BFRS_FAIL_SLAB"] = fail
    try:
        ch.generate_parity_into(segs, 30, 3, [np.empty(S, np.uint8) for _ in range(3)])
        sys.exit("encode: no injected failure")
    except bfrs.BfrsError as e:
        assert "injected" in str(e), e
    try:
        bfrs.recover_segment_rs30_3_into(ctx, slots, want, 7, np.empty(S, np.uint8))
        sys.exit("recover: no injected failure")
    except bfrs.BfrsError as e:
        assert "injected" in str(e), e
    del os.environ["BFRS_FAIL_SLAB"]
    outs = [np.empty(S, np.uint8) for _ in range(3)]
    ch.generate_parity_into(segs, 30, 3, outs)  # the one idle slot, reused
    assert all(np.array_equal(outs[j], want[j]) for j in range(3)), f"parity after fail {fail}"
    got = np.empty(S, np.uint8)
    bfrs.recover_segment_rs30_3_into(ctx, slots, want, 7, got)
    assert np.array_equal(got, segs[7]), f"restored after fail {fail}"
ctx.close()
print("slab-failure reuse ok")
'''


def test_failed_slab_call_leaves_its_slot_reusable():
    """a slab-pipelined wrapper that fails after queuing slabs (the
    measurement build's BFRS_FAIL_SLAB injects it after slab 0 or after the
    last slab) must leave nothing in flight on the slot it returns: the next
    call, on the same single idle slot, gives the oracle's parity and the
    original segment.  Runs in a child on libbfrs_ab.so (the product has no
    injection point)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "blockframe-rs_amd", "libbfrs_ab.so")):
        pytest.skip("libbfrs_ab.so not built (make -C blockframe-rs_amd/csrc ab)")
    env = dict(os.environ, BFRS_LIB="libbfrs_ab.so", BFRS_CODEC_SLOTS="1", BFRS_TEST_ROOT=root)
    r = subprocess.run([sys.executable, "-c", _SLAB_FAILURE_SCRIPT], capture_output=True,
                       text=True, timeout=180, env=env)
    assert r.returncode == 0 and "reuse ok" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])


_LDS_VARIANT_SCRIPT = r'''
import os, sys
import numpy as np
root = os.environ["BFRS_TEST_ROOT"]
sys.path.insert(0, os.path.join(root, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(root, "oracle"))
import bfrs, oracle
assert bfrs.LIB_PATH.endswith("libbfrs_ab.so"), bfrs.LIB_PATH
ctx = bfrs.Context(0)
rng = np.random.default_rng(0x1D5)
eng = oracle.ENGINE_AVX2 if oracle.lib().oracle_have_avx2() else oracle.ENGINE_SCALAR
n_cases = 0
# shard sizes: one chunk, a ragged wave run, ragged tiles with a tail, several
# read groups of whole tiles
sizes = [64, 64 * 63 + 10, 64 * 300 + 38, (1 << 20) + 64 * 3, (3 << 20) + 64 * 77 + 2]
for v in os.environ["LDS_VARIANTS"].split(","):
    os.environ["BFRS_KERNEL_VARIANT"] = v
    for k in (30, 29, 20, 19, 8, 7):   # odd k: padded to 30 / 20 / 8, unrotated
        for S in sizes:
            segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
            want = oracle.encode(segs, 3, eng)
            got = ctx.encode(segs, 3)
            assert all(np.array_equal(got[j], want[j]) for j in range(3)), (v, k, S, "encode")
            er = sorted(rng.choice(k, size=min(3, k), replace=False).tolist())
            rec = [w.copy() for w in want]
            if S > 64 and k > 3:   # a corrupted recovery shard: the crate decoder's linear map
                er = er[:2]
                rec[2][int(rng.integers(0, S))] ^= 0x5A
            orig = [None if i in er else segs[i] for i in range(k)]
            out = ctx.decode(orig, rec)
            ref = oracle.decode(orig, rec, eng)
            for i in er:
                assert np.array_equal(out[i], ref[i]), (v, k, S, "decode", i)
            n_cases += 2
    # one launch holding blocks of different n_in (the C2 / C4 last-block shape)
    S = (2 << 20) + 64 * 9
    ks = [30, 8, 20]
    segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(sum(ks))]
    outs = [np.empty(S, np.uint8) for _ in range(3 * len(ks))]
    ctx.encode_host_batch(ks, 3, S, segs, outs)
    off = 0
    for b, k in enumerate(ks):
        want = oracle.encode(segs[off:off + k], 3, eng)
        assert all(np.array_equal(outs[3 * b + j], want[j]) for j in range(3)), (v, "batch", k)
        off += k
    n_cases += len(ks)
# two tiles per workgroup (the measurement build's BFRS_TILES_PER_WG): the
# LDS-DMA kernels take one tile per workgroup only, so the launch falls back
# to v76's 8 KiB tiles and its grid must be sized for them
os.environ["BFRS_TILES_PER_WG"] = "2"
S = (1 << 20) + 64 * 3
segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(30)]
want = oracle.encode(segs, 3, eng)
got = ctx.encode(segs, 3)
assert all(np.array_equal(got[j], want[j]) for j in range(3)), "tiles_per_wg 2"
del os.environ["BFRS_TILES_PER_WG"]
n_cases += 1
ctx.close()
print(f"lds variants ok: {n_cases} cases")
'''


def test_lds_dma_variants_match_the_oracle():
    """Round 6: the measurement build's LDS-DMA input-ring
    kernels (v107-v109: 4 KiB per wave and input staged with
    global_load_lds_dwordx4) against the oracle before any timing is trusted:
    RS(k,3) encodes and decodes (incl. a corrupted recovery shard) for every
    unrolled size and its odd neighbour, shard sizes from one chunk to ragged
    multi-group runs with tails, and one launch mixing n_in 30 / 8 / 20.  Runs
    in a child on libbfrs_ab.so (the product does not carry them)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "blockframe-rs_amd", "libbfrs_ab.so")):
        pytest.skip("libbfrs_ab.so not built (make -C blockframe-rs_amd/csrc ab)")
    env = dict(os.environ, BFRS_LIB="libbfrs_ab.so", BFRS_TEST_ROOT=root,
               LDS_VARIANTS="107,108,109")
    r = subprocess.run([sys.executable, "-c", _LDS_VARIANT_SCRIPT], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and "lds variants ok" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])


_PIN_MALLOC_SCRIPT = r'''
import os, sys
import numpy as np
root = os.environ["BFRS_TEST_ROOT"]
sys.path.insert(0, os.path.join(root, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(root, "oracle"))
import bfrs, oracle
assert bfrs.LIB_PATH.endswith("libbfrs_ab.so"), bfrs.LIB_PATH
rng = np.random.default_rng(0x91A)
eng = oracle.ENGINE_AVX2 if oracle.lib().oracle_have_avx2() else oracle.ENGINE_SCALAR
for rnd in range(3):   # slots of >= 4 MiB freed and taken again, then the context
    ctx = bfrs.Context(0)
    for S in ((1 << 20) + 64 * 3 + 6, (6 << 20) + 38):
        segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(30)]
        want = oracle.encode(segs, 3, eng)
        got = ctx.encode(segs, 3)
        assert all(np.array_equal(got[j], want[j]) for j in range(3)), (rnd, S, "encode")
        orig = [None if i in (2, 17, 29) else segs[i] for i in range(30)]
        out = ctx.decode(orig, want)
        assert all(np.array_equal(out[i], segs[i]) for i in (2, 17, 29)), (rnd, S, "decode")
    ctx.close()
print("pin malloc ok")
'''


def test_large_pinned_buffers_from_hip_host_malloc():
    """Round 6 (review of pinned_free): a pinned buffer of >= 4 MiB is
    normally a registered huge-page mapping, but falls back to hipHostMalloc
    when the registration fails.  pinned_free must free such a buffer with
    hipHostFree, not unregister and munmap it.  The measurement build's
    hipHostMalloc mode (BFRS_PIN_MODE=malloc) forces the fallback for every
    codec slot.  Three contexts in turn, each with 1 MiB and 6 MiB RS(30,3)
    encodes and decodes checked against the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "blockframe-rs_amd", "libbfrs_ab.so")):
        pytest.skip("libbfrs_ab.so not built (make -C blockframe-rs_amd/csrc ab)")
    env = dict(os.environ, BFRS_LIB="libbfrs_ab.so", BFRS_TEST_ROOT=root, BFRS_PIN_MODE="malloc")
    r = subprocess.run([sys.executable, "-c", _PIN_MALLOC_SCRIPT], capture_output=True,
                       text=True, timeout=180, env=env)
    assert r.returncode == 0 and "pin malloc ok" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])


@pytest.mark.parametrize("n", [64 * 150 + 38, (16 << 20) + 64 * 5 + 38])
def test_host_batch_pinned_strided_rows_vs_oracle(ctx, oracle, n):
    """Pinned shard rows at a constant pitch (one pinned tensor, as the bench
    and config 4's host batches hand them over) go through the pipeline as
    2-D row copies (runtime.cpp copy_rows): every parity byte against the
    oracle, decodes whose erasures split the rows into runs, rows handed over
    in reverse order (a negative pitch: row by row), and recovery rows of
    another pinned tensor."""
    rng = np.random.default_rng(77)
    ks = [30, 8, 20]
    nseg = sum(ks)
    host = torch.empty(nseg, n, dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.from_numpy(rng.integers(0, 256, (nseg, n), dtype=np.uint8)))
    par = torch.empty(3 * len(ks), n, dtype=torch.uint8, pin_memory=True)
    rows = [host[s] for s in range(nseg)]
    ctx.encode_host_batch(ks, 3, n, rows, [par[i] for i in range(par.shape[0])])
    big = n > (1 << 20) and oracle.lib().oracle_have_avx2()
    eng = oracle.ENGINE_AVX2 if big else oracle.ENGINE_SCALAR
    blocks, off = [], 0
    for k in ks:
        blocks.append([host[off + i].numpy() for i in range(k)])
        off += k
    want = [oracle.encode(blk, 3, eng) for blk in blocks]
    for b in range(len(ks)):
        for j in range(3):
            assert np.array_equal(par[3 * b + j].numpy(), want[b][j]), (n, b, j)
    # reversed row order within each block: pitch -n, not merged
    par2 = torch.zeros_like(par)
    rev, off = [], 0
    for k in ks:
        rev += [host[off + i] for i in range(k)][::-1]
        off += k
    ctx.encode_host_batch(ks, 3, n, rev, [par2[i] for i in range(par2.shape[0])])
    for b, blk in enumerate(blocks):
        w = oracle.encode(blk[::-1], 3, eng)
        for j in range(3):
            assert np.array_equal(par2[3 * b + j].numpy(), w[j]), ("reversed", b, j)
    # decodes: erasures in the middle and at the ends of each block
    rest = torch.empty(3 * len(ks), n, dtype=torch.uint8, pin_memory=True)
    orig, outs, want_rows, off = [], [], [], 0
    for b, k in enumerate(ks):
        er = [0, k // 2, k - 1]
        for i in range(k):
            orig.append(None if i in er else host[off + i])
            outs.append(rest[3 * b + er.index(i)] if i in er else None)
            if i in er:
                want_rows.append((3 * b + er.index(i), off + i))
        off += k
    ctx.decode_host_batch(ks, 3, n, orig, [par[i] for i in range(par.shape[0])], outs)
    for r, s in want_rows:
        assert torch.equal(rest[r], host[s]), (n, r, s)


@pytest.mark.parametrize("k", list(range(1, 31)))
def test_every_three_erasure_pattern(ctx, oracle, k):
    """Every RS(k,3) shape a tier-3 block can have (k = 1..30: a full block or
    any last block) and all C(k + 3, 3) ways to lose 3 of its k + 3 shards
    (data and parity alike; 5,456 for k = 30, 46,375 in all), decoded on the
    GPU in device batches of up to 496 blocks that share one set of shards:
    every restored data shard equals the original (MDS decoding of a codeword
    is unique, so this is bit-exact with the crate by construction).  k = 30,
    20, 8 run the unrolled kernel, the others the looped subfield kernel;
    k <= 2 and k = 4 take LowRate.  The shard size is ragged (tail kernel
    included)."""
    import itertools
    from math import comb
    rng = np.random.default_rng(0x3E3 + k)
    n = 64 * 70 + 38
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    par = oracle.encode(data, 3)
    d_data = [torch.from_numpy(x).cuda() for x in data]
    d_par = [torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in par]
    patterns = list(itertools.combinations(range(k + 3), 3))
    checked = 0
    for c0 in range(0, len(patterns), 496):
        chunk = patterns[c0:c0 + 496]
        orig, rec, outs, want = [], [], [], []
        for er in chunk:
            for i in range(k):
                orig.append(None if i in er else d_data[i])
            for j in range(3):
                rec.append(None if k + j in er else d_par[j])
            for i in range(k):
                if i in er:
                    outs.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
                    want.append(i)
                else:
                    outs.append(None)
        ctx.decode_batch_dev([k] * len(chunk), 3, n, orig, rec, outs)
        got = torch.stack([o for o in outs if o is not None])
        ref = torch.stack([d_data[i] for i in want])
        bad = (got != ref).any(dim=1).nonzero().flatten().tolist()
        assert not bad, f"RS({k},3): {len(bad)} restored shards differ in patterns {c0}.."
        checked += got.shape[0]
    # patterns erasing e data shards (and 3 - e parity) restore e shards each
    assert checked == sum(e * comb(k, e) * comb(3, 3 - e) for e in range(4))


@pytest.mark.parametrize("k", list(range(1, 31)))
def test_inconsistent_inputs_follow_the_crates_decoder(ctx, oracle, k):
    """Decodes whose inputs are NOT a codeword (one present recovery shard
    corrupted): MDS uniqueness no longer fixes the output, so here the bytes
    are the crate decoder's own linear map of every shard it was given.  For
    every tier-3 block shape (k = 1..30) and 24 sampled erasure patterns (1-3
    erased data shards, the rest of the recovery present, one of those
    corrupted), one device batch per k against the oracle's restatement of
    the crate's decoder, byte for byte."""
    rng = np.random.default_rng(0xBAD0 + k)
    n = 64 * 70 + 38
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    par = [np.ascontiguousarray(p) for p in oracle.encode(data, 3)]
    cases = []
    for _ in range(24):
        e = int(rng.integers(1, min(3, k) + 1))
        er = sorted(rng.choice(k, e, replace=False).tolist())
        rec = [p.copy() for p in par]
        # drop recovery shards beyond what the erasures need, keep >= 1 to corrupt
        keep = sorted(rng.choice(3, int(rng.integers(e, 4)), replace=False).tolist())
        rec = [rec[j] if j in keep else None for j in range(3)]
        j = keep[int(rng.integers(0, len(keep)))]
        rec[j][int(rng.integers(0, n))] ^= int(rng.integers(1, 256))
        orig = [None if i in er else data[i] for i in range(k)]
        cases.append((orig, rec, er))
    d = lambda x: None if x is None else torch.from_numpy(np.ascontiguousarray(x)).cuda()
    outs = [[torch.empty(n, dtype=torch.uint8, device="cuda") if o is None else None for o in orig]
            for orig, _, _ in cases]
    ctx.decode_batch_dev([k] * len(cases), 3, n, [d(x) for c in cases for x in c[0]],
                         [d(x) for c in cases for x in c[1]], [o for oo in outs for o in oo])
    torch.cuda.synchronize()
    for (orig, rec, er), oo in zip(cases, outs):
        want = oracle.decode(orig, rec)
        for i in er:
            assert np.array_equal(oo[i].cpu().numpy(), want[i]), (k, er, i)


@pytest.mark.parametrize("k", [30, 8, 1])
def test_every_tail_length(ctx, oracle, k):
    """Every even tail length the crate allows (shard_bytes % 64 = 2, 4, ...,
    62) with whole chunks before it, in one device batch per k: encode against
    the oracle, and a decode of min(3, k) erased data shards against the
    originals.  The tail chunk's lo/hi split is the oracle's
    reading; the kernel must agree at every length."""
    rng = np.random.default_rng(0x7A11 + k)
    sizes = [64 * 9 + t for t in range(2, 64, 2)]
    for n in sizes:  # one launch per size (a batch shares its shard size)
        data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        d_data = [torch.from_numpy(x).cuda() for x in data]
        d_rec = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
        ctx.encode_batch_dev([k], 3, n, d_data, d_rec)
        want = oracle.encode(data, 3)
        for j in range(3):
            assert np.array_equal(d_rec[j].cpu().numpy(), want[j]), (k, n, j)
        er = list(range(min(3, k)))
        outs = [torch.empty(n, dtype=torch.uint8, device="cuda") if i in er else None
                for i in range(k)]
        ctx.decode_batch_dev([k], 3, n, [None if i in er else d_data[i] for i in range(k)],
                             d_rec, outs)
        torch.cuda.synchronize()
        for i in er:
            assert torch.equal(outs[i], d_data[i]), (k, n, i)
