"""GPU: one process driving several contexts.

BlockFrame is one Rust process whose rayon workers take independent blocks
(src/chunker/commit.rs:391-393).  bfrs_encode_host_batch_multi /
bfrs_decode_host_batch_multi spread a host-memory batch over several contexts
(context d: column stripe d of every shard), bfrs_commit_multi deals a tier-3
file's blocks over them.  The boxes have one GPU, so the tests open two or
three contexts on device 0: each has its own streams, HBM staging and host
thread, which is the multi-device code path; only the device ordinal differs.
Every test also has a "spread" form that puts context d on device
d % device_count: it runs wherever two or more GPUs are visible
and is skipped on the one-GPU boxes, so cross-device use stays untested until
a multi-GPU box runs the suite (README).
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
PLACEMENTS = ["device0", "spread"]


def _devices(bfrs, n, placement):
    """Device of each of n contexts: all on device 0, or spread over the
    visible GPUs (skipped with fewer than two)."""
    if placement == "spread":
        nd = bfrs.device_count()
        if nd < 2:
            pytest.skip("cross-device form: needs >= 2 visible GPUs (this box has one)")
        return [d % nd for d in range(n)]
    return [0] * n


@pytest.mark.parametrize("placement", PLACEMENTS)
def test_config4_host_batch_multi_golden(bfrs, placement):
    """BASELINE configs[3] (320 x 32 MiB = 10 x RS(30,3) + RS(20,3)) from
    pinned host memory through two contexts in this one process: parity equal
    to the golden digests of the unsplit oracle encode, and a 3-erasure decode
    of every block through the same two contexts restores the originals."""
    from bfrs import synth
    g = json.load(open(os.path.join(GOLDEN, "rs_large.json")))["c4_320x32MiB"]
    S, nseg = g["segment_size"], g["segments"]
    shapes = synth.block_shapes(nseg)
    assert shapes == g["blocks"]
    host = torch.empty(nseg, S, dtype=torch.uint8, pin_memory=True)
    row = torch.empty(S, dtype=torch.uint8, device="cuda")
    for s in range(nseg):
        synth.fill_segment_torch(row, g["seed"], s)
        host[s].copy_(row)
    del row
    par = torch.full((3 * len(shapes), S), 0xA5, dtype=torch.uint8, pin_memory=True)
    ctxs = [bfrs.Context(d) for d in _devices(bfrs, 2, placement)]
    try:
        bfrs.encode_host_batch_multi(ctxs, shapes, 3, S, [host[s] for s in range(nseg)],
                                     [par[i] for i in range(par.shape[0])])
        for b in range(len(shapes)):
            for j in range(3):
                h = hashlib.sha256(par[3 * b + j].numpy().tobytes()).hexdigest()
                assert h == g["parity_sha256"][b][j], (b, j)
        rng = np.random.default_rng(0xC4)
        rest = torch.empty(3 * len(shapes), S, dtype=torch.uint8, pin_memory=True)
        orig, outs, want, seg = [], [], [], 0
        for b, k in enumerate(shapes):
            er = sorted(rng.choice(k, 3, replace=False).tolist())
            for i in range(k):
                orig.append(None if i in er else host[seg + i])
                outs.append(rest[3 * b + er.index(i)] if i in er else None)
                if i in er:
                    want.append((3 * b + er.index(i), seg + i))
            seg += k
        bfrs.decode_host_batch_multi(ctxs, shapes, 3, S, orig, [par[i] for i in range(par.shape[0])],
                                     outs)
        for r, s in want:
            assert torch.equal(rest[r], host[s]), (r, s)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("placement", PLACEMENTS)
@pytest.mark.parametrize("n_ctx", [1, 2, 3, 5])
def test_host_batch_multi_stripes_vs_oracle(bfrs, oracle, n_ctx, placement):
    """Ragged shards (a tail chunk in the last stripe), more contexts than a
    narrow shard has chunks (idle contexts), mixed block sizes; every byte
    against the oracle."""
    rng = np.random.default_rng(n_ctx)
    ks = [30, 8, 1, 20]
    ctxs = [bfrs.Context(d) for d in _devices(bfrs, n_ctx, placement)]
    try:
        for n in (64 * 3 + 38, 8192 * 5 + 64 * 7 + 2, (1 << 20) + 6):
            host = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for k in ks]
            rec = [np.full(n, 0x5A, np.uint8) for _ in range(3 * len(ks))]
            bfrs.encode_host_batch_multi(ctxs, ks, 3, n, [x for blk in host for x in blk], rec)
            for b, blk in enumerate(host):
                want = oracle.encode(blk, 3)
                for j in range(3):
                    assert np.array_equal(rec[3 * b + j], want[j]), (n, b, j)
            orig, outs, erased = [], [], []
            for b, k in enumerate(ks):
                er = sorted(rng.choice(k, min(3, k), replace=False).tolist())
                erased.append(er)
                for i in range(k):
                    orig.append(None if i in er else host[b][i])
                    outs.append(np.zeros(n, np.uint8) if i in er else None)
            bfrs.decode_host_batch_multi(ctxs, ks, 3, n, orig, rec, outs)
            off = 0
            for b, k in enumerate(ks):
                for i in erased[b]:
                    assert np.array_equal(outs[off + i], host[b][i]), (n, b, i)
                off += k
    finally:
        for c in ctxs:
            c.close()


def test_multi_argument_errors(bfrs):
    c = bfrs.Context(0)
    x = np.zeros(128, np.uint8)
    with pytest.raises(bfrs.BfrsError):
        bfrs.encode_host_batch_multi([], [1], 3, 128, [x], [x.copy() for _ in range(3)])
    closed = bfrs.Context(0)
    closed.close()
    with pytest.raises(bfrs.BfrsError):
        bfrs.encode_host_batch_multi([c, closed], [1], 3, 128, [x], [x.copy() for _ in range(3)])
    with pytest.raises(bfrs.BfrsError) as e:  # not enough shards: checked before any work
        bfrs.decode_host_batch_multi([c, c], [2], 3, 128, [None, None], [x, None, None],
                                     [x.copy(), x.copy()])
    assert e.value.code == bfrs.E_NOT_ENOUGH_SHARDS
    c.close()


def _tree(d):
    out = {}
    for root, _, files in os.walk(d):
        for f in files:
            p = os.path.join(root, f)
            out[os.path.relpath(p, d)] = open(p, "rb").read()
    return out


@pytest.mark.parametrize("placement", PLACEMENTS)
@pytest.mark.parametrize("n_ctx,seg,size", [
    (2, 1 << 20, 200 * (1 << 20) + 12346),   # 7 blocks (last one 20 segments + a tail)
    (3, 1 << 20, 61 * (1 << 20)),            # 3 blocks, the last one segment
    (8, 64 << 10, 2 * 30 * (64 << 10)),      # more contexts than blocks
])
def test_commit_multi_equals_commit(bfrs, tmp_path, n_ctx, seg, size, placement):
    """bfrs_commit_multi over several contexts writes the same archive as
    bfrs_commit: every segment and parity file byte for byte, and the
    manifest except time_of_creation; the archive then reads back, checks
    Healthy and repairs like any other."""
    from bfrs import synth
    src = tmp_path / "big.bin"
    src.write_bytes(synth.segment_np(7, 0, size).tobytes())
    one = bfrs.Context(0)
    ctxs = [bfrs.Context(d) for d in _devices(bfrs, n_ctx, placement)]
    try:
        a = bfrs.commit(one, str(src), str(tmp_path / "single"), segment_size=seg, tier=3)
        b = bfrs.commit(ctxs, str(src), str(tmp_path / "multi"), segment_size=seg, tier=3)
        assert os.path.basename(a) == os.path.basename(b)  # {name}_{blake3 of the file}
        ta, tb = _tree(a), _tree(b)
        assert sorted(ta) == sorted(tb)
        for f in ta:
            if f == "manifest.json":
                ma, mb = json.loads(ta[f]), json.loads(tb[f])
                ma.pop("time_of_creation")
                mb.pop("time_of_creation")
                assert ma == mb
            else:
                assert ta[f] == tb[f], f
        assert bfrs.health_check(one, b)["status"] == "Healthy"
        # damage in two blocks, repaired through bfrs_repair_multi (blocks dealt
        # over the contexts, report summed), then through bfrs_repair
        seg0 = os.path.join(b, "blocks", "block_0", "segments", "segment_1.dat")
        par1 = os.path.join(b, "blocks", "block_1", "parity", "block_parity_2.dat")
        os.unlink(seg0)
        with open(par1, "r+b") as f:
            c = f.read(1)
            f.seek(0)
            f.write(bytes([c[0] ^ 0xFF]))
        rep = bfrs.repair(ctxs, b)
        assert rep["segments_repaired"] == 1 and rep["parity_repaired"] == 1, rep
        assert rep["blocks_checked"] == len([k for k in ta if k.endswith("block_parity_0.dat")])
        assert bfrs.health_check(one, b)["status"] == "Healthy"
        for f in (seg0, par1):
            assert open(f, "rb").read() == ta[os.path.relpath(f, b)]
        os.unlink(seg0)
        rep = bfrs.repair(one, b)
        assert rep["segments_repaired"] == 1 and bfrs.health_check(one, b)["status"] == "Healthy"
        assert open(seg0, "rb").read() == ta[os.path.relpath(seg0, b)]
    finally:
        one.close()
        for c in ctxs:
            c.close()
