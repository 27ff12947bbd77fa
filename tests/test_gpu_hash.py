"""GPU BLAKE3 (blake3_kernels.hip) vs the oracle: digests of device-resident
messages across chunk/group/reduction boundaries, subtree CVs (checked with
the pure-Python restatement and through bfrs_blake3_combine), batching of a
whole RS block, and argument errors."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K = 1024
G = 256 * K  # kernel-1 group
LENS = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 3000, 64 * K + 1, G - 1, G, G + 1,
        2 * G + 5, 1 << 20, (32 << 20) + 77, 32 << 20,
        512 * G, 512 * G + 1, 513 * G + 1000,  # 512+ groups: multi-level reduction
        # kernel 1 leaves 8-chunk (level-3) nodes of multi-group messages to
        # kernel 2: last groups of 4+1, 5, 8+1 and 9 chunks, exactly one
        # 512-node run, one run + 1 node
        G + 4 * K + 1, G + 5 * K, G + 8 * K + 1, G + 9 * K, 16 * G, 16 * G + 2 * K]


def _dev(a):
    return torch.from_numpy(a).to("cuda")


@pytest.mark.parametrize("n", LENS)
def test_gpu_blake3_single(ctx, oracle, n):
    a = np.random.default_rng(n % 9973).integers(0, 256, size=n, dtype=np.uint8)
    t = _dev(a) if n else torch.empty(0, dtype=torch.uint8, device="cuda")
    assert ctx.blake3_batch_dev([t]) == [oracle.blake3_hex(a)]


def test_gpu_blake3_batch_mixed(ctx, oracle):
    rng = np.random.default_rng(3)
    lens = [int(x) for x in rng.integers(0, 3 * G, size=40)] + [0, 1, 1024, G]
    arrs = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in lens]
    ts = [_dev(a) if a.size else torch.empty(0, dtype=torch.uint8, device="cuda") for a in arrs]
    want = [oracle.blake3_hex(a) for a in arrs]
    assert ctx.blake3_batch_dev(ts) == want
    # the prepared C-ABI call bench.py times: same digests, call after call
    call, dig = ctx.blake3_batch_dev_call(ts)
    for _ in range(2):
        dig[:] = 0
        call()
        assert [bytes(d).hex() for d in dig] == want


def test_gpu_blake3_rs_block(ctx, oracle):
    # one tier-3 block: 30 segments + 3 parity (4 MiB stand-ins), one call
    rng = np.random.default_rng(4)
    arrs = [rng.integers(0, 256, size=4 << 20, dtype=np.uint8) for _ in range(33)]
    ts = [_dev(a) for a in arrs]
    got = ctx.blake3_batch_dev(ts)
    assert got == [oracle.blake3_hex(a) for a in arrs]


@pytest.mark.parametrize("n", [1, 1024, 3000, G, G + 3, 3 * G])
def test_gpu_blake3_subtree_cv(ctx, n):
    import b3py
    a = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8)
    _, cvs = ctx.blake3_batch_dev([_dev(a)], with_cvs=True)
    if n <= 4 * K:
        assert cvs[0] == b3py.subtree_cv(a.tobytes(), 0)
    assert len(cvs[0]) == 32


@pytest.mark.parametrize("part,nparts,tail", [(G, 5, 777), (1 << 20, 3, 0), (4 * K, 9, 1)])
def test_gpu_file_hash_from_segment_cvs(ctx, bfrs, oracle, part, nparts, tail):
    # the whole-file digest (commit.rs:478) from per-segment CVs
    data = np.random.default_rng(part + tail).integers(0, 256, size=part * nparts + tail,
                                                       dtype=np.uint8)
    d = _dev(data)
    segs = [d[i:i + part] for i in range(0, data.size, part)]
    offs = [i * (part // K) for i in range(len(segs))]
    _, cvs = ctx.blake3_batch_dev(segs, with_cvs=True, chunk_offsets=offs)
    assert bfrs.blake3_combine(cvs) == oracle.blake3_hex(data)
    # at offset 0 the same call gives each segment's own digest
    assert ctx.blake3_batch_dev(segs) == [oracle.blake3_hex(data[i:i + part])
                                          for i in range(0, data.size, part)]


def test_gpu_blake3_errors(ctx, bfrs):
    t = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(bfrs.BfrsError) as e:
        ctx.blake3_batch_dev([t[1:]])
    assert e.value.code == bfrs.E_INVALID_ARGUMENT
    with pytest.raises(bfrs.BfrsError):
        bfrs.blake3_combine([b"\0" * 32])
