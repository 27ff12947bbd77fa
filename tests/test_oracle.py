"""CPU: pin the oracle before trusting it.

The reference pins no parity bytes; what is pinned:
  * SURVEY Appendix A.7 — independent KAT for RS(30,3), shard_bytes=128;
  * SURVEY Appendix A.6 — the generator G_30 and exp8 constants;
  * src/filestore/README.md:178 — RS(1,3) parity == copies of the data;
  * src/utils.rs:17-18 — blake3("blockframe") doctest KAT;
  * the BLAKE3 specification's test vectors (input byte i = i % 251);
  * src/merkle_tree/mod.rs:77-100 — parent = blake3(hex(l) ++ hex(r)), odd node paired with itself.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")

A7_P0 = ("5605235774c91b28ff48a41da09935d08583be6a84e525b0660cb2a432a3deb8e858bb22adc7f52d1e4fdf86"
         "cf33f6622b5505fc28172812b02d875937ebd52965e690575a0020a840781f69600fff65278db724ccf546bf"
         "fbc69e85bb74701cb3100c874ea429b5beb6354fe272378211577fbd435ec271f2ce278108573ebd")
A7_P1 = ("e4f3b308bc87779434d98670b77a798618ae0ea76c192831559a243086da040be2fd4d535e37c3aad7eb2002"
         "c58fa8c19324ca36e2e5130ea766271a264bbac0ecb13ae1e1540bc7e3d2bdc05a05a94e94732bc841cd8f3e"
         "97ad3c0639aca882b9975b11da54bef43112e897d3a969216f602a77d570256de585c15803f78def")
A7_P2 = ("dc19e8757d997c495d18a821b8ee455386c84ec69690223cbbd3036e5129b53a329e383b5857afe009ad19b9"
         "8c5b4073119e1135aad0aba2299c0a18f0c994afb61769a279ed92ec5ef11a0eb4afb2c16663e02c61db9af3"
         "babe90f1025abed229adabc4e17457c6979408b378c041d31522d6b482da0281ab3f94fd7235bce2")
A7_SHA = "af0a31fc6849a8c2d70bb02ba65bde41e81965a412e675ee1680d3c4516ccb12"

G30 = """0c 0f 0a 08 0a 0f 08 0c 0f 08 0a 0c 9b 92 84 8c bd b6 a5 af d6 db ca c6 f8 f7 e3 ed db ca
0f 0c 08 0a 0f 0a 0c 08 08 0f 0c 0a 92 9b 8c 84 b6 bd af a5 db d6 c6 ca f7 f8 ed e3 ca db
0a 08 0c 0f 08 0c 0a 0f 0a 0c 0f 08 84 8c 9b 92 a5 af bd b6 ca c6 d6 db e3 ed f8 f7 d6 c6"""

# BLAKE3 spec test_vectors.json, unkeyed hash (first 32 bytes), input[i] = i % 251
BLAKE3_SPEC = {
    0: "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    1: "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213",
    1023: "10108970eeda3eb932baac1428c7a2163b0e924c9a9e25b35bba72b28f70bd11",
    1024: "42214739f095a406f3fc83deb889744ac00df831c10daa55189b5d121c855af7",
    1025: "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444",
    2048: "e776b6028c7cd22a4d0ba182a8bf62205d2ef576467e838ed6f2529b85fba24a",
    2049: "5f4d72f40d7a5f82b15ca2b2e44b1de3c2ef86c426c95c1af0b6879522563030",
    3072: "b98cb0ff3623be03326b373de6b9095218513e64f1ee2edd2525c7ad1e5cffd2",
    3073: "7124b49501012f81cc7f11ca069ec9226cecb8a2c850cfe644e327d22d3e1cd3",
    4096: "015094013f57a5277b59d8475c0501042c0b642e531b0a1c8f58d2163229e969",
    4097: "9b4052b38f1c5fc8b1f9ff7ac7b27cd242487b3d890d15c96a1c25b8aa0fb995",
    5120: "9cadc15fed8b5d854562b26a9536d9707cadeda9b143978f319ab34230535833",
    8192: "aae792484c8efe4f19e2ca7d371d8c467ffb10748d8a5a1ae579948f718a2a63",
    31744: "62b6960e1a44bcc1eb1a611a8d6235b6b4b78f32e7abc4fb4c6cdcce94895c47",
    102400: "bc3e3d41a1146b069abffad3c0d44860cf664390afce4d9661f7902e7943e085",
}


def a7_inputs():
    return [np.array([(i * 131 + b * 7 + 3) & 0xFF for b in range(128)], dtype=np.uint8)
            for i in range(30)]


@pytest.mark.parametrize("engine", [0, 1])
def test_appendix_a7_kat(oracle, engine):
    if engine == 1 and not oracle.lib().oracle_have_avx2():
        pytest.skip("no AVX2")
    rec = oracle.encode(a7_inputs(), 3, engine=engine)
    assert [r.tobytes().hex() for r in rec] == [A7_P0, A7_P1, A7_P2]
    assert hashlib.sha256(b"".join(r.tobytes() for r in rec)).hexdigest() == A7_SHA


def test_generator_g30_and_prefix(oracle):
    want = [[int(x, 16) for x in row.split()] for row in G30.splitlines()]
    for k in (30, 20, 8, 5):
        for i in range(k):
            unit = [np.zeros(64, np.uint8) for _ in range(k)]
            unit[i][0] = 1  # symbol 0 of shard i = 1
            rec = oracle.encode(unit, 3)
            for j in range(3):
                sym = int(rec[j][0]) | int(rec[j][32]) << 8
                assert sym == want[j][i], (k, j, i)


def test_exp8_subfield(oracle):
    # exp8[t] = exp[257 t]
    assert [oracle.gf_exp(257 * t) for t in range(9)] == [0x01, 0x7a, 0x47, 0x74, 0x64, 0xdb,
                                                           0x4e, 0x15, 0x56]


def test_tower_identity_for_subfield_coefficients(oracle):
    """SURVEY A.5, used by the subfield kernel form and DESIGN §10's cost
    model: for c < 256 and x = L | H << 8,
    c*x = (m8(c, L ^ G(H)) ^ G(m8(c, H))) | m8(c, H) << 8, with
    G(h) = lo8((h << 8) ^ (h * 0x0100)) (whose high byte is 0)."""
    mul = oracle.gf_mul
    gamma = [((h << 8) ^ mul(h, 0x0100)) for h in range(256)]
    assert all(g >> 8 == 0 for g in gamma)
    rng = np.random.default_rng(5)
    for c in [1, 0x0c, 0x0f, 0x0a, 0x08, 0x9b, 0xd6, 0xf8, 0xff] + rng.integers(2, 256, 8).tolist():
        for x in rng.integers(0, 65536, 400).tolist() + [0, 0xFFFF, 0x0100, 0x00FF]:
            L, H = x & 0xFF, x >> 8
            hi = mul(c, H)
            lo = mul(c, L ^ gamma[H]) ^ gamma[hi]
            assert mul(c, x) == lo | hi << 8, (c, x)


def test_cantor_basis_recurrence(oracle):
    basis = [0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012, 0x6C98, 0x10D8,
             0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E]
    # Cantor element 2^i is basis vector i (log table convention); b_i^2 + b_i = b_{i-1}
    for i in range(1, 16):
        e = 1 << i
        assert oracle.gf_mul(e, e) ^ e == 1 << (i - 1)
    assert len(set(basis)) == 16


def test_rs13_is_replication(oracle):
    # src/filestore/README.md:178; SURVEY §0.4
    rng = np.random.default_rng(1)
    for n in (64, 128, 8_000_000 // 64 * 64 // 1000 * 64, 8000002 % 4096 + 2):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        rec = oracle.encode([d], 3)
        for r in rec:
            assert np.array_equal(r, d)


def test_default_rate_rule(oracle):
    assert oracle.use_high_rate(30, 3) and oracle.use_high_rate(8, 3) and oracle.use_high_rate(20, 3)
    assert not oracle.use_high_rate(1, 3) and not oracle.use_high_rate(2, 3)
    assert oracle.use_high_rate(3, 3) and not oracle.use_high_rate(4, 3)  # risk r2


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 20, 29, 30])
def test_decode_all_erasure_patterns(oracle, k):
    rng = np.random.default_rng(k)
    data = [rng.integers(0, 256, 128, dtype=np.uint8) for _ in range(k)]
    par = oracle.encode(data, 3)
    pats = list(itertools.combinations(range(k + 3), min(3, k)))
    if len(pats) > 800:  # C(33,3) = 5456; sample for runtime
        pats = [pats[i] for i in rng.choice(len(pats), 800, replace=False)]
    for er in pats:
        o = [None if i in er else data[i] for i in range(k)]
        r = [None if (k + j) in er else par[j] for j in range(3)]
        for i, a in oracle.decode(o, r).items():
            assert np.array_equal(a, data[i]), (k, er, i)


def _pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


@pytest.mark.parametrize("k,m", [(3, 3), (4, 3), (2, 2), (7, 5), (8, 8), (6, 8)])
def test_rates_agree_in_the_default_rate_tie(oracle, k, m):
    """Risk r2: DefaultRate's tie-break (next_pow2(k) == next_pow2(m)) picks
    between two rates that give the SAME bytes: both place the k originals in
    one coset of the size-c evaluation subspace and the m recovery shards in
    the neighbouring one, and the additive FFT's translation invariance maps
    one placement onto the other.  Encodes and decodes (including a decode of
    a corrupted, non-codeword recovery shard) agree byte for byte, so the tie
    rule cannot change BlockFrame's parity for a 3- or 4-segment last block."""
    assert _pow2(k) == _pow2(m)
    rng = np.random.default_rng(k * 100 + m)
    data = [rng.integers(0, 256, 192, dtype=np.uint8) for _ in range(k)]
    lo = oracle.encode(data, m, rate=oracle.RATE_LOW)
    hi = oracle.encode(data, m, rate=oracle.RATE_HIGH)
    assert all(np.array_equal(a, b) for a, b in zip(lo, hi))
    bad = [r.copy() for r in lo]
    bad[-1][::5] ^= 0x33
    for er in itertools.islice(itertools.combinations(range(k), min(k, m)), 0, 20):
        o = [None if i in er else data[i] for i in range(k)]
        for rec in (lo, bad):
            a = oracle.decode(o, rec, rate=oracle.RATE_LOW)
            b = oracle.decode(o, rec, rate=oracle.RATE_HIGH)
            assert all(np.array_equal(a[i], b[i]) for i in a), (er,)


def test_rates_differ_outside_the_tie(oracle):
    """The fixture above discriminates: off the tie the two rates' parity
    differs (so agreement in the tie is a property, not a no-op)."""
    rng = np.random.default_rng(9)
    for k, m in ((2, 3), (5, 3), (30, 3), (3, 5)):
        data = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(k)]
        lo = oracle.encode(data, m, rate=oracle.RATE_LOW)
        hi = oracle.encode(data, m, rate=oracle.RATE_HIGH)
        assert not all(np.array_equal(a, b) for a, b in zip(lo, hi)), (k, m)


def test_r2_fixture_reproduces_under_both_rates(oracle):
    """tests/golden/rs_r2.json (labelled r2-dependent) holds RS(3,3) and RS(4,3)
    parity under LowRate and HighRate; the oracle reproduces both, and the
    default rate's bytes are the labelled entry."""
    g = json.load(open(os.path.join(GOLDEN, "rs_r2.json")))
    assert "r2-dependent" in g["label"]
    for c in g["cases"]:
        orig = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in c["originals"]]
        for name, rate in (("low", oracle.RATE_LOW), ("high", oracle.RATE_HIGH)):
            rec = oracle.encode(orig, c["m"], rate=rate)
            assert [r.tobytes().hex() for r in rec] == c["rates"][name]["recovery"]
        dflt = oracle.encode(orig, c["m"])
        assert [r.tobytes().hex() for r in dflt] == c["rates"][c["this_build_default"]]["recovery"]


@pytest.mark.parametrize("k,m", [(3, 5), (7, 5), (5, 9), (3, 6), (6, 16)])
def test_lowrate_zero_padding_is_not_an_erasure(oracle, k, m):
    """LowRate with k not a power of two zero-pads the originals to c; the pad
    is a known zero of the codeword.  Every pattern of up to m erasures must
    round-trip (round 1 marked the pad as erased and lost c-k of the m)."""
    assert not oracle.use_high_rate(k, m) and _pow2(k) != k
    rng = np.random.default_rng(k * 7 + m)
    data = [rng.integers(0, 256, 128, dtype=np.uint8) for _ in range(k)]
    par = oracle.encode(data, m)
    for e in range(1, m + 1):
        for er in itertools.islice(itertools.combinations(range(k + m), e), 0, 60):
            o = [None if i in er else data[i] for i in range(k)]
            if all(x is not None for x in o):
                continue
            r = [None if (k + j) in er else par[j] for j in range(m)]
            if sum(x is not None for x in o + r) < k:
                continue
            for i, a in oracle.decode(o, r).items():
                assert np.array_equal(a, data[i]), (k, m, er, i)


def test_decode_not_enough_shards(oracle):
    data = [np.zeros(64, np.uint8) for _ in range(30)]
    par = oracle.encode(data, 3)
    with pytest.raises(ValueError):
        oracle.decode([None] * 4 + data[4:], par)


def test_avx2_engine_matches_scalar(oracle):
    if not oracle.lib().oracle_have_avx2():
        pytest.skip("no AVX2")
    rng = np.random.default_rng(3)
    for k, n in ((30, 4096), (8, 640), (3, 64), (2, 64)):
        d = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        a = oracle.encode(d, 3, engine=0)
        b = oracle.encode(d, 3, engine=1)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        o = [None, None] + d[2:]
        ra = oracle.decode(o, a, engine=0)
        rb = oracle.decode(o, a, engine=1)
        assert all(np.array_equal(ra[i], rb[i]) for i in ra)


def test_blake3_reference_kat(oracle):
    # src/utils.rs:17-18
    assert oracle.blake3_hex(b"blockframe") == \
        "c41e3ccb398783c24211ecea54ac84c2029d012165392c9deabbef3a597b8fb7"


@pytest.mark.parametrize("n", sorted(BLAKE3_SPEC))
def test_blake3_spec_vectors(oracle, n):
    d = (np.arange(n) % 251).astype(np.uint8)
    assert oracle.blake3_hex(d) == BLAKE3_SPEC[n]


def test_merkle_build_tree(oracle):
    # src/merkle_tree/mod.rs:77-100: parent = blake3(ascii(hex_l ++ hex_r)); odd -> self-pair
    a, b, c = (oracle.blake3_hex(x) for x in (b"a", b"b", b"c"))
    ab = oracle.blake3_hex((a + b).encode())
    cc = oracle.blake3_hex((c + c).encode())
    assert oracle.merkle_root_hex([a, b]) == ab
    assert oracle.merkle_root_hex([a, b, c]) == oracle.blake3_hex((ab + cc).encode())
    assert oracle.merkle_root_hex([a]) == a


def test_golden_small_reproduces(oracle):
    """The committed fixtures are what the (KAT-pinned) oracle produces."""
    g = json.load(open(os.path.join(GOLDEN, "rs_small.json")))
    for c in g["cases"]:
        orig = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in c["originals"]]
        rec = oracle.encode(orig, c["m"])
        assert [r.tobytes().hex() for r in rec] == c["recovery"], (c["k"], c["shard_bytes"])
        for d in c["decodes"]:
            o = [None if i in d["erased"] else orig[i] for i in range(c["k"])]
            r = [None if h is None else np.frombuffer(bytes.fromhex(h), np.uint8)
                 for h in d["recovery_used"]]
            out = oracle.decode(o, r)
            assert {str(i): a.tobytes().hex() for i, a in out.items()} == d["restored"]
            if not d["corrupt_recovery"]:
                for i, a in out.items():
                    assert np.array_equal(a, orig[i])
