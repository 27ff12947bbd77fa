"""RS parity as plain polynomial interpolation: a check of the oracle's
additive-FFT machinery that does not use its FFT, its skew factors or its
formal derivative.

reed-solomon-simd 3.1.0 (Leopard-style GF(2^16)) works on
points w_i of the field given, in the crate's representation, by the integer
i itself, and its transforms are:
- IFFT at offset b: from a polynomial's values at w_{b+i} (i < c) to its
  coefficients (degree < c);
- FFT at offset b: from those coefficients to the values at w_{b+i}.

So every recovery symbol follows from Lagrange interpolation alone:
- HighRate, c = next_pow2(m): original i sits at point c + i, zero-padded to
  whole chunks of c. Recovery j (at point j) is the XOR over the chunks of
  the chunk's interpolating polynomial (degree < c) evaluated at j
  (`rs_oracle.c:encode_high`: IFFT of each chunk at its offset, coefficients
  XOR-summed, one FFT at offset 0).
- LowRate, c = next_pow2(k): originals at points 0..k-1, zeros up to c.
  Recovery r is that polynomial evaluated at point c + r (`encode_low`).

This check shares the field tables (log/exp, pinned by App. A.6), the
64-byte lo/hi symbol layout and the rate rule with the oracle.  It shares
nothing of the transform, which is where a misreading of App. A.3 (skew
table, butterfly order, truncation) would hide.  It is test infrastructure
only.  Product-vs-oracle parity is covered by the GPU suite.
"""
import numpy as np
import pytest

ORDER = 65535


@pytest.fixture(scope="module")
def gf(oracle):
    exp = np.array([oracle.gf_exp(i) for i in range(ORDER)], np.int64)
    log = np.zeros(65536, np.int64)
    log[1:] = [oracle.gf_log(x) for x in range(1, 65536)]
    assert all(exp[log[x]] == x for x in (1, 2, 3, 255, 4097, 65535))
    return exp, log


def _symbols(shard):
    """64-byte chunks: bytes 0-31 are the low bytes of 32 symbols, 32-63 the
    high bytes (App. A.1)."""
    b = shard.reshape(-1, 2, 32).astype(np.int64)
    return (b[:, 0, :] | (b[:, 1, :] << 8)).reshape(-1)


def _bytes(sym):
    s = sym.reshape(-1, 32)
    return np.stack([s & 0xFF, s >> 8], axis=1).astype(np.uint8).reshape(-1)


def _lagrange_rows(gf, xs, ys):
    """logs of L_i(y) for y in ys, i over xs: prod_{l != i} (y + x_l) / (x_i + x_l)
    in characteristic 2 (addition is XOR)."""
    exp, log = gf
    xs = np.asarray(xs, np.int64)
    out = np.zeros((len(ys), len(xs)), np.int64)
    for a, y in enumerate(ys):
        for i, x in enumerate(xs):
            others = np.delete(xs, i)
            num = log[y ^ others].sum()
            den = log[x ^ others].sum()
            out[a, i] = (num - den) % ORDER
    return out


def _apply(gf, lrows, values):
    """XOR_i L_i(y) * v_i for every y (values: i x symbols, zeros allowed)."""
    exp, log = gf
    acc = np.zeros((lrows.shape[0], values.shape[1]), np.int64)
    nz = values != 0
    lv = log[values]
    for a in range(lrows.shape[0]):
        for i in range(values.shape[0]):
            prod = np.where(nz[i], exp[(lrows[a, i] + lv[i]) % ORDER], 0)
            acc[a] ^= prod
    return acc


def _next_pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


def interpolated_parity(gf, oracle, originals, m):
    k = len(originals)
    vals = np.stack([_symbols(o) for o in originals])
    if oracle.use_high_rate(k, m):
        c = _next_pow2(m)
        chunks = -(-k // c)
        padded = np.zeros((chunks * c, vals.shape[1]), np.int64)
        padded[:k] = vals
        rec = np.zeros((m, vals.shape[1]), np.int64)
        for q in range(chunks):
            xs = [c + q * c + i for i in range(c)]
            rec ^= _apply(gf, _lagrange_rows(gf, xs, list(range(m))), padded[q * c:(q + 1) * c])
    else:
        c = _next_pow2(k)
        padded = np.zeros((c, vals.shape[1]), np.int64)
        padded[:k] = vals
        rec = _apply(gf, _lagrange_rows(gf, list(range(c)), [c + r for r in range(m)]), padded)
    return [_bytes(r) for r in rec]


@pytest.mark.parametrize("k,m", [(30, 3), (8, 3), (20, 3), (4, 3), (3, 3), (2, 2), (1, 3),
                                 (3, 5), (5, 9), (7, 5), (17, 6), (64, 8), (6, 8)])
def test_oracle_parity_equals_lagrange_interpolation(gf, oracle, k, m):
    rng = np.random.default_rng(1000 * k + m)
    originals = [rng.integers(0, 256, 128, dtype=np.uint8) for _ in range(k)]
    want = interpolated_parity(gf, oracle, originals, m)
    got = oracle.encode(originals, m)
    for j in range(m):
        assert np.array_equal(got[j], want[j]), (k, m, j, oracle.use_high_rate(k, m))


def test_interpolation_check_discriminates(gf, oracle):
    """The check is not vacuous: parity built on the wrong points (original i
    at point i instead of c + i in HighRate) differs from the oracle."""
    rng = np.random.default_rng(5)
    originals = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(8)]
    vals = np.stack([_symbols(o) for o in originals])
    wrong = _apply(gf, _lagrange_rows(gf, list(range(4)), [0, 1, 2]), vals[:4]) ^ \
        _apply(gf, _lagrange_rows(gf, list(range(4, 8)), [0, 1, 2]), vals[4:])
    got = oracle.encode(originals, 3)
    assert not all(np.array_equal(got[j], _bytes(wrong[j])) for j in range(3))


# ---------------------------------------------------------------- decode as linear algebra
def _coef_logs(gf, oracle, k, m):
    """log of the coefficient of original i in recovery j (ORDER: zero):
    recovery_j = XOR_i coef[j][i] * original_i, from the interpolation above."""
    coef = np.full((m, k), ORDER, np.int64)
    if oracle.use_high_rate(k, m):
        c = _next_pow2(m)
        for q in range(-(-k // c)):
            xs = [c + q * c + i for i in range(c)]
            rows = _lagrange_rows(gf, xs, list(range(m)))
            for i in range(c):
                if q * c + i < k:
                    coef[:, q * c + i] = rows[:, i]
    else:
        c = _next_pow2(k)
        rows = _lagrange_rows(gf, list(range(c)), [c + r for r in range(m)])
        coef[:, :] = rows[:, :k]
    return coef


def _mul(gf, la, v):
    """exp(la) * v for a log la (ORDER: zero) and a symbol vector v."""
    exp, log = gf
    if la == ORDER:
        return np.zeros_like(v)
    return np.where(v != 0, exp[(la + log[v]) % ORDER], 0)


def _solve(gf, a_logs, rhs):
    """Gauss-Jordan over GF(2^16): a (e x e, logs, ORDER = 0) x = rhs (e x S)."""
    exp, log = gf
    e = a_logs.shape[0]
    a = np.where(a_logs == ORDER, 0, exp[a_logs % ORDER]).astype(np.int64)
    b = rhs.copy()
    for col in range(e):
        piv = next(r for r in range(col, e) if a[r, col])
        a[[col, piv]], b[[col, piv]] = a[[piv, col]], b[[piv, col]]
        inv = (ORDER - log[a[col, col]]) % ORDER
        a[col] = [0 if x == 0 else exp[(log[x] + inv) % ORDER] for x in a[col]]
        b[col] = _mul(gf, inv, b[col])
        for r in range(e):
            if r != col and a[r, col]:
                f = log[a[r, col]]
                a[r] ^= [0 if x == 0 else exp[(log[x] + f) % ORDER] for x in a[col]]
                b[r] ^= _mul(gf, f, b[col])
    return b


@pytest.mark.parametrize("k,m,erased,use,corrupt", [
    (30, 3, [4, 17, 29], [0, 1, 2], False),
    (30, 3, [0, 9], [2, 0], False),
    (30, 3, [5, 6, 7], [0, 1, 2], True),   # a corrupted (non-codeword) recovery shard
    (8, 3, [1], [1], True),
    (20, 3, [19, 0], [1, 2], False),
    (3, 5, [0, 2], [4, 1], True),          # LowRate
    (5, 9, [1, 2, 4], [8, 0, 3], False),
    (17, 6, [3, 11, 16, 0], [5, 1, 2, 3], True),
])
def test_oracle_decode_equals_linear_solve(gf, oracle, k, m, erased, use, corrupt):
    """With exactly k shards given (the survivors plus as many recovery shards as
    erasures), the restored originals are the unique solution of
    recovery_j = XOR_i coef[j][i] * original_i over the given j, whatever the
    decoder's algorithm (error locator, formal derivative, FFTs).  That holds
    for a corrupted recovery shard too, where the decode returns the
    non-codeword's solution."""
    rng = np.random.default_rng(7 * k + m + len(erased))
    originals = [rng.integers(0, 256, 128, dtype=np.uint8) for _ in range(k)]
    rec = [r.copy() for r in oracle.encode(originals, m)]
    if corrupt:
        rec[use[0]][int(rng.integers(0, 128))] ^= 0xA5
    orig_in = [None if i in erased else originals[i] for i in range(k)]
    rec_in = [rec[j] if j in use else None for j in range(m)]
    got = oracle.decode(orig_in, rec_in)
    coef = _coef_logs(gf, oracle, k, m)
    sym = {i: _symbols(originals[i]) for i in range(k) if i not in erased}
    rhs = []
    for j in use:
        r = _symbols(rec[j])
        for i, v in sym.items():
            r = r ^ _mul(gf, coef[j, i], v)
        rhs.append(r)
    x = _solve(gf, coef[np.ix_(use, erased)], np.stack(rhs))
    for a, i in enumerate(erased):
        assert np.array_equal(got[i], _bytes(x[a])), (k, m, i)
        if not corrupt:
            assert np.array_equal(got[i], originals[i])


def test_golden_fixtures_follow_the_algebra(gf, oracle):
    """The committed fixtures the GPU suite checks the product against
    (tests/golden/rs_small.json): every encode equals the interpolation, and
    every decode given exactly k shards equals the linear solve.  That covers
    the corrupted-recovery decodes and the ragged shard sizes (their tails
    padded into whole 64-byte chunks as App. A.1 lays them out)."""
    import json
    import os
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                        "rs_small.json")))["cases"]

    def chunked(b, n):  # a shard in the 64-byte chunk layout (tail rule of A.1)
        whole, tail = n // 64, n % 64
        out = np.zeros(-(-n // 64) * 64, np.uint8)
        out[:whole * 64] = b[:whole * 64]
        if tail:
            out[whole * 64:whole * 64 + tail // 2] = b[whole * 64:whole * 64 + tail // 2]
            out[whole * 64 + 32:whole * 64 + 32 + tail // 2] = b[whole * 64 + tail // 2:n]
        return out

    def unchunk(c, n):
        whole, tail = n // 64, n % 64
        out = np.zeros(n, np.uint8)
        out[:whole * 64] = c[:whole * 64]
        if tail:
            out[whole * 64:whole * 64 + tail // 2] = c[whole * 64:whole * 64 + tail // 2]
            out[whole * 64 + tail // 2:n] = c[whole * 64 + 32:whole * 64 + 32 + tail // 2]
        return out

    checked_dec = checked_corrupt = 0
    for case in cases:
        k, m, n = case["k"], case["m"], case["shard_bytes"]
        orig = [np.frombuffer(bytes.fromhex(h), np.uint8) for h in case["originals"]]
        want = interpolated_parity(gf, oracle, [chunked(o, n) for o in orig], m)
        assert [unchunk(w, n).tobytes().hex() for w in want] == case["recovery"], (k, m, n)
        coef = _coef_logs(gf, oracle, k, m)
        for d in case["decodes"]:
            er = [i for i in d["erased"] if i < k]  # indices >= k: recovery shards k + j
            use = [j for j, h in enumerate(d["recovery_used"]) if h is not None]
            if len(use) != len(er):
                continue  # more than k shards given: the decoder's choice, not algebra's
            rec = {j: _symbols(chunked(np.frombuffer(bytes.fromhex(d["recovery_used"][j]),
                                                     np.uint8), n)) for j in use}
            sym = {i: _symbols(chunked(orig[i], n)) for i in range(k) if i not in er}
            rhs = []
            for j in use:
                r = rec[j]
                for i, v in sym.items():
                    r = r ^ _mul(gf, coef[j, i], v)
                rhs.append(r)
            x = _solve(gf, coef[np.ix_(use, er)], np.stack(rhs))
            for a, i in enumerate(er):
                assert unchunk(_bytes(x[a]), n).tobytes().hex() == d["restored"][str(i)], \
                    (k, m, n, er)
            checked_dec += 1
            checked_corrupt += bool(d["corrupt_recovery"])
    assert checked_dec >= 60 and checked_corrupt >= 16  # of 21 cases' decodes (r4: 64, 16)


def test_survey_anchors_follow_from_the_algebra(gf, oracle):
    """SURVEY App. A.7's RS(30,3) KAT and A.6's generator G_30, derived from
    the interpolation model alone (points, layout and tables; no oracle
    encode): the model itself agrees with the survey's independent anchors."""
    import hashlib
    from test_oracle import A7_P0, A7_P1, A7_P2, A7_SHA, G30, a7_inputs
    rec = interpolated_parity(gf, oracle, a7_inputs(), 3)
    assert [r.tobytes().hex() for r in rec] == [A7_P0, A7_P1, A7_P2]
    assert hashlib.sha256(b"".join(r.tobytes() for r in rec)).hexdigest() == A7_SHA
    exp, _ = gf
    coef = _coef_logs(gf, oracle, 30, 3)
    want = [[int(x, 16) for x in row.split()] for row in G30.splitlines()]
    assert [[int(exp[c % ORDER]) for c in row] for row in coef] == want
