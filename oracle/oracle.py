"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end to oracle/liboracle.so (the C restatement of
reed-solomon-simd 3.1.0 and BLAKE3 in rs_oracle.c / blake3_oracle.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: the sanitizer build (make -C oracle sanitize -> liboracle_asan.so)
LIB_PATH = os.path.join(HERE, os.environ.get("ORACLE_LIB", "liboracle.so"))

ENGINE_SCALAR = 0
ENGINE_AVX2 = 1

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(ctypes.c_void_p)
        L.oracle_encode_engine.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_size_t, P, P]
        L.oracle_decode_engine.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_size_t, P, P, P]
        L.oracle_encode_rate.argtypes = [ctypes.c_int] + L.oracle_encode_engine.argtypes
        L.oracle_decode_rate.argtypes = [ctypes.c_int] + L.oracle_decode_engine.argtypes
        L.oracle_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                   ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                   ctypes.c_size_t, P, P, P]
        L.oracle_batch2.argtypes = L.oracle_batch.argtypes + [ctypes.c_int]
        L.oracle_use_high_rate.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_supported.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        for f in ("oracle_gf_exp", "oracle_gf_log"):
            getattr(L, f).argtypes = [ctypes.c_uint16]
            getattr(L, f).restype = ctypes.c_uint16
        L.oracle_gf_mul.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.oracle_gf_mul.restype = ctypes.c_uint16
        L.oracle_skew.argtypes = [ctypes.c_uint32]
        L.oracle_skew.restype = ctypes.c_uint16
        L.oracle_blake3_hex.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_merkle_root_hex.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        _lib = L
    return _lib


def _ptrs(arrs):
    """Array of raw pointers (None -> NULL) for a list of numpy uint8 arrays."""
    out = (ctypes.c_void_p * len(arrs))()
    for i, a in enumerate(arrs):
        out[i] = None if a is None else a.ctypes.data
    return out


def _as_u8(b):
    if b is None:
        return None
    a = np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else b,
                             dtype=np.uint8)
    return a


RATE_DEFAULT, RATE_LOW, RATE_HIGH = -1, 0, 1


def encode(originals, m=3, engine=ENGINE_SCALAR, rate=RATE_DEFAULT):
    """RS(k,m) encode of k equal-length shards -> list of m recovery arrays.
    rate: DefaultRate (the crate's choice) or a forced Low/HighRate (r2 fixtures)."""
    orig = [_as_u8(o) for o in originals]
    k = len(orig)
    n = orig[0].size if k else 0
    rec = [np.zeros(n, dtype=np.uint8) for _ in range(m)]
    rc = lib().oracle_encode_rate(engine, rate, k, m, n, _ptrs(orig), _ptrs(rec))
    if rc != 0:
        raise ValueError(f"oracle_encode rc={rc}")
    return rec


def decode(originals, recovery, engine=ENGINE_SCALAR, rate=RATE_DEFAULT):
    """originals: k entries (None = missing); recovery: m entries (None = missing).
    Returns {index: restored array} for each missing original."""
    orig = [_as_u8(o) for o in originals]
    rec = [_as_u8(r) for r in recovery]
    k, m = len(orig), len(rec)
    present = [a for a in orig + rec if a is not None]
    n = present[0].size
    out = [np.zeros(n, dtype=np.uint8) if o is None else None for o in orig]
    outp = (ctypes.c_void_p * k)()
    for i, a in enumerate(out):
        outp[i] = None if a is None else a.ctypes.data
    rc = lib().oracle_decode_rate(engine, rate, k, m, n, _ptrs(orig), _ptrs(rec), outp)
    if rc != 0:
        raise ValueError(f"oracle_decode rc={rc}")
    return {i: a for i, a in enumerate(out) if a is not None}


def use_high_rate(k, m):
    return bool(lib().oracle_use_high_rate(k, m))


def gf_mul(a, b):
    return int(lib().oracle_gf_mul(a, b))


def gf_exp(i):
    return int(lib().oracle_gf_exp(i))


def gf_log(x):
    return int(lib().oracle_gf_log(x))


def blake3_hex(data) -> str:
    a = _as_u8(data) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)
    buf = ctypes.create_string_buffer(65)
    lib().oracle_blake3_hex(a.ctypes.data if a.size else None, a.size, buf)
    return buf.value.decode()


def merkle_root_hex(leaves) -> str:
    """src/merkle_tree/mod.rs:77-100 over hex-string leaves."""
    cat = "".join(leaves).encode()
    buf = ctypes.create_string_buffer(65)
    rc = lib().oracle_merkle_root_hex(cat, len(leaves), buf)
    if rc != 0:
        raise ValueError("merkle_root_hex failed")
    return buf.value.decode()


def batch(engine, decode_, threads, ks, m, shard_bytes, orig, rec, out, copies=False):
    """Multi-threaded block-parallel driver (CPU baseline).  orig/rec/out are
    per-block lists of numpy arrays (or None).  copies: also make the
    reference wrappers' input/output copies around every block."""
    nb = len(ks)
    keep = []
    def tbl(lists):
        arr = (ctypes.c_void_p * nb)()
        for b, lst in enumerate(lists):
            p = _ptrs(lst)
            keep.append(p)
            arr[b] = ctypes.cast(p, ctypes.c_void_p)
        return arr
    karr = (ctypes.c_uint32 * nb)(*ks)
    rc = lib().oracle_batch2(engine, int(decode_), threads, nb, karr, m, shard_bytes,
                             ctypes.cast(tbl(orig), ctypes.POINTER(ctypes.c_void_p)),
                             ctypes.cast(tbl(rec), ctypes.POINTER(ctypes.c_void_p)),
                             ctypes.cast(tbl(out), ctypes.POINTER(ctypes.c_void_p)),
                             int(copies))
    if rc != 0:
        raise ValueError(f"oracle_batch rc={rc}")
