"""bfrs — Python binding of the MI355X BlockFrame Reed-Solomon C-ABI.

Thin ctypes layer over blockframe-rs_amd/libbfrs.so (include/bfrs.h), used by
the tests and bench.py.  It mirrors the reference's codec surface:

    ReedSolomonEncoder / ReedSolomonDecoder   (reed-solomon-simd 3.1.0, as called at
                                               src/chunker/generate.rs:37-49,84-96 and
                                               src/filestore/recovery.rs:58-69,152-170)
    Chunker.generate_parity(_segmented)       (src/chunker/generate.rs:26-104)
    recover_segment_rs13 / recover_segment_rs30_3  (src/filestore/recovery.rs:43-173)

All arithmetic runs in the HIP kernels of libbfrs.so.  If the library is
missing, import fails loudly; if no GPU is present, every codec call raises
BfrsError(BFRS_E_NO_DEVICE).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import sys
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# BFRS_LIB: another in-tree build of the library (A/B of two builds on one box)
LIB_PATH = os.path.join(os.path.dirname(_HERE), os.environ.get("BFRS_LIB", "libbfrs.so"))

# Error codes (include/bfrs.h)
OK = 0
E_DIFFERENT_SHARD_SIZE = -1
E_DUPLICATE_ORIGINAL_SHARD_INDEX = -2
E_DUPLICATE_RECOVERY_SHARD_INDEX = -3
E_INVALID_ORIGINAL_SHARD_INDEX = -4
E_INVALID_RECOVERY_SHARD_INDEX = -5
E_INVALID_SHARD_SIZE = -6
E_NOT_ENOUGH_SHARDS = -7
E_TOO_FEW_ORIGINAL_SHARDS = -8
E_TOO_MANY_ORIGINAL_SHARDS = -9
E_UNSUPPORTED_SHARD_COUNT = -10
E_WRAPPER = -20
E_INVALID_ARGUMENT = -30
E_HIP = -31
E_NO_DEVICE = -32
E_NOMEM = -33
E_NOT_RESTORED = -34
E_NOT_FOUND = -35

# Every symbol include/bfrs.h declares (tests check the library exports them).
EXPORTS = (
    "bfrs_abi_version", "bfrs_strerror", "bfrs_last_error", "bfrs_device_count", "bfrs_open",
    "bfrs_close", "bfrs_synchronize", "bfrs_shard_pitch",
    "bfrs_use_high_rate", "bfrs_encode_coefficient",
    "bfrs_plan_decode", "bfrs_encoder_new", "bfrs_encoder_add_original_shard",
    "bfrs_encoder_encode", "bfrs_encoder_recovery", "bfrs_encoder_free", "bfrs_decoder_new",
    "bfrs_decoder_add_original_shard", "bfrs_decoder_add_recovery_shard", "bfrs_decoder_decode",
    "bfrs_decoder_restored_original", "bfrs_decoder_free", "bfrs_encode", "bfrs_decode",
    "bfrs_encode_batch_dev", "bfrs_decode_batch_dev", "bfrs_encode_host_batch",
    "bfrs_decode_host_batch", "bfrs_encode_host_batch_multi", "bfrs_decode_host_batch_multi",
    "bfrs_generate_parity",
    "bfrs_generate_parity_segmented", "bfrs_recover_segment_rs13", "bfrs_recover_segment_rs30_3",
    "bfrs_blake3_hex", "bfrs_blake3_batch_dev", "bfrs_blake3_combine", "bfrs_merkle_root_hex", "bfrs_manifest_check", "bfrs_commit", "bfrs_commit_multi", "bfrs_repair", "bfrs_repair_multi", "bfrs_health_check",
    "bfrs_store_list", "bfrs_store_find", "bfrs_batch_health_check", "bfrs_archive_open",
    "bfrs_archive_size", "bfrs_archive_stat", "bfrs_archive_read", "bfrs_archive_stats_get", "bfrs_archive_close",
)

SIZE_MAX = ctypes.c_size_t(-1).value


class BfrsError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


_lib: Optional[ctypes.CDLL] = None

# Live handles, for the ordered close at interpreter exit.
# Left to the garbage collector, objects still alive at exit are finalised in
# no particular order -- a context's __del__ may run before that of an
# archive handle whose prefetch threads still use it -- or not at all, so the
# HIP runtime's own teardown would meet live streams and pinned memory.
import atexit
import weakref

_LIVE_ARCHIVES: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_CODECS: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_CONTEXTS: "weakref.WeakSet" = weakref.WeakSet()


def close_all() -> None:
    """Close every live handle in dependency order: archive handles (their
    prefetch threads are joined), then encoder / decoder objects, then each
    context after a device synchronize.  Registered with atexit; safe to call
    more than once."""
    for a in list(_LIVE_ARCHIVES):
        try:
            a.close()
        except Exception:
            pass
    for o in list(_LIVE_CODECS):
        try:
            o.free()
        except Exception:
            pass
    for c in list(_LIVE_CONTEXTS):
        try:
            if c.handle:
                c.synchronize()
        except Exception:
            pass
        try:
            c.close()
        except Exception:
            pass


atexit.register(close_all)


class RepairReport(ctypes.Structure):
    """bfrs_repair_report (include/bfrs.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("blocks_checked", "segments_checked",
                                               "segments_repaired", "parity_repaired",
                                               "unrecoverable_blocks")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class ArchiveAttr(ctypes.Structure):
    """bfrs_archive_attr (include/bfrs.h)."""
    _fields_ = [("size", ctypes.c_uint64), ("segment_size", ctypes.c_uint64),
                ("segments", ctypes.c_uint64), ("blocks", ctypes.c_uint64),
                ("tier", ctypes.c_int32), ("reserved", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class ArchiveStats(ctypes.Structure):
    """bfrs_archive_stats (include/bfrs.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("hits", "misses", "verified", "recoveries",
                                               "recovered_segments", "bytes_served", "prefetched")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_pp = ctypes.POINTER(ctypes.c_void_p)


def _torch_runtime_first() -> None:
    """Load PyTorch's ROCm runtime before libbfrs.so when torch is installed.

    torch bundles its own HIP/ROCr libraries.  If libbfrs.so (linked against
    /opt/rocm) loads first, the two HIP runtimes end up with separate device
    state and whichever initialises the GPU second sees no device (measured on
    the MI355X boxes: `bfrs.lib(); torch.cuda.is_available(); bfrs.Context(0)`
    fails with BFRS_E_NO_DEVICE).  Loaded in the other order they share the
    process's ROCr and both work, so the binding imports torch first.  Hosts
    without torch (a Rust caller of the C-ABI) are unaffected."""
    import importlib.util
    if "torch" not in sys.modules and importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libbfrs.so not built at {LIB_PATH}; run __graft_entry__.build()")
        _torch_runtime_first()
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "bfrs_abi_version": ([], ctypes.c_int),
            "bfrs_strerror": ([ctypes.c_int], ctypes.c_char_p),
            "bfrs_last_error": ([], ctypes.c_char_p),
            "bfrs_device_count": ([], ctypes.c_int),
            "bfrs_shard_pitch": ([_sz], _sz),
            "bfrs_open": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
            "bfrs_close": ([_vp], None),
            "bfrs_synchronize": ([_vp], ctypes.c_int),
            "bfrs_use_high_rate": ([_sz, _sz], ctypes.c_int),
            "bfrs_encode_coefficient": ([_sz, _sz, _sz, _sz, ctypes.POINTER(ctypes.c_uint16)],
                                        ctypes.c_int),
            "bfrs_plan_decode": ([_sz, _sz, _vp, _vp, _vp, _sz, ctypes.POINTER(_sz),
                                  ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_encoder_new": ([_vp, _sz, _sz, _sz, ctypes.POINTER(_vp)], ctypes.c_int),
            "bfrs_encoder_add_original_shard": ([_vp, _vp, _sz], ctypes.c_int),
            "bfrs_encoder_encode": ([_vp], ctypes.c_int),
            "bfrs_encoder_recovery": ([_vp, _sz, ctypes.POINTER(_vp), ctypes.POINTER(_sz)],
                                      ctypes.c_int),
            "bfrs_encoder_free": ([_vp], None),
            "bfrs_decoder_new": ([_vp, _sz, _sz, _sz, ctypes.POINTER(_vp)], ctypes.c_int),
            "bfrs_decoder_add_original_shard": ([_vp, _sz, _vp, _sz], ctypes.c_int),
            "bfrs_decoder_add_recovery_shard": ([_vp, _sz, _vp, _sz], ctypes.c_int),
            "bfrs_decoder_decode": ([_vp], ctypes.c_int),
            "bfrs_decoder_restored_original": ([_vp, _sz, ctypes.POINTER(_vp),
                                                ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_decoder_free": ([_vp], None),
            "bfrs_encode": ([_vp, _sz, _sz, _sz, _pp, _pp], ctypes.c_int),
            "bfrs_decode": ([_vp, _sz, _sz, _sz, _pp, _pp, _pp], ctypes.c_int),
            "bfrs_encode_batch_dev": ([_vp, _sz, ctypes.POINTER(ctypes.c_uint32), _sz, _sz, _pp,
                                       _pp, _vp], ctypes.c_int),
            "bfrs_decode_batch_dev": ([_vp, _sz, ctypes.POINTER(ctypes.c_uint32), _sz, _sz, _pp,
                                       _pp, _pp, _vp], ctypes.c_int),
            "bfrs_encode_host_batch": ([_vp, _sz, ctypes.POINTER(ctypes.c_uint32), _sz, _sz, _pp,
                                        _pp], ctypes.c_int),
            "bfrs_decode_host_batch": ([_vp, _sz, ctypes.POINTER(ctypes.c_uint32), _sz, _sz, _pp,
                                        _pp, _pp], ctypes.c_int),
            "bfrs_encode_host_batch_multi": ([_pp, _sz, _sz, ctypes.POINTER(ctypes.c_uint32), _sz,
                                              _sz, _pp, _pp], ctypes.c_int),
            "bfrs_decode_host_batch_multi": ([_pp, _sz, _sz, ctypes.POINTER(ctypes.c_uint32), _sz,
                                              _sz, _pp, _pp, _pp], ctypes.c_int),
            "bfrs_commit_multi": ([_pp, _sz, ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.c_int,
                                   ctypes.c_char_p, _sz], ctypes.c_int),
            "bfrs_generate_parity": ([_vp, _pp, ctypes.POINTER(_sz), _sz, _sz, _sz, _pp,
                                      ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_generate_parity_segmented": ([_vp, _vp, _sz, _pp, ctypes.POINTER(_sz)],
                                               ctypes.c_int),
            "bfrs_recover_segment_rs13": ([_vp, _pp, ctypes.POINTER(_sz), _sz, _sz, _vp,
                                           ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_recover_segment_rs30_3": ([_vp, _pp, ctypes.POINTER(_sz), _sz, _pp,
                                             ctypes.POINTER(_sz), _sz, _sz, _vp,
                                             ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_blake3_hex": ([_vp, _sz, ctypes.c_int, ctypes.c_char_p], ctypes.c_int),
            "bfrs_blake3_batch_dev": ([_vp, _sz, _pp, ctypes.POINTER(_sz), _vp, _vp, _vp, _vp],
                                      ctypes.c_int),
            "bfrs_blake3_combine": ([_vp, _sz, ctypes.c_char_p], ctypes.c_int),
            "bfrs_merkle_root_hex": ([ctypes.c_char_p, _sz, ctypes.c_char_p], ctypes.c_int),
            "bfrs_manifest_check": ([ctypes.c_char_p, _sz, ctypes.POINTER(ctypes.c_int),
                                     ctypes.c_char_p, _sz, ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_commit": ([_vp, ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.c_int,
                             ctypes.c_char_p, _sz],
                            ctypes.c_int),
            "bfrs_health_check": ([_vp, ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)],
                                  ctypes.c_int),
            "bfrs_repair": ([_vp, ctypes.c_char_p, ctypes.POINTER(RepairReport)], ctypes.c_int),
            "bfrs_repair_multi": ([_pp, _sz, ctypes.c_char_p, ctypes.POINTER(RepairReport)],
                                  ctypes.c_int),
            "bfrs_store_list": ([ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)],
                                ctypes.c_int),
            "bfrs_store_find": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, _sz,
                                 ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_batch_health_check": ([_vp, ctypes.c_char_p, ctypes.c_char_p, _sz,
                                         ctypes.POINTER(_sz)], ctypes.c_int),
            "bfrs_archive_open": ([_vp, ctypes.c_char_p, _sz, ctypes.c_int, ctypes.POINTER(_vp)],
                                  ctypes.c_int),
            "bfrs_archive_size": ([_vp, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "bfrs_archive_stat": ([ctypes.c_char_p, ctypes.POINTER(ArchiveAttr)], ctypes.c_int),
            "bfrs_archive_read": ([_vp, ctypes.c_uint64, _sz, _vp, ctypes.POINTER(_sz)],
                                  ctypes.c_int),
            "bfrs_archive_stats_get": ([_vp, ctypes.POINTER(ArchiveStats)], ctypes.c_int),
            "bfrs_archive_close": ([_vp], None),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != OK:
        msg = lib().bfrs_last_error().decode(errors="replace")
        raise BfrsError(rc, msg or lib().bfrs_strerror(rc).decode())


def _ptr_array(ptrs: Sequence[Optional[int]]):
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return ctypes.cast(arr, _pp), arr


def _host_ptr(buf) -> int:
    """Address of a host buffer (bytes / bytearray / numpy array)."""
    import numpy as np
    if isinstance(buf, np.ndarray):
        if not buf.flags.c_contiguous:
            raise ValueError("host buffer must be C-contiguous")
        return buf.ctypes.data
    if isinstance(buf, bytes):
        return ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    if isinstance(buf, bytearray):
        return ctypes.addressof((ctypes.c_char * len(buf)).from_buffer(buf))
    raise TypeError(f"unsupported host buffer type {type(buf)}")


def _out_nbytes(buf) -> int:
    """Size of a writable output buffer (numpy array or bytearray)."""
    import numpy as np
    if isinstance(buf, np.ndarray):
        if not buf.flags.writeable:  # e.g. np.frombuffer(bytes): the library would write into it
            raise ValueError("output buffer is read-only")
        return buf.nbytes
    if isinstance(buf, bytearray):
        return len(buf)
    raise TypeError(f"output buffer must be a numpy array or bytearray, not {type(buf)}")


def _as_np(buf):
    import numpy as np
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def use_high_rate(original_count: int, recovery_count: int) -> bool:
    rc = lib().bfrs_use_high_rate(original_count, recovery_count)
    if rc < 0:
        raise BfrsError(rc, "unsupported shard count")
    return rc == 1


def encode_coefficient(k: int, m: int, j: int, i: int) -> int:
    c = ctypes.c_uint16()
    _check(lib().bfrs_encode_coefficient(k, m, j, i, ctypes.byref(c)))
    return c.value


def plan_decode(k: int, m: int, orig_present, rec_present):
    """Decode coefficient matrix (rows = missing originals, cols = present
    recovery then present originals) as a list of lists."""
    op = (ctypes.c_uint8 * k)(*[1 if x else 0 for x in orig_present])
    rp = (ctypes.c_uint8 * m)(*[1 if x else 0 for x in rec_present])
    rows, cols = _sz(), _sz()
    _check(lib().bfrs_plan_decode(k, m, op, rp, None, 0, ctypes.byref(rows), ctypes.byref(cols)))
    n = rows.value * cols.value
    buf = (ctypes.c_uint16 * max(1, n))()
    _check(lib().bfrs_plan_decode(k, m, op, rp, buf, n, ctypes.byref(rows), ctypes.byref(cols)))
    return [[buf[r * cols.value + c] for c in range(cols.value)] for r in range(rows.value)]


def device_count() -> int:
    return int(lib().bfrs_device_count())


def shard_pitch(shard_bytes: int) -> int:
    """bfrs_shard_pitch: byte distance between consecutive shards of one allocation."""
    return int(lib().bfrs_shard_pitch(shard_bytes))


def empty_shards(n: int, shard_bytes: int, device="cuda"):
    """n shards of shard_bytes as rows of one device allocation, shard_pitch apart.

    Returns a (n, shard_bytes) uint8 view with row stride shard_pitch(shard_bytes):
    one column of many 32 MiB shards then spreads over the HBM channels
     instead of aliasing onto the same ones."""
    import torch
    pitch = shard_pitch(shard_bytes)
    buf = torch.empty(max(1, n * pitch), dtype=torch.uint8, device=device)
    return buf.as_strided((n, shard_bytes), (pitch, 1))


class Context:
    """A bfrs_ctx on one HIP device (no CPU fallback)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().bfrs_open(device, ctypes.byref(h)))
        self.handle = h
        self.device = device
        _LIVE_CONTEXTS.add(self)

    def close(self) -> None:
        """bfrs_close: archive handles still open on the context are detached
        by the library (their threads joined; later reads fail), codec objects
        stay valid to free."""
        if self.handle:
            lib().bfrs_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self) -> None:
        _check(lib().bfrs_synchronize(self.handle))

    # ---- device-resident batch API (torch tensors or raw device addresses)
    @staticmethod
    def _addr(t) -> Optional[int]:
        if t is None:
            return None
        return t if isinstance(t, int) else t.data_ptr()

    def encode_batch_dev(self, original_counts, recovery_count, shard_bytes, d_originals,
                         d_recovery, stream=None) -> None:
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._addr(t) for t in d_originals])
        pr, kr = _ptr_array([self._addr(t) for t in d_recovery])
        _check(lib().bfrs_encode_batch_dev(self.handle, len(original_counts), ks, recovery_count,
                                           shard_bytes, po, pr,
                                           _stream_handle(stream, list(d_originals) + list(d_recovery))))

    def decode_batch_dev(self, original_counts, recovery_count, shard_bytes, d_originals,
                         d_recovery, d_restored, stream=None) -> None:
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._addr(t) for t in d_originals])
        pr, kr = _ptr_array([self._addr(t) for t in d_recovery])
        pd, kd = _ptr_array([self._addr(t) for t in d_restored])
        _check(lib().bfrs_decode_batch_dev(self.handle, len(original_counts), ks, recovery_count,
                                           shard_bytes, po, pr, pd,
                                           _stream_handle(stream, list(d_originals) + list(d_recovery)
                                                          + list(d_restored))))

    def prepare_encode(self, original_counts, recovery_count, shard_bytes, d_originals,
                       d_recovery):
        """Pre-built argument arrays for repeated bfrs_encode_batch_dev calls on
        the same buffers (bench loops); returns f(stream_handle)."""
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._addr(t) for t in d_originals])
        pr, kr = _ptr_array([self._addr(t) for t in d_recovery])
        fn, h, n = lib().bfrs_encode_batch_dev, self.handle, len(original_counts)

        def call(stream_handle=None, _keep=(ks, ko, kr)):
            _check(fn(h, n, ks, recovery_count, shard_bytes, po, pr, stream_handle))
        return call

    def prepare_decode(self, original_counts, recovery_count, shard_bytes, d_originals,
                       d_recovery, d_restored):
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._addr(t) for t in d_originals])
        pr, kr = _ptr_array([self._addr(t) for t in d_recovery])
        pd, kd = _ptr_array([self._addr(t) for t in d_restored])
        fn, h, n = lib().bfrs_decode_batch_dev, self.handle, len(original_counts)

        def call(stream_handle=None, _keep=(ks, ko, kr, kd)):
            _check(fn(h, n, ks, recovery_count, shard_bytes, po, pr, pd, stream_handle))
        return call

    def blake3_batch_dev(self, d_msgs, lens=None, stream=None, with_cvs=False,
                         chunk_offsets=None):
        """BLAKE3 of device messages (torch uint8 tensors, or addresses with
        `lens`).  Returns hex digests, plus 32-byte subtree CVs if with_cvs;
        chunk_offsets places each message inside an enclosing one (CVs)."""
        import numpy as np
        n = len(d_msgs)
        if lens is None:
            lens = [t.numel() for t in d_msgs]
        pm, km = _ptr_array([self._addr(t) if l else None for t, l in zip(d_msgs, lens)])
        ls = (_sz * max(1, n))(*lens)
        dig = np.zeros(max(1, n) * 32, np.uint8)
        cvs = np.zeros(max(1, n) * 32, np.uint8) if with_cvs else None
        offs = None if chunk_offsets is None else (ctypes.c_uint64 * max(1, n))(*chunk_offsets)
        _check(lib().bfrs_blake3_batch_dev(self.handle, n, pm, ls, offs, dig.ctypes.data,
                                           cvs.ctypes.data if with_cvs else None,
                                           _stream_handle(stream, [t for t in d_msgs
                                                                   if not isinstance(t, int)])))
        hexes = [dig[32 * i:32 * i + 32].tobytes().hex() for i in range(n)]
        if with_cvs:
            return hexes, [cvs[32 * i:32 * i + 32].tobytes() for i in range(n)]
        return hexes

    def blake3_batch_dev_call(self, d_msgs, stream=None):
        """bfrs_blake3_batch_dev with its arguments marshalled once: returns
        (call, digests), where call() hashes the same device messages again
        into the numpy array digests (n x 32 bytes) and raises BfrsError on
        failure.  For timing the library call without Python's per-call
        marshalling (bench.py); the tensors must outlive call."""
        import numpy as np
        n = len(d_msgs)
        lens = [t.numel() for t in d_msgs]
        pm, km = _ptr_array([self._addr(t) if l else None for t, l in zip(d_msgs, lens)])
        ls = (_sz * max(1, n))(*lens)
        dig = np.zeros((max(1, n), 32), np.uint8)
        st = _stream_handle(stream, list(d_msgs))
        fn, h, out = lib().bfrs_blake3_batch_dev, self.handle, dig.ctypes.data

        def call(_keep=(km, ls, dig)):
            # _keep: the pointer arrays AND the digest array `out` points into
            # stay alive as long as call does, whatever the caller keeps
            _check(fn(h, n, pm, ls, None, out, None, st))
        return call, dig[:n]

    # ---- host-memory batch API (host buffers: numpy arrays or CPU torch tensors)
    @staticmethod
    def _haddr(t) -> Optional[int]:
        if t is None:
            return None
        if isinstance(t, int):
            return t
        if hasattr(t, "data_ptr"):
            return t.data_ptr()
        return _host_ptr(t)

    @staticmethod
    def _check_host_bufs(bufs, shard_bytes, writable, what):
        """The C-ABI takes bare pointers: every host buffer the binding passes
        must hold shard_bytes contiguous bytes (and be writable for outputs)."""
        import numpy as np
        for t in bufs:
            if t is None or isinstance(t, int):
                continue
            if hasattr(t, "data_ptr"):  # CPU torch tensor
                if t.device.type != "cpu" or not t.is_contiguous():
                    raise ValueError(f"{what}: host tensors must be contiguous CPU tensors")
                n = t.numel() * t.element_size()
            elif isinstance(t, np.ndarray):
                if writable and not t.flags.writeable:
                    raise ValueError(f"{what}: output buffer is read-only")
                n = t.nbytes
            elif isinstance(t, (bytes, bytearray)):
                if writable and isinstance(t, bytes):
                    raise ValueError(f"{what}: output buffer is read-only (bytes)")
                n = len(t)
            else:
                raise TypeError(f"{what}: unsupported host buffer type {type(t)}")
            if n < shard_bytes:
                raise ValueError(f"{what}: buffer of {n} bytes < shard_bytes {shard_bytes}")

    def encode_host_batch(self, original_counts, recovery_count, shard_bytes, originals,
                          recovery_out) -> None:
        self._check_host_bufs(originals, shard_bytes, False, "encode_host_batch")
        self._check_host_bufs(recovery_out, shard_bytes, True, "encode_host_batch")
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._haddr(t) for t in originals])
        pr, kr = _ptr_array([self._haddr(t) for t in recovery_out])
        _check(lib().bfrs_encode_host_batch(self.handle, len(original_counts), ks, recovery_count,
                                            shard_bytes, po, pr))

    def decode_host_batch(self, original_counts, recovery_count, shard_bytes, originals,
                          recovery, restored_out) -> None:
        self._check_host_bufs(list(originals) + list(recovery), shard_bytes, False,
                              "decode_host_batch")
        self._check_host_bufs(restored_out, shard_bytes, True, "decode_host_batch")
        ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
        po, ko = _ptr_array([self._haddr(t) for t in originals])
        pr, kr = _ptr_array([self._haddr(t) for t in recovery])
        pd, kd = _ptr_array([self._haddr(t) for t in restored_out])
        _check(lib().bfrs_decode_host_batch(self.handle, len(original_counts), ks, recovery_count,
                                            shard_bytes, po, pr, pd))

    # ---- one-shot host API (numpy in, numpy out)
    def encode(self, originals, recovery_count=3):
        import numpy as np
        orig = [_as_np(o) for o in originals]
        n = orig[0].size
        rec = [np.empty(n, dtype=np.uint8) for _ in range(recovery_count)]
        po, ko = _ptr_array([o.ctypes.data for o in orig])
        pr, kr = _ptr_array([r.ctypes.data for r in rec])
        _check(lib().bfrs_encode(self.handle, len(orig), recovery_count, n, po, pr))
        return rec

    def decode(self, originals, recovery):
        import numpy as np
        orig = [None if o is None else _as_np(o) for o in originals]
        rec = [None if r is None else _as_np(r) for r in recovery]
        n = next(a.size for a in orig + rec if a is not None)
        out = [np.empty(n, dtype=np.uint8) if o is None else None for o in orig]
        po, ko = _ptr_array([None if o is None else o.ctypes.data for o in orig])
        pr, kr = _ptr_array([None if r is None else r.ctypes.data for r in rec])
        pd, kd = _ptr_array([None if a is None else a.ctypes.data for a in out])
        _check(lib().bfrs_decode(self.handle, len(orig), len(rec), n, po, pr, pd))
        return {i: a for i, a in enumerate(out) if a is not None}


def _stream_handle(stream, tensors=()) -> Optional[int]:
    """None -> torch's current stream when torch tensors are passed (so the
    codec is ordered after the kernels that produced them), else HIP's
    default stream (the C-ABI's NULL)."""
    if stream is None:
        if any(hasattr(t, "data_ptr") for t in tensors):
            import torch
            return torch.cuda.current_stream().cuda_stream
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


def _live_codec(obj):
    """The object's handle; its context must still be open (include/bfrs.h:
    a codec object may only be freed after bfrs_close)."""
    if not getattr(obj, "handle", None):
        raise BfrsError(E_INVALID_ARGUMENT, "codec object already freed")
    if not obj.ctx.handle:
        raise BfrsError(E_INVALID_ARGUMENT, "the codec object's context is closed")
    return obj.handle


def _view(fn, owner, index):
    """A read-only numpy view of a codec object's pinned row.  The view keeps
    `owner` (the encoder / decoder) alive: the row belongs to the object's
    codec slot, which goes back to the pool (or is freed) when the object is
    freed, so a view that outlived its object would read another object's
    bytes or freed memory."""
    import numpy as np
    p, n = ctypes.c_void_p(), _sz()
    _check(fn(owner._h(), index, ctypes.byref(p), ctypes.byref(n)))
    buf = (ctypes.c_uint8 * n.value).from_address(p.value)
    buf._bfrs_owner = owner  # the array's base is buf, buf holds the object
    a = np.frombuffer(buf, dtype=np.uint8)
    a.flags.writeable = False
    return a


class ReedSolomonEncoder:
    """reed_solomon_simd::ReedSolomonEncoder over the HIP path."""

    def __init__(self, ctx: Context, original_count: int, recovery_count: int, shard_bytes: int):
        h = ctypes.c_void_p()
        _check(lib().bfrs_encoder_new(ctx.handle, original_count, recovery_count, shard_bytes,
                                      ctypes.byref(h)))
        self.handle, self.ctx, self.recovery_count = h, ctx, recovery_count
        _LIVE_CODECS.add(self)

    def free(self) -> None:
        if getattr(self, "handle", None):
            lib().bfrs_encoder_free(self.handle)
            self.handle = None

    def __del__(self):
        self.free()

    def _h(self):
        return _live_codec(self)

    def add_original_shard(self, shard) -> None:
        a = _as_np(shard)
        _check(lib().bfrs_encoder_add_original_shard(self._h(), a.ctypes.data, a.size))

    def encode(self) -> "ReedSolomonEncoder":
        _check(lib().bfrs_encoder_encode(self._h()))
        return self

    def recovery_view(self, index: int):
        """Recovery shard `index` as a read-only numpy view of the encoder's
        pinned row (valid until the next call on this encoder), no copy."""
        return _view(lib().bfrs_encoder_recovery, self, index)

    def recovery_iter(self):
        for j in range(self.recovery_count):
            p, n = ctypes.c_void_p(), _sz()
            _check(lib().bfrs_encoder_recovery(self._h(), j, ctypes.byref(p), ctypes.byref(n)))
            yield ctypes.string_at(p, n.value)


class ReedSolomonDecoder:
    """reed_solomon_simd::ReedSolomonDecoder over the HIP path."""

    def __init__(self, ctx: Context, original_count: int, recovery_count: int, shard_bytes: int):
        h = ctypes.c_void_p()
        _check(lib().bfrs_decoder_new(ctx.handle, original_count, recovery_count, shard_bytes,
                                      ctypes.byref(h)))
        self.handle, self.ctx = h, ctx
        _LIVE_CODECS.add(self)

    def free(self) -> None:
        if getattr(self, "handle", None):
            lib().bfrs_decoder_free(self.handle)
            self.handle = None

    def __del__(self):
        self.free()

    def _h(self):
        return _live_codec(self)

    def add_original_shard(self, index: int, shard) -> None:
        a = _as_np(shard)
        _check(lib().bfrs_decoder_add_original_shard(self._h(), index, a.ctypes.data, a.size))

    def add_recovery_shard(self, index: int, shard) -> None:
        a = _as_np(shard)
        _check(lib().bfrs_decoder_add_recovery_shard(self._h(), index, a.ctypes.data, a.size))

    def decode(self) -> "ReedSolomonDecoder":
        _check(lib().bfrs_decoder_decode(self._h()))
        return self

    def restored_view(self, index: int):
        """Restored original `index` as a read-only numpy view (valid until the
        next add/decode call), or None if it was not restored."""
        try:
            return _view(lib().bfrs_decoder_restored_original, self, index)
        except BfrsError as e:
            if e.code == E_NOT_RESTORED:
                return None
            raise

    def restored_original(self, index: int) -> Optional[bytes]:
        p, n = ctypes.c_void_p(), _sz()
        rc = lib().bfrs_decoder_restored_original(self._h(), index, ctypes.byref(p),
                                                  ctypes.byref(n))
        if rc == E_NOT_RESTORED:
            return None
        _check(rc)
        return ctypes.string_at(p, n.value)


class Chunker:
    """The codec-facing part of src/chunker (generate.rs)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def generate_parity(self, segments, data_shards: int, parity_shards: int):
        import numpy as np
        segs = [_as_np(s) for s in segments]
        maxlen = max((s.size for s in segs), default=0)
        outs = [np.empty(maxlen, dtype=np.uint8) for _ in range(parity_shards)]
        self.generate_parity_into(segs, data_shards, parity_shards, outs)
        return [o.tobytes() for o in outs]

    def generate_parity_into(self, segments, data_shards: int, parity_shards: int, outs) -> int:
        """generate_parity writing into caller buffers (each >= the longest
        segment), as a Rust caller of the C-ABI would; returns the parity length."""
        segs = [_as_np(s) for s in segments]
        if len(outs) < parity_shards or any(
                _out_nbytes(o) < max((s.size for s in segs), default=0) for o in outs):
            raise ValueError("generate_parity_into: output buffers too small")
        ps, ks = _ptr_array([s.ctypes.data if s.size else None for s in segs])
        lens = (_sz * max(1, len(segs)))(*[s.size for s in segs])
        po, ko = _ptr_array([_host_ptr(o) for o in outs])
        plen = _sz()
        _check(lib().bfrs_generate_parity(self.ctx.handle, ps, lens, len(segs), data_shards,
                                          parity_shards, po, ctypes.byref(plen)))
        return plen.value

    def generate_parity_segmented(self, segment_data):
        import numpy as np
        a = _as_np(segment_data)
        padded = (a.size + 63) // 64 * 64
        outs = [np.empty(max(1, padded), dtype=np.uint8) for _ in range(3)]
        po, ko = _ptr_array([o.ctypes.data for o in outs])
        plen = _sz()
        _check(lib().bfrs_generate_parity_segmented(self.ctx.handle,
                                                    a.ctypes.data if a.size else None, a.size,
                                                    po, ctypes.byref(plen)))
        return [o[:plen.value].tobytes() for o in outs]


def recover_segment_rs13(ctx: Context, parity_shards, expected_size: Optional[int] = None) -> bytes:
    """src/filestore/recovery.rs:43-79"""
    import numpy as np
    ps = [_as_np(p) for p in parity_shards]
    n = max((p.size for p in ps), default=0)
    out = np.empty(max(1, n), dtype=np.uint8)
    pp, kp = _ptr_array([p.ctypes.data for p in ps])
    lens = (_sz * max(1, len(ps)))(*[p.size for p in ps])
    olen = _sz()
    _check(lib().bfrs_recover_segment_rs13(ctx.handle, pp, lens, len(ps),
                                           SIZE_MAX if expected_size is None else expected_size,
                                           out.ctypes.data, ctypes.byref(olen)))
    return out[:olen.value].tobytes()


def recover_segment_rs30_3(ctx: Context, valid_segments, block_parity, target_index: int) -> bytes:
    """src/filestore/recovery.rs:118-173 (valid_segments: 30 slots, None = missing)."""
    import numpy as np
    segs = [None if s is None else _as_np(s) for s in valid_segments]
    par = [_as_np(p) for p in block_parity]
    sizes = [s.size for s in segs if s is not None] + [p.size for p in par]
    out = np.empty(max(1, max(sizes, default=0)), dtype=np.uint8)
    n = recover_segment_rs30_3_into(ctx, segs, par, target_index, out)
    return out[:n].tobytes()


def recover_segment_rs30_3_into(ctx: Context, valid_segments, block_parity, target_index: int,
                                out) -> int:
    """recover_segment_rs30_3 writing into a caller buffer (>= the largest
    shard), as a Rust caller of the C-ABI would; returns the restored length."""
    segs = [None if s is None else _as_np(s) for s in valid_segments]
    par = [_as_np(p) for p in block_parity]
    n = max([s.size for s in segs if s is not None] + [p.size for p in par], default=0)
    if _out_nbytes(out) < n:
        raise ValueError("recover_segment_rs30_3_into: output buffer too small")
    ps, ks = _ptr_array([None if s is None else s.ctypes.data for s in segs])
    slens = (_sz * max(1, len(segs)))(*[0 if s is None else s.size for s in segs])
    pp, kp = _ptr_array([p.ctypes.data for p in par])
    plens = (_sz * max(1, len(par)))(*[p.size for p in par])
    olen = _sz()
    _check(lib().bfrs_recover_segment_rs30_3(ctx.handle, ps, slens, len(segs), pp, plens,
                                             len(par), target_index, _host_ptr(out),
                                             ctypes.byref(olen)))
    return olen.value


# ---- integrity helpers + archive pipeline (src/utils.rs, src/merkle_tree,
# src/chunker/commit.rs, src/filestore/health.rs, src/mount) ----------------

def blake3_hex(data, threads: int = 1) -> str:
    """blake3_hash_bytes (src/utils.rs:22-28)."""
    a = _as_np(data)
    out = ctypes.create_string_buffer(65)
    _check(lib().bfrs_blake3_hex(a.ctypes.data if a.size else None, a.size, threads, out))
    return out.value.decode()


def blake3_combine(cvs) -> str:
    """Digest of a message from the subtree CVs (32 bytes each) of its parts."""
    raw = b"".join(bytes(c) for c in cvs)
    out = ctypes.create_string_buffer(65)
    _check(lib().bfrs_blake3_combine(raw, len(raw) // 32, out))
    return out.value.decode()


def merkle_root_hex(leaves) -> str:
    """MerkleTree::from_hashes(leaves).get_root() (src/merkle_tree/mod.rs:56-100)."""
    leaves = list(leaves)
    if any(len(h) != 64 for h in leaves):
        raise ValueError("leaves must be 64-char hex digests")
    out = ctypes.create_string_buffer(65)
    _check(lib().bfrs_merkle_root_hex("".join(leaves).encode(), len(leaves), out))
    return out.value.decode()


def archive_stat(archive_dir: str) -> dict:
    """The mount's getattr geometry of an archive (src/mount/filesystem_unix.rs:
    153-174): size, tier, segment_size, segments, blocks.  Host only."""
    a = ArchiveAttr()
    _check(lib().bfrs_archive_stat(os.fsencode(archive_dir), ctypes.byref(a)))
    return a.as_dict()


def manifest_check(text) -> tuple:
    """ManifestFile::new + validate (src/merkle_tree/manifest.rs:47-88).
    Returns (valid, canonical_json)."""
    raw = text.encode() if isinstance(text, str) else bytes(text)
    valid, need = ctypes.c_int(), _sz()
    _check(lib().bfrs_manifest_check(raw, len(raw), ctypes.byref(valid), None, 0,
                                     ctypes.byref(need)))
    out = ctypes.create_string_buffer(need.value)
    _check(lib().bfrs_manifest_check(raw, len(raw), ctypes.byref(valid), out, len(out),
                                     ctypes.byref(need)))
    return bool(valid.value), out.value.decode()


def commit(ctx, file_path: str, archive_root: str, segment_size: int = 0,
           tier: int = 0) -> str:
    """Chunker::commit (src/chunker/commit.rs:593-613); tier 1/2/3 forces
    commit_tiny/commit_segmented/commit_blocked.  Returns the archive directory.
    `ctx` may be a list of contexts (one per device): bfrs_commit_multi deals a
    tier-3 file's blocks over them from this one process (commit.rs:391-393)."""
    out = ctypes.create_string_buffer(4096)
    if isinstance(ctx, (list, tuple)):
        pc, kc = _ctx_array(ctx)
        _check(lib().bfrs_commit_multi(pc, len(ctx), os.fsencode(file_path),
                                       os.fsencode(archive_root), segment_size, tier, out,
                                       len(out)))
    else:
        _check(lib().bfrs_commit(ctx.handle, os.fsencode(file_path), os.fsencode(archive_root),
                                 segment_size, tier, out, len(out)))
    return out.value.decode()


def _ctx_array(ctxs):
    for c in ctxs:
        if not isinstance(c, Context) or not c.handle:
            raise BfrsError(E_INVALID_ARGUMENT, "a context of the list is closed or not a Context")
    return _ptr_array([c.handle.value if isinstance(c.handle, ctypes.c_void_p) else c.handle
                       for c in ctxs])


def encode_host_batch_multi(ctxs, original_counts, recovery_count, shard_bytes, originals,
                            recovery_out) -> None:
    """bfrs_encode_host_batch_multi: one host-memory batch over several contexts
    (normally one per device) from this process, context d taking the 64-B
    column stripe d of every shard (include/bfrs.h)."""
    Context._check_host_bufs(originals, shard_bytes, False, "encode_host_batch_multi")
    Context._check_host_bufs(recovery_out, shard_bytes, True, "encode_host_batch_multi")
    pc, kc = _ctx_array(ctxs)
    ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
    po, ko = _ptr_array([Context._haddr(t) for t in originals])
    pr, kr = _ptr_array([Context._haddr(t) for t in recovery_out])
    _check(lib().bfrs_encode_host_batch_multi(pc, len(ctxs), len(original_counts), ks,
                                              recovery_count, shard_bytes, po, pr))


def decode_host_batch_multi(ctxs, original_counts, recovery_count, shard_bytes, originals,
                            recovery, restored_out) -> None:
    """bfrs_decode_host_batch_multi (see encode_host_batch_multi)."""
    Context._check_host_bufs(list(originals) + list(recovery), shard_bytes, False,
                             "decode_host_batch_multi")
    Context._check_host_bufs(restored_out, shard_bytes, True, "decode_host_batch_multi")
    pc, kc = _ctx_array(ctxs)
    ks = (ctypes.c_uint32 * len(original_counts))(*original_counts)
    po, ko = _ptr_array([Context._haddr(t) for t in originals])
    pr, kr = _ptr_array([Context._haddr(t) for t in recovery])
    pd, kd = _ptr_array([Context._haddr(t) for t in restored_out])
    _check(lib().bfrs_decode_host_batch_multi(pc, len(ctxs), len(original_counts), ks,
                                              recovery_count, shard_bytes, po, pr, pd))


def repair(ctx, archive_dir: str) -> dict:
    """FileStore::repair (src/filestore/health.rs:470-495), intended semantics.
    `ctx` may be a list of contexts: bfrs_repair_multi deals a tier-3 archive's
    blocks over them from this one process."""
    rep = RepairReport()
    if isinstance(ctx, (list, tuple)):
        pc, kc = _ctx_array(ctx)
        _check(lib().bfrs_repair_multi(pc, len(ctx), os.fsencode(archive_dir), ctypes.byref(rep)))
    else:
        _check(lib().bfrs_repair(ctx.handle, os.fsencode(archive_dir), ctypes.byref(rep)))
    return rep.as_dict()


def health_check(ctx: Context, archive_dir: str) -> dict:
    """FileStore::health_check (src/filestore/health.rs:111-438), intended semantics."""
    import json
    return json.loads(_json_call(lib().bfrs_health_check, ctx.handle, os.fsencode(archive_dir)))


_JSON_GUESS = 1 << 18


def _json_call(f, *args) -> str:
    """JSON output convention (*needed = length + 1; a short buffer gets a
    truncated report).  One call into a buffer that fits any usual report; a
    second only if it was too short — a size query first would run the whole
    check (every shard hashed) twice."""
    need = _sz()
    out = ctypes.create_string_buffer(_JSON_GUESS)
    _check(f(*args, out, len(out), ctypes.byref(need)))
    if need.value > len(out):
        out = ctypes.create_string_buffer(need.value)
        _check(f(*args, out, len(out), ctypes.byref(need)))
    return out.value.decode()


class FileStore:
    """FileStore's discovery over an archive root (src/filestore/mod.rs:81-154,
    health.rs:45-74): get_all / find / batch_health_check."""

    def __init__(self, store_path: str):
        self.store_path = store_path

    def get_all(self) -> list:
        import json
        return json.loads(_json_call(lib().bfrs_store_list, os.fsencode(self.store_path)))

    def find(self, file_name: str) -> dict:
        """The first archived file named file_name (with its archive "dir");
        BfrsError(E_NOT_FOUND, "File '<name>' not found") otherwise."""
        d = _json_call(lib().bfrs_store_find, os.fsencode(self.store_path), file_name.encode())
        return next(f for f in self.get_all() if f["dir"] == d)

    def batch_health_check(self, ctx: Context) -> dict:
        import json
        return json.loads(_json_call(lib().bfrs_batch_health_check, ctx.handle,
                                     os.fsencode(self.store_path)))


class Archive:
    """Read-path core of the FUSE mount (src/mount/filesystem_unix.rs:176-305):
    offset reads through an LRU segment cache with BLAKE3 verification and GPU
    reconstruction of corrupt/missing segments."""

    def __init__(self, ctx: Context, archive_dir: str, cache_segments: int = 64,
                 write_back: bool = False):
        self.ctx = ctx
        h = _vp()
        _check(lib().bfrs_archive_open(ctx.handle, os.fsencode(archive_dir), cache_segments,
                                       1 if write_back else 0, ctypes.byref(h)))
        self.handle = h.value
        self._read = lib().bfrs_archive_read
        _LIVE_ARCHIVES.add(self)

    @property
    def size(self) -> int:
        n = ctypes.c_uint64()
        _check(lib().bfrs_archive_size(self.handle, ctypes.byref(n)))
        return n.value

    def read_into(self, offset: int, out) -> int:
        import numpy as np
        a = out if isinstance(out, np.ndarray) else np.frombuffer(out, dtype=np.uint8)
        if a.nbytes and not a.flags.c_contiguous:
            raise ValueError("read_into: destination must be C-contiguous")
        if not a.flags.writeable:  # bytes, or a read-only view: never write into it
            raise ValueError("read_into: destination is read-only")
        return self.read_into_ptr(offset, a.__array_interface__["data"][0] if a.nbytes else 0,
                                  a.nbytes)

    def read_into_ptr(self, offset: int, addr: int, size: int) -> int:
        """bfrs_archive_read into host memory at `addr` (the FUSE reply buffer's
        role): no per-call buffer objects, so a request loop measures the read
        path rather than Python."""
        n = _sz()  # per call: readers on other threads share this handle
        _check(self._read(self.handle, offset, size, addr or None, ctypes.byref(n)))
        return n.value

    def read(self, offset: int, size: int) -> bytes:
        import numpy as np
        buf = np.empty(max(1, size), dtype=np.uint8)
        n = self.read_into(offset, buf[:size])
        return buf[:n].tobytes()

    def stats(self) -> dict:
        st = ArchiveStats()
        _check(lib().bfrs_archive_stats_get(self.handle, ctypes.byref(st)))
        return st.as_dict()

    def close(self) -> None:
        if self.handle:
            lib().bfrs_archive_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
