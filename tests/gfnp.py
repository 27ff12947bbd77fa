"""numpy helpers for tests: crate shard layout <-> GF(2^16) symbols, and a
vectorised symbol-matrix product used only to check the planner's matrices
against the oracle on the CPU (never as a product path)."""
import numpy as np


def to_symbols(shard: np.ndarray) -> np.ndarray:
    """64-byte chunk layout (shard length multiple of 64)."""
    c = shard.reshape(-1, 64).astype(np.uint32)
    return (c[:, :32] | (c[:, 32:] << 8)).reshape(-1)


def from_symbols(sym: np.ndarray) -> np.ndarray:
    s = sym.reshape(-1, 32)
    out = np.empty((s.shape[0], 64), dtype=np.uint8)
    out[:, :32] = s & 0xFF
    out[:, 32:] = s >> 8
    return out.reshape(-1)


def gf_mul_vec(x: np.ndarray, c: int, exp, log) -> np.ndarray:
    if c == 0:
        return np.zeros_like(x)
    lc = int(log[c])
    s = log[x].astype(np.uint32) + lc
    s = (s + (s >> 16)) & 0xFFFF
    r = exp[s]
    r[x == 0] = 0
    return r


def apply_matrix(mat, inputs, exp, log):
    """rows of mat x list of input shards -> list of output shards."""
    syms = [to_symbols(a) for a in inputs]
    outs = []
    for row in mat:
        acc = np.zeros_like(syms[0])
        for c, s in zip(row, syms):
            acc ^= gf_mul_vec(s, c, exp, log)
        outs.append(from_symbols(acc))
    return outs
