"""Minimal pure-Python BLAKE3 (test-only, small inputs): subtree chaining
values of message parts, to pin bfrs_blake3_combine without a GPU.  Follows
the BLAKE3 specification (compression, chunk/parent flags, left-complete tree)."""
import struct

IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB,
      0x5BE0CD19)
PERM = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
START, END, PARENT, ROOT = 1, 2, 4, 8
M32 = 0xFFFFFFFF


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _g(v, a, b, c, d, x, y):
    v[a] = (v[a] + v[b] + x) & M32
    v[d] = _rotr(v[d] ^ v[a], 16)
    v[c] = (v[c] + v[d]) & M32
    v[b] = _rotr(v[b] ^ v[c], 12)
    v[a] = (v[a] + v[b] + y) & M32
    v[d] = _rotr(v[d] ^ v[a], 8)
    v[c] = (v[c] + v[d]) & M32
    v[b] = _rotr(v[b] ^ v[c], 7)


def compress(cv, block, counter, blen, flags):
    m = list(struct.unpack("<16I", block.ljust(64, b"\0")))
    v = list(cv) + list(IV[:4]) + [counter & M32, counter >> 32, blen, flags]
    for r in range(7):
        _g(v, 0, 4, 8, 12, m[0], m[1]); _g(v, 1, 5, 9, 13, m[2], m[3])
        _g(v, 2, 6, 10, 14, m[4], m[5]); _g(v, 3, 7, 11, 15, m[6], m[7])
        _g(v, 0, 5, 10, 15, m[8], m[9]); _g(v, 1, 6, 11, 12, m[10], m[11])
        _g(v, 2, 7, 8, 13, m[12], m[13]); _g(v, 3, 4, 9, 14, m[14], m[15])
        m = [m[p] for p in PERM]
    return [v[i] ^ v[i + 8] for i in range(8)]


def chunk_cv(data, index):
    cv = list(IV)
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    for j, b in enumerate(blocks):
        flags = (START if j == 0 else 0) | (END if j == len(blocks) - 1 else 0)
        cv = compress(cv, b, index, len(b), flags)
    return cv


def parent_cv(l, r):
    return compress(list(IV), struct.pack("<16I", *l, *r), 0, 64, PARENT)


def subtree_cv(data, chunk0):
    """Non-root CV of the subtree over `data` starting at chunk `chunk0`."""
    nodes = [chunk_cv(data[i:i + 1024], chunk0 + i // 1024) for i in range(0, len(data), 1024)] \
        or [chunk_cv(b"", chunk0)]
    while len(nodes) > 1:
        nxt = [parent_cv(nodes[i], nodes[i + 1]) for i in range(0, len(nodes) - 1, 2)]
        if len(nodes) % 2:
            nxt.append(nodes[-1])
        nodes = nxt
    return struct.pack("<8I", *nodes[0])
