"""BLAKE3 specification restatement in plain Python -- TEST INFRASTRUCTURE ONLY.

This module is part of the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.  The
product path (``spacedrive_amd`` + ``libsdcas.so``) never imports or calls it.

What it restates
----------------
The reference hashes through the third-party ``blake3`` crate, version 1.4.1
(``/root/reference/Cargo.lock:625-628``, declared at ``core/Cargo.toml:63``).  The crate
is not vendored in ``/root/reference`` and no Rust toolchain exists in this image, so
the crate is restated here from the published BLAKE3 specification (hash mode,
``derive_key`` mode, 7 rounds, 1 KiB chunks, binary tree with "left subtree = largest
power of two" split, CV stack as in the spec's reference implementation).

Call sites it stands in for:
  * ``Hasher::new/update/finalize`` -- ``core/src/object/cas.rs:24,25,29,38,44,58,61``,
    ``core/src/object/validation/hash.rs:12,16,21``
  * ``Hash::to_hex`` (lowercase) -- ``cas.rs:61``, ``hash.rs:21``
  * ``blake3::derive_key`` -- ``crates/crypto/src/types.rs:166`` (pinned by the KAT
    ``DERIVE_B3_EXPECTED`` at ``crates/crypto/src/keys/hashing.rs:210-213``)

Pinning
-------
``tests/test_oracle.py`` checks this module against the only in-repo BLAKE3 vector
(``derive_b3``, ``crates/crypto/src/keys/hashing.rs:323-328``) and against the
published official BLAKE3 test-vector hashes (input ``i % 251``) for lengths that
cross the block, chunk and multi-level tree boundaries.  The tree here is built with
the spec's incremental CV stack -- deliberately NOT the level-wise pairwise merge the
GPU kernels use -- so agreement between the two is itself a check of the kernels'
tree shape.
"""

from __future__ import annotations

import struct

MASK = 0xFFFFFFFF

IV = (
    0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
    0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19,
)

MSG_PERMUTATION = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)

CHUNK_START = 1 << 0
CHUNK_END = 1 << 1
PARENT = 1 << 2
ROOT = 1 << 3
KEYED_HASH = 1 << 4
DERIVE_KEY_CONTEXT = 1 << 5
DERIVE_KEY_MATERIAL = 1 << 6

BLOCK_LEN = 64
CHUNK_LEN = 1024
OUT_LEN = 32


def _rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & MASK


def _g(s: list, a: int, b: int, c: int, d: int, mx: int, my: int) -> None:
    s[a] = (s[a] + s[b] + mx) & MASK
    s[d] = _rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & MASK
    s[b] = _rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + my) & MASK
    s[d] = _rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & MASK
    s[b] = _rotr(s[b] ^ s[c], 7)


def _round(s: list, m: list) -> None:
    _g(s, 0, 4, 8, 12, m[0], m[1])
    _g(s, 1, 5, 9, 13, m[2], m[3])
    _g(s, 2, 6, 10, 14, m[4], m[5])
    _g(s, 3, 7, 11, 15, m[6], m[7])
    _g(s, 0, 5, 10, 15, m[8], m[9])
    _g(s, 1, 6, 11, 12, m[10], m[11])
    _g(s, 2, 7, 8, 13, m[12], m[13])
    _g(s, 3, 4, 9, 14, m[14], m[15])


def compress(cv, block_words, counter: int, block_len: int, flags: int) -> list:
    """One BLAKE3 compression; returns the 16-word extended output."""
    s = [
        cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
        IV[0], IV[1], IV[2], IV[3],
        counter & MASK, (counter >> 32) & MASK, block_len, flags,
    ]
    m = list(block_words)
    for r in range(7):
        _round(s, m)
        if r != 6:
            m = [m[MSG_PERMUTATION[i]] for i in range(16)]
    for i in range(8):
        s[i] ^= s[i + 8]
        s[i + 8] ^= cv[i]
    return s


def words_from_block(block: bytes) -> list:
    block = block + bytes(BLOCK_LEN - len(block))
    return list(struct.unpack("<16I", block))


class _Output:
    __slots__ = ("cv", "block_words", "counter", "block_len", "flags")

    def __init__(self, cv, block_words, counter, block_len, flags):
        self.cv, self.block_words = cv, block_words
        self.counter, self.block_len, self.flags = counter, block_len, flags

    def chaining_value(self) -> list:
        return compress(self.cv, self.block_words, self.counter, self.block_len, self.flags)[:8]

    def root_bytes(self, out_len: int = OUT_LEN) -> bytes:
        out = bytearray()
        ctr = 0
        while len(out) < out_len:
            w = compress(self.cv, self.block_words, ctr, self.block_len, self.flags | ROOT)
            out += struct.pack("<16I", *w)
            ctr += 1
        return bytes(out[:out_len])


class _ChunkState:
    def __init__(self, key, chunk_counter: int, flags: int):
        self.cv = list(key)
        self.chunk_counter = chunk_counter
        self.block = bytearray()
        self.blocks_compressed = 0
        self.flags = flags

    def len(self) -> int:
        return BLOCK_LEN * self.blocks_compressed + len(self.block)

    def _start_flag(self) -> int:
        return CHUNK_START if self.blocks_compressed == 0 else 0

    def update(self, data: bytes) -> None:
        while data:
            if len(self.block) == BLOCK_LEN:
                w = words_from_block(bytes(self.block))
                self.cv = compress(self.cv, w, self.chunk_counter, BLOCK_LEN,
                                   self.flags | self._start_flag())[:8]
                self.blocks_compressed += 1
                self.block = bytearray()
            take = min(BLOCK_LEN - len(self.block), len(data))
            self.block += data[:take]
            data = data[take:]

    def output(self) -> _Output:
        return _Output(self.cv, words_from_block(bytes(self.block)), self.chunk_counter,
                       len(self.block), self.flags | self._start_flag() | CHUNK_END)


def _parent_output(left, right, key, flags) -> _Output:
    return _Output(list(key), list(left) + list(right), 0, BLOCK_LEN, PARENT | flags)


class Hasher:
    """Incremental BLAKE3 hasher (spec reference structure: CV stack)."""

    def __init__(self, key=IV, flags: int = 0):
        self.key = list(key)
        self.flags = flags
        self.chunk = _ChunkState(self.key, 0, flags)
        self.cv_stack: list = []

    def _add_chunk_cv(self, new_cv, total_chunks: int) -> None:
        while total_chunks & 1 == 0:
            new_cv = _parent_output(self.cv_stack.pop(), new_cv, self.key,
                                    self.flags).chaining_value()
            total_chunks >>= 1
        self.cv_stack.append(new_cv)

    def update(self, data: bytes) -> "Hasher":
        data = bytes(data)
        while data:
            if self.chunk.len() == CHUNK_LEN:
                cv = self.chunk.output().chaining_value()
                total = self.chunk.chunk_counter + 1
                self._add_chunk_cv(cv, total)
                self.chunk = _ChunkState(self.key, total, self.flags)
            take = min(CHUNK_LEN - self.chunk.len(), len(data))
            self.chunk.update(data[:take])
            data = data[take:]
        return self

    def finalize(self, out_len: int = OUT_LEN) -> bytes:
        out = self.chunk.output()
        for left in reversed(self.cv_stack):
            out = _parent_output(left, out.chaining_value(), self.key, self.flags)
        return out.root_bytes(out_len)


def blake3(data: bytes, out_len: int = OUT_LEN) -> bytes:
    return Hasher().update(data).finalize(out_len)


def derive_key(context: str, material: bytes, out_len: int = OUT_LEN) -> bytes:
    ctx_key_bytes = Hasher(IV, DERIVE_KEY_CONTEXT).update(context.encode()).finalize(32)
    ctx_key = struct.unpack("<8I", ctx_key_bytes)
    return Hasher(ctx_key, DERIVE_KEY_MATERIAL).update(material).finalize(out_len)


# --- level-wise tree (the shape the GPU kernels use), kept here only so tests can
# --- compare it against the CV-stack shape above for every chunk count.

def chunk_cv(chunk: bytes, counter: int, is_root: bool) -> list:
    """CV (or root output words) of one chunk, compressing block by block."""
    nblocks = max(1, (len(chunk) + BLOCK_LEN - 1) // BLOCK_LEN)
    cv = list(IV)
    for b in range(nblocks):
        blk = chunk[b * BLOCK_LEN:(b + 1) * BLOCK_LEN]
        fl = (CHUNK_START if b == 0 else 0) | (CHUNK_END if b == nblocks - 1 else 0)
        if is_root and b == nblocks - 1:
            fl |= ROOT
        cv = compress(cv, words_from_block(blk), counter, len(blk), fl)[:8]
    return cv


def levelwise_hash(data: bytes) -> bytes:
    """Hash by level-wise pairwise merge with the odd tail carried up unchanged."""
    n = max(1, (len(data) + CHUNK_LEN - 1) // CHUNK_LEN)
    if n == 1:
        return struct.pack("<8I", *chunk_cv(data, 0, True))
    level = [chunk_cv(data[i * CHUNK_LEN:(i + 1) * CHUNK_LEN], i, False) for i in range(n)]
    while len(level) > 1:
        root = len(level) == 2
        nxt = []
        for i in range(0, len(level) - 1, 2):
            fl = PARENT | (ROOT if root else 0)
            nxt.append(compress(IV, list(level[i]) + list(level[i + 1]), 0, BLOCK_LEN, fl)[:8])
        if len(level) & 1:
            nxt.append(level[-1])
        level = nxt
    return struct.pack("<8I", *level[0])
