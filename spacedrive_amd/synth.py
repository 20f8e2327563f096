"""Synthetic file libraries for benchmarks and parity tests.

A library is three arrays per file -- ``sizes`` (u64), ``cids`` (content id, u64) and
``twins`` (u32 twin tag) -- computed from the GLOBAL file index with a counter-based
hash, so any rank can describe its own shard of a 10 M-file library without the rest.
File contents are never stored: byte ``o`` of content ``cid`` is generated on demand by
``csrc/synth.hip`` (device) or ``oracle/sd_oracle.c`` (CPU checker) from the same
splitmix64 stream.

Planted structure: ``dup_frac`` of files are exact copies (same size and content) of
another file's base content, and ``twin_frac`` of sampled-size files are "sample twins"
of their predecessor: same size and same bytes inside every sample window of
cas.rs:35-58, one byte different outside -- same cas_id, different checksum.
"""
from __future__ import annotations

import numpy as np

SMALL_MAX = 102400          # cas.rs:15, hashed whole when size <= this
SAMPLED_MAX = 4 << 30       # 4 GiB upper end of the sampled-size distribution
EDGE_SIZES = [0, 1, 55, 56, 57, 63, 64, 65, 1015, 1016, 1017, 2040, 2041, 16376, 16377, 65536,
              102399, 102400, 102401, 131072, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (1 << 32) + 1]
LIB_SEED = 0x51DE_5EED
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _mix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _u01(idx: np.ndarray, stream: int, seed: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = _mix(idx.astype(np.uint64) * _GOLD ^ np.uint64((seed * 0x1000193 + stream) & 0xFFFFFFFFFFFFFFFF))
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def _loguniform(u: np.ndarray, lo: int, hi: int) -> np.ndarray:
    a, b = np.log(lo), np.log(hi + 1.0)
    v = np.floor(np.exp(a + u * (b - a))).astype(np.uint64)
    return np.clip(v, lo, hi)


def base_sizes(idx: np.ndarray, small_frac: float, seed: int) -> np.ndarray:
    u_cat = _u01(idx, 1, seed)
    u_sz = _u01(idx, 2, seed)
    small = _loguniform(u_sz, 1, SMALL_MAX)
    big = _loguniform(u_sz, SMALL_MAX + 1, SAMPLED_MAX)
    return np.where(u_cat < small_frac, small, big)


def library(start: int, n: int, n_total: int, small_frac: float = 0.6, dup_frac: float = 0.10,
            twin_frac: float = 0.01, edge: bool = True, seed: int = LIB_SEED):
    """Files [start, start+n) of an n_total-file library -> (sizes, cids, twins)."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    sizes = base_sizes(idx, small_frac, seed)
    cids = idx.copy()
    twins = np.zeros(n, np.uint32)
    # exact duplicates of another file's base content (may live on another shard)
    dup = _u01(idx, 3, seed) < dup_frac
    with np.errstate(over="ignore"):
        tgt = (_mix(idx * _GOLD ^ np.uint64(seed + 4)) % np.uint64(max(n_total, 1))).astype(np.uint64)
    tsz = base_sizes(tgt, small_frac, seed)
    sizes = np.where(dup, tsz, sizes)
    cids = np.where(dup, tgt, cids)
    # sample twins of the predecessor (sampled sizes only)
    prev = np.where(idx > 0, idx - np.uint64(1), idx)
    psz = base_sizes(prev, small_frac, seed)
    twin = (~dup) & (_u01(idx, 5, seed) < twin_frac) & (psz > SMALL_MAX) & (idx > 0)
    sizes = np.where(twin, psz, sizes)
    cids = np.where(twin, prev, cids)
    twins = np.where(twin, (idx % np.uint64(254) + np.uint64(1)).astype(np.uint32), twins)
    if edge:  # the edge sizes are always part of the library
        k = np.arange(len(EDGE_SIZES))
        sel = (k >= start) & (k < start + n)
        pos = (k[sel] - start).astype(np.int64)
        sizes[pos] = np.array(EDGE_SIZES, np.uint64)[sel]
        cids[pos] = k[sel].astype(np.uint64)
        twins[pos] = 0
    return sizes.astype(np.uint64), cids.astype(np.uint64), twins.astype(np.uint32)


def small_library(start: int, n: int, seed: int = LIB_SEED, **kw):
    """configs[1]: files <= 100 KiB, whole-content cas_id."""
    return library(start, n, kw.pop("n_total", start + n), small_frac=1.0, edge=False, seed=seed, **kw)


def sampled_library(start: int, n: int, seed: int = LIB_SEED, **kw):
    """configs[2]: files > 100 KiB, sampled cas_id."""
    return library(start, n, kw.pop("n_total", start + n), small_frac=0.0, edge=False, seed=seed, **kw)


def sample_windows(size: int):
    """(file offset, length) of the byte windows generate_cas_id reads from a file of
    `size` bytes, in message order (cas.rs:27-58): the whole file, or head / 4 samples /
    tail."""
    if size <= SMALL_MAX:
        return [(0, size)]
    jump = (size - 2 * 8192) // 4
    return [(0, 8192)] + [(8192 + k * jump, 10240) for k in range(4)] + [(size - 8192, 8192)]


def write_files(directory: str, sizes, staged: np.ndarray, extents: np.ndarray, prefix: str = "f"):
    """Materialise synthetic files from their staged cas messages: a whole-content file is
    its message minus the 8-byte header; a sampled file is written sparse (ftruncate to
    its size, then only the windows generate_cas_id reads), so multi-GB files cost only
    their 56 KiB of sampled bytes.  Returns the paths."""
    import os
    paths = []
    for i, size in enumerate(np.asarray(sizes, np.uint64).tolist()):
        p = os.path.join(directory, f"{prefix}{i:07d}")
        off = int(extents["msg_offset"][i]) + 8
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            if size > SMALL_MAX:
                os.ftruncate(fd, size)
            for fo, ln in sample_windows(size):
                if ln:
                    os.pwrite(fd, staged[off:off + ln].tobytes(), fo)
                off += ln
        finally:
            os.close(fd)
        paths.append(p)
    return paths
