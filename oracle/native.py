"""ctypes loader for oracle/build/libsd_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.  The
C restatement it loads is documented in oracle/sd_oracle.c.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libsd_oracle.so")
_lib = None

EXTENT_DTYPE = np.dtype([("size", "<u8"), ("msg_offset", "<u8"), ("msg_len", "<u4"), ("kind", "<u4")])


def build() -> None:
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, U64, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.sdo_blake3.argtypes = [P, ctypes.c_size_t, P]
        L.sdo_cas_message_len.argtypes = [U64]
        L.sdo_cas_message_len.restype = U64
        L.sdo_synth_fill.argtypes = [U64, ctypes.c_uint32, U64, U64, P]
        L.sdo_synth_cas_message.argtypes = [U64, ctypes.c_uint32, U64, P]
        L.sdo_synth_cas_message.restype = U64
        L.sdo_cas_ids_staged.argtypes = [P, P, U64, P, I]
        L.sdo_cas_ids_synth.argtypes = [P, P, P, U64, P, I]
        L.sdo_cas_ids_synth_simd.argtypes = [P, P, P, U64, P, I, I]
        L.sdo_cas_ids_synth_simd.restype = I
        L.sdo_checksums.argtypes = [P, P, P, U64, P, I]
        L.sdo_checksums_synth.argtypes = [P, P, P, U64, P, I]
        L.sdo_stage_synth.argtypes = [P, P, P, P, U64, P]
        L.sdo_cas_ids_staged_simd.argtypes = [P, P, U64, P, I, I]
        L.sdo_cas_ids_staged_simd.restype = I
        L.sdo_checksums_simd.argtypes = [P, P, P, U64, P, I, I]
        L.sdo_checksums_simd.restype = I
        L.sdo_cas_ids_files.argtypes = [P, P, U64, P, P, I, I]
        L.sdo_cas_ids_files.restype = I
        L.sdo_file_checksums.argtypes = [P, U64, P, P, I, I]
        L.sdo_file_checksums.restype = I
        L.sdo_checksum_synth_mt.argtypes = [U64, U64, ctypes.c_uint32, I, I, P]
        L.sdo_checksum_synth_mt.restype = I
        L.sdo_checksum_mt.argtypes = [P, U64, I, I, P]
        L.sdo_checksum_mt.restype = I
        L.sdo_simd_level.argtypes = [I]
        L.sdo_simd_level.restype = I
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def blake3(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    lib().sdo_blake3(buf, len(data), out)
    return out.raw


def synth_bytes(cid: int, twin: int, offset: int, length: int) -> bytes:
    out = np.empty(length, np.uint8)
    lib().sdo_synth_fill(cid, twin, offset, length, _p(out))
    return out.tobytes()


def cas_message(cid: int, twin: int, size: int) -> bytes:
    out = np.empty(8 + min(size, 102400) if size <= 102400 else 57352, np.uint8)
    n = lib().sdo_synth_cas_message(cid, twin, size, _p(out))
    return out[:n].tobytes()


def cas_ids_synth(sizes, cids, twins=None, nthreads: int = 1) -> np.ndarray:
    sizes = np.ascontiguousarray(sizes, np.uint64)
    cids = np.ascontiguousarray(cids, np.uint64)
    tw = None if twins is None else np.ascontiguousarray(twins, np.uint32)
    out = np.empty((len(sizes), 8), np.uint8)
    lib().sdo_cas_ids_synth(_p(sizes), _p(cids), _p(tw), len(sizes), _p(out), nthreads)
    return out


def cas_ids_synth_simd(sizes, cids, twins=None, nthreads: int = 1, simd: int = -1) -> np.ndarray:
    """cas_ids_synth with the SIMD hasher (itself checked against the scalar one in
    tests/test_oracle.py) -- for library-scale parity runs."""
    sizes = np.ascontiguousarray(sizes, np.uint64)
    cids = np.ascontiguousarray(cids, np.uint64)
    tw = None if twins is None else np.ascontiguousarray(twins, np.uint32)
    out = np.empty((len(sizes), 8), np.uint8)
    lib().sdo_cas_ids_synth_simd(_p(sizes), _p(cids), _p(tw), len(sizes), _p(out), nthreads, simd)
    return out


def cas_ids_staged(staged: np.ndarray, extents: np.ndarray, nthreads: int = 1, simd: int = 0) -> np.ndarray:
    """simd: 0 scalar (the checker), -1 best available SIMD, 1 AVX2, 2 AVX-512."""
    out = np.empty((len(extents), 8), np.uint8)
    lib().sdo_cas_ids_staged_simd(_p(staged), _p(extents), len(extents), _p(out), nthreads, simd)
    return out


def cas_ids_files(paths, sizes, nthreads: int = 1, simd: int = -1):
    """generate_cas_id over files on disk with the reference's read schedule (cas.rs:27-58)
    -> (cas_id bytes [n, 8], sd_file_status [n])."""
    n = len(paths)
    sizes = np.ascontiguousarray(sizes, np.uint64)
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    out = np.zeros((n, 8), np.uint8)
    status = np.zeros(n, np.int32)
    lib().sdo_cas_ids_files(arr, _p(sizes), n, _p(out), _p(status), nthreads, simd)
    return out, status


def file_checksums(paths, nthreads: int = 1, simd: int = -1):
    """file_checksum over files on disk with the reference's read schedule (hash.rs:10-24:
    1 MiB read calls until a short one) -> (32-byte hashes [n, 32], sd_file_status [n])."""
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    out = np.zeros((n, 32), np.uint8)
    status = np.zeros(n, np.int32)
    lib().sdo_file_checksums(arr, n, _p(out), _p(status), nthreads, simd)
    return out, status


def checksum_synth_mt(size: int, cid: int, twin: int = 0, nthreads: int = 8, simd: int = -1) -> bytes:
    """Full BLAKE3 of one synthetic file, chunk-parallel on nthreads (multi-GiB files)."""
    out = ctypes.create_string_buffer(32)
    lib().sdo_checksum_synth_mt(size, cid, twin, nthreads, simd, out)
    return out.raw


def checksum_mt(data: np.ndarray, size: int, nthreads: int = 8, simd: int = -1) -> bytes:
    """Full BLAKE3 of data[:size] (any uint8 array, e.g. a memmap), chunk-parallel."""
    out = ctypes.create_string_buffer(32)
    lib().sdo_checksum_mt(_p(data), size, nthreads, simd, out)
    return out.raw


def simd_level(requested: int = -1) -> int:
    return lib().sdo_simd_level(requested)


def checksums_simd(data: np.ndarray, offsets, lens, nthreads: int = 1, simd: int = -1) -> np.ndarray:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    out = np.empty((len(offsets), 32), np.uint8)
    lib().sdo_checksums_simd(_p(data), _p(offsets), _p(lens), len(offsets), _p(out), nthreads, simd)
    return out


def checksums(data: np.ndarray, offsets, lens, nthreads: int = 1) -> np.ndarray:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    out = np.empty((len(offsets), 32), np.uint8)
    lib().sdo_checksums(_p(data), _p(offsets), _p(lens), len(offsets), _p(out), nthreads)
    return out


def checksums_synth(sizes, cids, twins=None, nthreads: int = 1) -> np.ndarray:
    sizes = np.ascontiguousarray(sizes, np.uint64)
    cids = np.ascontiguousarray(cids, np.uint64)
    tw = None if twins is None else np.ascontiguousarray(twins, np.uint32)
    out = np.empty((len(sizes), 32), np.uint8)
    lib().sdo_checksums_synth(_p(sizes), _p(cids), _p(tw), len(sizes), _p(out), nthreads)
    return out


def stage_synth(sizes, cids, twins, offsets, total: int, nthreads: int = 1) -> np.ndarray:
    """Host buffer holding the exact cas messages of synthetic files at `offsets`; with
    nthreads > 1 the files are split into contiguous ranges written by that many threads
    (each message lands at its own absolute offset, so the ranges never overlap)."""
    sizes = np.ascontiguousarray(sizes, np.uint64)
    cids = np.ascontiguousarray(cids, np.uint64)
    tw = None if twins is None else np.ascontiguousarray(twins, np.uint32)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    buf = np.zeros(total + 64, np.uint8)
    n = len(sizes)
    nthreads = max(1, min(int(nthreads), n // 1024 or 1))
    if nthreads == 1:
        lib().sdo_stage_synth(_p(sizes), _p(cids), _p(tw), _p(offsets), n, _p(buf))
        return buf
    import threading
    cuts = np.linspace(0, n, nthreads + 1).astype(np.int64)

    def run(a, b):
        lib().sdo_stage_synth(_p(sizes[a:b]), _p(cids[a:b]), None if tw is None else _p(tw[a:b]),
                              _p(offsets[a:b]), b - a, _p(buf))

    th = [threading.Thread(target=run, args=(int(cuts[i]), int(cuts[i + 1]))) for i in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return buf
