"""The library's CPU path (libsdcas.so ``sd_cpu_*``), with the names and error behaviour of
``spacedrive_amd.cas``: for a node without a gfx950 device, and what the latency policy
uses for few concurrent single-file calls.

Same file-read semantics as the GPU path (cas.rs:23-62, hash.rs:10-24); the hashing is
the library's own host BLAKE3 (csrc/cpu_blake3.cpp: AVX-512 / AVX2 / SSE2 chunk lanes).
It needs no device and no torch device state.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Union

import numpy as np

from ._native import SD_FILE_OK, check, hex_results, lib, path_array
from .cas import _status_error

THREADS = 16  # host threads for batches (the CPU share of one GPU on an MI355X node)


def simd_lanes() -> int:
    """Chunk lanes of the host hasher on this CPU (16 AVX-512, 8 AVX2, 4 SSE2)."""
    return int(lib().sd_cpu_simd_lanes())


def generate_cas_ids(paths: Sequence[Union[str, os.PathLike]], sizes: Sequence[int],
                     nthreads: int = THREADS) -> List[Union[str, OSError]]:
    n = len(paths)
    if n != len(sizes):
        raise ValueError("paths and sizes differ in length")
    if n == 0:
        return []
    sizes_a = np.ascontiguousarray(sizes, dtype=np.uint64)
    status = np.zeros(n, np.int32)
    keep, arr = path_array(paths)
    out = ctypes.create_string_buffer(17 * n)
    check(lib().sd_cpu_cas_ids_files(arr, sizes_a.ctypes.data, n, out, status.ctypes.data, nthreads))
    return hex_results(out, 16, status, paths, _status_error)


def generate_cas_id(path: Union[str, os.PathLike], size: int) -> str:
    """cas.rs:23 on the calling thread."""
    out = ctypes.create_string_buffer(17)
    st = ctypes.c_int32(0)
    check(lib().sd_cpu_cas_id_path(os.fsencode(path), int(size), out, ctypes.byref(st)))
    if st.value != SD_FILE_OK:
        raise _status_error(st.value, os.fsdecode(path))
    return out.raw[:16].decode()


def file_checksums(paths: Sequence[Union[str, os.PathLike]],
                   nthreads: int = THREADS) -> List[Union[str, OSError]]:
    n = len(paths)
    if n == 0:
        return []
    keep, arr = path_array(paths)
    out = ctypes.create_string_buffer(65 * n)
    status = np.zeros(n, np.int32)
    check(lib().sd_cpu_file_checksums(arr, n, out, status.ctypes.data, nthreads))
    return hex_results(out, 64, status, paths, _status_error)


def file_checksum(path: Union[str, os.PathLike]) -> str:
    """hash.rs:10 on the calling thread."""
    out = ctypes.create_string_buffer(65)
    st = ctypes.c_int32(0)
    check(lib().sd_cpu_file_checksum_path(os.fsencode(path), out, ctypes.byref(st)))
    if st.value != SD_FILE_OK:
        raise _status_error(st.value, os.fsdecode(path))
    return out.raw[:64].decode()


def cas_ids_staged(staged: np.ndarray, extents: np.ndarray, status: Optional[np.ndarray] = None,
                   nthreads: int = THREADS) -> List[str]:
    """sd_cpu_cas_ids over host-staged messages (extents as stage_plan builds them)."""
    n = len(extents)
    out = ctypes.create_string_buffer(17 * max(n, 1))
    check(lib().sd_cpu_cas_ids(staged.ctypes.data, staged.nbytes, extents.ctypes.data, n, out,
                               None if status is None else status.ctypes.data, nthreads))
    raw = out.raw  # one copy: each .raw access copies the whole buffer
    return [raw[17 * i:17 * i + 16].decode() for i in range(n)]


def blake3(data: bytes) -> bytes:
    """Full 32-byte BLAKE3 of a host buffer (sd_cpu_checksums of one range)."""
    buf = np.frombuffer(bytes(data) + bytes(64), np.uint8)
    offs = np.zeros(1, np.uint64)
    lens = np.array([len(data)], np.uint64)
    out = np.zeros(32, np.uint8)
    check(lib().sd_cpu_checksums(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1, out.ctypes.data, 1))
    return out.tobytes()
