"""Host-side mirror of the reference's content-addressing interface.

Same names, argument meaning and error behaviour as the Rust functions they replace:

* ``generate_cas_id(path, size) -> str``  -- core/src/object/cas.rs:23-62
  (16 lowercase hex chars; the ``size`` argument is hashed as le64 exactly as given,
  and selects whole-file (``size <= 102400``) or sampled hashing).
* ``file_checksum(path) -> str``          -- core/src/object/validation/hash.rs:10-24
  (64 lowercase hex chars).
* ``FileMetadata.new(path)``              -- core/src/object/file_identifier/mod.rs:59-97
  (``cas_id`` is ``None`` for an empty file; directories are rejected).

Files are read with the reference's semantics whatever their length: ``size`` is only
hashed (le64) and picks the branch; a whole-kind file contributes every byte it holds
(``fs::read``, cas.rs:29), a sampled one its head and samples by ``read_exact`` and its
tail at ``SeekFrom::End(-8192)`` (cas.rs:31-58); a checksum hashes 1 MiB reads until a
short one (hash.rs:14-20).  I/O errors surface as ``OSError`` (the reference's
``io::Error``); a sample or header past the end of the file raises
``UnexpectedEofError`` (``read_exact``'s ``io::ErrorKind::UnexpectedEof``, cas.rs:36,43,
56).  The batched variants return one result or exception per input, which lets callers
keep the reference's per-caller policy (identifier: log and drop,
file_identifier/mod.rs:127-128; validator: abort the step, validator_job.rs:147-149).

Batches hash on the GPU (libsdcas.so's HIP kernels).  The single-file calls follow the
library's latency policy (include/sd_cas.h, sd_cas_id_path): hashed on the calling
thread by the library's CPU path while few calls are in flight, coalesced into GPU
batches beyond that.  ``spacedrive_amd.cpu`` exposes the CPU path explicitly (a node
without the device).
"""
from __future__ import annotations

import ctypes
import errno as _errno
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import numpy as np

from ._native import (SD_FILE_IO_ERROR, SD_FILE_OK, SD_FILE_SHORT_READ, check, hex_results, lib, path_array)
from .device import _ptr, default_context

MINIMUM_FILE_SIZE = 1024 * 100  # cas.rs:15
STAGE_THREADS = 16  # host reader threads (the CPU share of one GPU on an MI355X node)


class UnexpectedEofError(OSError):
    """io::ErrorKind::UnexpectedEof from read_exact (cas.rs:36,43,56)."""


def _status_error(st: int, path: str) -> OSError:
    code = st & 0xFFFF
    if code == SD_FILE_SHORT_READ:
        return UnexpectedEofError(_errno.EIO, "failed to fill whole buffer", path)
    if code == SD_FILE_IO_ERROR:
        err = (st >> 16) & 0xFFFF
        return OSError(err, os.strerror(err), path)
    return OSError(_errno.EIO, f"sd_cas status {st}", path)


def generate_cas_ids(paths: Sequence[Union[str, os.PathLike]], sizes: Sequence[int],
                     device: Optional[int] = None) -> List[Union[str, OSError]]:
    """Batched generate_cas_id: one cas_id string or OSError per (path, size)."""
    n = len(paths)
    if n != len(sizes):
        raise ValueError("paths and sizes differ in length")
    if n == 0:
        return []
    ctx = default_context(device)
    sizes_a = np.ascontiguousarray(sizes, dtype=np.uint64)
    status = np.zeros(n, np.int32)
    keep, arr = path_array(paths)
    out = ctypes.create_string_buffer(17 * n)
    # library-side pread of header/samples/tail (or the whole file) on its stager pool,
    # overlapped window by window with the H2D copies and kernels
    check(lib().sd_cas_ids_files(ctx.handle, arr, _ptr(sizes_a), n, out, _ptr(status), STAGE_THREADS))
    return hex_results(out, 16, status, paths, _status_error)


def generate_cas_id(path: Union[str, os.PathLike], size: int, device: Optional[int] = None) -> str:
    """cas.rs:23 ``generate_cas_id(path, size) -> Result<String, io::Error>``.

    The single-file latency path (watcher / non_indexed callers): concurrent calls from
    any number of threads are coalesced into GPU batches by the library (sd_cas_id_path)."""
    ctx = default_context(device)
    out = ctypes.create_string_buffer(17)
    st = ctypes.c_int32(0)
    check(lib().sd_cas_id_path(ctx.handle, os.fsencode(path), int(size), out, ctypes.byref(st)))
    if st.value != SD_FILE_OK:
        raise _status_error(st.value, os.fsdecode(path))
    return out.raw[:16].decode()


def file_checksums(paths: Sequence[Union[str, os.PathLike]],
                   device: Optional[int] = None) -> List[Union[str, OSError]]:
    """Batched file_checksum: one 64-hex string or OSError per path."""
    n = len(paths)
    if n == 0:
        return []
    ctx = default_context(device)
    keep, arr = path_array(paths)
    out = ctypes.create_string_buffer(65 * n)
    status = np.zeros(n, np.int32)
    check(lib().sd_file_checksums(ctx.handle, arr, n, out, _ptr(status)))
    return hex_results(out, 64, status, paths, _status_error)


def file_checksum(path: Union[str, os.PathLike], device: Optional[int] = None) -> str:
    """hash.rs:10 ``file_checksum(path) -> Result<String, io::Error>`` (coalesced like
    generate_cas_id: sd_file_checksum_path)."""
    ctx = default_context(device)
    out = ctypes.create_string_buffer(65)
    st = ctypes.c_int32(0)
    check(lib().sd_file_checksum_path(ctx.handle, os.fsencode(path), out, ctypes.byref(st)))
    if st.value != SD_FILE_OK:
        raise _status_error(st.value, os.fsdecode(path))
    return out.raw[:64].decode()


def cas_ids_files_stats(device: Optional[int] = None) -> dict:
    """Routes taken by generate_cas_ids (sd_cas_ids_files) on the device's default context:
    calls hashed on the CPU path by the batch-size policy ("batch_cpu_max") and calls that
    went through the GPU."""
    v = np.zeros(2, np.uint64)
    check(lib().sd_cas_ids_files_stats(default_context(device).handle, _ptr(v)))
    return {"cpu": int(v[0]), "gpu": int(v[1])}


def cas_ids_host_stats(device: Optional[int] = None) -> dict:
    """Files hashed by sd_cas_ids (messages in host memory) on the GPU and by the host threads
    that co-hash beside it ("host_cohash_threads"), since the context was created."""
    v = np.zeros(2, np.uint64)
    check(lib().sd_cas_ids_stats(default_context(device).handle, _ptr(v)))
    return {"gpu_files": int(v[0]), "host_files": int(v[1])}


def checksums_host_stats(device: Optional[int] = None) -> dict:
    """Bytes hashed by sd_checksums (ranges in host memory) on the GPU and by the host threads
    that co-hash beside it ("host_cohash_threads"), since the context was created."""
    v = np.zeros(2, np.uint64)
    check(lib().sd_checksums_stats(default_context(device).handle, _ptr(v)))
    return {"gpu_bytes": int(v[0]), "host_bytes": int(v[1])}


def coalescer_stats(device: Optional[int] = None) -> dict:
    """Latency-path counters of the device's default context: single-file requests, the
    GPU batches they were coalesced into, the largest batch, and requests hashed on the
    CPU path."""
    v = np.zeros(4, np.uint64)
    check(lib().sd_coalescer_stats(default_context(device).handle, _ptr(v)))
    return {"requests": int(v[0]), "batches": int(v[1]), "max_batch": int(v[2]), "cpu": int(v[3])}


def file_checksums_stats(device: Optional[int] = None) -> dict:
    """Routes taken by file_checksums (sd_file_checksums_routes): calls on the CPU path by the
    batch policy ("checksum_cpu_max"), calls through the GPU alone, and calls split between
    the GPU route and the CPU path ("checksum_hybrid_threads")."""
    v = np.zeros(3, np.uint64)
    check(lib().sd_file_checksums_routes(default_context(device).handle, _ptr(v)))
    return {"cpu": int(v[0]), "gpu": int(v[1]), "hybrid": int(v[2])}


def file_checksums_bytes(device: Optional[int] = None) -> dict:
    """sd_file_checksums_bytes: file bytes the GPU route hashed, and the CPU path inside split calls."""
    v = np.zeros(2, np.uint64)
    check(lib().sd_file_checksums_bytes(default_context(device).handle, _ptr(v)))
    return {"gpu": int(v[0]), "cpu_in_split": int(v[1])}


def file_checksums_learned(device: Optional[int] = None) -> dict:
    """sd_file_checksums_learned: the GB/s the context learned for the split and for the CPU
    path alone ("checksum_split_adapt"), and how many calls each was counted for."""
    v = np.zeros(4, np.float64)
    check(lib().sd_file_checksums_learned(default_context(device).handle, _ptr(v)))
    return {"split_GBps": float(v[0]), "cpu_GBps": float(v[1]), "split_calls": int(v[2]), "cpu_calls": int(v[3])}


def checksums_learned(device: Optional[int] = None) -> dict:
    """sd_checksums_learned: the GB/s the context learned for sd_checksums' co-hashed calls
    and for the CPU path alone ("checksum_split_adapt"), and how many calls each was counted for."""
    v = np.zeros(4, np.float64)
    check(lib().sd_checksums_learned(default_context(device).handle, _ptr(v)))
    return {"cohash_GBps": float(v[0]), "cpu_GBps": float(v[1]), "cohash_calls": int(v[2]), "cpu_calls": int(v[3])}


def set_tuning(key: str, value: int) -> None:
    """sd_cas_set_tuning (process-wide knobs, include/sd_cas.h)."""
    check(lib().sd_cas_set_tuning(key.encode(), int(value)))


def get_tuning(key: str) -> int:
    """sd_cas_get_tuning."""
    v = ctypes.c_int32(0)
    check(lib().sd_cas_get_tuning(key.encode(), ctypes.byref(v)))
    return int(v.value)


@dataclass
class FileMetadata:
    """file_identifier/mod.rs:50-55 (kind detection is out of scope: SURVEY.md §2)."""

    cas_id: Optional[str]
    size: int

    @staticmethod
    def new(path: Union[str, os.PathLike], device: Optional[int] = None) -> "FileMetadata":
        r = FileMetadata.batch([path], device)[0]
        if isinstance(r, OSError):
            raise r
        return r

    @staticmethod
    def batch(paths: Sequence[Union[str, os.PathLike]],
              device: Optional[int] = None) -> List[Union["FileMetadata", OSError]]:
        """mod.rs:59-97 for a whole identifier step: stat, skip empty files, hash the rest."""
        out: List[Union[FileMetadata, OSError, None]] = [None] * len(paths)
        todo, sizes = [], []
        for i, p in enumerate(paths):
            try:
                st = os.stat(p)
            except OSError as e:  # mod.rs:65-67
                out[i] = e
                continue
            if os.path.isdir(p):  # mod.rs:69-72
                raise AssertionError("We can't generate cas_id for directories")
            if st.st_size == 0:  # mod.rs:80-88
                out[i] = FileMetadata(None, 0)
            else:
                todo.append(i)
                sizes.append(st.st_size)
        if todo:
            ids = generate_cas_ids([paths[i] for i in todo], sizes, device)
            for i, s, r in zip(todo, sizes, ids):
                out[i] = r if isinstance(r, OSError) else FileMetadata(r, s)
        return out  # type: ignore[return-value]
