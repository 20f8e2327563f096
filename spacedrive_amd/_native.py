"""Loader for the in-tree HIP library ``spacedrive_amd/libsdcas.so`` (C ABI: include/sd_cas.h).

Importing the product path without the built library raises (there is no Python
fallback).  The library's GPU entry points fail with SD_ERR_DEVICE without a gfx950
device; its sd_cpu_* entry points are the explicit CPU path (include/sd_cas.h).

torch is imported first on purpose: the torch wheel ships its own ``libamdhip64.so.7``
and the library's ``NEEDED libamdhip64.so.7`` must bind to that same copy, so that one
HIP runtime serves torch's allocations, streams and RCCL and our kernels alike.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- must precede the CDLL load (one HIP runtime per process)

HERE = os.path.dirname(os.path.abspath(__file__))
# SD_CAS_LIB: an alternative build of the same library (the sanitizer build of
# scripts/sanitize_pytest.sh); the default is the in-tree gfx950 build
LIB_PATH = os.environ.get("SD_CAS_LIB") or os.path.join(HERE, "libsdcas.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "sd_cas.h")

SD_OK = 0
RC_NAMES = {0: "SD_OK", -1: "SD_ERR_INVALID", -2: "SD_ERR_DEVICE", -3: "SD_ERR_NOMEM",
            -4: "SD_ERR_INTERNAL", -5: "SD_ERR_COMM", -6: "SD_ERR_CAPACITY"}
SD_ERR_CAPACITY = -6
SD_FILE_OK, SD_FILE_SKIPPED_EMPTY, SD_FILE_IO_ERROR, SD_FILE_SHORT_READ, SD_FILE_CHANGED = 0, 1, 2, 3, 4
SD_KIND_WHOLE, SD_KIND_SAMPLED = 1, 2
SAMPLED_MSG_LEN = 57352
STAGE_ALIGN = 128


class SdCasError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"{RC_NAMES.get(rc, rc)}: {msg}")
        self.rc = rc


class Extent(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint64), ("msg_offset", ctypes.c_uint64),
                ("msg_len", ctypes.c_uint32), ("kind", ctypes.c_uint32)]


_lib = None

P = ctypes.c_void_p
U64 = ctypes.c_uint64
U32 = ctypes.c_uint32
I32 = ctypes.c_int
SZ = ctypes.c_size_t
PU64 = ctypes.POINTER(ctypes.c_uint64)

# (name, restype, argtypes) -- exactly the exports of include/sd_cas.h
SIGNATURES = [
    ("sd_cas_abi_version", I32, []),
    ("sd_cas_last_error", ctypes.c_char_p, []),
    ("sd_cas_ctx_create", I32, [I32, ctypes.POINTER(P)]),
    ("sd_cas_ctx_destroy", None, [P]),
    ("sd_cas_host_alloc", I32, [P, U64, ctypes.POINTER(P)]),
    ("sd_cas_host_free", None, [P, P]),
    ("sd_cas_stage_plan", I32, [P, SZ, P, PU64]),
    ("sd_cas_stage_file", I32, [ctypes.c_char_p, P, P, ctypes.POINTER(ctypes.c_int32)]),
    ("sd_cas_stage_files", I32, [P, P, SZ, P, P, I32]),
    ("sd_cas_ids", I32, [P, P, U64, P, SZ, P, P]),
    ("sd_cas_ids_files", I32, [P, P, P, SZ, P, P, I32]),
    ("sd_cas_ids_files_stats", I32, [P, P]),
    ("sd_cas_hashes_files", I32, [P, P, P, SZ, P, P, P, I32]),
    ("sd_cas_batch_create", I32, [P, P, SZ, ctypes.POINTER(P)]),
    ("sd_cas_batch_destroy", None, [P]),
    ("sd_cas_batch_run", I32, [P, P, P, P, P]),
    ("sd_cas_batch_run_part", I32, [P, P, I32, P, P, P]),
    ("sd_cas_batch_stats", I32, [P, P]),
    ("sd_checksum_batch_create", I32, [P, P, P, SZ, ctypes.POINTER(P)]),
    ("sd_checksum_batch_destroy", None, [P]),
    ("sd_checksum_batch_run", I32, [P, P, P, P, P]),
    ("sd_checksum_batch_stats", I32, [P, P]),
    ("sd_file_checksums", I32, [P, P, SZ, P, P]),
    ("sd_checksums", I32, [P, P, P, P, SZ, P]),
    ("sd_cas_id_path", I32, [P, ctypes.c_char_p, U64, P, ctypes.POINTER(ctypes.c_int32)]),
    ("sd_file_checksum_path", I32, [P, ctypes.c_char_p, P, ctypes.POINTER(ctypes.c_int32)]),
    ("sd_coalescer_stats", I32, [P, P]),
    ("sd_cpu_simd_lanes", I32, []),
    ("sd_cpu_cas_ids", I32, [P, U64, P, SZ, P, P, I32]),
    ("sd_cpu_cas_ids_files", I32, [P, P, SZ, P, P, I32]),
    ("sd_cpu_checksums", I32, [P, P, P, SZ, P, I32]),
    ("sd_cpu_file_checksums", I32, [P, SZ, P, P, I32]),
    ("sd_cpu_cas_id_path", I32, [ctypes.c_char_p, U64, P, ctypes.POINTER(ctypes.c_int32)]),
    ("sd_cpu_file_checksum_path", I32, [ctypes.c_char_p, P, ctypes.POINTER(ctypes.c_int32)]),
    ("sd_dedup_partition", I32, [P, P, P, U64, U64, I32, P, P, PU64, P]),
    ("sd_dedup_group", I32, [P, P, U64, I32, P, PU64, P]),
    ("sd_dedup_owners", I32, [P, P, U64, P, U64, P, P]),
    ("sd_comm_id", I32, [P]),
    ("sd_comm_create", I32, [P, P, I32, I32, ctypes.POINTER(P)]),
    ("sd_comm_destroy", None, [P]),
    ("sd_comm_group_create", I32, [I32, ctypes.POINTER(P)]),
    ("sd_comm_group_destroy", None, [P]),
    ("sd_comm_create_local", I32, [P, P, I32, ctypes.POINTER(P)]),
    ("sd_comm_set_timing", I32, [P, I32]),
    ("sd_comm_last_phases", I32, [P, P]),
    ("sd_cas_dedup_mgpu", I32, [P, P, P, P, U64, U64, U64, P, P, P, U64, PU64, PU64, P]),
    ("sd_split_range", I32, [U64, I32, I32, PU64, PU64, PU64]),
    ("sd_shard_plan", I32, [P, SZ, I32, P]),
    ("sd_split_checksum_create", I32, [P, U64, I32, I32, ctypes.POINTER(P)]),
    ("sd_split_checksum_destroy", None, [P]),
    ("sd_split_checksum_leaves", I32, [P, P, P, P, P]),
    ("sd_split_checksum_root", I32, [P, P, P, P, P]),
    ("sd_split_checksum_mgpu", I32, [P, P, P, P, P, P, P]),
    ("sd_cpu_split_leaves", I32, [P, U64, I32, I32, P, I32]),
    ("sd_cpu_split_root", I32, [P, U64, P]),
    ("sd_synth_stage_cas", I32, [P, P, P, P, P, SZ, P, P]),
    ("sd_synth_fill", I32, [P, U64, U32, U64, P, P]),
    ("sd_synth_fill_at", I32, [P, U64, U32, U64, U64, P, P]),
    ("sd_device_malloc", I32, [P, U64, ctypes.POINTER(P)]),
    ("sd_device_free", None, [P, P]),
    ("sd_memcpy", I32, [P, P, P, U64, P]),
    ("sd_stream_sync", I32, [P, P]),
    ("sd_cas_batch_time", I32, [P, P, P, P, I32, P, ctypes.POINTER(ctypes.c_float)]),
    ("sd_checksum_batch_time", I32, [P, P, P, P, I32, P, ctypes.POINTER(ctypes.c_float)]),
    ("sd_valu_peak", I32, [P, ctypes.POINTER(ctypes.c_double)]),
    ("sd_cas_set_tuning", I32, [ctypes.c_char_p, I32]),
    ("sd_cas_get_tuning", I32, [ctypes.c_char_p, ctypes.POINTER(I32)]),
    ("sd_file_checksums_stats", I32, [P, P]),
    ("sd_file_checksums_routes", I32, [P, P]),
    ("sd_file_checksums_bytes", I32, [P, P]),
    ("sd_file_checksums_learned", I32, [P, P]),
    ("sd_checksums_learned", I32, [P, P]),
    ("sd_cas_ids_stats", I32, [P, P]),
    ("sd_checksums_stats", I32, [P, P]),
    ("sd_read_probe", I32, [P, P, U64, I32, P]),
    ("sd_host_cpu_budget", I32, [P]),
    ("sd_host_numa", I32, [P]),
    ("sd_comm_rccl_info", I32, [ctypes.POINTER(I32), ctypes.c_char_p, SZ]),
]


def host_cpu_budget() -> dict:
    """The library's host thread budget (sd_host_cpu_budget)."""
    out = (ctypes.c_int * 5)()
    check(lib().sd_host_cpu_budget(out))
    return {"budget": out[0], "affinity": out[1], "cgroup_quota_cpus": out[2] / 1000.0 if out[2] else None,
            "local_world_size": out[3], "overridden": bool(out[4])}


def host_numa() -> dict:
    """Where the library's own threads run (sd_host_numa)."""
    out = (ctypes.c_int * 3)()
    check(lib().sd_host_numa(out))
    return {"placed": bool(out[0]), "cpus": out[1], "device_node": out[2]}


def rccl_info() -> dict:
    """The RCCL that serves libsdcas's communicators in this process (sd_comm_rccl_info)."""
    v = ctypes.c_int(0)
    buf = ctypes.create_string_buffer(4096)
    check(lib().sd_comm_rccl_info(ctypes.byref(v), buf, len(buf)))
    code = v.value
    return {"version_code": code, "version": f"{code // 10000}.{code // 100 % 100}.{code % 100}",
            "path": os.path.realpath(buf.value.decode()) if buf.value else None}


def lib():
    """The loaded library; raises ImportError (no fallback) if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). spacedrive_amd has no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != SD_OK:
        msg = lib().sd_cas_last_error()
        raise SdCasError(rc, msg.decode() if msg else "")


def path_array(paths) -> tuple:
    """(keepalive, char** address) for n paths: one NUL-joined buffer and a u64 pointer array
    computed from its NUL positions with numpy.  A ctypes array of n separately encoded
    strings costs ~0.7 us per path in Python (24 ms for the identifier's 32768-file
    look-ahead call, more than the library's own work); this costs ~0.05 us.  Paths are
    encoded as os.fsencode does (utf-8, surrogateescape); a path holding a NUL raises
    ValueError, as open() does."""
    import numpy as np
    n = len(paths)
    try:
        buf = ("\0".join(paths) + "\0").encode("utf-8", "surrogateescape")
    except TypeError:  # PathLike or bytes entries
        buf = b"\0".join(os.fsencode(p) for p in paths) + b"\0"
    ends = np.flatnonzero(np.frombuffer(buf, np.uint8) == 0)
    if len(ends) != max(n, 1):
        raise ValueError("embedded null byte in a path")
    base = ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    ptrs = np.empty(max(n, 1), np.uint64)
    ptrs[0] = base
    ptrs[1:] = ends[:-1].astype(np.uint64) + np.uint64(base + 1)
    return (buf, ptrs), ptrs.ctypes.data


def hex_results(out, width: int, status, paths, err) -> list:
    """The n NUL-terminated hex strings of `width` chars in `out` (a ctypes string buffer),
    with err(status, path) in place of each entry whose status is not SD_FILE_OK."""
    import numpy as np
    n = len(paths)
    bad = np.flatnonzero(np.asarray(status[:n]) != SD_FILE_OK).tolist()
    if not bad:  # every entry is `width` hex chars + NUL: one C-level split
        res = ctypes.string_at(out, (width + 1) * n - 1).decode("latin-1").split("\0")
        if len(res) == n and all(len(r) == width for r in (res[0], res[-1])):
            return res
    res = np.frombuffer(out, dtype=f"S{width + 1}", count=n).astype(f"U{width}").tolist()
    for i in bad:
        res[i] = err(int(status[i]), os.fsdecode(paths[i]))
    return res
