"""Device-level interface over libsdcas.so: contexts, prepared batches, device buffers.

Device memory and streams are torch tensors / torch streams (plumbing only); every byte
of hashing runs in the gfx950 kernels of ``csrc/cas_kernels.hip``.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from ._native import Extent, SdCasError, check, lib

EXTENT_DTYPE = np.dtype([("size", "<u8"), ("msg_offset", "<u8"), ("msg_len", "<u4"), ("kind", "<u4")])
assert EXTENT_DTYPE.itemsize == ctypes.sizeof(Extent) == 24


def _ptr(x) -> Optional[int]:
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return int(x)


def _stream(stream) -> Optional[int]:
    """The HIP stream handle a wrapper passes to the C ABI.  A stream other than the
    current one is first ordered after the work queued so far on the current stream (an
    event recorded there, waited on by `stream`): the inputs a caller just produced --
    torch fills, copies, kernels on the current stream -- are complete before the
    library's kernels read them, with no manual wait_stream.  The reverse order (the
    outputs, consumed back on the current stream) stays the caller's, as in torch."""
    cur = torch.cuda.current_stream()
    if stream is None:
        return cur.cuda_stream
    s = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(int(stream))
    if s.cuda_stream != cur.cuda_stream:
        s.wait_stream(cur)
    return s.cuda_stream


def stage_plan(sizes) -> tuple:
    """cas.rs:25-58 message layout for files of these sizes -> (extents, staged_bytes)."""
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    ext = np.zeros(len(sizes), dtype=EXTENT_DTYPE)
    total = ctypes.c_uint64(0)
    check(lib().sd_cas_stage_plan(_ptr(sizes), len(sizes), _ptr(ext), ctypes.byref(total)))
    return ext, int(total.value)


class Context:
    """One per device and process; thread-safe (sd_cas_ctx)."""

    def __init__(self, device: Optional[int] = None):
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        h = ctypes.c_void_p()
        check(lib().sd_cas_ctx_create(device, ctypes.byref(h)))
        self.handle = h

    def close(self) -> None:
        if self.handle:
            lib().sd_cas_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- batches
    def cas_batch(self, extents: np.ndarray) -> "CasBatch":
        return CasBatch(self, extents)

    def checksum_batch(self, offsets, lens) -> "ChecksumBatch":
        return ChecksumBatch(self, offsets, lens)

    # -------------------------------------------------------------- files -> device hashes
    def hashes_files(self, paths, sizes, d_hash32, d_valid=None, nthreads: int = 16) -> np.ndarray:
        """sd_cas_hashes_files: generate_cas_id's messages of these files hashed into
        d_hash32 (device, n x 32 B; the cas_id is each row's first 8 bytes) and, if given,
        d_valid (device, n B: hashed and not empty).  Returns the int32 status per file."""
        from ._native import path_array
        n = len(paths)
        status = np.zeros(max(n, 1), np.int32)
        keep, arr = path_array(paths)
        sz = np.ascontiguousarray(sizes, dtype=np.uint64)
        assert d_hash32.numel() >= 32 * n and (d_valid is None or d_valid.numel() >= n)
        # the library writes the rows from its own streams: whatever the caller queued on
        # the current stream (e.g. the buffers' zero fills) must be done first
        torch.cuda.current_stream().synchronize()
        check(lib().sd_cas_hashes_files(self.handle, arr, _ptr(sz), n, _ptr(d_hash32),
                                        None if d_valid is None else _ptr(d_valid), _ptr(status), nthreads))
        return status[:n]

    # -------------------------------------------------------------- synthetic data
    def synth_stage_cas(self, d_sizes, d_cids, d_twins, d_extents, n, d_staged, stream=None) -> None:
        check(lib().sd_synth_stage_cas(self.handle, _ptr(d_sizes), _ptr(d_cids), _ptr(d_twins),
                                       _ptr(d_extents), n, _ptr(d_staged), _stream(stream)))

    def synth_fill(self, cid: int, twin: int, length: int, d_out, stream=None, offset: int = 0) -> None:
        """bytes [offset, offset + length) of synthetic content (cid, twin) -> d_out"""
        check(lib().sd_synth_fill_at(self.handle, cid, twin, offset, length, _ptr(d_out), _stream(stream)))

    def valu_peak(self) -> float:
        v = ctypes.c_double(0)
        check(lib().sd_valu_peak(self.handle, ctypes.byref(v)))
        return float(v.value)

    # -------------------------------------------------------------- dedup
    def dedup_partition(self, d_hash32, d_valid, n: int, base: int, nparts: int, d_counts, d_records,
                        stream=None) -> int:
        nv = ctypes.c_uint64(0)
        check(lib().sd_dedup_partition(self.handle, _ptr(d_hash32), _ptr(d_valid), n, base, nparts,
                                       _ptr(d_counts), _ptr(d_records), ctypes.byref(nv), _stream(stream)))
        return int(nv.value)

    def dedup_group(self, d_records, m: int, d_rep, stream=None, index_sorted: bool = False) -> int:
        ng = ctypes.c_uint64(0)
        check(lib().sd_dedup_group(self.handle, _ptr(d_records), m, 1 if index_sorted else 0, _ptr(d_rep),
                                   ctypes.byref(ng), _stream(stream)))
        return int(ng.value)

    def dedup_owners(self, d_records, m: int, d_rep, d_owner, chunk_size: int = 100, stream=None) -> None:
        check(lib().sd_dedup_owners(self.handle, _ptr(d_records), m, _ptr(d_rep), chunk_size, _ptr(d_owner),
                                    _stream(stream)))

    def dedup_mgpu(self, comm: "Comm", d_hash32, d_valid, n: int, base: int, d_records, d_rep, d_owner,
                   capacity: int, chunk_size: int = 100, stream=None):
        """sd_cas_dedup_mgpu: partition -> RCCL all-to-all -> group -> owners on this rank.
        Returns (m, n_groups); raises SdCasError (SD_ERR_CAPACITY) on every rank when some
        rank's capacity is short -- then ``.needed`` is this rank's requirement."""
        m = ctypes.c_uint64(0)
        ng = ctypes.c_uint64(0)
        rc = lib().sd_cas_dedup_mgpu(self.handle, comm.handle, _ptr(d_hash32), _ptr(d_valid), n, base, chunk_size,
                                     _ptr(d_records), _ptr(d_rep), _ptr(d_owner), capacity, ctypes.byref(m),
                                     ctypes.byref(ng), _stream(stream))
        try:
            check(rc)
        except SdCasError as e:
            e.needed = int(m.value)
            raise
        return int(m.value), int(ng.value)


class CommGroup:
    """sd_comm_group: the in-process rendezvous of ``nranks`` ranks that are threads of one
    process (one Comm per thread, each on its own Context).  Close it after its Comms."""

    def __init__(self, nranks: int):
        h = ctypes.c_void_p()
        check(lib().sd_comm_group_create(nranks, ctypes.byref(h)))
        self.handle, self.nranks = h, nranks

    def close(self) -> None:
        if self.handle:
            lib().sd_comm_group_destroy(self.handle)
            self.handle = None


class Comm:
    """libsdcas's communicator (sd_comm): one per rank, on its context's device -- RCCL, or
    the in-process transport of a CommGroup."""

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(Comm.ID_BYTES)
        check(lib().sd_comm_id(buf))
        return buf.raw

    def __init__(self, ctx: Context, uid: Optional[bytes], nranks: int, rank: int,
                 group: Optional["CommGroup"] = None):
        """RCCL (``uid`` from ``unique_id()`` on one rank) or, with ``group``, the in-process
        transport (sd_comm_create_local: the ranks are threads of this process)."""
        h = ctypes.c_void_p()
        if group is not None:
            assert group.nranks == nranks
            check(lib().sd_comm_create_local(ctx.handle, group.handle, rank, ctypes.byref(h)))
        else:
            assert uid is not None and len(uid) == Comm.ID_BYTES
            check(lib().sd_comm_create(ctx.handle, uid, nranks, rank, ctypes.byref(h)))
        self.handle, self.nranks, self.rank, self.group = h, nranks, rank, group

    PHASES = ("partition", "allgather_rows", "host_turnaround", "sendrecv", "group_owners")  # SD_DEDUP_PHASES

    def set_timing(self, on: bool) -> None:
        """sd_comm_set_timing: record HIP events at the phases of each sd_cas_dedup_mgpu call."""
        check(lib().sd_comm_set_timing(self.handle, 1 if on else 0))

    def last_phases(self) -> dict:
        """sd_comm_last_phases: the last timed call's phase durations (ms), by name."""
        ms = (ctypes.c_float * len(Comm.PHASES))()
        check(lib().sd_comm_last_phases(self.handle, ms))
        return {k: float(v) for k, v in zip(Comm.PHASES, ms)}

    def close(self) -> None:
        if self.handle:
            lib().sd_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class CasBatch:
    """Prepared cas_id batch (sd_cas_batch): run over device-resident staged messages."""

    def __init__(self, ctx: Context, extents: np.ndarray):
        self.ctx = ctx
        self.extents = np.ascontiguousarray(extents, dtype=EXTENT_DTYPE)
        h = ctypes.c_void_p()
        check(lib().sd_cas_batch_create(ctx.handle, _ptr(self.extents), len(self.extents), ctypes.byref(h)))
        self.handle = h
        st = np.zeros(8, np.uint64)
        check(lib().sd_cas_batch_stats(h, _ptr(st)))
        (self.n, self.n_sampled, self.n_whole, self.whole_chunks, self.compressions,
         self.msg_bytes, self.full_items, self.tail_items) = (int(v) for v in st)

    def run(self, d_staged: torch.Tensor, d_hash32: torch.Tensor, stream=None) -> None:
        assert d_hash32.numel() >= 32 * self.n and d_staged.is_cuda and d_hash32.is_cuda
        check(lib().sd_cas_batch_run(self.ctx.handle, self.handle, _ptr(d_staged), _ptr(d_hash32),
                                     _stream(stream)))

    def run_part(self, parts: int, d_staged: torch.Tensor, d_hash32: torch.Tensor, stream=None) -> None:
        """parts: 1 = sampled-file kernel only, 2 = whole-file kernels only."""
        check(lib().sd_cas_batch_run_part(self.ctx.handle, self.handle, parts, _ptr(d_staged), _ptr(d_hash32),
                                          _stream(stream)))

    def time(self, d_staged, d_hash32, iters: int, stream=None) -> float:
        ms = ctypes.c_float(0)
        check(lib().sd_cas_batch_time(self.ctx.handle, self.handle, _ptr(d_staged), _ptr(d_hash32), iters,
                                      _stream(stream), ctypes.byref(ms)))
        return float(ms.value)

    def close(self) -> None:
        if self.handle:
            lib().sd_cas_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class ChecksumBatch:
    """Prepared full-file checksum batch (sd_checksum_batch) over byte ranges of one buffer."""

    def __init__(self, ctx: Context, offsets, lens):
        self.ctx = ctx
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint64)
        h = ctypes.c_void_p()
        check(lib().sd_checksum_batch_create(ctx.handle, _ptr(self.offsets), _ptr(self.lens), len(self.lens),
                                             ctypes.byref(h)))
        self.handle = h
        st = np.zeros(4, np.uint64)
        check(lib().sd_checksum_batch_stats(h, _ptr(st)))
        self.n, self.total_bytes, self.compressions, self.blocks = (int(v) for v in st)

    def run(self, d_data: torch.Tensor, d_hash32: torch.Tensor, stream=None) -> None:
        assert d_hash32.numel() >= 32 * self.n
        check(lib().sd_checksum_batch_run(self.ctx.handle, self.handle, _ptr(d_data), _ptr(d_hash32),
                                          _stream(stream)))

    def time(self, d_data, d_hash32, iters: int, stream=None) -> float:
        ms = ctypes.c_float(0)
        check(lib().sd_checksum_batch_time(self.ctx.handle, self.handle, _ptr(d_data), _ptr(d_hash32), iters,
                                           _stream(stream), ctypes.byref(ms)))
        return float(ms.value)

    def close(self) -> None:
        if self.handle:
            lib().sd_checksum_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class SplitChecksum:
    """One file's checksum over the ranks of a communicator (sd_split_checksum): this rank
    hashes its block range to CVs; the gathered CVs reduce to the file's BLAKE3."""

    def __init__(self, ctx: Context, total_len: int, nranks: int = 1, rank: int = 0):
        from .split import split_range
        self.ctx = ctx
        self.total_len, self.nranks, self.rank = int(total_len), nranks, rank
        self.offset, self.len, self.cv_bytes = split_range(total_len, nranks, rank)
        h = ctypes.c_void_p()
        check(lib().sd_split_checksum_create(ctx.handle, self.total_len, nranks, rank, ctypes.byref(h)))
        self.handle = h

    def leaves(self, d_slice: torch.Tensor, d_cvs: torch.Tensor, stream=None) -> None:
        assert d_cvs.numel() >= self.cv_bytes and d_slice.numel() >= self.len
        check(lib().sd_split_checksum_leaves(self.ctx.handle, self.handle, _ptr(d_slice), _ptr(d_cvs),
                                             _stream(stream)))

    def root(self, d_cvs: torch.Tensor, d_hash32: torch.Tensor, stream=None) -> None:
        assert d_cvs.numel() >= self.cv_bytes and d_hash32.numel() >= 32
        check(lib().sd_split_checksum_root(self.ctx.handle, self.handle, _ptr(d_cvs), _ptr(d_hash32),
                                           _stream(stream)))

    def mgpu(self, comm: "Comm", d_slice: torch.Tensor, d_cvs: torch.Tensor, d_hash32: torch.Tensor,
             stream=None) -> None:
        assert d_cvs.numel() >= self.cv_bytes and d_slice.numel() >= self.len and d_hash32.numel() >= 32
        check(lib().sd_split_checksum_mgpu(self.ctx.handle, comm.handle, self.handle, _ptr(d_slice), _ptr(d_cvs),
                                           _ptr(d_hash32), _stream(stream)))

    def close(self) -> None:
        if self.handle:
            lib().sd_split_checksum_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_default: dict = {}


def default_context(device: Optional[int] = None) -> Context:
    if device is None:
        device = torch.cuda.current_device()
    ctx = _default.get(device)
    if ctx is None:
        ctx = _default[device] = Context(device)
    return ctx
