"""One file's checksum over many ranks (a file's 1 MiB blocks shard
naturally).

``file_checksum`` (core/src/object/validation/hash.rs:10-24) is BLAKE3 of the file's bytes.
BLAKE3's tree makes every 1 MiB block's chaining value (CV) a function of that block's
bytes and position only, so rank r of R can hash its contiguous block range
[r*q, min((r+1)*q, nb)), q = ceil(nb / R), without seeing the rest of the file; the CVs of
all ranks laid end to end in rank order are the file's block CVs, and one reduce gives the
file's hash -- the same 64-hex string ``file_checksum`` returns.  The exchange is 32 bytes
per MiB of file (1 MB for 32 GiB).

Backends, all with the same block partition (``split_range`` = the C ABI's sd_split_range):
* ``SplitChecksum.mgpu`` (device.py): leaves + in-place ncclAllGather + root inside
  libsdcas over its RCCL communicator -- the MI355X path;
* ``checksum_split`` here: the same steps with the gather through ``torch.distributed``
  (all_gather), on the device (nccl) or on host cores (gloo + the library's
  CPU leaves/root) -- the statement the CPU tests run at world sizes 2 and 3.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from ._native import check, lib

BLOCK = 1 << 20


def split_range(total_len: int, nranks: int, rank: int) -> Tuple[int, int, int]:
    """(offset, len, cv_bytes): the file bytes rank `rank` holds and the CV buffer size."""
    o, n, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().sd_split_range(int(total_len), nranks, rank, ctypes.byref(o), ctypes.byref(n), ctypes.byref(c)))
    return o.value, n.value, c.value


def cpu_leaves(slice_bytes: np.ndarray, total_len: int, nranks: int, rank: int, nthreads: int = 16) -> np.ndarray:
    """This rank's block CVs on host cores: a uint8 array of cv_bytes, its own slots set."""
    _, length, cv_bytes = split_range(total_len, nranks, rank)
    s = np.ascontiguousarray(slice_bytes, dtype=np.uint8)
    assert s.size >= length
    cvs = np.zeros(cv_bytes, np.uint8)
    check(lib().sd_cpu_split_leaves(s.ctypes.data if s.size else None, int(total_len), nranks, rank,
                                    cvs.ctypes.data, nthreads))
    return cvs


def cpu_root(cvs: np.ndarray, total_len: int) -> bytes:
    c = np.ascontiguousarray(cvs, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    check(lib().sd_cpu_split_root(c.ctypes.data, int(total_len), out))
    return out.raw


def _gather_slots(cvs, r: int, R: int, q: int, group) -> None:
    """In place: every rank's q CV slots into their rank-ordered places."""
    import torch.distributed as dist
    rows = cvs.view(R, q * 32)
    dist.all_gather(list(rows.unbind(0)), rows[r].clone(), group=group)


def checksum_split(slice_data, total_len: int, ctx=None, group=None) -> str:
    """file_checksum of a file of `total_len` bytes whose range ``split_range(total_len, R, r)``
    this rank holds in `slice_data` (a uint8 torch tensor: on the device with `ctx`, else on
    the host), collective over the torch.distributed group.  Returns the 64-hex hash on
    every rank."""
    import torch
    import torch.distributed as dist
    R = dist.get_world_size(group) if dist.is_initialized() else 1
    r = dist.get_rank(group) if dist.is_initialized() else 0
    off, length, cv_bytes = split_range(total_len, R, r)
    q = cv_bytes // (32 * R)
    if ctx is not None:
        from .device import SplitChecksum
        sc = SplitChecksum(ctx, total_len, R, r)
        try:
            cvs = torch.zeros(cv_bytes, dtype=torch.uint8, device=slice_data.device)
            sc.leaves(slice_data, cvs)
            if R > 1:
                _gather_slots(cvs, r, R, q, group)
            out = torch.empty(32, dtype=torch.uint8, device=slice_data.device)
            sc.root(cvs, out)
            torch.cuda.synchronize(slice_data.device)
            return bytes(out.cpu().numpy()).hex()
        finally:
            sc.close()
    cvs = torch.from_numpy(cpu_leaves(slice_data.numpy(), total_len, R, r))
    if R > 1:
        _gather_slots(cvs, r, R, q, group)
    return cpu_root(cvs.numpy(), total_len).hex()


def file_checksum_split(path, ctx=None, group=None) -> str:
    """file_checksum (hash.rs:10-24) of one file on disk, computed by all ranks of the group:
    every rank stats the file, preads only its own byte range ``split_range(len, R, r)`` and
    hashes it (on the device with `ctx`, else on host cores); the block CVs are gathered and
    every rank returns the 64-hex hash.  For a file that is not being written: the ranks
    must see the same length (it is checked across the group)."""
    import os

    import torch
    import torch.distributed as dist
    R = dist.get_world_size(group) if dist.is_initialized() else 1
    r = dist.get_rank(group) if dist.is_initialized() else 0
    total = os.stat(path).st_size
    if R > 1:
        lens = [None] * R
        dist.all_gather_object(lens, total, group=group)
        if len(set(lens)) != 1:
            raise OSError(f"{path}: length differs across ranks {lens} (the file is changing)")
    off, length, _ = split_range(total, R, r)
    buf = np.zeros(length + 64, np.uint8)  # zero padding past the slice (the kernels' rule)
    fd = os.open(path, os.O_RDONLY)
    try:
        got = 0
        mv = memoryview(buf)
        while got < length:
            k = os.preadv(fd, [mv[got:length]], off + got)
            if k == 0:
                raise OSError(f"{path}: shorter than its length {total} (the file is changing)")
            got += k
    finally:
        os.close(fd)
    t = torch.from_numpy(buf)
    if ctx is not None:
        dev = torch.device("cuda", torch.cuda.current_device())
        t = t.to(dev)
    return checksum_split(t, total, ctx=ctx, group=group)
