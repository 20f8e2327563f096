"""Post-hash duplicate grouping across GPUs.

Reference semantics (core/src/object/file_identifier/mod.rs:136-333): after hashing a
step's files, each file_path is linked to an Object that already owns an equal cas_id,
otherwise a new Object is created; size-0 files (cas_id None, mod.rs:80-88) never
dedup.  The partition of files into equal-cas_id groups is what this module computes,
bit-exactly; which member becomes the Object is a policy of the caller (the reference's
choice depends on 100-row chunking and HashMap order, §8(e)), here the smallest global
file index of the group (the "Object-link candidate").

Multi-GPU: files are sharded by index; each rank buckets its records
``(cas_id as big-endian u64, global index)`` by cas_id prefix (device kernel
``sd_dedup_partition``), the records move to the rank owning their prefix range, and
each rank sorts and groups its bucket (``sd_dedup_group``) and assigns Objects
(``sd_dedup_owners``).  Two transports for the exchange:

* ``dedup_shard_rccl`` -- the product path on GPUs: the whole step behind the C ABI
  (``sd_cas_dedup_mgpu``): an RCCL all-gather of the count matrix, then grouped
  ncclSend/ncclRecv of the records (the all-to-all over xGMI), on libsdcas's own RCCL
  communicator (``make_comm``), so a Rust host drives the same code;
* ``dedup_shard`` -- the same step with the exchange in ``torch.distributed``
  (``all_to_all_single``), which also runs on "gloo" for the CPU tests.

No other collective exists on the data path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_plan(sizes, nranks: int) -> np.ndarray:
    """Contiguous index ranges of balanced hashing cost for a library scan over `nranks`
    GPUs (sd_shard_plan): rank r hashes files [bounds[r], bounds[r+1]).  The cost of a file
    is the BLAKE3 compressions of its cas message."""
    import ctypes
    from ._native import check, lib
    s = np.ascontiguousarray(sizes, dtype=np.uint64)
    bounds = np.zeros(nranks + 1, np.uint64)
    check(lib().sd_shard_plan(s.ctypes.data if s.size else None, ctypes.c_size_t(s.size), nranks, bounds.ctypes.data))
    return bounds


def dest_of(keys: np.ndarray, nparts: int) -> np.ndarray:
    """Destination rank of a cas_id key: its top 16 bits scaled to nparts (contiguous ranges)."""
    return (((keys >> np.uint64(48)) * np.uint64(nparts)) >> np.uint64(16)).astype(np.int64)


def keys_from_hashes(h32: np.ndarray) -> np.ndarray:
    """First 8 hash bytes as a big-endian u64 (== the hex cas_id's lexicographic order)."""
    return h32[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)


def exchange(send_records: torch.Tensor, send_counts: torch.Tensor,
             group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All-to-all of records grouped by destination.

    send_records: int64 [m, 2] (key, global index) ordered by destination rank;
    send_counts:  int64 [world] records per destination.  Returns the received records.
    Works for any backend whose tensors live on the device of ``send_records``.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return send_records
    if dist.get_backend(group) == "gloo" and send_records.is_cuda:
        # CPU transport (tests / single-GPU rehearsal): same exchange, host tensors
        dev = send_records.device
        return exchange(send_records.cpu(), send_counts.cpu(), group).to(dev)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rc = recv_counts.cpu().tolist()
    sc = send_counts.cpu().tolist()
    out = torch.empty((int(sum(rc)), 2), dtype=send_records.dtype, device=send_records.device)
    dist.all_to_all_single(out, send_records, output_split_sizes=rc, input_split_sizes=sc, group=group)
    return out


def group_device(ctx, records: torch.Tensor, index_sorted: bool = False) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Sort received records by (cas_id, index) and map each to its group's smallest index."""
    m = records.shape[0]
    rep = torch.empty(max(m, 1), dtype=torch.int64, device=records.device)
    ng = ctx.dedup_group(records, m, rep, index_sorted=index_sorted)
    return records, rep[:m], ng


def shards_ascend(n_local: int, global_base: int, group: Optional[dist.ProcessGroup] = None,
                   device=None) -> bool:
    """True when every rank's index range [base, base + n) ends before the next rank's
    starts: the records received in rank order are then in ascending index order."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return True
    mine = torch.tensor([global_base, n_local], dtype=torch.int64, device=device)
    rows = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine, group=group)
    r = torch.stack(rows).cpu().tolist()
    return all(r[k][0] + r[k][1] <= r[k + 1][0] for k in range(world - 1))


def dedup_shard(ctx, d_hash32: torch.Tensor, d_valid: Optional[torch.Tensor], n_local: int, global_base: int,
                group: Optional[dist.ProcessGroup] = None, index_sorted: Optional[bool] = None):
    """Full distributed step on one rank: partition -> exchange -> group -> Object owners.

    Returns (records int64 [m, 2] sorted by (key, index), rep int64 [m], n_groups,
    owner int64 [m]) for the cas_id prefix range this rank owns; owner is the file whose
    Object each record links to under the reference's chunk-of-100 rule
    (spacedrive_amd/identifier.py).  ``index_sorted``: whether the shards' index ranges
    ascend with the rank (checked with one small all-gather when None).
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dev = d_hash32.device
    if index_sorted is None:
        gloo = world > 1 and dist.get_backend(group) == "gloo"
        index_sorted = shards_ascend(n_local, global_base, group, "cpu" if gloo else dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    recs = torch.empty((max(n_local, 1), 2), dtype=torch.int64, device=dev)
    nv = ctx.dedup_partition(d_hash32, d_valid, n_local, global_base, world, counts, recs)
    recv = exchange(recs[:nv], counts, group)
    # the partition is stable: with ascending shards the received records are in index
    # order, and one stable cas_id sort suffices
    records, rep, ng = group_device(ctx, recv, index_sorted=index_sorted)
    # identifier.object_owners is the torch statement of the same rule (tests compare them)
    owners = torch.empty(max(records.shape[0], 1), dtype=torch.int64, device=dev)
    ctx.dedup_owners(records, records.shape[0], rep, owners)
    return records, rep, ng, owners[:records.shape[0]]


def make_comm(ctx, group: Optional[dist.ProcessGroup] = None):
    """libsdcas's RCCL communicator over the ranks of ``group``: rank 0's ncclUniqueId is
    broadcast through torch.distributed, then every rank joins (sd_comm_create)."""
    from .device import Comm
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    uid = [Comm.unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0, group=group)
    return Comm(ctx, uid[0], world, rank)


class RcclDedup:
    """sd_cas_dedup_mgpu with reusable output buffers (grown when a rank needs more)."""

    def __init__(self, ctx, comm, device, capacity: int = 0):
        self.ctx, self.comm, self.device = ctx, comm, device
        self.capacity = 0
        self._alloc(capacity)

    def _alloc(self, cap: int) -> None:
        cap = max(int(cap), 1)
        if cap > self.capacity:
            self.records = torch.empty((cap, 2), dtype=torch.int64, device=self.device)
            self.rep = torch.empty(cap, dtype=torch.int64, device=self.device)
            self.owner = torch.empty(cap, dtype=torch.int64, device=self.device)
            self.capacity = cap

    def __call__(self, d_hash32, d_valid, n_local: int, global_base: int, chunk_size: int = 100, stream=None):
        from ._native import SD_ERR_CAPACITY, SdCasError
        for _ in range(2):
            try:
                m, ng = self.ctx.dedup_mgpu(self.comm, d_hash32, d_valid, n_local, global_base, self.records,
                                            self.rep, self.owner, self.capacity, chunk_size, stream)
                return self.records[:m], self.rep[:m], ng, self.owner[:m]
            except SdCasError as e:
                if e.rc != SD_ERR_CAPACITY:
                    raise
                # every rank stopped before the exchange: all retry, each with room for its need
                self._alloc(max(e.needed, self.capacity) * 5 // 4 + 1024)
        raise RuntimeError("sd_cas_dedup_mgpu: capacity still short after regrowing")


def dedup_shard_rccl(ctx, comm, d_hash32: torch.Tensor, d_valid: Optional[torch.Tensor], n_local: int,
                     global_base: int, capacity: Optional[int] = None):
    """dedup_shard through the C ABI's RCCL exchange (sd_cas_dedup_mgpu); same outputs."""
    runner = RcclDedup(ctx, comm, d_hash32.device, capacity if capacity is not None else n_local + 4096)
    return runner(d_hash32, d_valid, n_local, global_base)


# ------------------------------------------------------------------ host reference
def partition_host(keys: np.ndarray, idx: np.ndarray, nparts: int):
    """Host mirror of sd_dedup_partition: stable, grouped by destination, input order within one."""
    d = dest_of(keys, nparts)
    order = np.argsort(d, kind="stable")
    counts = np.bincount(d, minlength=nparts).astype(np.int64)
    recs = np.stack([keys[order].view(np.int64), idx[order].astype(np.int64)], axis=1)
    return recs, counts


def group_host(records: np.ndarray):
    """Host mirror of sd_dedup_group: sort by (key, index); rep = min index of the group."""
    if len(records) == 0:
        return records, np.zeros(0, np.int64), 0
    k = records[:, 0].view(np.uint64)
    i = records[:, 1]
    order = np.lexsort((i, k))
    r = records[order]
    ks = r[:, 0].view(np.uint64)
    head = np.ones(len(r), bool)
    head[1:] = ks[1:] != ks[:-1]
    head_pos = np.maximum.accumulate(np.where(head, np.arange(len(r)), 0))
    return r, r[head_pos, 1], int(head.sum())
