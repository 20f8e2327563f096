"""One rank's part of a multi-GPU library scan from files on disk: the file identifier
(core/src/object/file_identifier/mod.rs:57-333) over a whole library, one process per GPU.

    bounds = dedup.shard_plan(sizes, R)                  # contiguous, cost-balanced shards
    rank r: sd_cas_hashes_files(its files)               # cas_id messages read as cas.rs does,
                                                         # hashed into device rows
            sd_cas_dedup_mgpu(rows, comm)                # cas_id-prefix all-to-all over RCCL,
                                                         # grouping, chunk-of-100 Object rule
Every rank returns its shard's cas_ids (status per file as generate_cas_id's Result) and
the groups / Object owners of the cas_id prefix range it owns.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import dedup
from .cas import _status_error
from ._native import SD_FILE_OK


def scan_library(ctx, paths: Sequence[str], sizes, comm=None, group: Optional[dist.ProcessGroup] = None,
                 chunk_size: int = 100, nthreads: int = 16) -> dict:
    """This rank's share of the scan of the whole library (`paths`, `sizes` as the walker's
    metadata reported them; the same lists on every rank).  With `comm` (libsdcas's RCCL
    communicator, dedup.make_comm) the exchange runs inside the library; without it, over
    torch.distributed.  Returns {"shard": (lo, hi), "cas_ids": [str | OSError] for files
    lo..hi-1, "records": int64 [m, 2] (cas_id key, global index) sorted, "rep": [m],
    "owner": [m], "n_groups": int}."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    bounds = dedup.shard_plan(sizes, world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    n = hi - lo
    dev = torch.device("cuda", torch.cuda.current_device())
    d_hash = torch.zeros((max(n, 1), 32), dtype=torch.uint8, device=dev)
    d_valid = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    status = ctx.hashes_files(list(paths[lo:hi]), sizes[lo:hi], d_hash, d_valid, nthreads=nthreads)
    if comm is not None:
        runner = dedup.RcclDedup(ctx, comm, dev, capacity=n * 5 // 4 + 4096)
        recs, rep, ng, owner = runner(d_hash, d_valid, n, lo, chunk_size=chunk_size)
    else:
        recs, rep, ng, owner = dedup.dedup_shard(ctx, d_hash, d_valid, n, lo, group)
    h = d_hash[:n].cpu().numpy()
    ids = [h[i, :8].tobytes().hex() if status[i] == SD_FILE_OK else _status_error(int(status[i]), str(paths[lo + i]))
           for i in range(n)]
    return {"shard": (lo, hi), "cas_ids": ids, "records": recs, "rep": rep, "owner": owner, "n_groups": ng}
