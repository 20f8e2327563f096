"""The N > 1 dedup path on CPU: file-sharded records exchanged by cas_id prefix over a
world-size-2 (and 3) gloo group must reproduce the single-process grouping exactly
(SURVEY.md §8(e)).  The device kernels behind partition/group are checked against the
same host mirrors on the GPU (tests/test_gpu_parity.py::test_dedup_group_matches_host)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from spacedrive_amd.dedup import dest_of, exchange, group_host, partition_host


def _keys(n_total, seed=3):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 1 << 63, n_total, dtype=np.int64).astype(np.uint64) * np.uint64(2)
    dup = rng.random(n_total) < 0.25
    src = rng.integers(0, n_total, n_total)
    keys[dup] = keys[src[dup]]  # duplicates across shards
    keys[:5] = np.uint64(0xFFFF_FFFF_FFFF_FFFF)  # top of the prefix range
    keys[5:9] = np.uint64(0)
    return keys


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = _keys(world * n_per)[rank * n_per:(rank + 1) * n_per]
        idx = np.arange(rank * n_per, (rank + 1) * n_per, dtype=np.int64)
        valid = np.ones(n_per, bool)
        valid[::97] = False  # empty files never dedup
        recs, counts = partition_host(keys[valid], idx[valid], world)
        recv = exchange(torch.from_numpy(recs), torch.from_numpy(counts))
        r, rep, ng = group_host(recv.numpy())
        np.save(os.path.join(outdir, f"r{rank}.npy"), np.concatenate([r, rep[:, None]], axis=1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the driver's node, rehearsed on gloo
def test_distributed_grouping_equals_single_process(tmp_path, world):
    n_per = 4000
    mp.start_processes(_worker, args=(world, _free_port(), n_per, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    n_total = world * n_per
    keys = _keys(n_total)
    idx = np.arange(n_total, dtype=np.int64)
    valid = np.ones(n_total, bool)
    for r in range(world):
        valid[r * n_per:(r + 1) * n_per][::97] = False
    ref, ref_rep, ref_ng = group_host(np.stack([keys[valid].view(np.int64), idx[valid]], axis=1))
    parts = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    # each rank owns a contiguous cas_id prefix range, in rank order
    for r, p in enumerate(parts):
        assert np.all(dest_of(p[:, 0].view(np.uint64), world) == r)
    got = np.concatenate(parts)
    assert np.array_equal(got[:, :2], ref)
    assert np.array_equal(got[:, 2], ref_rep)
    # grouping semantics: rep is the smallest index with an equal cas_id
    k = ref[:, 0]
    for i in np.nonzero(np.r_[True, k[1:] != k[:-1]])[0][:200]:
        same = ref[k == k[i]]
        assert ref_rep[i] == same[:, 1].min()


def test_single_rank_exchange_is_identity():
    recs = torch.arange(10, dtype=torch.int64).view(5, 2)
    assert exchange(recs, torch.tensor([5])) is recs


def _ascend_worker(rank, world, port, outdir):
    from spacedrive_amd.dedup import shards_ascend
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = [shards_ascend(100, rank * 100),          # contiguous, ascending
               shards_ascend(100, (world - 1 - rank) * 100),  # descending: received records not index-sorted
               shards_ascend(100, rank * 50)]            # overlapping ranges
        np.save(os.path.join(outdir, f"a{rank}.npy"), np.array(res))
    finally:
        dist.destroy_process_group()


def test_shards_ascend_is_checked_across_ranks(tmp_path):
    """the index-sorted grouping fast path is taken only when every rank's
    [base, base + n) ends before the next rank's starts (checked by one all-gather)."""
    world = 3
    mp.start_processes(_ascend_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert np.load(tmp_path / f"a{r}.npy").tolist() == [True, False, False]


def test_shard_plan_balances_hashing_cost():
    """sd_shard_plan: contiguous, ascending, complete, and balanced in BLAKE3 compressions
    (a sampled file costs 953, a small one 1..146) to within one file's cost per boundary."""
    from spacedrive_amd.dedup import shard_plan
    from spacedrive_amd import synth

    def cost(s):
        m = 8 + s if s <= 102400 else 57352
        c = max(1, -(-m // 1024))
        last = m - (c - 1) * 1024
        return (c - 1) * 16 + max(1, -(-last // 64)) + (c - 1)

    sizes, _, _ = synth.library(0, 50_000, 50_000)
    sizes = np.asarray(sizes, np.uint64)
    sizes[:20000] = 5  # a skewed library: small files first, then the mixture
    costs = np.array([cost(int(s)) for s in sizes])
    for R in (1, 2, 3, 8, 64):
        b = shard_plan(sizes, R).astype(np.int64)
        assert b[0] == 0 and b[-1] == len(sizes) and np.all(np.diff(b) >= 0)
        per = np.array([costs[b[r]:b[r + 1]].sum() for r in range(R)])
        assert per.max() - per.min() <= 2 * costs.max(), (R, per.min(), per.max())
    assert list(shard_plan(np.zeros(0, np.uint64), 3)) == [0, 0, 0, 0]
