"""bench.py's N > 1 self-checks, rehearsed with more ranks on CPU (gloo, world 2 and 8):
the key-slice parity of the exchange (bench.dedup_parity, with its row gathers of uneven
sizes) must accept a correct multi-rank dedup and reject a corrupted one on every rank.
The device kernels behind the real exchange are covered by the GPU tests; here the
exchanged records come from the host mirrors (dedup.partition_host / exchange /
group_host / identifier.object_owners), so the test isolates the bench's own gathering,
grouping and broadcast logic at the rank counts the driver runs (the N > 1
branch must not meet its first 8-rank run untested)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _library_hashes(world, n_per, seed=17):
    """32-byte hash rows for the whole library: duplicates across shards, and 1 in 8 rows
    forced into bench.dedup_parity's key slice (bits 40..47 of the cas_id key == 0)."""
    rng = np.random.default_rng(seed)
    n = world * n_per
    h = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    dup = rng.random(n) < 0.3
    src = rng.integers(0, n, n)
    h[dup] = h[src[dup]]
    h[rng.random(n) < 0.125, 2] = 0  # key byte 2 = bits 40..47 of the big-endian key
    return h


def _worker(rank, world, port, n_per, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from spacedrive_amd import identifier
        from spacedrive_amd.dedup import exchange, group_host, keys_from_hashes, partition_host
        bench.DIST = True
        h = _library_hashes(world, n_per)[rank * n_per:(rank + 1) * n_per]
        start = rank * n_per
        valid = np.ones(n_per, bool)
        valid[::97] = False  # empty files never dedup
        keys = keys_from_hashes(h)
        idx = np.arange(start, start + n_per, dtype=np.int64)
        recs, counts = partition_host(keys[valid], idx[valid], world)
        recv = exchange(torch.from_numpy(recs), torch.from_numpy(counts))
        r, rep, _ = group_host(recv.numpy())
        owners = identifier.object_owners(torch.from_numpy(r[:, 1].copy()), torch.from_numpy(rep.copy()))
        d_hash = torch.from_numpy(h.reshape(-1).copy())
        d_valid = torch.from_numpy(valid.astype(np.uint8))
        args = (d_hash, d_valid, n_per, start, torch.from_numpy(r.copy()), torch.from_numpy(rep.copy()))
        ok = bench.dedup_parity(*args, owners, world, torch.device("cpu"), "torch")
        # a wrong Object owner for one record inside the slice, on the last rank only
        bad_owners = owners.clone()
        if rank == world - 1:
            sel = np.nonzero(((r[:, 0].view(np.uint64) >> np.uint64(40)) & np.uint64(0xFF)) == 0)[0]
            bad_owners[int(sel[0])] += 1
        bad = bench.dedup_parity(*args, bad_owners, world, torch.device("cpu"), "torch")
        # uneven row counts through bench._gather_rows
        rows = bench._gather_rows(torch.full((rank + 1, 2), rank, dtype=torch.int64), world, "cpu")
        gathered = [int(x.shape[0]) for x in rows]
        np.save(os.path.join(outdir, f"p{rank}.npy"),
                np.array([ok["parity"], bad["parity"], ok.get("records", -1), gathered == list(range(1, world + 1))],
                         dtype=np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_dedup_parity_at_world(tmp_path, world):
    n_per = 2500
    mp.start_processes(_worker, args=(world, _free_port(), n_per, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    assert all(int(x[0]) == 1 for x in res), "a correct exchange must pass on every rank"
    assert all(int(x[1]) == 0 for x in res), "a corrupted owner must fail on every rank"
    assert int(res[0][2]) > 100  # rank 0 checked a real slice of records from every rank
    assert all(int(x[3]) == 1 for x in res)
