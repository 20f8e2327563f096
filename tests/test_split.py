"""One file's checksum over many ranks (VERDICT r1 missing #7) on CPU:
the block partition (sd_split_range), the library's CPU leaves + root for every rank count
against the oracle's BLAKE3 of the whole file, and the torch.distributed statement over
world-size 2 and 3 gloo groups.  The device leaves/root and the RCCL gather are checked on
the GPU (tests/test_gpu_parity.py::test_split_checksum_*)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import native
from spacedrive_amd._native import SdCasError
from spacedrive_amd.split import BLOCK, checksum_split, cpu_leaves, cpu_root, file_checksum_split, split_range

SIZES = [0, 1, 1023, 1024, 1025, BLOCK - 1, BLOCK, BLOCK + 1, 2 * BLOCK, 5 * BLOCK + 3, 17 * BLOCK,
         33 * BLOCK + 12345]


def _data(total, seed=1):
    d = np.random.default_rng(seed + total).integers(0, 256, total + 64, dtype=np.uint8)
    d[total:] = 0
    return d


def _oracle(d, total):
    return native.checksums_simd(d, [0], [total], nthreads=4)[0].tobytes()


def test_split_range_partition():
    for total in SIZES + [(1 << 40) + 7]:
        nb = max(1, -(-total // BLOCK))
        for R in (1, 2, 3, 5, 8, 64):
            q = -(-nb // R)
            end = 0
            for r in range(R):
                off, ln, cv = split_range(total, R, r)
                assert cv == R * q * 32
                assert off == min(total, min(nb, r * q) * BLOCK) and off == end  # contiguous, in rank order
                end = off + ln
            assert end == total
    with pytest.raises(SdCasError):
        split_range(10, 2, 2)
    with pytest.raises(SdCasError):
        split_range(10, 0, 0)


@pytest.mark.parametrize("total", SIZES)
def test_cpu_split_equals_whole_file_blake3(total):
    d = _data(total)
    want = _oracle(d, total)
    for R in (1, 2, 3, 4, 7):
        cvs = None
        for r in range(R):
            off, ln, cv_bytes = split_range(total, R, r)
            mine = cpu_leaves(d[off:off + ln], total, R, r, nthreads=3)
            q = cv_bytes // (32 * R)
            if cvs is None:
                cvs = np.zeros(cv_bytes, np.uint8)
            cvs[r * q * 32:(r + 1) * q * 32] = mine[r * q * 32:(r + 1) * q * 32]
        assert cpu_root(cvs, total) == want, (total, R)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = []
        for total in (3 * BLOCK + 5, 10 * BLOCK, 100):
            d = _data(total, seed=7)
            off, ln, _ = split_range(total, world, rank)
            res.append(checksum_split(torch.from_numpy(d[off:off + ln].copy()), total))
        res.append(file_checksum_split(os.path.join(outdir, "file.bin")))  # each rank reads its range
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write("\n".join(res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the driver's node, rehearsed on gloo
def test_checksum_split_over_gloo(tmp_path, world):
    fdata = _data(5 * BLOCK + 999, seed=9)[:5 * BLOCK + 999]
    (tmp_path / "file.bin").write_bytes(fdata.tobytes())
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    want = [_oracle(_data(t, seed=7), t).hex() for t in (3 * BLOCK + 5, 10 * BLOCK, 100)]
    want.append(_oracle(_data(5 * BLOCK + 999, seed=9), 5 * BLOCK + 999).hex())
    for r in range(world):
        assert open(tmp_path / f"r{r}.txt").read().split("\n") == want, r
