"""Full-size parity: the 10 M-file library (configs[4]) and the configs[3] checksums, bit-exact.

BASELINE.json's target is "bit-exact cas_ids and checksums for 10M synthetic files".
This runs the whole 10 M-file library the 8-GPU bench hashes -- the same per-rank shards
(``synth.library(rank * n, n, 10 M)``), one after another on one GPU -- and compares:

* every file's cas_id (8 bytes) with the oracle's (oracle/sd_oracle.c, SIMD hasher over
  messages it builds from the generator itself; checked against the scalar oracle in
  tests/test_oracle.py);
* the dedup exchange: each shard is partitioned on the device into 8 cas_id-prefix
  buckets exactly as its rank would send them (sd_dedup_partition), the buckets are
  concatenated in source-rank order as the all-to-all delivers them, and each is grouped
  on the device (sd_dedup_group).  Records, representatives and group counts must equal
  the host grouping of the ORACLE's cas_ids;
* the same exchange through the library's own multi-rank code: the 8 shards' hashes go to
  8 ranks that are threads of this process on the in-process communicator
  (sd_comm_create_local; RCCL refuses 8 ranks on one GPU), each calls sd_cas_dedup_mgpu
  (partition, gathered count matrix, per-peer record copies, grouping, Object rule) and its
  records, representatives and owners must equal the host grouping + object_owners of the
  oracle's cas_ids of the prefix range it owns;
* configs[3]: the 16 x 4 GiB validator files bench.py times (content ids 10000..10015)
  plus a mixed 2-8 GiB set, full 32-byte BLAKE3 vs the chunk-parallel C oracle.

The oracle is the checker here, never the thing measured.  Usage on the GPU box:

    python scripts/parity_full.py [--files 10000000] [--shards 8] [--out gpurun_out/parity.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GiB = 1 << 30
CK_BENCH = [(4 * GiB, 10_000 + i, 0) for i in range(16)]  # bench.py configs[3], rank 0
CK_MIXED = [(2 * GiB + 1, 20_001, 0), (3 * GiB + 777, 20_002, 3), (5 * GiB - 3, 20_003, 0),
            (6 * GiB + 12345, 20_004, 1), (8 * GiB, 20_005, 0)]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cas_library(ctx, n_total: int, shards: int, nthreads: int) -> dict:
    import spacedrive_amd as sd
    from oracle import native
    from spacedrive_amd import synth
    from spacedrive_amd.dedup import dest_of, group_host

    n = n_total // shards
    assert n * shards == n_total
    ids = np.empty((n_total, 8), np.uint8)
    buckets = [[] for _ in range(shards)]  # device-partitioned records, per destination, in source order
    d_hash = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    counts = torch.empty(shards, dtype=torch.int64, device="cuda")
    recs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    all_sizes = np.empty(n_total, np.uint64)
    t_gpu = 0.0
    shard_hashes, shard_valid = [], []  # per rank, for the in-process sd_cas_dedup_mgpu
    for s in range(shards):
        start = s * n
        sizes, cids, twins = synth.library(start, n, n_total)
        all_sizes[start:start + n] = sizes
        ext, total = sd.stage_plan(sizes)
        d_staged = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        d_ext = torch.from_numpy(ext.view(np.uint8).copy()).cuda()
        ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                            torch.from_numpy(twins.astype(np.int32)).cuda(), d_ext, n, d_staged)
        batch = ctx.cas_batch(ext)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch.run(d_staged, d_hash)
        d_valid = torch.from_numpy((sizes != 0).astype(np.uint8)).cuda()  # size 0: no cas_id (mod.rs:80-88)
        nv = ctx.dedup_partition(d_hash, d_valid, n, start, shards, counts, recs)
        torch.cuda.synchronize()
        t_gpu += time.perf_counter() - t0
        ids[start:start + n] = d_hash.view(n, 32)[:, :8].cpu().numpy()
        shard_hashes.append(d_hash.clone())
        shard_valid.append(d_valid)
        c = counts.cpu().numpy()
        r = recs[:nv].cpu().numpy()
        off = np.concatenate([[0], np.cumsum(c)])
        for d in range(shards):
            buckets[d].append(r[off[d]:off[d + 1]])
        batch.close()
        del d_staged, d_ext
        log(f"shard {s}: {n} files ({batch.n_sampled} sampled) hashed + partitioned")
    torch.cuda.empty_cache()

    # the oracle's cas_ids of the same 10 M files, built from the generator on the host
    t0 = time.perf_counter()
    want = np.empty_like(ids)
    for s in range(shards):
        sizes, cids, twins = synth.library(s * n, n, n_total)
        want[s * n:(s + 1) * n] = native.cas_ids_synth_simd(sizes, cids, twins, nthreads=nthreads)
    t_cpu = time.perf_counter() - t0
    bad = np.nonzero((ids != want).any(axis=1))[0]
    log(f"cas_ids: {len(bad)} mismatches of {n_total} (oracle {t_cpu:.1f}s on {nthreads} threads)")

    # dedup: device buckets grouped on the device vs the host grouping of the oracle's ids
    valid = all_sizes != 0
    keys = want.copy().view(">u8").reshape(-1).astype(np.uint64)
    gidx = np.arange(n_total, dtype=np.int64)
    dest = dest_of(keys, shards)
    groups = rep_mismatch = rec_mismatch = 0
    dup_files = 0
    host_groups = []
    for d in range(shards):
        got = np.concatenate(buckets[d]) if buckets[d] else np.zeros((0, 2), np.int64)
        sel = valid & (dest == d)
        host = np.stack([keys[sel].view(np.int64), gidx[sel]], axis=1)
        hr, hrep, hng = group_host(host)
        host_groups.append((hr, hrep, hng))
        dr = torch.from_numpy(got).cuda()
        drep = torch.empty(max(len(got), 1), dtype=torch.int64, device="cuda")
        ng = ctx.dedup_group(dr, len(got), drep, index_sorted=True)
        torch.cuda.synchronize()
        dr_h, drep_h = dr.cpu().numpy(), drep[:len(got)].cpu().numpy()
        rec_mismatch += int(len(dr_h) != len(hr) or not np.array_equal(dr_h, hr))
        rep_mismatch += int(len(drep_h) != len(hrep) or not np.array_equal(drep_h, hrep))
        groups += ng
        assert ng == hng or rec_mismatch, (d, ng, hng)
        dup_files += int((hrep != hr[:, 1]).sum())
    del buckets
    exchange = exchange_inprocess(shard_hashes, shard_valid, n, shards, host_groups)
    del shard_hashes, shard_valid
    torch.cuda.empty_cache()
    return {"files": n_total, "shards": shards, "files_per_shard": n, "cas_id_mismatches": int(len(bad)),
            "first_mismatches": [int(i) for i in bad[:10]],
            "empty_files": int((~valid).sum()), "sampled_files": int((all_sizes > 102400).sum()),
            "dedup": {"records": int(valid.sum()), "groups": int(groups), "duplicate_files": dup_files,
                      "bucket_record_mismatches": rec_mismatch, "bucket_rep_mismatches": rep_mismatch},
            "exchange_inprocess": exchange,
            "gpu_s": t_gpu, "oracle_s": t_cpu, "oracle_threads": nthreads}


def exchange_inprocess(hashes, valids, n: int, shards: int, host_groups) -> dict:
    """sd_cas_dedup_mgpu over `shards` ranks that are threads of this process (one context and
    stream each, the in-process communicator), rank r holding shard r's hashes; every rank's
    output vs the host grouping (+ the chunk-of-100 Object rule) of its prefix range."""
    import threading
    from spacedrive_amd import dedup
    from spacedrive_amd.device import Comm, CommGroup, Context
    from spacedrive_amd.identifier import object_owners
    group = CommGroup(shards)
    ctxs = [Context(0) for _ in range(shards)]
    comms = [Comm(ctxs[r], None, shards, r, group=group) for r in range(shards)]
    for c in comms:
        c.set_timing(True)
    out, errs = [None] * shards, []

    def rank(r):
        try:
            st = torch.cuda.Stream()
            runner = dedup.RcclDedup(ctxs[r], comms[r], hashes[r].device, capacity=n * 5 // 4)
            res = []
            for _ in range(2):  # the second call reuses the buffers (and times the warm exchange)
                t0 = time.perf_counter()
                recs, rep, ng, own = runner(hashes[r], valids[r], n, r * n, stream=st)
                st.synchronize()
                res.append(time.perf_counter() - t0)
            out[r] = (recs.cpu().numpy(), rep.cpu().numpy(), ng, own.cpu().numpy(), res, comms[r].last_phases())
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    try:
        ts = [threading.Thread(target=rank, args=(r,)) for r in range(shards)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
    finally:
        for c in comms:
            c.close()
        group.close()
        for c in ctxs:
            c.close()
    mism = {"records": 0, "reps": 0, "groups": 0, "owners": 0}
    per_rank = []
    for r in range(shards):
        recs, rep, ng, own, secs, phases = out[r]
        hr, hrep, hng = host_groups[r]
        want_own = object_owners(torch.from_numpy(hr[:, 1].copy()), torch.from_numpy(hrep), 100).numpy()
        mism["records"] += int(not np.array_equal(recs, hr))
        mism["reps"] += int(not np.array_equal(rep, hrep))
        mism["groups"] += int(ng != hng)
        mism["owners"] += int(not np.array_equal(own, want_own))
        per_rank.append({"records": int(len(recs)), "groups": int(ng), "call_ms": [x * 1e3 for x in secs],
                         "phases_ms": phases})
    return {"ranks": shards, "transport": "in-process (sd_comm_create_local), all ranks on one GPU",
            "rank_mismatches": mism, "parity": not any(mism.values()), "per_rank": per_rank}


def checksums(ctx, files, nthreads: int) -> dict:
    from oracle import native
    offs, off = [], 0
    for L, _, _ in files:
        offs.append(off)
        off = (off + L + 64 + 63) // 64 * 64
    d = torch.empty(off + 64, dtype=torch.uint8, device="cuda")
    for (L, cid, tw), o in zip(files, offs):
        ctx.synth_fill(cid, tw, L, d[o:])
    cb = ctx.checksum_batch(offs, [f[0] for f in files])
    h = torch.zeros(len(files) * 32, dtype=torch.uint8, device="cuda")
    cb.run(d, h)
    torch.cuda.synchronize()
    got = h.cpu().numpy().reshape(-1, 32)
    cb.close()
    del d
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    rows = []
    for (L, cid, tw), g in zip(files, got):
        w = native.checksum_synth_mt(L, cid, tw, nthreads=nthreads)
        rows.append({"size": L, "content_id": cid, "twin": tw, "checksum": g.tobytes().hex(), "equal": g.tobytes() == w})
    return {"files": len(files), "bytes": sum(f[0] for f in files), "mismatches": sum(not r["equal"] for r in rows),
            "oracle_s": time.perf_counter() - t0, "per_file": rows}


def run(n_total: int = 10_000_000, shards: int = 8, nthreads: int = 16, with_checksums: bool = True) -> dict:
    import spacedrive_amd as sd
    ctx = sd.default_context(0)
    out = {"what": "full-size parity vs the oracle (scripts/parity_full.py)",
           "cas": cas_library(ctx, n_total, shards, nthreads)}
    if with_checksums:
        out["checksum_configs3"] = checksums(ctx, CK_BENCH, nthreads)
        out["checksum_mixed"] = checksums(ctx, CK_MIXED, nthreads)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--files", type=int, default=10_000_000)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--no-checksums", action="store_true")
    p.add_argument("--out", default="")
    a = p.parse_args()
    t0 = time.time()
    r = run(a.files, a.shards, a.threads, not a.no_checksums)
    r["wall_s"] = time.time() - t0
    s = json.dumps(r)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    ok = r["cas"]["cas_id_mismatches"] == 0 and r["cas"]["dedup"]["bucket_record_mismatches"] == 0 \
        and r["cas"]["dedup"]["bucket_rep_mismatches"] == 0 and r["cas"]["exchange_inprocess"]["parity"] \
        and all(r.get(k, {"mismatches": 0})["mismatches"] == 0 for k in ("checksum_configs3", "checksum_mixed"))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
