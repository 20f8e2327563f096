"""bench.py -- cas_id files/s (+ checksum GB/s) on 1..8 MI355X, one process per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[4], weak-scaled): a 10 M-file synthetic library with the
configs[0] mixture (60 % of files <= 100 KiB hashed whole, 40 % sampled), sharded by file
index: each GPU owns ``--files-per-gpu`` (default 1 250 000 = 10 M / 8) files, so N = 8 is
the full 10 M-file library.  One step = hash every file of the shard (sampled kernel +
whole-file kernels) + the dedup exchange (partition by cas_id prefix, all-to-all of the
records over RCCL, sort + group).  Inputs are resident in HBM before timing (generated on
device from the counter-based generator; host staging + PCIe is reported separately in
DESIGN.md, never as `value`).

After the timed steps, rank 0 (N = 1 only) times the CPU baseline (oracle/sd_oracle.c,
the C restatement of cas.rs + blake3) on a bounded sample of the same files, and every
rank times configs[3] (full-file checksums of 16 x 4 GiB files) as `checksum`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
# int32 VALU: 157.3 TF fp32 vector peak (MI355X_MICROARCH.md) counts packed FMA (2 flop x 2
# lanes); BLAKE3's add/xor/alignbit have no packed 32-bit forms: 256 CU x 64 lanes x 2.4 GHz
VALU_PEAK_TOPS = 256 * 64 * 2.4e9 / 1e12
SAMPLED_MSG = 57352


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--files-per-gpu", type=int, default=1_250_000)
    p.add_argument("--checksum-gib", type=int, default=64, help="configs[3] size per GPU; 0 = skip")
    p.add_argument("--checksum-steps", type=int, default=5)
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target seconds per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (rehearsal)")
    p.add_argument("--share-gpu", action="store_true", help="map every rank onto the visible GPUs (rehearsal)")
    p.add_argument("--config-files", type=int, default=1_000_000,
                   help="N=1 only: files of the configs[1] (small) and configs[2] (sampled) kernel legs; 0 = skip")
    p.add_argument("--config-reps", type=int, default=5)
    p.add_argument("--file-backed-files", type=int, default=20000,
                   help="N=1 only: time the drop-in from files on disk (pread stager + sd_cas_ids) on this many "
                        "files of the shard, beside the reference's read schedule on the CPU; 0 = skip")
    p.add_argument("--host-staged-files", type=int, default=0,
                   help="N=1 only: also time the PCIe-inclusive drop-in path on this many files (DESIGN.md)")
    return p.parse_args()


def pmc_traffic(kernels):
    """HBM bytes per launch (summed over the given kernels) from the committed rocprofv3
    PMC summary of the same bench command (profiles/pmc_summary.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(path))
        return sum(d["kernels"][k]["hbm_bytes_per_launch"] for k in ([kernels] if isinstance(kernels, str) else kernels))
    except Exception:
        return None


def cpu_baseline(sizes, cids, twins, seconds: float):
    """Oracle C restatement on the host, hash only over pre-staged messages.

    Uses the SIMD multi-chunk hasher (oracle/sd_oracle_simd.c: AVX-512 16-way / AVX2 8-way
    hash_many, the strategy of the reference's blake3 crate), so the baseline is the
    reference's arithmetic at its own CPU speed, not a scalar strawman."""
    from oracle import native
    from spacedrive_amd.device import stage_plan
    threads = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU
    level = native.simd_level(-1)

    def rate(nthreads, n0):
        n = n0
        while True:
            s, c, t = sizes[:n], cids[:n], twins[:n]
            ext, total = stage_plan(s)
            buf = native.stage_synth(s, c, t, ext["msg_offset"], total)
            t0 = time.perf_counter()
            native.cas_ids_staged(buf, ext, nthreads=nthreads, simd=-1)
            dt = time.perf_counter() - t0
            if dt >= seconds * 0.5 or n >= len(sizes):
                return n, dt, float(ext["msg_len"].astype(np.float64).sum())
            n = min(len(sizes), int(n * max(2.0, seconds / max(dt, 1e-3))))

    n1, dt1, b1 = rate(1, 2000)
    nT, dtT, bT = rate(threads, 20000)
    simd = {0: "scalar", 1: "AVX2 8-way", 2: "AVX-512 16-way"}[level]
    return {
        "value": nT / dtT, "unit": "files/s", "cores": threads, "kind": "port",
        "sample": f"first {nT} files of this shard (same mixture), messages pre-staged in host RAM, hash only; "
                  f"C restatement of cas.rs + blake3 with {simd} multi-chunk hash_many (oracle/sd_oracle_simd.c) "
                  f"on {threads} threads; {bT / dtT / 1e9:.2f} GB/s of message bytes",
        "single_thread": {"value": n1 / dt1, "unit": "files/s", "cores": 1, "sample_files": n1,
                          "GBps": b1 / dt1 / 1e9},
        "simd": simd,
    }


def host_staged(ctx, ext, d_staged, batch, k, dev):
    """PCIe-inclusive drop-in path: the first k files' messages in pinned host memory ->
    sd_cas_ids (plan, H2D, kernels, D2H, hex).  Reported apart from `value`."""
    import ctypes
    from spacedrive_amd._native import check, lib
    k = min(k, len(ext))
    nbytes = int(ext["msg_offset"][k - 1]) + int(ext["msg_len"][k - 1])
    nbytes = (nbytes + 63) // 64 * 64
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(d_staged[:nbytes])
    sub = np.ascontiguousarray(ext[:k])
    out = ctypes.create_string_buffer(17 * k)
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dbuf.copy_(host, non_blocking=True)  # warm the copy path
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dbuf.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = time.perf_counter() - t0
    del dbuf
    check(lib().sd_cas_ids(ctx.handle, host.data_ptr(), nbytes, sub.ctypes.data, k, out, None))  # warm-up
    t0 = time.perf_counter()
    check(lib().sd_cas_ids(ctx.handle, host.data_ptr(), nbytes, sub.ctypes.data, k, out, None))
    e2e_s = time.perf_counter() - t0
    return {"files": k, "bytes": nbytes, "h2d_GBps": nbytes / h2d_s / 1e9, "h2d_ms": h2d_s * 1e3,
            "end_to_end_files_per_s": k / e2e_s, "end_to_end_ms": e2e_s * 1e3,
            "note": "sd_cas_ids from pinned host memory: host plan + H2D + kernels + D2H + hex, one call, "
                    "not overlapped; the reference's own cost is reading the files (6 preads per sampled file)"}


def config_leg(ctx, which: str, nfiles: int, reps: int, dev, stream, valu_peak: float):
    """configs[1] (1 M files <= 100 KiB, whole-content cas_id) or configs[2] (1 M files
    > 100 KiB, sampled cas_id) on this GPU: kernel-only files/s over device-resident
    staged messages, timed with HIP events on the launch stream, plus determinism of the
    full 32-byte hashes across runs (a size-independent property; bit-exactness vs the
    oracle is pinned by tests/test_gpu_parity.py on the same generator)."""
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    gen = synth.small_library if which == "small" else synth.sampled_library
    sizes, cids, twins = gen(0, nfiles)
    ext, total = sd.stage_plan(sizes)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, nfiles, d_staged, stream)
    b = ctx.cas_batch(ext)
    h0 = torch.zeros(nfiles * 32, dtype=torch.uint8, device=dev)
    h1 = torch.zeros(nfiles * 32, dtype=torch.uint8, device=dev)
    b.run(d_staged, h0, stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(reps):
        b.run(d_staged, h1, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    deterministic = bool(torch.equal(h0, h1))
    valu = b.compressions * 672 / (ms * 1e-3)
    res = {"workload": ("configs[1]: 1M files <= 100 KiB, whole-content cas_id (log-uniform sizes 1..102400)"
                        if which == "small" else
                        "configs[2]: 1M files > 100 KiB, sampled cas_id (log-uniform sizes 102401..4 GiB)"),
           "files": nfiles, "kernel_ms": ms, "files_per_s": nfiles / (ms * 1e-3),
           "msg_GBps": b.msg_bytes / (ms * 1e-3) / 1e9, "compressions": b.compressions,
           "valu_frac": valu / 1e12 / VALU_PEAK_TOPS,
           "valu_frac_of_measured_peak": valu / valu_peak if valu_peak else None,
           "kernels": ["k_cas_sampled"] if which == "sampled" else ["k_whole_items", "k_whole_merge8"],
           "deterministic": deterministic}
    del d_staged, h0, h1, b
    torch.cuda.empty_cache()
    assert deterministic, which
    return res


def _fs_type(path: str) -> str:
    best, fstype = "", "?"
    try:
        for line in open("/proc/mounts"):
            parts = line.split()
            if len(parts) > 2 and path.startswith(parts[1]) and len(parts[1]) > len(best):
                best, fstype = parts[1], parts[2]
    except OSError:
        pass
    return fstype


def file_backed(ctx, sizes, ext, d_staged, k: int, with_cpu: bool):
    """The drop-in path from files on disk, as identifier_job_step would drive it
    (file_identifier/mod.rs:107-134): the first k files of this shard are written to a
    scratch directory (sampled files sparse: only the windows cas.rs reads are
    materialised), then timed end to end -- stage (sd_cas_stage_files: head / 4 samples /
    tail by pread on 16 threads into pinned memory) + sd_cas_ids (H2D, kernels, D2H, hex)
    -- and, as the CPU baseline, the reference's own read schedule (open, read_exact,
    seek; cas.rs:27-58) + the SIMD C restatement on 1 and 16 threads.  Both read from
    the page cache (files just written).  The two outputs are asserted equal."""
    import ctypes
    import shutil
    import tempfile
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    from spacedrive_amd._native import check, lib
    k = min(k, len(sizes))
    sub_sizes = np.ascontiguousarray(sizes[:k])
    sub_ext, total = sd.stage_plan(sub_sizes)
    nbytes = int(ext["msg_offset"][k - 1]) + int(ext["msg_len"][k - 1])
    host = d_staged[:nbytes].cpu().numpy()  # messages in the shard layout (same offsets)
    base = "/dev/shm"
    try:
        st = os.statvfs(base)
        if st.f_bavail * st.f_frsize < 4 * nbytes:
            base = None
    except OSError:
        base = None
    d = tempfile.mkdtemp(prefix="sd_fb_", dir=base)
    try:
        t0 = time.perf_counter()
        paths = synth.write_files(d, sub_sizes, host, ext[:k])
        write_s = time.perf_counter() - t0
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        pin = ctypes.c_void_p()
        check(L.sd_cas_host_alloc(ctx.handle, total, ctypes.byref(pin)))
        out = ctypes.create_string_buffer(17 * k)
        status = np.zeros(k, np.int32)
        threads = 16
        runs = []
        try:
            for _ in range(3):  # first run warms the stager's threads and the context's slots
                status[:] = 0
                t0 = time.perf_counter()
                check(L.sd_cas_stage_files(arr, sub_ext.ctypes.data, k, pin, status.ctypes.data, threads))
                t1 = time.perf_counter()
                check(L.sd_cas_ids(ctx.handle, pin, total, sub_ext.ctypes.data, k, out, status.ctypes.data))
                t2 = time.perf_counter()
                runs.append((t1 - t0, t2 - t1))
        finally:
            L.sd_cas_host_free(ctx.handle, pin)
        assert (status == 0).all(), np.unique(status)
        stage_s = min(r[0] for r in runs[1:])
        hash_s = min(r[1] for r in runs[1:])
        gpu_ids = [out.raw[17 * i:17 * i + 16].decode() for i in range(k)]
        # the pipelined path-based drop-in: stager pool preads window k+1 while window k
        # is copied and hashed (sd_cas_ids_files)
        out2 = ctypes.create_string_buffer(17 * k)
        st2 = np.zeros(k, np.int32)
        sz = np.ascontiguousarray(sub_sizes, np.uint64)
        pipe = []
        for _ in range(3):
            t0 = time.perf_counter()
            check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, out2, st2.ctypes.data, threads))
            pipe.append(time.perf_counter() - t0)
        assert (st2 == 0).all() and out2.raw == out.raw
        pipe_s = min(pipe[1:])
        res = {"files": k, "dir_fs": _fs_type(d), "write_s": write_s,
               "message_bytes": int(sub_ext["msg_len"].astype(np.int64).sum()),
               "gpu": {"files_per_s": k / pipe_s, "ms": pipe_s * 1e3, "stage_threads": threads,
                       "note": "sd_cas_ids_files: pread on the library's stager pool into pinned windows, "
                               "overlapped with H2D + kernels + D2H + hex; best of 2 warm runs",
                       "unpipelined": {"files_per_s": k / (stage_s + hash_s), "stage_ms": stage_s * 1e3,
                                       "hash_ms": hash_s * 1e3,
                                       "note": "sd_cas_stage_files then sd_cas_ids, one after the other"}}}
        if with_cpu:
            from oracle import native
            cpu = {}
            for nt in (1, threads):
                t0 = time.perf_counter()
                got, cst = native.cas_ids_files(paths, sub_sizes, nthreads=nt, simd=-1)
                dt = time.perf_counter() - t0
                cpu[f"threads_{nt}"] = {"files_per_s": k / dt, "seconds": dt}
            assert (cst == 0).all()
            want = [got[i].tobytes().hex() for i in range(k)]
            res["cpu_reference_schedule"] = cpu
            res["equal_to_cpu"] = want == gpu_ids
            assert res["equal_to_cpu"], "file-backed GPU cas_ids differ from the CPU restatement"
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:  # rehearsal of the N-rank path on a box with fewer GPUs
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    import spacedrive_amd as sd
    from spacedrive_amd import dedup, synth

    ctx = sd.Context(local)
    n = args.files_per_gpu
    start, n_total = rank * n, world * n
    t_setup = time.time()
    sizes, cids, twins = synth.library(start, n, n_total)
    ext, total = sd.stage_plan(sizes)
    dev = torch.device("cuda", local)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, n, d_staged)
    batch = ctx.cas_batch(ext)
    d_hash = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_valid = torch.from_numpy((sizes != 0).astype(np.uint8)).to(dev)  # size 0: no cas_id (mod.rs:80-88)
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s: {n} files ({batch.n_sampled} sampled), "
        f"{batch.msg_bytes / 1e9:.2f} GB of messages, {batch.compressions / 1e9:.3f} G compressions")

    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    split = True  # separate launches: the dominant kernel is timed on its own

    def step(k=None):
        if k is not None:
            ev[k][0].record(stream)
        if split:
            batch.run_part(1, d_staged, d_hash, stream)  # k_cas_sampled
            if k is not None:
                ev[k][1].record(stream)
            batch.run_part(2, d_staged, d_hash, stream)  # whole-file leaf + tree kernels
        else:
            batch.run(d_staged, d_hash, stream)
            if k is not None:
                ev[k][1].record(stream)
        if k is not None:
            ev[k][2].record(stream)
        r = dedup.dedup_shard(ctx, d_hash.view(n, 32), d_valid, n, start)
        if k is not None:
            ev[k][3].record(stream)
        return r

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        res = step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    def avg(a, b):
        return sum(ev[k][a].elapsed_time(ev[k][b]) for k in range(args.steps)) / args.steps
    hash_ms, sampled_ms, dedup_ms = avg(0, 2), avg(0, 1), avg(2, 3)
    recs, rep, n_groups, owners = res
    # every valid file lands on exactly one rank; groups never straddle ranks
    tot = torch.tensor([recs.shape[0], n_groups, int((sizes != 0).sum())], dtype=torch.int64,
                       device=dev if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(tot)
    dedup_totals = {"records": int(tot[0]), "groups": int(tot[1]), "valid_files": int(tot[2]),
                    "records_on_rank0": int(recs.shape[0]),
                    "objects_created_on_rank0": int((owners == recs[:, 1]).sum())}
    assert dedup_totals["records"] == dedup_totals["valid_files"], dedup_totals
    files_total = n_total * args.steps
    value = files_total / elapsed

    # roofline of the dominant kernel, k_cas_sampled (81 % of the shard's compressions),
    # timed on its own with HIP events on its launch stream: 953 compressions x 672 VALU
    # lane-ops per sampled file; bytes = 57 352 B message read + 32 B hash written per file
    valu_peak = ctx.valu_peak()
    if split:
        dom_kernel, dom_ms = "k_cas_sampled", sampled_ms
        dom_comp = 953 * batch.n_sampled
        dom_bytes = batch.n_sampled * (SAMPLED_MSG + 32)
    else:
        dom_kernel, dom_ms = "hash phase", hash_ms
        dom_comp, dom_bytes = batch.compressions, batch.msg_bytes + 32 * n
    dom_valu = dom_comp * 672 / (dom_ms * 1e-3)
    dom_gbps = dom_bytes / (dom_ms * 1e-3) / 1e9
    hash_bytes = batch.msg_bytes + 32 * n
    hash_valu = batch.compressions * 672 / (hash_ms * 1e-3)
    phase = ["k_cas_sampled", "k_whole_items", "k_whole_merge8"]
    traffic = pmc_traffic(dom_kernel) if split else pmc_traffic(phase)

    out = {
        "metric": "cas_id files/sec (10M synthetic files) + checksum GB/s at 1/2/4/8 MI355X",
        "value": value, "unit": "files/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic (device-generated, SURVEY.md 8(d) generator)",
        "config": {"workload": f"10M-file library mixture (configs[0] mix: 60% <=100KiB whole-content, 40% sampled; "
                               f"10% dups, 1% sample twins), {n} files per GPU, step = hash shard + "
                               f"cas_id-prefix all-to-all dedup + Object owners (chunk-of-100 rule)",
                   "files_per_gpu": n, "global_files": n_total, "parallelism": f"file-sharded x{world}"},
        "roofline": {"bound": "valu", "achieved": dom_valu / 1e12, "peak": VALU_PEAK_TOPS,
                     "unit": "T int32 VALU lane-ops/s", "frac": dom_valu / 1e12 / VALU_PEAK_TOPS,
                     "traffic": traffic, "kernel": dom_kernel, "kernel_ms": dom_ms,
                     "algorithmic": {"compressions_per_launch": dom_comp, "lane_ops_per_compression": 672,
                                     "bytes_per_launch": dom_bytes,
                                     "per_unit": "sampled file: 953 compressions, 57352 B read + 32 B written"},
                     "measured_valu_peak": valu_peak / 1e12,
                     "frac_of_measured_peak": dom_valu / valu_peak if valu_peak else None,
                     "hbm": {"achieved": dom_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                             "frac": dom_gbps / HBM_PEAK_GBPS},
                     "phase": {"kernels": phase, "ms": hash_ms, "compressions": batch.compressions,
                               "bytes": hash_bytes, "achieved": hash_valu / 1e12,
                               "frac": hash_valu / 1e12 / VALU_PEAK_TOPS,
                               "traffic": pmc_traffic(phase)}},
        "kernels": {"hash_ms": hash_ms, "sampled_ms": sampled_ms if split else None,
                    "whole_ms": hash_ms - sampled_ms if split else None, "dedup_and_exchange_ms": dedup_ms,
                    "host_overhead_ms": elapsed / args.steps * 1e3 - hash_ms - dedup_ms,
                    "sampled_files": batch.n_sampled, "whole_files": batch.n_whole},
        "dedup": dedup_totals,
    }
    if rank == 0 and world == 1 and args.host_staged_files > 0:
        out["host_staged"] = host_staged(ctx, ext, d_staged, batch, args.host_staged_files, dev)
    if rank == 0 and world == 1 and args.file_backed_files > 0:
        out["file_backed"] = file_backed(ctx, sizes, ext, d_staged, args.file_backed_files,
                                         with_cpu=not args.no_cpu_baseline)
    del d_staged, recs, rep, owners
    torch.cuda.empty_cache()

    # configs[3]: validator checksums, 16 files of (G/16) GiB per GPU
    if args.checksum_gib > 0:
        nf = 16
        flen = (args.checksum_gib << 30) // nf
        d_data = torch.empty(nf * flen + 128, dtype=torch.uint8, device=dev)
        offs = [i * flen for i in range(nf)]
        for i in range(nf):
            ctx.synth_fill(10_000 + start + i, 0, flen, d_data[offs[i]:])
        cb = ctx.checksum_batch(offs, [flen] * nf)
        d_sum = torch.empty(nf * 32, dtype=torch.uint8, device=dev)
        cb.run(d_data, d_sum, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(args.checksum_steps):
            cb.run(d_data, d_sum, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ck_ms = e0.elapsed_time(e1) / args.checksum_steps
        gbps = cb.total_bytes / (ck_ms * 1e-3) / 1e9
        tot = torch.tensor([gbps], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(tot)
        out["checksum"] = {"GBps": float(tot.item()), "unit": "GB/s", "per_gpu_GBps": gbps, "ms_per_run": ck_ms,
                           "workload": f"configs[3]: {nf} x {flen >> 30} GiB files per GPU, full-file BLAKE3",
                           "roofline": {"bound": "valu",
                                        "achieved": cb.compressions * 672 / (ck_ms * 1e-3) / 1e12,
                                        "peak": VALU_PEAK_TOPS, "unit": "T int32 VALU lane-ops/s",
                                        "frac": cb.compressions * 672 / (ck_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS,
                                        "hbm": {"achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                                "frac": gbps / HBM_PEAK_GBPS}},
                           "traffic": pmc_traffic("k_ck_leaf")}
        del d_data
        torch.cuda.empty_cache()

    if world == 1 and args.config_files > 0:
        out["configs"] = {k: config_leg(ctx, k, args.config_files, args.config_reps, dev, stream, valu_peak)
                          for k in ("small", "sampled")}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sizes, cids, twins, args.cpu_seconds)
        if "cpu_reference_schedule" in out.get("file_backed", {}):
            out["cpu_baseline"]["file_backed"] = dict(out["file_backed"]["cpu_reference_schedule"],
                                                      files=out["file_backed"]["files"],
                                                      note="reference read schedule from files (page cache)")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
