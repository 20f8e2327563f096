"""The library's CPU path (libsdcas.so sd_cpu_*, no device) and its GPU-free host logic
(the stager, the sequential reader) against the oracle: the reference's read semantics
for files whose length differs from the size argument (cas.rs:23-62), hash.rs's read
loop, the goldens, and every SIMD width the host has."""
import ctypes
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from oracle import blake3_spec as b3
from oracle import cas_spec as cs
from spacedrive_amd import cpu
from spacedrive_amd._native import SD_FILE_CHANGED, SD_FILE_OK, SD_FILE_SHORT_READ, check, lib
from spacedrive_amd.cas import UnexpectedEofError
from spacedrive_amd.device import stage_plan
from tests.test_oracle import LENGTH_MISMATCH_CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pat(n):
    return bytes(i % 251 for i in range(n))


def test_cpu_blake3_official_vectors(golden):
    for n, h in golden["blake3_official"]["hash"].items():
        assert cpu.blake3(pat(int(n))).hex() == h, n


def test_cpu_blake3_vs_oracle_sizes(oracle_native):
    rng = np.random.default_rng(3)
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 16 * 1024, 16 * 1024 + 1, 17 * 1024,
              33 * 1024 + 5, 57352, 102408, 1 << 20, (1 << 20) + 1, 3 * (1 << 20) + 777]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert cpu.blake3(d) == oracle_native.blake3(d), n


@pytest.mark.parametrize("lanes", [4, 8, 16])
def test_cpu_simd_widths(lanes):
    """Each chunk-lane width (SSE2 4, AVX2 8, AVX-512 16) the host supports, in a child
    process (the width is picked once per process)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from spacedrive_amd import cpu\n"
            "from oracle import native\n"
            "import numpy as np\n"
            "print(cpu.simd_lanes())\n"
            "rng = np.random.default_rng(9)\n"
            "for n in [0, 1025, 4096, 16 * 1024 + 3, 40000, 57352, 300001]:\n"
            "    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()\n"
            "    assert cpu.blake3(d) == native.blake3(d), n\n"
            # cas batches: the chunks of many messages packed across the lanes together
            "from spacedrive_amd.device import stage_plan\n"
            "sizes = np.concatenate([np.arange(0, 2100, 7), [102399, 102400, 102401, 5 << 20]]).astype(np.uint64)\n"
            "rng.shuffle(sizes)\n"
            "cids = np.arange(len(sizes), dtype=np.uint64) + 77\n"
            "ext, total = stage_plan(sizes)\n"
            "buf = native.stage_synth(sizes, cids, None, ext['msg_offset'], total)\n"
            "want = [r.tobytes().hex() for r in native.cas_ids_staged(buf, ext)]\n"
            "for nt in (1, 3):\n"
            "    assert cpu.cas_ids_staged(buf, ext, nthreads=nt) == want, nt\n") % ROOT
    env = dict(os.environ, SD_CPU_LANES=str(lanes))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = int(r.stdout.split()[0])
    assert got <= lanes
    if got < lanes:
        pytest.skip(f"host CPU runs {got} lanes at most")


def test_cpu_cas_ids_staged_goldens(golden, oracle_native):
    files = golden["cas_synth"]["files"]
    sizes = np.array([f["size"] for f in files], np.uint64)
    cids = np.array([f["content_id"] for f in files], np.uint64)
    twins = np.array([f["twin"] for f in files], np.uint32)
    ext, total = stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    got = cpu.cas_ids_staged(buf, ext)
    assert got == [f["cas_id"] for f in files]


def test_cpu_checksums_block_parallel_ranges(oracle_native):
    """sd_cpu_checksums splits a range of >= 8 MiB into 1 MiB block tasks beside the small
    ranges' tasks (one huge range no longer runs on one thread): ranges either side of the
    split threshold, a ragged tail, an odd offset and an empty range, on 1 and 8 threads,
    against the oracle's BLAKE3 of each range."""
    rng = np.random.default_rng(11)
    lens = [(8 << 20) - 1, 8 << 20, (8 << 20) + 1, 12345, 0, (9 << 20) + 777, 64]
    offs, o = [], 0
    for L in lens:
        offs.append(o)
        o += L + 3  # odd starts
    data = rng.integers(0, 256, o + 64, dtype=np.uint8)
    offs_a, lens_a = np.array(offs, np.uint64), np.array(lens, np.uint64)
    want = [oracle_native.blake3(data[a:a + L].tobytes()) for a, L in zip(offs, lens)]
    for nt in (1, 8):
        out = np.zeros((len(lens), 32), np.uint8)
        check(lib().sd_cpu_checksums(data.ctypes.data, offs_a.ctypes.data, lens_a.ctypes.data, len(lens),
                                     out.ctypes.data, nt))
        assert [r.tobytes() for r in out] == want, nt


def test_cpu_paths_of_a_directory(tmp_path):
    """A directory given as a file: File::open succeeds on Linux and the first read fails
    with EISDIR, so generate_cas_id (whole or sampled size) and file_checksum return that
    io::Error (cas.rs:29,36; hash.rs:16): SD_FILE_IO_ERROR with errno 21, on either side of a
    regular file hashed as usual."""
    import errno
    content = bytes(i % 251 for i in range(200_000))
    (tmp_path / "sub").mkdir()
    (tmp_path / "f").write_bytes(content)
    paths = [str(tmp_path / "sub"), str(tmp_path / "f"), str(tmp_path / "sub")]
    sizes = np.array([4096, 200_000, 200_000], np.uint64)
    arr = (ctypes.c_char_p * 3)(*[os.fsencode(p) for p in paths])
    want = {"cas": cs.generate_cas_id_file(content, 200_000), "checksum": cs.file_checksum(content)}
    for name, call, width in (
            ("cas", lambda o, st: lib().sd_cpu_cas_ids_files(arr, sizes.ctypes.data, 3, o, st.ctypes.data, 2), 17),
            ("checksum", lambda o, st: lib().sd_cpu_file_checksums(arr, 3, o, st.ctypes.data, 2), 65)):
        out = ctypes.create_string_buffer(width * 3)
        st = np.zeros(3, np.int32)
        check(call(out, st))
        assert [(int(x) & 0xFFFF, int(x) >> 16) for x in st] == [
            (2, errno.EISDIR), (SD_FILE_OK, 0), (2, errno.EISDIR)], name
        assert out.raw[width:2 * width - 1].decode() == want[name], name


def _write(tmp_path, name, content):
    p = tmp_path / name
    p.write_bytes(content)
    return str(p)


def test_cpu_cas_ids_files_length_mismatch(tmp_path, oracle_native):
    """cas.rs with stale sizes (SURVEY.md §3 CS4/CS5 callers pass metadata that may lag the
    file): every case of tests/test_oracle.py, batched and single-file, equals the oracle's
    read schedule."""
    paths, sizes, contents = [], [], []
    for i, (flen, size) in enumerate(LENGTH_MISMATCH_CASES):
        content = cs.synth_bytes(900 + i, 0, 0, flen)
        paths.append(_write(tmp_path, f"m{i}", content))
        sizes.append(size)
        contents.append(content)
    paths.append(str(tmp_path / "missing"))
    sizes.append(10)
    want, wst = oracle_native.cas_ids_files(paths, np.array(sizes, np.uint64), nthreads=2)
    got = cpu.generate_cas_ids(paths, sizes, nthreads=4)
    for i in range(len(paths)):
        if wst[i] == 0:
            assert got[i] == want[i].tobytes().hex(), (i, LENGTH_MISMATCH_CASES[i])
            assert cpu.generate_cas_id(paths[i], sizes[i]) == got[i]
        elif wst[i] == SD_FILE_SHORT_READ:
            assert isinstance(got[i], UnexpectedEofError), i
        else:
            assert isinstance(got[i], FileNotFoundError), i
    assert wst[-1] != 0 and (wst[:-1] == 3).sum() == 2  # two UnexpectedEof cases, one ENOENT


def test_cpu_file_checksums_vs_oracle(tmp_path, oracle_native):
    MiB = 1 << 20
    sizes = [0, 1, 1024, 1025, MiB - 1, MiB, MiB + 1, 2 * MiB, 5 * MiB + 77]
    paths = [_write(tmp_path, f"c{i}", oracle_native.synth_bytes(50 + i, 0, 0, s)) for i, s in enumerate(sizes)]
    paths.insert(3, str(tmp_path / "nope"))
    want, wst = oracle_native.file_checksums(paths, nthreads=2)
    got = cpu.file_checksums(paths, nthreads=3)
    assert isinstance(got[3], FileNotFoundError) and wst[3] != 0
    for i in range(len(paths)):
        if i != 3:
            assert wst[i] == 0 and got[i] == want[i].tobytes().hex(), i
            assert cpu.file_checksum(paths[i]) == got[i]


@pytest.mark.parametrize("piece_kib", [0, 64, 100, 256, 1024, 4096])
def test_cpu_file_checksums_read_pieces(tmp_path, oracle_native, piece_kib):
    """"cpu_read_piece_kib": the CPU path reads and hashes each 1 MiB block of a large file
    in pieces (round 5); every piece size -- a divisor of the block, one that is not (100),
    the whole block, more than it -- gives the oracle's checksums."""
    import spacedrive_amd as sd
    MiB = 1 << 20
    sizes = [8 * MiB, 9 * MiB + 123, 17 * MiB - 1]
    paths = [_write(tmp_path, f"p{i}", oracle_native.synth_bytes(70 + i, 0, 0, s)) for i, s in enumerate(sizes)]
    want, wst = oracle_native.file_checksums(paths, nthreads=2)
    keep = sd.get_tuning("cpu_read_piece_kib")
    try:
        sd.set_tuning("cpu_read_piece_kib", piece_kib)
        got = cpu.file_checksums(paths, nthreads=4)
    finally:
        sd.set_tuning("cpu_read_piece_kib", keep)
    assert (wst == 0).all() and got == [w.tobytes().hex() for w in want]


def test_cpu_file_checksum_of_a_pipe(tmp_path):
    """hash.rs stops at the first short read: a FIFO (st_size 0) hashes what one read returns."""
    fifo = str(tmp_path / "fifo")
    os.mkfifo(fifo)
    payload = cs.synth_bytes(98, 0, 0, 4000)

    def writer():
        with open(fifo, "wb", buffering=0) as f:
            f.write(payload)

    t = threading.Thread(target=writer)
    t.start()
    got = cpu.file_checksum(fifo)
    t.join()
    assert got == b3.blake3(payload).hex()


# -------------------------------------------------------------- the staging ABI (host only)
def _stage(path, ext_row, staged):
    st = ctypes.c_int32(-1)
    check(lib().sd_cas_stage_file(os.fsencode(path), ctypes.c_void_p(ext_row), ctypes.c_void_p(staged.ctypes.data),
                                  ctypes.byref(st)))
    return st.value


def test_stage_file_length_mismatch(tmp_path):
    """sd_cas_stage_file: a whole-kind extent is in/out (msg_len = 8 + the bytes read);
    a file longer than the extent's room reports SD_FILE_CHANGED; a sampled file's tail
    comes from its real end."""
    for i, (flen, size) in enumerate(LENGTH_MISMATCH_CASES):
        content = cs.synth_bytes(900 + i, 0, 0, flen)
        p = _write(tmp_path, f"s{i}", content)
        ext, total = stage_plan(np.array([size], np.uint64))
        staged = np.full(total + 64, 0xAB, np.uint8)
        st = _stage(p, ext.ctypes.data, staged)
        try:
            msg = cs.cas_message_file(content, size)
        except cs.UnexpectedEof:
            assert st == SD_FILE_SHORT_READ, i
            continue
        if size <= 102400 and flen > size:
            assert st == SD_FILE_CHANGED, i
            continue
        assert st == SD_FILE_OK, i
        assert int(ext["msg_len"][0]) == len(msg), i
        assert staged[:len(msg)].tobytes() == msg, i
        pad = (len(msg) + 63) // 64 * 64
        assert not staged[len(msg):pad].any(), i


def test_cpu_cas_ids_on_restaged_shorter_files(tmp_path):
    """Shorter whole files staged with their planned extents, then hashed with the
    updated extents: equals the reference's fs::read message."""
    sizes = [100, 5000, 102400]
    flens = [10, 4000, 70000]
    paths = [_write(tmp_path, f"r{i}", cs.synth_bytes(60 + i, 0, 0, flens[i])) for i in range(3)]
    ext, total = stage_plan(np.array(sizes, np.uint64))
    staged = np.zeros(total + 64, np.uint8)
    arr = (ctypes.c_char_p * 3)(*[os.fsencode(p) for p in paths])
    status = np.full(3, -1, np.int32)
    check(lib().sd_cas_stage_files(arr, ext.ctypes.data, 3, staged.ctypes.data, status.ctypes.data, 2))
    assert (status == 0).all()
    got = cpu.cas_ids_staged(staged, ext)
    for i in range(3):
        assert got[i] == cs.generate_cas_id_file(cs.synth_bytes(60 + i, 0, 0, flens[i]), sizes[i])


def test_cpu_cas_id_of_a_pipe(tmp_path, oracle_native):
    """The CPU path reads a pipe as fs::read does (cas.rs:29): every byte until the writer
    closes, hashed after le64(size) -- here the metadata length 0 of a FIFO."""
    import threading
    from spacedrive_amd import cpu
    data = bytes(range(256)) * 700
    fifo = str(tmp_path / "pipe")
    os.mkfifo(fifo)

    def writer():
        with open(fifo, "wb") as f:
            for o in range(0, len(data), 4000):
                f.write(data[o:o + 4000])

    t = threading.Thread(target=writer)
    t.start()
    try:
        got = cpu.generate_cas_id(fifo, 0)
    finally:
        t.join()
    assert got == oracle_native.blake3(bytes(8) + data)[:8].hex()


def _sparse_sampled(tmp_path, name, size, cid):
    """a sparse file of `size` bytes holding the generator's bytes only where
    generate_cas_id reads (cas.rs:31-58); None where the filesystem refuses the size"""
    from spacedrive_amd import synth
    p = str(tmp_path / name)
    try:
        with open(p, "wb") as f:
            f.truncate(size)
            for off, ln in synth.sample_windows(size):
                f.seek(off)
                f.write(cs.synth_bytes(cid, 0, off, ln))
    except OSError:  # EFBIG: the filesystem's largest file
        return None
    return p


def test_cpu_cas_ids_files_past_a_tebibyte(tmp_path, oracle_native):
    """Sampled files of 1 TiB and more on disk (sparse), through the product's file readers
    (the CPU path and the stager that feeds the GPU route): 64-bit pread offsets up to the
    footer at size - 8192, equal to the Python spec and to the oracle's read schedule."""
    sizes = [(1 << 40) + 12345, (1 << 42) + 3, (1 << 43) - 1]
    made = [(s, _sparse_sampled(tmp_path, f"tb{i}", s, 990 + i)) for i, s in enumerate(sizes)]
    made = [(s, p, 990 + i) for i, (s, p) in enumerate(made) if p]
    if not made:
        pytest.skip("the filesystem refuses files of 1 TiB")
    paths = [p for _, p, _ in made]
    szs = [s for s, _, _ in made]
    want = [cs.generate_cas_id(cs.synth_reader(c), s) for s, _, c in made]
    assert cpu.generate_cas_ids(paths, szs, nthreads=2) == want
    got, st = oracle_native.cas_ids_files(paths, np.array(szs, np.uint64), nthreads=2)
    assert not st.any() and [g.tobytes().hex() for g in got] == want
    # the stager (sd_cas_stage_files: the GPU route's reader) stages the spec's messages
    ext, total = stage_plan(np.array(szs, np.uint64))
    staged = np.zeros(total + 64, np.uint8)
    status = np.zeros(len(paths), np.int32)
    arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    check(lib().sd_cas_stage_files(arr, ext.ctypes.data, len(paths), staged.ctypes.data, status.ctypes.data, 2))
    assert not status.any()
    for i, (s, _, c) in enumerate(made):
        o, L = int(ext["msg_offset"][i]), int(ext["msg_len"][i])
        assert staged[o:o + L].tobytes() == cs.cas_message(cs.synth_reader(c), s)
