"""The C ABI boundary on a machine without a GPU: the library loads, exports exactly what
include/sd_cas.h declares, its host-only planning works, and the GPU entry points fail
loudly without a device (the CPU path is the separate, explicit sd_cpu_* family)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from spacedrive_amd import _native
from spacedrive_amd._native import SdCasError, check, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(_native.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sd_[a-z0-9_]+)\s*\(", src)))


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_abi():
    fns = declared_functions()
    for must in ("sd_cas_ctx_create", "sd_cas_ids", "sd_cas_batch_run", "sd_checksum_batch_run",
                 "sd_file_checksums", "sd_dedup_partition", "sd_dedup_group", "sd_cas_stage_plan"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    exp = exported_symbols()
    missing = [f for f in declared_functions() if f not in exp]
    assert not missing, missing
    # and the Python binding covers the whole header
    assert sorted(n for n, _, _ in _native.SIGNATURES) == declared_functions()


def test_library_loads_and_binds():
    L = lib()
    assert L.sd_cas_abi_version() == 2
    for name, _, _ in _native.SIGNATURES:
        assert getattr(L, name) is not None


def test_stage_plan_layout():
    # cas.rs:25-58: 8 + size (<= 102400) or 57352; 64-byte aligned offsets
    sizes = np.array([0, 1, 102400, 102401, 5 << 30, 1000], np.uint64)
    from spacedrive_amd.device import stage_plan
    ext, total = stage_plan(sizes)
    assert list(ext["msg_len"]) == [8, 9, 102408, 57352, 57352, 1008]
    assert list(ext["kind"]) == [1, 1, 1, 2, 2, 1]
    assert all(int(o) % 64 == 0 for o in ext["msg_offset"])
    ends = ext["msg_offset"] + ext["msg_len"]
    assert np.all(ext["msg_offset"][1:] >= ends[:-1])
    assert total % 64 == 0 and total >= int(ends[-1])


def test_stage_file_host_only(tmp_path):
    # staging needs no device: pread of header / samples / tail into the extent
    from oracle import cas_spec as cs
    from spacedrive_amd.device import stage_plan
    sizes = [100, 102400, 300000]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"f{i}"
        p.write_bytes(cs.synth_bytes(40 + i, 0, 0, s))
        paths.append(p)
    ext, total = stage_plan(np.array(sizes, np.uint64))
    staged = np.full(total, 0xAB, np.uint8)
    for i, p in enumerate(paths):
        st = ctypes.c_int32(-1)
        check(lib().sd_cas_stage_file(os.fsencode(p), ctypes.c_void_p(ext.ctypes.data + 24 * i),
                                      ctypes.c_void_p(staged.ctypes.data), ctypes.byref(st)))
        assert st.value == 0
        msg = cs.cas_message(cs.synth_reader(40 + i), sizes[i])
        o = int(ext["msg_offset"][i])
        assert staged[o:o + len(msg)].tobytes() == msg
        pad_end = (o + len(msg) + 63) // 64 * 64
        assert not staged[o + len(msg):pad_end].any()  # zero padding


def test_stage_file_errors(tmp_path):
    from spacedrive_amd.device import stage_plan
    ext, total = stage_plan(np.array([200000], np.uint64))
    staged = np.zeros(total, np.uint8)
    st = ctypes.c_int32(-1)
    check(lib().sd_cas_stage_file(b"/nonexistent/x", ctypes.c_void_p(ext.ctypes.data),
                                  ctypes.c_void_p(staged.ctypes.data), ctypes.byref(st)))
    assert st.value & 0xFFFF == _native.SD_FILE_IO_ERROR and (st.value >> 16) == 2  # ENOENT
    short = tmp_path / "short"
    short.write_bytes(b"x" * 150000)  # planned 200000: the last sample (145904..156144) runs past EOF
    check(lib().sd_cas_stage_file(os.fsencode(short), ctypes.c_void_p(ext.ctypes.data),
                                  ctypes.c_void_p(staged.ctypes.data), ctypes.byref(st)))
    assert st.value == _native.SD_FILE_SHORT_READ


def test_invalid_arguments_do_not_cross_boundary():
    rc = lib().sd_cas_stage_plan(None, 3, None, None)
    assert rc == -1 and b"null" in lib().sd_cas_last_error()
    out = (ctypes.c_double * 4)()
    rc = lib().sd_file_checksums_learned(None, out)  # no context: refused before any HIP call
    assert rc == -1 and b"null" in lib().sd_cas_last_error()
    rc = lib().sd_checksums_learned(None, out)
    assert rc == -1 and b"null" in lib().sd_cas_last_error()


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_gpu_entry_points_fail_without_a_device():
    h = ctypes.c_void_p()
    with pytest.raises(SdCasError) as e:
        check(lib().sd_cas_ctx_create(0, ctypes.byref(h)))
    assert e.value.rc == -2


def test_unknown_tuning_key_is_rejected():
    assert lib().sd_cas_set_tuning(b"whole_variant", 3) == -1  # the A/B kernel variants are gone
    assert lib().sd_cas_set_tuning(b"sampled_variant", 0) == -1
    assert lib().sd_cas_set_tuning(b"files_window_mb", 32) == 0
    # the batch-size policy between the latency and the throughput kernels
    assert lib().sd_cas_set_tuning(b"sampled_wave_max", 6144) == 0
    assert lib().sd_cas_set_tuning(b"whole_wave_max", 512) == 0
    # sd_cas_ids_files' batch-size policy (CPU path at or below it)
    assert lib().sd_cas_set_tuning(b"batch_cpu_max", 4096) == 0


def test_stage_files_threaded_equals_single(tmp_path):
    # sd_cas_stage_files on 8 threads == sd_cas_stage_file one by one, incl. error statuses
    from oracle import cas_spec as cs
    from spacedrive_amd.device import stage_plan
    sizes = [1, 1000, 102400, 102401, 250000, 77, 0, 150000]
    paths = []
    for i, sz in enumerate(sizes):
        p = tmp_path / f"g{i}"
        p.write_bytes(cs.synth_bytes(70 + i, 0, 0, sz if i != 7 else 140000))  # last: shorter than planned
        paths.append(str(p))
    paths.append(str(tmp_path / "missing"))
    sizes.append(5000)
    ext, total = stage_plan(np.array(sizes, np.uint64))
    a = np.full(total, 0x11, np.uint8)
    b = np.full(total, 0x22, np.uint8)
    st_a = np.zeros(len(sizes), np.int32)
    for i, p in enumerate(paths):
        st = ctypes.c_int32()
        check(lib().sd_cas_stage_file(os.fsencode(p), ctypes.c_void_p(ext.ctypes.data + 24 * i),
                                      ctypes.c_void_p(a.ctypes.data), ctypes.byref(st)))
        st_a[i] = st.value
    arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    st_b = np.full(len(sizes), -7, np.int32)
    check(lib().sd_cas_stage_files(arr, ext.ctypes.data, len(paths), b.ctypes.data, st_b.ctypes.data, 8))
    assert list(st_a) == list(st_b)
    # file 7 is 140000 B planned as 150000: every sample fits and the tail is read at the
    # file's real end (SeekFrom::End, cas.rs:54) -- the reference returns an id
    assert st_b[7] == _native.SD_FILE_OK and (st_b[8] & 0xFFFF) == _native.SD_FILE_IO_ERROR
    for i in range(8):
        o, L = int(ext["msg_offset"][i]), int(ext["msg_len"][i])
        content = cs.synth_bytes(70 + i, 0, 0, sizes[i] if i != 7 else 140000)
        assert a[o:o + L].tobytes() == b[o:o + L].tobytes() == cs.cas_message_file(content, sizes[i])


def _header_param_counts():
    src = open(_native.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(sd_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


RUST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "rust")


def _rust_decls():
    src = open(os.path.join(RUST, "sd-cas-sys", "src", "lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    return src, re.findall(r"pub fn (sd_[a-z0-9_]+)\s*\(([^)]*)\)", block, flags=re.S)


def test_rust_shim_matches_header():
    """integration/rust/sd-cas-sys (the binding a maintainer adds as crates/sd-cas-sys)
    declares only functions the header has, with the header's parameter counts, and the
    new round-2 exports: the CPU path, the RCCL exchange, host-memory checksums."""
    src, decls = _rust_decls()
    hdr = _header_param_counts()
    for name, args in decls:
        n = 0 if not args.strip() else args.count(",") + 1 - (1 if args.strip().endswith(",") else 0)
        assert name in hdr, name
        assert hdr[name] == n, (name, hdr[name], n)
    names = {n for n, _ in decls}
    for must in ("sd_cas_ids_files", "sd_cas_id_path", "sd_file_checksums", "sd_file_checksum_path", "sd_checksums",
                 "sd_cpu_cas_ids_files", "sd_cpu_file_checksums", "sd_cpu_cas_id_path", "sd_cpu_file_checksum_path",
                 "sd_comm_id", "sd_comm_create", "sd_comm_destroy", "sd_cas_dedup_mgpu"):
        assert must in names, must
    hdr_src = open(_native.HEADER).read()
    abi = re.search(r"#define SD_CAS_ABI_VERSION (\d+)", hdr_src).group(1)
    assert f"SD_CAS_ABI_VERSION: c_int = {abi};" in src
    for c, v in (("SD_FILE_CHANGED", 4), ("SD_ERR_CAPACITY", -6), ("SD_COMM_ID_BYTES", 128)):
        assert re.search(rf"{c}\b[^;]*= {v};", src), c
    # no panic on a GPU-less node -- ctx() returns a Result, the safe layer
    # routes to the CPU path
    ctx_fn = src[src.index("pub fn ctx()"):src.index("pub fn last_error()")]
    assert "-> Result<&'static Ctx, io::Error>" in ctx_fn
    assert not re.search(r"\b(assert|assert_eq|panic|unwrap|expect)\b", ctx_fn)
    for safe, cpu in (("cas_ids_blocking", "sd_cpu_cas_ids_files"), ("cas_id_blocking", "sd_cpu_cas_id_path"),
                      ("checksums_blocking", "sd_cpu_file_checksums"),
                      ("checksum_blocking", "sd_cpu_file_checksum_path")):
        body = src[src.index(f"pub fn {safe}("):]
        body = body[:body.index("\n}\n")]
        assert cpu in body and "Err(_) =>" in body, safe


def test_rust_step_excerpts_use_the_shim():
    """The batched identifier step (file_identifier/mod.rs:100-134) and validator step
    (validation/validator_job.rs:126-168) call the batched functions core/cas.rs and
    core/hash.rs define, keep the reference's per-file error policies, and keep the
    100-row chunking that Object linking depends on."""
    core = os.path.join(RUST, "core")
    cas, hsh = open(os.path.join(core, "cas.rs")).read(), open(os.path.join(core, "hash.rs")).read()
    ident = open(os.path.join(core, "file_identifier_step.rs")).read()
    valid = open(os.path.join(core, "validator_step.rs")).read()
    assert "pub async fn generate_cas_ids(" in cas and "pub async fn generate_cas_id(" in cas
    assert "pub async fn file_checksums(" in hsh and "pub async fn file_checksum(" in hsh
    assert "generate_cas_ids(to_hash).await" in ident
    assert 'error!("Failed to extract file metadata' in ident  # log and drop (mod.rs:127-128)
    assert "md.len() != 0" in ident  # empty files are not hashed (mod.rs:80-88)
    assert "CHUNK_SIZE stays" in ident
    # the identifier reaches the GPU by looking ahead, K orphans per hashing call
    # (spacedrive_amd/identifier.py IdentifierJob is the tested statement of it)
    assert "pub const LOOKAHEAD: i64 = 32_768;" in ident and ".take(LOOKAHEAD)" in ident
    assert "#[serde(skip)]" in ident and "lookahead.take(file_paths)" in ident
    assert ".order_by(file_path::id::order(SortOrder::Asc))" in ident  # the reference's query order
    from spacedrive_amd.identifier import LOOKAHEAD
    assert LOOKAHEAD == 32768
    assert "file_checksums(full_paths.clone()).await" in valid
    assert "ValidatorError::FileIO(FileIOError::from((full_path, e))))?" in valid  # `?` per file (:147-149)


def test_path_array_and_hex_results(tmp_path):
    """The batched wrappers' marshalling: path_array's char** holds every path as os.fsencode
    gives it (str, bytes, PathLike, non-UTF-8 bytes), rejects an embedded NUL like open();
    hex_results returns the hex strings and the caller's error for each failed status --
    and the CPU path called through them hashes real files like the single-file call."""
    import pathlib
    from spacedrive_amd import cpu
    from spacedrive_amd._native import hex_results, path_array
    paths = ["/a/b", b"/c\xff/d", pathlib.Path("/e f/é"), "/" + "x" * 300]
    keep, arr = path_array(paths)
    ptrs = np.ctypeslib.as_array((ctypes.c_uint64 * len(paths)).from_address(arr))
    assert [ctypes.string_at(int(p)) for p in ptrs] == [os.fsencode(p) for p in paths]
    with pytest.raises(ValueError):
        path_array(["ok", "bad\0path"])
    out = ctypes.create_string_buffer(b"".join(b"%016x\0" % i for i in range(5)), 17 * 5)
    st = np.array([0, 0, 2 | (2 << 16), 0, 0], np.int32)
    got = hex_results(out, 16, st, ["p0", "p1", "p2", "p3", "p4"], lambda s, p: (s, p))
    assert got == ["%016x" % 0, "%016x" % 1, (st[2], "p2"), "%016x" % 3, "%016x" % 4]
    assert hex_results(out, 16, np.zeros(5, np.int32), ["p"] * 5, None) == ["%016x" % i for i in range(5)]
    files = []
    for i, n in enumerate([1, 5000, 102401, 0]):
        f = tmp_path / f"f{i}"
        f.write_bytes(bytes((j * 7 + i) % 251 for j in range(n)))
        files.append(str(f))
    files.append(str(tmp_path / "missing"))
    sizes = [os.path.getsize(f) if os.path.exists(f) else 10 for f in files]
    batch = cpu.generate_cas_ids(files, sizes)
    for f, s, r in zip(files, sizes, batch):
        if os.path.exists(f):
            assert r == cpu.generate_cas_id(f, s)
        else:
            assert isinstance(r, OSError) and r.filename == f


def test_host_cpu_budget_caps_and_override():
    """The host thread budget: resolved from this process's CPUs, at
    least 1 and at most its affinity mask; "host_cpu_budget" > 0 replaces it and 0 restores
    the resolved value; a CPU-path call with more threads than the budget gives the same
    results (it is clamped, not refused)."""
    import spacedrive_amd as sd
    b = sd.host_cpu_budget()
    assert 1 <= b["budget"] <= b["affinity"] == len(os.sched_getaffinity(0)) and not b["overridden"]
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    assert b["local_world_size"] == max(1, lw)
    data = np.random.default_rng(3).integers(0, 256, 5 << 20, dtype=np.uint8)
    offs = np.array([0, 1 << 20, 3 << 20], np.uint64)
    lens = np.array([1 << 20, (2 << 20) + 7, 12345], np.uint64)
    want = np.zeros((3, 32), np.uint8)
    check(lib().sd_cpu_checksums(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, 3, want.ctypes.data, 1))
    try:
        sd.set_tuning("host_cpu_budget", 2)
        assert sd.host_cpu_budget()["budget"] == 2 and sd.host_cpu_budget()["overridden"]
        got = np.zeros((3, 32), np.uint8)
        check(lib().sd_cpu_checksums(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, 3, got.ctypes.data, 64))
        assert np.array_equal(got, want)
    finally:
        sd.set_tuning("host_cpu_budget", 0)
    assert sd.host_cpu_budget() == b


def test_host_cpu_budget_divides_by_local_world_size():
    """Each of the node's ranks gets its share: a process started as one of 4 local ranks
    (LOCAL_WORLD_SIZE=4, as torch.distributed.run sets it) resolves min(affinity share,
    quota / 4), the affinity split only when the mask holds every online CPU (a narrower
    mask is a per-rank binding)."""
    import math
    import sys
    code = ("import os, json, spacedrive_amd as sd; "
            "print(json.dumps(sd.host_cpu_budget()))")
    env = dict(os.environ, LOCAL_WORLD_SIZE="4")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).stdout
    import json
    b = json.loads(out.strip().splitlines()[-1])
    aff = b["affinity"]
    cpus = aff // 4 if aff >= os.cpu_count() else aff
    if b["cgroup_quota_cpus"]:
        cpus = min(cpus, max(1, math.ceil(b["cgroup_quota_cpus"] - 1e-9)) // 4)
    assert b["local_world_size"] == 4 and b["budget"] == max(1, cpus)


def test_host_cpu_budget_keeps_a_bound_ranks_mask():
    """A rank bound to its own CPUs (taskset / numactl / --cpu-bind: a mask narrower than
    the machine) keeps that mask as its share; it is not divided by LOCAL_WORLD_SIZE a second
    time."""
    import json
    import sys
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2 or len(cpus) < os.cpu_count():
        pytest.skip("needs an unbound process on a machine of >= 2 CPUs")
    mine = cpus[:2]
    code = ("import os, json; os.sched_setaffinity(0, %r); import spacedrive_amd as sd; "
            "print(json.dumps(sd.host_cpu_budget()))" % (mine,))
    env = dict(os.environ, LOCAL_WORLD_SIZE="8")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).stdout
    b = json.loads(out.strip().splitlines()[-1])
    assert b["affinity"] == 2
    want = 2
    if b["cgroup_quota_cpus"]:
        import math
        want = min(want, max(1, math.ceil(b["cgroup_quota_cpus"] - 1e-9) // 8))
    assert b["budget"] == max(1, want)


def test_host_numa_without_a_context_places_nothing():
    """The library's threads are placed on a device's NUMA node only once a context exists
    (sd_cas_ctx_create reads the node); the CPU path alone leaves them where they are, and
    "numa_pin" is an ordinary tuning key."""
    import spacedrive_amd as sd
    from spacedrive_amd._native import host_numa
    if os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK):
        pytest.skip("GPU present: a context may exist")
    assert host_numa() == {"placed": False, "cpus": 0, "device_node": -1}
    keep = sd.get_tuning("numa_pin")
    assert keep == 0  # opt-in
    sd.set_tuning("numa_pin", 1)
    sd.set_tuning("numa_pin", keep)


@pytest.mark.parametrize("lang,std", [("c", "-std=c99"), ("c", "-std=c11"), ("c++", "-std=c++11"), ("c++", "-std=c++17")])
def test_header_compiles_strict(tmp_path, lang, std):
    """include/sd_cas.h is the boundary a Rust (bindgen / hand-written extern "C"), C or C++
    host includes: it compiles on its own under strict ISO modes with every warning an
    error, and links against the in-tree library (every function a host would call
    resolves)."""
    src = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    src.write_text('#include "sd_cas.h"\n'
                   "int main(void) { return sd_cas_abi_version() > 0 ? 0 : 1; }\n")
    cc = "gcc" if lang == "c" else "g++"
    lib_dir = os.path.join(ROOT, "spacedrive_amd")
    r = subprocess.run([cc, std, "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                        str(src), "-L", lib_dir, "-lsdcas", "-Wl,-rpath," + lib_dir, "-o", str(tmp_path / "t")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert subprocess.run([str(tmp_path / "t")], timeout=60).returncode == 0
