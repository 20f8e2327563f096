"""The C ABI from plain C (examples/cas_files.c, built by __graft_entry__.build()): the
program a C or FFI host would write, run on real files.  Without a device it takes the
library's CPU path (sd_cpu_*); on the GPU box the same binary uses the device (-m gpu).
Both against the oracle (the reference's read schedule and BLAKE3)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "cas_files")
SIZES = [0, 1, 1016, 102400, 102401, 300001, (1 << 20) + 3]


def _run(args):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} missing: run __graft_entry__.build()")
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return [ln.split("  ", 1) for ln in r.stdout.splitlines()]


def _check(tmp_path, oracle_native, extra):
    rng = np.random.default_rng(3)
    paths, blobs = [], []
    for i, n in enumerate(SIZES):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        (tmp_path / f"f{i}").write_bytes(data)
        paths.append(str(tmp_path / f"f{i}"))
        blobs.append(data)
    want, st = oracle_native.cas_ids_files(paths, np.array(SIZES, np.uint64), nthreads=2)
    assert not st.any()
    missing = str(tmp_path / "missing")
    got = _run(extra + paths + [missing])
    assert [g[1] for g in got] == paths + [missing]
    assert [g[0] for g in got[:-1]] == [w.tobytes().hex() for w in want]
    assert got[-1][0] == "error(2/2)"  # SD_FILE_IO_ERROR with ENOENT
    got = _run(extra + ["-c"] + paths)
    assert [g[0] for g in got] == [oracle_native.blake3(b).hex() for b in blobs]


def test_c_client_cpu_path(tmp_path, oracle_native):
    _check(tmp_path, oracle_native, ["--cpu"])


@pytest.mark.gpu
def test_c_client_gpu(tmp_path, oracle_native):
    _check(tmp_path, oracle_native, [])
