"""The identifier job with look-ahead hashing (spacedrive_amd/identifier.py IdentifierJob) vs a
literal restatement of the reference's job (oracle/identifier_spec.py identifier_job_replay:
file_identifier_job.rs:80-309, mod.rs:100-392) fed with the oracle's own cas_ids.

Files on disk: duplicates inside one step and across steps, empty files (own Object, never
linked), and files whose metadata fails (dropped and left orphan) -- among them a step's
LAST row, which the reference's cursor (`id >= last id`) queries and hashes again.  The
per-step (created, linked) counts and every file's Object must be equal for every
look-ahead size, and a job paused and resumed with an empty cache must end the same."""
import os

import numpy as np
import pytest

from oracle.identifier_spec import ERR, identifier_job_replay
from spacedrive_amd import identifier
from spacedrive_amd.identifier import IdentifierJob


def _library(root, n=2345, seed=11):
    """n orphan paths: contents drawn from a small pool (duplicates), some empty, some missing."""
    rng = np.random.default_rng(seed)
    pool = []
    for k in range(400):
        size = int(rng.choice([1, 57, 1016, 1017, 4096, 65536, 102400, 102401, 150000, 300000]))
        pool.append(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
    paths = []
    for i in range(n):
        p = os.path.join(root, f"f{i:05d}")
        if i % 97 == 5 or i in (99, 199, 200, 1299):  # metadata fails: dangling symlink (stat: ENOENT)
            os.symlink(os.path.join(root, "missing", str(i)), p)
        elif i % 41 == 3:
            open(p, "wb").close()  # empty: cas_id None (mod.rs:80-88)
        else:
            src = i - 1 if i % 13 == 0 and i else int(rng.integers(0, len(pool)))  # adjacent copies too
            data = open(paths[src], "rb").read() if i % 13 == 0 and i and os.path.isfile(paths[src]) \
                else pool[src % len(pool)]
            with open(p, "wb") as f:
                f.write(data)
        paths.append(p)
    return paths


def _oracle_outcomes(paths):
    from oracle import native
    res = [None] * len(paths)
    todo, sizes = [], []
    for i, p in enumerate(paths):
        try:
            st = os.stat(p)
        except OSError:
            res[i] = ERR
            continue
        if st.st_size:
            todo.append(i)
            sizes.append(st.st_size)
    ids, status = native.cas_ids_files([paths[i] for i in todo], sizes, nthreads=4)
    for k, i in enumerate(todo):
        res[i] = ids[k].tobytes().hex() if status[k] == 0 else ERR
    return res


@pytest.fixture(scope="module")
def library(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("identifier_job"))
    paths = _library(root)
    want_owner, want_stats, queried = identifier_job_replay(_oracle_outcomes(paths))
    return paths, want_owner, want_stats, queried


def _cpu_metadata():
    from spacedrive_amd import cpu
    return identifier._stat_then_hash(lambda p, s: cpu.generate_cas_ids(p, s, nthreads=4))


def _check(job, want_owner, want_stats):
    assert job.step_stats == want_stats
    assert job.owner == want_owner


@pytest.mark.parametrize("k", [100, 1000, 32768])
def test_lookahead_job_equals_reference_job(library, k):
    paths, want_owner, want_stats, queried = library
    job = IdentifierJob(paths, lookahead=k, metadata=_cpu_metadata()).run()
    _check(job, want_owner, want_stats)
    # the dropped last rows were queried twice by the reference's cursor rule
    assert sum(len(q) for q in queried) > len(paths) - sum(o is None for o in want_owner)
    # one batched call per `k` orphans (plus small calls for re-queried rows)
    assert max(job.hash_calls) <= max(k, 100)
    if k >= len(paths):
        assert job.hash_calls[0] == len(paths)


def test_lookahead_job_resumes_from_its_cursor(library):
    paths, want_owner, want_stats, _ = library
    first = IdentifierJob(paths, lookahead=1000, metadata=_cpu_metadata()).run(max_steps=7)
    st = first.resume_state()
    assert len(first.cache) > 0  # hashed ahead of the pause, then dropped with the job
    second = IdentifierJob(paths, lookahead=1000, metadata=_cpu_metadata(), cursor=st["cursor"], owner=st["owner"],
                           cas_owner=st["cas_owner"], step_stats=st["step_stats"]).run()
    _check(second, want_owner, want_stats)
    # the resumed job re-hashes from its cursor, nothing before it
    assert second.hash_calls[0] <= len(paths) - st["cursor"]


def test_job_replay_without_errors_is_the_chunked_replay():
    from oracle.identifier_spec import identifier_replay
    rng = np.random.default_rng(3)
    cas = [None if rng.random() < 0.05 else format(int(rng.integers(0, 300)), "x") for _ in range(2001)]
    o1, s1 = identifier_replay(cas)
    o2, s2, q = identifier_job_replay(cas)
    assert o1 == o2 and s1 == s2 and all(len(x) == 100 for x in q[:-1])


@pytest.mark.gpu
def test_lookahead_job_on_the_gpu_route(library):
    """The default metadata: stat + generate_cas_ids (sd_cas_ids_files); a look-ahead call of
    more than batch_cpu_max files takes the GPU route."""
    import spacedrive_amd as sd
    paths, want_owner, want_stats, _ = library
    keep = sd.get_tuning("batch_cpu_max")
    sd.set_tuning("batch_cpu_max", 1000)  # this library (2345 files) is one call above the threshold
    try:
        before = sd.cas_ids_files_stats()
        job = IdentifierJob(paths, lookahead=32768).run()
        after = sd.cas_ids_files_stats()
    finally:
        sd.set_tuning("batch_cpu_max", keep)
    _check(job, want_owner, want_stats)
    assert job.hash_calls[0] > 1000 and after["gpu"] > before["gpu"]
