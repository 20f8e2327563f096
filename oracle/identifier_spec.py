"""Restatement of identifier_job_step's Object link/create logic -- TEST INFRASTRUCTURE ONLY.

Follows /root/reference/core/src/object/file_identifier/mod.rs:136-333 literally, over
file_paths in `id` order taken CHUNK_SIZE = 100 at a time (mod.rs:36;
get_orphan_file_paths orders by id and takes 100, file_identifier_job.rs:286-309):

  1. write every file_path's cas_id (mod.rs:144-165);
  2. existing_objects = Objects owning a file_path whose cas_id is among the chunk's
     unique cas_ids (mod.rs:168-175), in DB (creation) order;
  3. each file_path with a cas_id links to the FIRST existing object with an equal
     cas_id (mod.rs:189-225);
  4. every file_path whose cas_id is None (empty file) or not owned by an existing
     object gets a NEW Object of its own (mod.rs:229-333) -- so duplicates inside one
     chunk each get a separate Object.

The reference creates a chunk's new Objects in HashMap order (mod.rs:134), so which of
several same-chunk duplicates a later chunk links to is unspecified there; this
restatement creates them in index order (lowest index first), and the product rule in
spacedrive_amd/identifier.py uses the same tie-break.  Counts per chunk are exact.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

CHUNK_SIZE = 100


def _assign_step(chunk, cas_of, objects, obj_cas, out):
    """mod.rs:136-333 for one step's rows (their cas_ids known): link to existing Objects,
    create the rest.  Returns (created, linked)."""
    unique = {cas_of[i] for i in chunk if cas_of[i] is not None}
    existing = [o for o in range(len(objects)) if obj_cas[o] & unique]
    existing_cas = set()
    for o in existing:
        existing_cas |= obj_cas[o]
    linked = 0
    for i in chunk:
        c = cas_of[i]
        if c is None:
            continue
        o = next((o for o in existing if c in obj_cas[o]), None)
        if o is not None:
            out[i] = o
            objects[o].append(i)
            linked += 1
    created = 0
    for i in chunk:
        c = cas_of[i]
        if c is None or c not in existing_cas:
            o = len(objects)
            objects.append([i])
            obj_cas.append({c} if c is not None else set())
            out[i] = o
            created += 1
    return created, linked


def identifier_replay(cas_ids: Sequence[Optional[str]], chunk_size: int = CHUNK_SIZE
                      ) -> Tuple[List[int], List[Tuple[int, int]]]:
    """cas_ids in file_path.id order -> (object id per file, [(created, linked)] per chunk)."""
    n = len(cas_ids)
    objects: List[List[int]] = []      # object id -> file indices
    obj_cas: List[set] = []            # object id -> cas_ids of its file_paths
    out: List[int] = [-1] * n
    stats = []
    for start in range(0, n, chunk_size):
        stats.append(_assign_step(range(start, min(n, start + chunk_size)), cas_ids, objects, obj_cas, out))
    # name every object by the file that created it
    return [objects[o][0] for o in out], stats


ERR = object()  # a file whose FileMetadata::new failed (mod.rs:127-128: logged, dropped)


def identifier_job_replay(results: Sequence, chunk_size: int = CHUNK_SIZE):
    """The whole identifier JOB over orphan file_paths 0..n-1 (their ids), with per-file
    hashing outcomes `results[i]` = cas_id str, None (empty file, no cas_id) or ERR:
      * init: task_count = ceil(orphans / 100) steps, cursor = the first orphan's id
        (file_identifier_job.rs:120-171);
      * each step: orphans (no Object yet) with id >= cursor, in id order, at most 100
        (get_orphan_file_paths, :286-309; orphan_path_filters :245-268); none -> EarlyFinish
        (:196-203);
      * a file whose metadata failed is dropped from the step and stays an orphan
        (mod.rs:119-134); the rest link or create (mod.rs:136-333);
      * cursor = the id of the step's last row (mod.rs:384-392) -- so a dropped file that
        was its step's last row is queried (and hashed) again by the next step.
    Returns (owner file index per file or None if never assigned, [(created, linked)] per
    step, [rows queried per step])."""
    n = len(results)
    objects: List[List[int]] = []
    obj_cas: List[set] = []
    out: List[int] = [-1] * n
    stats, queried = [], []
    if n == 0:
        return [], [], []
    steps = (n + chunk_size - 1) // chunk_size
    cursor = 0
    for _ in range(steps):
        rows = [i for i in range(cursor, n) if out[i] < 0][:chunk_size]
        if not rows:
            break  # EarlyFinish
        queried.append(rows)
        ok = [i for i in rows if results[i] is not ERR]
        cas_of = {i: results[i] for i in ok}
        stats.append(_assign_step(ok, cas_of, objects, obj_cas, out))
        cursor = rows[-1]
    return [objects[o][0] if o >= 0 else None for o in out], stats, queried
