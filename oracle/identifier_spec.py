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


def identifier_replay(cas_ids: Sequence[Optional[str]], chunk_size: int = CHUNK_SIZE
                      ) -> Tuple[List[int], List[Tuple[int, int]]]:
    """cas_ids in file_path.id order -> (object id per file, [(created, linked)] per chunk)."""
    n = len(cas_ids)
    objects: List[List[int]] = []      # object id -> file indices
    obj_cas: List[set] = []            # object id -> cas_ids of its file_paths
    out: List[int] = [-1] * n
    stats = []
    for start in range(0, n, chunk_size):
        chunk = range(start, min(n, start + chunk_size))
        unique = {cas_ids[i] for i in chunk if cas_ids[i] is not None}
        existing = [o for o in range(len(objects)) if obj_cas[o] & unique]
        existing_cas = set()
        for o in existing:
            existing_cas |= obj_cas[o]
        linked = 0
        for i in chunk:
            c = cas_ids[i]
            if c is None:
                continue
            o = next((o for o in existing if c in obj_cas[o]), None)
            if o is not None:
                out[i] = o
                objects[o].append(i)
                linked += 1
        created = 0
        for i in chunk:
            c = cas_ids[i]
            if c is None or c not in existing_cas:
                o = len(objects)
                objects.append([i])
                obj_cas.append({c} if c is not None else set())
                out[i] = o
                created += 1
        stats.append((created, linked))
    # name every object by the file that created it
    return [objects[o][0] for o in out], stats
