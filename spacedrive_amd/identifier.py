"""Object assignment from the GPU dedup output, with the reference's chunk-of-100 rule.

identifier_job_step (core/src/object/file_identifier/mod.rs:136-333) processes orphan
file_paths in id order, 100 per step (mod.rs:36).  Within one step, a file whose cas_id
already belongs to an Object from an EARLIER step links to it; every other file --
including duplicates inside the same step and empty files -- gets a new Object of its
own.  With `rep` = the smallest index of a file's equal-cas_id group (sd_dedup_group),
that is, per file i:

    owner(i) = i      if chunk(i) == chunk(rep(i))   (created in the cas_id's first step)
               rep(i) otherwise                      (linked to the first step's Object)

-- one elementwise pass on the device, no per-chunk DB round trips.  The objects are
named by the index of the file that created them.  Checked against a literal
restatement of mod.rs:136-333 (oracle/identifier_spec.py) in tests/test_identifier.py.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch

CHUNK_SIZE = 100  # file_identifier/mod.rs:36
LOOKAHEAD = 32768  # orphans hashed per generate_cas_ids call by the look-ahead identifier


def object_owners(index: torch.Tensor, rep: torch.Tensor, chunk_size: int = CHUNK_SIZE) -> torch.Tensor:
    """owner file index per record (records of non-empty files; empty files own themselves)."""
    same_step = torch.div(index, chunk_size, rounding_mode="floor") == torch.div(rep, chunk_size,
                                                                                  rounding_mode="floor")
    return torch.where(same_step, index, rep)


def step_counts(index: torch.Tensor, owner: torch.Tensor, n_files: int, empty_index: torch.Tensor = None,
                chunk_size: int = CHUNK_SIZE):
    """(created, linked) per identifier step, as identifier_job_step returns them (mod.rs:335)."""
    steps = (n_files + chunk_size - 1) // chunk_size
    chunk = torch.div(index, chunk_size, rounding_mode="floor")
    created = torch.bincount(chunk[owner == index], minlength=steps)
    linked = torch.bincount(chunk[owner != index], minlength=steps)
    if empty_index is not None and empty_index.numel():
        created = created + torch.bincount(torch.div(empty_index, chunk_size, rounding_mode="floor"),
                                           minlength=steps)
    return created, linked


# ------------------------------------------------------------------ the identifier job
# A file's outcome of FileMetadata::new (mod.rs:59-97): its cas_id (None for an empty
# file) or the OSError that makes the step log and drop it (mod.rs:127-128).
Outcome = Union[Optional[str], OSError]


def _stat_then_hash(hash_batch: Callable[[List[str], List[int]], List[Union[str, OSError]]]):
    """FileMetadata::new for many files: stat (mod.rs:65-67), no hash for an empty file
    (mod.rs:80-88), ONE batched generate_cas_ids for the rest."""
    def run(paths: Sequence[str]) -> List[Outcome]:
        out: List[Outcome] = [None] * len(paths)
        todo, sizes = [], []
        for i, p in enumerate(paths):
            try:
                st = os.stat(p)
            except OSError as e:
                out[i] = e
                continue
            if st.st_size:
                todo.append(i)
                sizes.append(st.st_size)
        if todo:
            for i, r in zip(todo, hash_batch([paths[i] for i in todo], sizes)):
                out[i] = r
        return out
    return run


@dataclass
class IdentifierJob:
    """The file_identifier job over one location's orphan file_paths, with look-ahead hashing.

    The job is the reference's (file_identifier_job.rs:80-243): ``steps`` = ceil(orphans /
    100) at init, each step queries the orphans with ``id >= cursor`` in id order, at most
    CHUNK_SIZE (get_orphan_file_paths, :286-309), links or creates their Objects
    (identifier_job_step, mod.rs:100-336) and moves the cursor to the step's last row
    (mod.rs:384-392); a file whose metadata fails is dropped from its step and stays an
    orphan (mod.rs:127-128).  Only the hashing is new: a step whose rows are not all in the
    look-ahead cache hashes the next ``lookahead`` orphans from its cursor that are not
    cached, in ONE batched call (generate_cas_ids: the GPU route, from 4097 files on), and
    the steps take their outcomes from the cache, each consumed once.  The 100-row steps,
    their queries and the Object rule are unchanged, so the Objects equal the reference's.
    A resumed job (``cursor`` / ``objects`` restored, cache empty) re-hashes from its cursor,
    as the reference does (file_identifier_job.rs:53-68).

    ``orphans``: the location's orphan paths in file_path.id order (id = position).
    ``metadata``: paths -> outcomes; default = stat + the library's generate_cas_ids."""

    orphans: Sequence[str]
    lookahead: int = LOOKAHEAD
    metadata: Optional[Callable[[Sequence[str]], List[Outcome]]] = None
    chunk_size: int = CHUNK_SIZE
    cursor: int = 0
    owner: List[Optional[int]] = field(default_factory=list)   # object (named by its creator) per file
    cas_owner: Dict[str, int] = field(default_factory=dict)   # cas_id -> Object, for later links
    step_stats: List[Tuple[int, int]] = field(default_factory=list)
    hash_calls: List[int] = field(default_factory=list)       # files per batched hashing call
    cache: Dict[int, Outcome] = field(default_factory=dict)

    def __post_init__(self):
        if self.metadata is None:
            from .cas import generate_cas_ids
            self.metadata = _stat_then_hash(generate_cas_ids)
        if not self.owner:
            self.owner = [None] * len(self.orphans)
        self.steps = (len(self.orphans) + self.chunk_size - 1) // self.chunk_size

    def _query(self, k: int) -> List[int]:
        """orphans with id >= cursor, in id order, at most k (orphan_path_filters, :245-268)"""
        out = []
        for i in range(self.cursor, len(self.orphans)):
            if self.owner[i] is None:
                out.append(i)
                if len(out) == k:
                    break
        return out

    def step(self) -> Optional[Tuple[int, int]]:
        """One execute_step (file_identifier_job.rs:174-230); None = EarlyFinish."""
        rows = self._query(self.chunk_size)
        if not rows:
            return None
        if any(i not in self.cache for i in rows):  # look ahead from the cursor
            todo = [i for i in self._query(max(self.lookahead, self.chunk_size)) if i not in self.cache]
            self.hash_calls.append(len(todo))
            for i, r in zip(todo, self.metadata([self.orphans[i] for i in todo])):
                self.cache[i] = r
        outcome = {i: self.cache.pop(i) for i in rows}
        ok = [i for i in rows if not isinstance(outcome[i], OSError)]  # mod.rs:127-128
        # mod.rs:136-333: link to an Object of an earlier step, else create one per file
        linked = 0
        for i in ok:
            c = outcome[i]
            if c is not None and c in self.cas_owner:
                self.owner[i] = self.cas_owner[c]
                linked += 1
        created = 0
        for i in ok:
            c = outcome[i]
            if self.owner[i] is None:
                self.owner[i] = i
                created += 1
                if c is not None and c not in self.cas_owner:
                    self.cas_owner[c] = i  # the lowest index of the step creates the linked-to Object
        self.cursor = rows[-1]
        self.step_stats.append((created, linked))
        return created, linked

    def run(self, max_steps: Optional[int] = None) -> "IdentifierJob":
        """The job's step loop (job/mod.rs:622-856) for its remaining steps."""
        todo = self.steps - len(self.step_stats)
        if max_steps is not None:
            todo = min(todo, max_steps)
        for _ in range(todo):
            if self.step() is None:
                break
        return self

    def resume_state(self) -> dict:
        """What the reference persists across a pause (JobState: the run metadata's cursor and
        the DB's Object links); the look-ahead cache is not part of it."""
        return {"cursor": self.cursor, "owner": list(self.owner), "cas_owner": dict(self.cas_owner),
                "step_stats": list(self.step_stats)}
