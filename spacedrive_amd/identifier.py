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

import torch

CHUNK_SIZE = 100  # file_identifier/mod.rs:36


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
