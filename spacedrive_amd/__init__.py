"""spacedrive_amd -- MI355X-native content addressing for Spacedrive.

The hot path of the reference (cavellblood/spacedrive):
  * ``generate_cas_id``  core/src/object/cas.rs:23-62      (sampled BLAKE3 cas_id)
  * ``file_checksum``    core/src/object/validation/hash.rs:10-24 (full-file BLAKE3)
  * the post-hash cas_id -> Object grouping, sharded over GPUs by cas_id prefix
re-implemented as hand-written gfx950 HIP kernels behind the C ABI in include/sd_cas.h
(``libsdcas.so``).  See DESIGN.md.
"""
from ._native import SdCasError, host_cpu_budget, lib, rccl_info  # noqa: F401  (ImportError if libsdcas.so is missing)
from . import cpu  # noqa: F401  (the library's explicit CPU path, sd_cpu_*)
from . import split  # noqa: F401  (one file's checksum over many ranks)
from .cas import (FileMetadata, UnexpectedEofError, cas_ids_files_stats, cas_ids_host_stats, checksums_host_stats,  # noqa: F401
                  checksums_learned,
                  coalescer_stats, file_checksum,
                  file_checksums, file_checksums_bytes, file_checksums_learned, file_checksums_stats, generate_cas_id, generate_cas_ids, get_tuning, set_tuning)
from .device import CasBatch, ChecksumBatch, Context, SplitChecksum, default_context, stage_plan  # noqa: F401

__all__ = ["generate_cas_id", "generate_cas_ids", "file_checksum", "file_checksums", "FileMetadata",
           "UnexpectedEofError", "Context", "CasBatch", "ChecksumBatch", "default_context", "stage_plan",
           "SdCasError", "cas_ids_files_stats", "cas_ids_host_stats", "checksums_host_stats", "file_checksums_stats", "file_checksums_learned", "checksums_learned", "coalescer_stats",
           "set_tuning", "get_tuning", "host_cpu_budget", "rccl_info",
           "cpu"]
