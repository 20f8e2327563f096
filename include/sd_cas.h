/*
 * sd_cas.h -- C ABI of the MI355X content-addressing library (libsdcas.so).
 *
 * Drop-in boundary for Spacedrive's content-addressing hot path:
 *   generate_cas_id  /root/reference/core/src/object/cas.rs:23
 *       pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) -> Result<String, io::Error>
 *   file_checksum    /root/reference/core/src/object/validation/hash.rs:10
 *       pub async fn file_checksum(path: impl AsRef<Path>) -> Result<String, io::Error>
 * The Rust signatures stay as they are; a thin shim crate calls these
 * entry points inside tokio::task::spawn_blocking, and a batched sibling replaces the
 * per-file join_all of identifier_job_step (core/src/object/file_identifier/mod.rs:107-134).
 *
 * Conventions:
 *   - plain pointers and sizes only; the caller owns every buffer; nothing is retained
 *     after a call returns (batches are explicit objects the caller destroys);
 *   - every entry point is thread-safe and re-entrant: a context hands each call its own
 *     stream and scratch from an internal pool; no C++ exception crosses the ABI (the
 *     analogue of the reference FFI's panic::catch_unwind fence,
 *     apps/mobile/modules/sd-core/ios/crate/src/lib.rs:36-86);
 *   - return value: SD_OK (0) or a negative sd_rc for the whole call; per-file outcomes go
 *     to an int32 status array (sd_file_status);
 *   - `stream` arguments are hipStream_t passed as void*; NULL is HIP's null (default)
 *     stream, as everywhere in HIP.  Device-pointer entry points only enqueue work on it
 *     and do not synchronise (the dedup calls return host counts and so do sync it);
 *   - the GPU entry points need a gfx950 device (sd_cas_ctx_create fails with SD_ERR_DEVICE
 *     otherwise); the sd_cpu_* entry points are the library's CPU path:
 *     the same results from the host cores, for a node without the device and for the
 *     latency path's single-file callers.  No GPU entry point falls back to them silently;
 *     sd_cas_id_path / sd_file_checksum_path route a call to the CPU by a documented,
 *     tunable policy ("latency_cpu_max") and count it in sd_coalescer_stats.
 *
 * File-read semantics (the reference's, whatever the file's length): a whole-kind cas
 * message is le64(size) || every byte fs::read returns (cas.rs:25,29) -- the file may be
 * shorter or longer than `size`; a sampled message reads head and samples with read_exact
 * at their traced offsets and the tail at seek(End(-8192)), the file's real end (cas.rs:
 * 31-58); a checksum hashes what 1 MiB read calls return until one returns fewer
 * (hash.rs:14-20).
 */
#ifndef SD_CAS_H
#define SD_CAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SD_CAS_ABI_VERSION 2

/* cas.rs:10-15 */
#define SD_SAMPLE_COUNT 4u
#define SD_SAMPLE_SIZE 10240u
#define SD_HEADER_OR_FOOTER_SIZE 8192u
#define SD_MINIMUM_FILE_SIZE 102400u
/* le64 header + head + 4 samples + tail */
#define SD_SAMPLED_MSG_LEN 57352u
/* sd_cas_stage_plan starts staged messages on this alignment (one 128-byte cache line, so
 * a lane's 2 KiB chunk pair is whole lines) and zero-pads them up to it.  The kernels need
 * only 16-byte aligned offsets (sd_extent.msg_offset) and zero padding to a 64-byte boundary. */
#define SD_STAGE_ALIGN 128u

typedef enum sd_rc {
    SD_OK = 0,
    SD_ERR_INVALID = -1,  /* bad argument (null pointer, misaligned extent, ...) */
    SD_ERR_DEVICE = -2,   /* HIP / device error, or no gfx950 device */
    SD_ERR_NOMEM = -3,    /* device or pinned-host allocation failed */
    SD_ERR_INTERNAL = -4, /* unexpected exception caught at the boundary, or a HIP call
                             attempted on a private-fd-table worker thread */
    SD_ERR_COMM = -5,     /* collective (RCCL) failure */
    SD_ERR_CAPACITY = -6  /* sd_cas_dedup_mgpu: some rank's output capacity is too small (every
                             rank returns it, before the exchange; *m_out = own requirement) */
} sd_rc;

/* per-file status, mapped back to io::ErrorKind by the Rust shim */
typedef enum sd_file_status {
    SD_FILE_OK = 0,
    SD_FILE_SKIPPED_EMPTY = 1, /* FileMetadata::new skips len 0 (file_identifier/mod.rs:80-88) */
    SD_FILE_IO_ERROR = 2,      /* open/read failed: errno in the high 16 bits */
    SD_FILE_SHORT_READ = 3,    /* read_exact hit EOF: io::ErrorKind::UnexpectedEof (cas.rs:36,43,56) */
    SD_FILE_CHANGED = 4        /* staging only (sd_cas_stage_file/_files): the whole-kind file holds
                                  more bytes than its extent's room (it grew since the caller's
                                  stat); the reference hashes them all -- re-stage it with a larger
                                  extent, or use sd_cas_ids_files / sd_cas_id_path, which do */
} sd_file_status;

typedef enum sd_kind {
    SD_KIND_WHOLE = 1,  /* size <= 102400: le64(size) || whole file          (cas.rs:27-29) */
    SD_KIND_SAMPLED = 2 /* size  > 102400: le64(size) || head || 4 samples || tail (cas.rs:30-58) */
} sd_kind;

/* One file of a cas batch: where its hashed message sits in the staged buffer. 24 bytes. */
typedef struct sd_extent {
    uint64_t size;       /* file size as passed to generate_cas_id (hashed as le64)  */
    uint64_t msg_offset; /* byte offset of the message in the staged buffer (16-B aligned) */
    uint32_t msg_len;    /* SAMPLED: 57352; WHOLE: 8 + the bytes staged (planned 8 + size) */
    uint32_t kind;       /* sd_kind                                                  */
} sd_extent;

typedef struct sd_cas_ctx sd_cas_ctx;
typedef struct sd_cas_batch sd_cas_batch;
typedef struct sd_checksum_batch sd_checksum_batch;

/* ---------------------------------------------------------------- context */
int sd_cas_abi_version(void);
/* The host thread budget: the most host threads one call of this
 * process starts -- readers, CPU-path workers and co-hashing threads alike.  Resolved once
 * as min(affinity share, quota share), at least 1: the CPUs in the affinity mask, divided by
 * LOCAL_WORLD_SIZE (the ranks sharing the node's host; 1 when unset) only when the mask holds
 * every CPU of its scope -- the online CPUs, or the cgroup cpuset when that is smaller (a
 * narrower mask is a per-rank binding); and the tightest cgroup CPU quota
 * from the process's cgroup up, rounded up, divided by LOCAL_WORLD_SIZE.  The tuning key
 * "host_cpu_budget" > 0 replaces it.  out[5]: [0] the budget, [1] affinity CPUs, [2] cgroup
 * quota in milli-CPUs (0 = none), [3] LOCAL_WORLD_SIZE, [4] 1 if the tuning key set it. */
int sd_host_cpu_budget(int out[5]);
/* Where the library's own threads run: out[0] = 1 when they are placed on the CPUs of the
 * NUMA node of the first context's device (within each thread's own affinity mask; tuning
 * "numa_pin", default 0 = not placed), out[1] = those CPUs, out[2] = the device's node (-1
 * unknown).  Callers' threads are never moved; with "numa_pin" 0 no thread is. */
int sd_host_numa(int out[3]);
/* last error message of the calling thread ("" if none) */
const char* sd_cas_last_error(void);
int sd_cas_ctx_create(int device, sd_cas_ctx** out);
void sd_cas_ctx_destroy(sd_cas_ctx* ctx);
/* pinned host staging memory (fastest H2D); free with sd_cas_host_free */
int sd_cas_host_alloc(sd_cas_ctx* ctx, uint64_t bytes, void** out);
void sd_cas_host_free(sd_cas_ctx* ctx, void* p);

/* ---------------------------------------------------------------- staging (host) */
/* Layout of the cas messages of n files (cas.rs:25-58): fills extents_out[n] and the
 * staged-buffer size.  Pure host arithmetic; no device needed. */
int sd_cas_stage_plan(const uint64_t* sizes, size_t n, sd_extent* extents_out,
                      uint64_t* total_bytes_out);
/* Shards a library of n files (by global index, as the multi-GPU scan does) over nranks
 * ranks in contiguous index ranges of balanced hashing cost: the cost
 * of a file is the BLAKE3 compressions of its cas message (953 for every sampled file,
 * 1..146 for a small one).  bounds_out[nranks + 1]: rank r hashes [bounds[r], bounds[r+1]),
 * bounds ascending (sd_cas_dedup_mgpu's index-ordered fast path).  Pure host arithmetic. */
int sd_shard_plan(const uint64_t* sizes, size_t n, int nranks, uint64_t* bounds_out);
/* Reads one file into its extent exactly as generate_cas_id does (le64 header, then the
 * whole file until EOF, or head/samples by read_exact and the tail at the file's real end),
 * zero-padding to the next 64-byte boundary.  The extent is in/out: for a whole-kind file
 * msg_len becomes 8 + the bytes read, which may be fewer than planned (the file is shorter
 * than `size`; room = the planned msg_len - 8).  Sets *status to an sd_file_status
 * (SD_FILE_CHANGED when the file holds more than the room); returns SD_OK unless
 * arguments are invalid. */
int sd_cas_stage_file(const char* path, sd_extent* ext, uint8_t* staged, int32_t* status);
/* The same for n files on nthreads threads (the reference does these reads one tokio
 * blocking-pool hop at a time: cas.rs:29-58).  status[n] receives each file's outcome. */
int sd_cas_stage_files(const char* const* paths, sd_extent* extents, size_t n, uint8_t* staged,
                       int32_t* status, int nthreads);

/* ---------------------------------------------------------------- cas ids */
/* Drop-in batch: staged messages in host memory (pinned or pageable) -> n cas_ids as
 * 16 lowercase hex chars + NUL (cas.rs:61), 17 bytes per file.  status may be NULL;
 * entries whose status[i] != SD_FILE_OK on input are skipped and left untouched.  Whole-
 * kind messages of any length are accepted (longer than 8 + 102400 B: hashed by the
 * chunk-parallel checksum kernels).  A call of >= 8192 files is PCIe-bound, and feeding
 * the GPU costs the host only DMA, so "host_cohash_threads" (default 15; 0 = GPU only)
 * host threads hash files from the end of the list on the library's CPU path meanwhile,
 * the GPU taking windows from the front until the two meet; sd_cas_ids_stats counts the
 * files each side hashed. */
int sd_cas_ids_stats(sd_cas_ctx* ctx, uint64_t out[2]); /* files hashed: [0] GPU, [1] host threads */
int sd_cas_ids(sd_cas_ctx* ctx, const uint8_t* staged, uint64_t staged_bytes,
               const sd_extent* extents, size_t n, char* out_hex17, int32_t* status);

/* Path-based drop-in batch (SURVEY.md §8(b)'s "library does pread" entry): n (path,
 * size) pairs -> cas_ids, sizes as the caller's metadata reported them (the size is
 * hashed as given, cas.rs:25).  The library plans the messages, preads them on a
 * persistent pool of nthreads stager threads into pinned windows ("files_window_mb",
 * default 32), and overlaps staging window k+1 with window k's H2D copy and kernels.
 * status[n] (required) receives each file's sd_file_status.  Batch-size policy: a call of
 * at most "batch_cpu_max" files (default 4096; 0 = never) is hashed by
 * sd_cpu_cas_ids_files on nthreads host threads instead, which returns the same ids sooner
 * for an identifier step (100 files: ~0.1 ms vs ~0.3 ms from the page cache). */
int sd_cas_ids_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n,
                     char* out_hex17, int32_t* status, int nthreads);
/* Calls of sd_cas_ids_files on this context so far: out[0] on the CPU path (batch-size
 * policy), out[1] through the GPU. */
int sd_cas_ids_files_stats(sd_cas_ctx* ctx, uint64_t out[2]);
/* The same, with the full 32-byte hashes left in device memory for a multi-GPU library
 * scan (sd_cas_dedup_mgpu takes them as they are): d_hash32 (device, n x 32 bytes) row i =
 * file i's hash when status[i] == SD_FILE_OK (other rows untouched); d_valid (device, n
 * bytes, may be NULL) = 1 for the files the identifier dedups -- hashed and not empty
 * (file_identifier/mod.rs:80-88).  Returns when the rows are written. */
int sd_cas_hashes_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n,
                        uint8_t* d_hash32, uint8_t* d_valid, int32_t* status, int nthreads);

/* Prepared batch for device-resident data: builds the work lists for these extents once
 * (host arithmetic + one upload).  extents are host pointers. */
int sd_cas_batch_create(sd_cas_ctx* ctx, const sd_extent* extents, size_t n, sd_cas_batch** out);
void sd_cas_batch_destroy(sd_cas_batch* batch);
/* Enqueue the hashing of a prepared batch: d_staged (device, >= staged size) ->
 * d_hash32 (device, n x 32 bytes: the full BLAKE3 hash; the cas_id is its first 8).
 * The batch holds the device scratch its kernels pass between them (subtree chaining
 * values), so runs of ONE batch must be ordered: the same stream, or an event between
 * streams.  Its sampled and whole parts use separate scratch and may overlap each other
 * (run_part on two streams).  Separate batches are independent. */
int sd_cas_batch_run(sd_cas_ctx* ctx, const sd_cas_batch* batch, const uint8_t* d_staged,
                     uint8_t* d_hash32, void* stream);
/* Same, restricted to one part of the batch (bitmask): SD_PART_SAMPLED runs only the
 * sampled-file kernels, SD_PART_WHOLE only the whole-file kernels (lets a caller time
 * each part with events on `stream`). */
#define SD_PART_SAMPLED 1
#define SD_PART_WHOLE 2
int sd_cas_batch_run_part(sd_cas_ctx* ctx, const sd_cas_batch* batch, int parts, const uint8_t* d_staged,
                          uint8_t* d_hash32, void* stream);
/* Statistics of a prepared batch: [0] files, [1] sampled files, [2] whole files,
 * [3] chunks of whole files, [4] BLAKE3 compressions, [5] message bytes, [6] full-pair
 * and [7] tail work items of the whole-file kernel (its launch shape). */
int sd_cas_batch_stats(const sd_cas_batch* batch, uint64_t out[8]);

/* ---------------------------------------------------------------- checksums */
/* Full-file BLAKE3 (hash.rs:10-24) of n files that are byte ranges of one device
 * buffer.  offsets/lens are HOST arrays; each range must start 16-byte aligned and the
 * buffer must be readable up to the next 64-byte boundary after each range.  Start ranges
 * on SD_STAGE_ALIGN (128 B, a whole cache line) for full speed: a range that starts mid-line
 * hashes about 5% slower (every line-pair load straddles two lines; scripts/ck_align_probe.py). */
int sd_checksum_batch_create(sd_cas_ctx* ctx, const uint64_t* offsets, const uint64_t* lens,
                             size_t n, sd_checksum_batch** out);
void sd_checksum_batch_destroy(sd_checksum_batch* batch);
int sd_checksum_batch_run(sd_cas_ctx* ctx, const sd_checksum_batch* batch, const uint8_t* d_data,
                          uint8_t* d_hash32, void* stream);
/* [0] files, [1] total bytes, [2] BLAKE3 compressions, [3] 1 MiB leaf blocks */
int sd_checksum_batch_stats(const sd_checksum_batch* batch, uint64_t out[4]);
/* Drop-in over host memory (pinned or pageable; hash.rs:10-24 on data already read):
 * full BLAKE3 of n byte ranges of `data` -> 65-byte hex each.  Ranges start 16-byte
 * aligned (ranges of 1 MiB or more are placed on 128-B device lines whatever their host
 * start); no page that holds no range byte is read (a range may end where `data` ends, and
 * `data` may have unmapped holes between ranges; bytes between two ranges on a page they
 * share may be copied).  Consecutive ranges are copied 256 MiB window at a time, larger
 * ranges stream; two windows alternate so the H2D copies overlap the kernels.  In calls of
 * >= 1 GiB, "host_cohash_threads" host threads (default 15; 0 = GPU only) hash ranges from
 * the end on the CPU path meanwhile (ranges of >= 8 MiB block-parallel), the GPU taking
 * them from the front until the two meet; one range of >= 256 MiB, the one nearest the
 * predicted meeting point, is shared 1 MiB block by block.  Such a call
 * ("checksum_split_adapt" k > 0, default 8) runs co-hashed or on the CPU path alone
 * (sd_cpu_checksums on the host budget's threads), whichever this context has measured
 * faster: each once (a warm-up call, then a counted one), then the faster by an EWMA of
 * its GB/s, the other every k-th call; results are identical either way (round 6). */
int sd_checksums(sd_cas_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, size_t n,
                 char* out_hex65);
/* bytes sd_checksums hashed so far on this context: [0] by the GPU, [1] by host threads --
 * the co-hashing threads, and every byte of a call the learned route sent to the CPU path
 * (their share of a call: the host_share of the bench's with-H2D rows) */
int sd_checksums_stats(sd_cas_ctx* ctx, uint64_t out[2]);
/* what the context learned for sd_checksums' co-hash-eligible calls: [0] the co-hashed
 * call's GB/s, [1] the CPU path's, [2] / [3] how many calls each was counted for */
int sd_checksums_learned(sd_cas_ctx* ctx, double out[4]);
/* Drop-in: checksums of n files on disk -> 65-byte lowercase hex each (hash.rs:21-23);
 * status[n] required.  Each file is read as hash.rs reads it: 1 MiB read calls until a
 * short one -- for a regular file its bytes up to EOF, read with parallel preads
 * ("read_threads"); a pipe or device sequentially.  Small files are packed many per
 * pinned window, large ones (or ones that grow while read) streamed window by window,
 * whatever their final length; two windows alternate so host reads overlap the H2D
 * copies and the kernels (the readers stream each piece through a cache-resident buffer into
 * the pinned window, "checksum_stage_hot" 1).  Batch policy: with "checksum_hybrid_threads"
 * g > 0 (default 6), a call whose regular files of >= 8 MiB add up to >= 512 MiB is split
 * between the GPU and the CPU path on the 16 "read_threads" at once, claimed by 1 MiB blocks
 * ("checksum_split_blocks" 1): a thread that finds one of g GPU slots free reads a run of up
 * to 32 blocks of a file into it (fewer slots under a smaller host budget); otherwise it
 * hashes the small files, then single blocks, on the CPU path; each file's root is merged
 * from both sides' block CVs -- from the page cache 1.13-1.43x the CPU path alone
 * (round 4's whole-file claims, "checksum_split_blocks" 0: 0.9-1.24x).  On a
 * host whose threads hash fast the split can lose to them (0.93x on one box), so by default
 * ("checksum_split_adapt" 8) such a call takes the split or the CPU path alone by the context's
 * recent GB/s of each: each route once, then the faster, the other every 8th call (the
 * routes give identical results).  Any other call of at most "checksum_cpu_max" files is
 * hashed by sd_cpu_file_checksums on "read_threads" threads -- by default every such call,
 * because from the page cache the host's threads hash faster than PCIe can carry the bytes
 * to the GPU; "checksum_cpu_max" 0 = the GPU route alone for every call. */
int sd_file_checksums_stats(sd_cas_ctx* ctx, uint64_t out[2]);  /* calls: [0] CPU path, [1] GPU */
int sd_file_checksums_routes(sd_cas_ctx* ctx, uint64_t out[3]); /* [0] CPU path, [1] GPU, [2] split */
/* bytes (stat lengths) of the files [0] the GPU route hashed (GPU-only and split calls) and
 * [1] the CPU path hashed inside split calls: the split's share on this host */
int sd_file_checksums_bytes(sd_cas_ctx* ctx, uint64_t out[2]);
/* what the context learned for the calls the split applies to ("checksum_split_adapt"):
 * [0] the split's GB/s, [1] the CPU path's (EWMAs of counted calls), [2] / [3] how many
 * calls each was counted for (each route's first call is a warm-up and not counted) */
int sd_file_checksums_learned(sd_cas_ctx* ctx, double out[4]);
int sd_file_checksums(sd_cas_ctx* ctx, const char* const* paths, size_t n, char* out_hex65,
                      int32_t* status);

/* ---------------------------------------------------------------- latency path */
/* Single-file generate_cas_id (cas.rs:23) / file_checksum (hash.rs:10) for the
 * reference's per-file callers -- the location watcher (core/src/location/manager/
 * watcher/utils.rs:235,393,438-446) and non_indexed::walk (core/src/location/
 * non_indexed.rs:164-187).  Blocking and thread-safe.  Policy: while fewer than
 * "latency_cpu_max" (default 16; 0 = never) single-file calls are in flight on the
 * context, a call is hashed on the calling thread by the CPU path -- one GPU round trip
 * per file costs more than hashing it; beyond that, concurrent calls are coalesced by a
 * dispatcher thread into one batch per window (tuning "coalesce_window_us", default 200,
 * or "coalesce_max" requests, default 4096), handed to sd_cas_ids_files /
 * sd_file_checksums -- whose batch policies route it ("batch_cpu_max",
 * "checksum_cpu_max": with the defaults a coalesced batch is hashed on the CPU path by
 * the dispatcher's 16 threads; with them at 0, on the GPU).  Return SD_OK with *status =
 * sd_file_status (the hex is written only for SD_FILE_OK). */
int sd_cas_id_path(sd_cas_ctx* ctx, const char* path, uint64_t size, char* out_hex17, int32_t* status);
int sd_file_checksum_path(sd_cas_ctx* ctx, const char* path, char* out_hex65, int32_t* status);
/* [0] single-file requests, [1] batches they were coalesced into (each routed by the batch
 * policies), [2] largest batch, [3] requests hashed on their caller's thread (CPU path) */
int sd_coalescer_stats(sd_cas_ctx* ctx, uint64_t out[4]);

/* ---------------------------------------------------------------- CPU path (no device) */
/* The library's own host BLAKE3 (AVX-512 16-lane / AVX2 8-lane / SSE2 4-lane chunk
 * hashing, picked at run time) with the same file-read semantics as the GPU path.  No
 * context needed; nthreads host threads (the caller's included). */
int sd_cpu_simd_lanes(void);
/* sd_cas_ids on the host: staged messages -> 17-byte hex cas_ids (status as sd_cas_ids) */
int sd_cpu_cas_ids(const uint8_t* staged, uint64_t staged_bytes, const sd_extent* extents, size_t n,
                   char* out_hex17, int32_t* status, int nthreads);
/* sd_cas_ids_files on the host: (path, size) pairs -> cas_ids; status[n] required */
int sd_cpu_cas_ids_files(const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17,
                         int32_t* status, int nthreads);
/* full BLAKE3 of n byte ranges of one host buffer -> 32 raw bytes each (the 1 MiB blocks
 * of a range of >= 8 MiB are tasks of their own when nthreads > 1) */
int sd_cpu_checksums(const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, size_t n,
                     uint8_t* out_hash32, int nthreads);
/* sd_file_checksums on the host: paths -> 65-byte hex; status[n] required */
int sd_cpu_file_checksums(const char* const* paths, size_t n, char* out_hex65, int32_t* status, int nthreads);
/* one file on the calling thread (the latency path's CPU route) */
int sd_cpu_cas_id_path(const char* path, uint64_t size, char* out_hex17, int32_t* status);
int sd_cpu_file_checksum_path(const char* path, char* out_hex65, int32_t* status);

/* ---------------------------------------------------------------- dedup (post-hash) */
/* Bucket records (cas_id as big-endian u64 of the first 8 hash bytes, global file
 * index) by the top bits of the cas_id for an all-to-all over nparts ranks.
 * d_hash32: n x 32 bytes on device; d_valid: n bytes (0 = skip, e.g. empty files;
 * may be NULL).  Writes d_counts[nparts] (u64) and d_records[n] (2 x u64 each,
 * grouped by destination, stable within a destination).  Returns the number of valid
 * records in *n_valid (host). */
int sd_dedup_partition(sd_cas_ctx* ctx, const uint8_t* d_hash32, const uint8_t* d_valid,
                       uint64_t n, uint64_t global_index_base, int nparts, uint64_t* d_counts,
                       uint64_t* d_records, uint64_t* n_valid, void* stream);
/* Group received records by cas_id: sorts d_records[m] (in place) by (cas_id, index) and
 * writes d_rep[m] (u64): for each record, the smallest global index with an equal
 * cas_id -- the Object-link candidate (file_identifier/mod.rs:168-225 semantics up to
 * the chunk-of-100 rule).  Returns the number of groups.
 * flags: SD_DEDUP_INDEX_SORTED promises the records are already in ascending index
 * order -- true for sd_dedup_partition's output after an all-to-all in rank order over
 * contiguous index shards -- and saves one radix sort. */
#define SD_DEDUP_INDEX_SORTED 1
int sd_dedup_group(sd_cas_ctx* ctx, uint64_t* d_records, uint64_t m, int flags, uint64_t* d_rep,
                   uint64_t* n_groups, void* stream);
/* Object owner per grouped record (d_records / d_rep as sd_dedup_group leaves them), the
 * reference's link-or-create rule for identifier steps of `chunk_size` files
 * (file_identifier/mod.rs:36,136-333): d_owner[i] = index if index / chunk_size ==
 * rep / chunk_size (the group's first step creates an Object per file), else rep (a later
 * step links to it).  Asynchronous on `stream`; no host sync. */
int sd_dedup_owners(sd_cas_ctx* ctx, const uint64_t* d_records, uint64_t m, const uint64_t* d_rep,
                    uint64_t chunk_size, uint64_t* d_owner, void* stream);

/* ---------------------------------------------------------------- multi-GPU dedup (RCCL) */
/* One process (or thread) per GPU, files sharded by global index.  The
 * communicator is RCCL's: rank 0 calls sd_comm_id (ncclGetUniqueId) and hands the 128
 * bytes to every rank out of band; each rank calls sd_comm_create (ncclCommInitRank,
 * collective) on its context's device. */
#define SD_COMM_ID_BYTES 128
typedef struct sd_comm sd_comm;
int sd_comm_id(uint8_t* out_id /* SD_COMM_ID_BYTES */);
int sd_comm_create(sd_cas_ctx* ctx, const uint8_t* id, int nranks, int rank, sd_comm** out);
void sd_comm_destroy(sd_comm* comm);
/* In-process communicator: the ranks are threads of ONE process (each with its own context,
 * on one device or several) that share an sd_comm_group.  Every collective below has the
 * same semantics over it; the exchange is device-to-device copies between the ranks'
 * buffers, ordered by a host barrier (a rank whose thread never arrives makes its peers
 * return SD_ERR_COMM after 120 s).  For a host that drives several GPUs from one process,
 * and for rehearsing N ranks on one GPU, which RCCL refuses.  Destroy every member comm
 * before the group. */
typedef struct sd_comm_group sd_comm_group;
int sd_comm_group_create(int nranks, sd_comm_group** out);
void sd_comm_group_destroy(sd_comm_group* group);
int sd_comm_create_local(sd_cas_ctx* ctx, sd_comm_group* group, int rank, sd_comm** out);
/* The whole post-hash step of one rank, collective over the communicator: partition its n
 * records by cas_id prefix (sd_dedup_partition), all-gather the count matrix and the
 * shards' index ranges (ncclAllGather), exchange the 16-byte records with grouped
 * ncclSend / ncclRecv -- the all-to-all over xGMI --, then group the records this rank
 * receives (sd_dedup_group; index order is exploited when the shards' ranges ascend with
 * the rank) and assign their Objects (sd_dedup_owners, identifier steps of chunk_size).
 * Outputs hold `capacity` entries: d_records_out 2 x u64 each (sorted by (cas_id,
 * index)), d_rep_out and d_owner_out u64 each; *m_out = the records this rank owns,
 * *n_groups_out = its groups.  If any rank's capacity is too small, every rank returns
 * SD_ERR_CAPACITY before the record exchange, with *m_out = its own requirement (and
 * SD_ERR_INTERNAL together if any rank's partition counts disagree with its valid records:
 * the gathered rows carry both, so no rank is left waiting in the exchange).  Runs on
 * `stream`; returns after the group counts are known (host sync).  Over RCCL, each wait for
 * the peers is bounded by the tuning key "comm_timeout_ms" (300 000; 0 = unbounded): a peer
 * that died or hung, or an RCCL asynchronous error, makes the call return SD_ERR_COMM naming
 * the step, and the communicator is broken from then on -- later calls on it return
 * SD_ERR_COMM, and sd_comm_destroy releases nothing of it (work may still be queued against
 * it; the host is expected to exit).  Overlapping it with the
 * next batch's hashing (a second stream) pays only with the hashing stream at the higher
 * priority (107.5 vs 103.9-104.3 M files/s with equal priorities). */
int sd_cas_dedup_mgpu(sd_cas_ctx* ctx, sd_comm* comm, const uint8_t* d_hash32, const uint8_t* d_valid, uint64_t n,
                      uint64_t global_index_base, uint64_t chunk_size, uint64_t* d_records_out, uint64_t* d_rep_out,
                      uint64_t* d_owner_out, uint64_t capacity, uint64_t* m_out, uint64_t* n_groups_out,
                      void* stream);
/* Phase timing of sd_cas_dedup_mgpu (diagnostics): with timing on, each call records HIP
 * events on its stream at the phase boundaries; sd_comm_last_phases waits for the last
 * call's events and returns the SD_DEDUP_PHASES durations in ms, in order:
 *   [0] partition (kernels), [1] all-gather of the rows + their copy to the host,
 *   [2] host turnaround: the stream idles from the rows' arrival until the host, having read
 *       them, has queued the exchange (the call's one mid-call sync),
 *   [3] grouped ncclSend / ncclRecv of the records, [4] group + Object owners. */
#define SD_DEDUP_PHASES 5
/* The RCCL that serves sd_comm in this process: *version = ncclGetVersion's code (e.g.
 * 22606 = 2.26.6) and path_out = the shared object its symbols were bound to (librccl.so.1
 * is one soname: a host that loaded another RCCL first -- torch's ProcessGroupNCCL -- has
 * libsdcas's communicators served by that one).  path_out may be NULL. */
int sd_comm_rccl_info(int* version, char* path_out, size_t path_cap);
int sd_comm_set_timing(sd_comm* comm, int on);
int sd_comm_last_phases(sd_comm* comm, float* ms_out /* SD_DEDUP_PHASES */);

/* ---------------------------------------------------------------- one file over many GPUs */
/* file_checksum (hash.rs:10-24) of ONE file whose bytes are spread over the ranks of a
 * communicator (a file's 1 MiB blocks shard naturally).  The file's
 * total_len bytes are cut into nb = max(1, ceil(total_len / 1 MiB)) blocks; rank r of R
 * holds blocks [r*q, min((r+1)*q, nb)) with q = ceil(nb / R) -- sd_split_range gives its
 * byte range [offset, offset + len) and the CV buffer size, R * q * 32 bytes.  Each rank
 * hashes its blocks to their 32-byte chaining values at block index b of the CV buffer
 * (a block's CV depends only on its bytes and its position, not on the total); the
 * buffers of all ranks laid end to end in rank order are the file's block CVs in order,
 * and one reduce gives the BLAKE3 of the whole file, bit-identical to file_checksum's.
 * A file of one block (total_len <= 1 MiB) is held by rank 0, whose "CV" slot 0 then
 * holds the root hash itself.  GPU-free. */
int sd_split_range(uint64_t total_len, int nranks, int rank, uint64_t* offset, uint64_t* len,
                   uint64_t* cv_bytes);
typedef struct sd_split_checksum sd_split_checksum;
int sd_split_checksum_create(sd_cas_ctx* ctx, uint64_t total_len, int nranks, int rank,
                             sd_split_checksum** out);
void sd_split_checksum_destroy(sd_split_checksum* split);
/* This rank's blocks -> d_cvs (device, cv_bytes; only this rank's slots are written).
 * d_slice = the rank's `len` bytes (device, 16-byte aligned, zero-padded to the next
 * 64-byte boundary).  Asynchronous on `stream`. */
int sd_split_checksum_leaves(sd_cas_ctx* ctx, const sd_split_checksum* split, const uint8_t* d_slice,
                             uint8_t* d_cvs, void* stream);
/* All ranks' CVs (device, every slot filled) -> the 32-byte file hash (device).
 * Asynchronous on `stream`; one call at a time per split object. */
int sd_split_checksum_root(sd_cas_ctx* ctx, sd_split_checksum* split, const uint8_t* d_cvs,
                           uint8_t* d_hash32, void* stream);
/* Collective over the communicator (nranks / rank must match the split's): leaves, an
 * in-place ncclAllGather of the CV slots (32 B per MiB of file: 1 MB per 32 GiB), root.
 * Every rank gets the hash.  Asynchronous on `stream`. */
int sd_split_checksum_mgpu(sd_cas_ctx* ctx, sd_comm* comm, sd_split_checksum* split, const uint8_t* d_slice,
                           uint8_t* d_cvs, uint8_t* d_hash32, void* stream);
/* The same two steps on host cores (host pointers). */
int sd_cpu_split_leaves(const uint8_t* slice, uint64_t total_len, int nranks, int rank, uint8_t* cvs,
                        int nthreads);
int sd_cpu_split_root(const uint8_t* cvs, uint64_t total_len, uint8_t* out_hash32);

/* ---------------------------------------------------------------- synthetic data */
/* Device generator of SURVEY.md §8(d) (seed 0x5D5DCA51D, splitmix64 counter stream),
 * for benchmarks and parity tests: writes the exact cas message of each synthetic file
 * (content id cids[i], twin tag twins[i]) into its extent.  All arrays device. */
int sd_synth_stage_cas(sd_cas_ctx* ctx, const uint64_t* d_sizes, const uint64_t* d_cids,
                       const uint32_t* d_twins, const sd_extent* d_extents, size_t n,
                       uint8_t* d_staged, void* stream);
/* bytes [0, len) of synthetic content (cid, twin) -> d_out (device) */
int sd_synth_fill(sd_cas_ctx* ctx, uint64_t cid, uint32_t twin, uint64_t len, uint8_t* d_out,
                  void* stream);
/* bytes [offset, offset + len) of the same content -> d_out (offset and d_out 8-aligned) */
int sd_synth_fill_at(sd_cas_ctx* ctx, uint64_t cid, uint32_t twin, uint64_t offset, uint64_t len,
                     uint8_t* d_out, void* stream);

/* ---------------------------------------------------------------- device utilities */
int sd_device_malloc(sd_cas_ctx* ctx, uint64_t bytes, void** out);
void sd_device_free(sd_cas_ctx* ctx, void* p);
int sd_memcpy(sd_cas_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream);
int sd_stream_sync(sd_cas_ctx* ctx, void* stream);
/* Time `iters` back-to-back runs of a prepared batch with HIP events on `stream`:
 * *ms_total = elapsed milliseconds (kernel time on that stream, no host sync inside). */
int sd_cas_batch_time(sd_cas_ctx* ctx, const sd_cas_batch* batch, const uint8_t* d_staged,
                      uint8_t* d_hash32, int iters, void* stream, float* ms_total);
int sd_checksum_batch_time(sd_cas_ctx* ctx, const sd_checksum_batch* batch, const uint8_t* d_data,
                           uint8_t* d_hash32, int iters, void* stream, float* ms_total);
/* Process-wide knobs (results are identical for every value): "coalesce_window_us"
 * (200), "coalesce_max" (4096) and "latency_cpu_max" (16) of the latency path;
 * "files_window_mb" (32) of sd_cas_ids_files; "read_threads" (16) of sd_file_checksums;
 * "dedup_variant" (sd_dedup_group) 0 =
 * rocPRIM radix sort, 1 = LDS buckets with the radix sort as overflow fallback (default);
 * "sampled_wave_max" (6144) / "whole_wave_max" (512): a cas batch with at most that many
 * sampled / whole-kind files takes the latency kernels (one wave or workgroup per file),
 * a larger one the throughput kernels -- read when the batch is planned; "batch_cpu_max"
 * (4096): sd_cas_ids_files calls of at most that many files take the CPU path;
 * "files_ring" (4): pinned window buffers sd_cas_ids_files' readers may fill ahead of the
 * copies; "files_stage_hot" (1): its readers read each file into a per-thread buffer and
 * stream-copy it into the window (0 = read straight into the window); "checksum_cpu_max" (2147483647): sd_file_checksums calls of at most that many
 * files take the CPU path (sd_cpu_file_checksums on "read_threads" threads; 0 = the GPU
 * route always); "checksum_hybrid_threads" (6): GPU slots -- threads feeding the GPU at once
 * -- when sd_file_checksums splits a large call with the CPU path (0 = never split);
 * "checksum_stage_hot" (1): sd_file_checksums' GPU-route readers deliver through a
 * cache-resident buffer and streaming stores (0 = pread straight into the pinned window);
 * "cpu_read_piece_kib" (256): the CPU path reads and hashes each 1 MiB block of a large file
 * in pieces of this many KiB, each hashed while still in the core's L2 (0 = one 1 MiB read,
 * then the hash; 256 measured 1.04-1.07x, profiles/r5/r5d_hybrid.json);
 * "checksum_split_blocks" (1): sd_file_checksums' split claims work by 1 MiB blocks (the
 * GPU's "checksum_hybrid_threads" slots take runs of blocks while free, the host threads
 * single blocks); 0 = by whole files (round 4);
 * "checksum_split_adapt" (8): a call the split applies to takes the split or the CPU path
 * alone, learned per context from the GB/s of its past calls -- each once, then the faster,
 * the other every k-th call to keep its rate current; 0 = always the split;
 * "host_cohash_threads" (15): host threads hashing beside the GPU in sd_cas_ids calls of
 * >= 8192 files and sd_checksums calls of >= 1 GiB (0 = the GPU alone; never more than the
 * host budget less one in sd_cas_ids, less 3/16 of it (at least one) in sd_checksums -- 13
 * of 16 measured best there); "host_cpu_budget" (0 = resolved, see sd_host_cpu_budget): the cap
 * on every call's host threads -- thread counts callers pass (nthreads) and the knobs above
 * are clamped to it; "comm_timeout_ms" (300000): the longest sd_cas_dedup_mgpu waits for its
 * RCCL peers (0 = no bound).  Unknown keys fail with SD_ERR_INVALID. */
int sd_cas_set_tuning(const char* key, int value);
int sd_cas_get_tuning(const char* key, int* value);
/* Read-only probe over d_buf[0, bytes) (bytes a multiple of 4096) for calibrating the
 * PMC byte counters on this kernel family's access patterns: pattern 0 = coalesced
 * 16 B/lane streaming, pattern 1 = one lane per 1 KiB chunk reading 4 x 16 B per 64-byte
 * block (the hashing kernels' pattern), pattern 2 = pattern 1 with 2 chunks per lane,
 * pattern 3 = pattern 0 with its loads marked non-temporal. */
int sd_read_probe(sd_cas_ctx* ctx, const uint8_t* d_buf, uint64_t bytes, int pattern, void* stream);
/* VALU ceiling of the kernels' BLAKE3 G instruction mix (asm, registers only, 8 waves per SIMD):
 * measured lane-ops/s on this device. */
int sd_valu_peak(sd_cas_ctx* ctx, double* lane_ops_per_s);

#ifdef __cplusplus
}
#endif
#endif /* SD_CAS_H */
