//! Raw FFI mirror of `include/sd_cas.h` (ABI version 2) plus a small safe layer used by
//! `core/src/object/cas.rs`, `core/src/object/validation/hash.rs`, the batched identifier
//! step (`file_identifier_step.rs`) and the batched validator step (`validator_step.rs`).
//!
//! Conventions follow the reference's own FFI (`apps/mobile/modules/sd-core/ios/crate/
//! src/lib.rs:36-86`): plain pointers and sizes, no panics across the boundary.  Behind
//! the ABI, libsdcas catches every C++ exception and returns a negative `sd_rc`.
//!
//! Routing: with a gfx950 device, batches go to the GPU entry points and single files to
//! `sd_cas_id_path` / `sd_file_checksum_path` (the library's latency policy: CPU while few
//! calls are in flight, coalesced GPU batches beyond).  Without one, [`ctx`] returns an
//! error (it never panics) and every call takes the library's CPU path (`sd_cpu_*`): the
//! same results from the host cores.
#![allow(non_camel_case_types)]
use std::ffi::{CStr, CString};
use std::io;
use std::os::raw::{c_char, c_int, c_void};
use std::os::unix::ffi::OsStrExt;
use std::path::Path;
use std::sync::{Arc, OnceLock};

#[repr(C)]
pub struct sd_cas_ctx {
    _p: [u8; 0],
}

#[repr(C)]
pub struct sd_comm {
    _p: [u8; 0],
}
#[repr(C)]
pub struct sd_comm_group {
    _p: [u8; 0],
}

#[repr(C)]
pub struct sd_split_checksum {
    _p: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct sd_extent {
    pub size: u64,
    pub msg_offset: u64,
    pub msg_len: u32,
    pub kind: u32,
}

pub const SD_CAS_ABI_VERSION: c_int = 2;
pub const SD_OK: c_int = 0;
pub const SD_ERR_DEVICE: c_int = -2;
pub const SD_ERR_CAPACITY: c_int = -6;
pub const SD_FILE_OK: i32 = 0;
pub const SD_FILE_SKIPPED_EMPTY: i32 = 1;
pub const SD_FILE_IO_ERROR: i32 = 2;
pub const SD_FILE_SHORT_READ: i32 = 3;
pub const SD_FILE_CHANGED: i32 = 4;
pub const SD_COMM_ID_BYTES: usize = 128;

extern "C" {
    pub fn sd_cas_abi_version() -> c_int;
    pub fn sd_cas_last_error() -> *const c_char;
    // the host thread budget every call is capped by; "host_cpu_budget" sets it
    pub fn sd_host_cpu_budget(out: *mut c_int) -> c_int;
    // where the library's own threads run (the device's NUMA node; tuning "numa_pin")
    pub fn sd_host_numa(out: *mut c_int) -> c_int;
    pub fn sd_cas_set_tuning(key: *const c_char, value: c_int) -> c_int;
    pub fn sd_cas_ctx_create(device: c_int, out: *mut *mut sd_cas_ctx) -> c_int;
    pub fn sd_cas_ctx_destroy(ctx: *mut sd_cas_ctx);
    pub fn sd_cas_stage_plan(sizes: *const u64, n: usize, ext: *mut sd_extent, total: *mut u64) -> c_int;
    pub fn sd_cas_ids_files(ctx: *mut sd_cas_ctx, paths: *const *const c_char, sizes: *const u64, n: usize,
                            out_hex17: *mut c_char, status: *mut i32, nthreads: c_int) -> c_int;
    pub fn sd_cas_hashes_files(ctx: *mut sd_cas_ctx, paths: *const *const c_char, sizes: *const u64, n: usize,
                               d_hash32: *mut u8, d_valid: *mut u8, status: *mut i32, nthreads: c_int) -> c_int;
    pub fn sd_cas_id_path(ctx: *mut sd_cas_ctx, path: *const c_char, size: u64, out_hex17: *mut c_char,
                          status: *mut i32) -> c_int;
    pub fn sd_file_checksums(ctx: *mut sd_cas_ctx, paths: *const *const c_char, n: usize,
                             out_hex65: *mut c_char, status: *mut i32) -> c_int;
    pub fn sd_file_checksum_path(ctx: *mut sd_cas_ctx, path: *const c_char, out_hex65: *mut c_char,
                                 status: *mut i32) -> c_int;
    pub fn sd_checksums(ctx: *mut sd_cas_ctx, data: *const u8, offsets: *const u64, lens: *const u64, n: usize,
                        out_hex65: *mut c_char) -> c_int;
    // the validator's split: bytes the GPU route and the CPU path hashed
    pub fn sd_file_checksums_bytes(ctx: *mut sd_cas_ctx, out: *mut u64) -> c_int;
    // what the context learned for the split vs the CPU path ("checksum_split_adapt")
    pub fn sd_file_checksums_learned(ctx: *mut sd_cas_ctx, out: *mut f64) -> c_int;
    // what the context learned for sd_checksums' co-hashed calls vs the CPU path alone
    pub fn sd_checksums_learned(ctx: *mut sd_cas_ctx, out: *mut f64) -> c_int;
    // the CPU path (no device)
    pub fn sd_cpu_simd_lanes() -> c_int;
    pub fn sd_cpu_cas_ids_files(paths: *const *const c_char, sizes: *const u64, n: usize, out_hex17: *mut c_char,
                                status: *mut i32, nthreads: c_int) -> c_int;
    pub fn sd_cpu_file_checksums(paths: *const *const c_char, n: usize, out_hex65: *mut c_char, status: *mut i32,
                                 nthreads: c_int) -> c_int;
    pub fn sd_cpu_cas_id_path(path: *const c_char, size: u64, out_hex17: *mut c_char, status: *mut i32) -> c_int;
    pub fn sd_cpu_file_checksum_path(path: *const c_char, out_hex65: *mut c_char, status: *mut i32) -> c_int;
    // multi-GPU dedup over RCCL (one process per GPU)
    pub fn sd_comm_id(out_id: *mut u8) -> c_int;
    pub fn sd_comm_create(ctx: *mut sd_cas_ctx, id: *const u8, nranks: c_int, rank: c_int,
                          out: *mut *mut sd_comm) -> c_int;
    pub fn sd_comm_destroy(comm: *mut sd_comm);
    pub fn sd_comm_rccl_info(version: *mut c_int, path_out: *mut c_char, path_cap: usize) -> c_int;
    // the same collectives with the ranks as threads of one process (several GPUs, one process)
    pub fn sd_comm_group_create(nranks: c_int, out: *mut *mut sd_comm_group) -> c_int;
    pub fn sd_comm_group_destroy(group: *mut sd_comm_group);
    pub fn sd_comm_create_local(ctx: *mut sd_cas_ctx, group: *mut sd_comm_group, rank: c_int,
                                out: *mut *mut sd_comm) -> c_int;
    pub fn sd_cas_dedup_mgpu(ctx: *mut sd_cas_ctx, comm: *mut sd_comm, d_hash32: *const u8, d_valid: *const u8,
                             n: u64, global_index_base: u64, chunk_size: u64, d_records_out: *mut u64,
                             d_rep_out: *mut u64, d_owner_out: *mut u64, capacity: u64, m_out: *mut u64,
                             n_groups_out: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_shard_plan(sizes: *const u64, n: usize, nranks: c_int, bounds_out: *mut u64) -> c_int;
    // one file's checksum over many GPUs (its 1 MiB blocks sharded by rank)
    pub fn sd_split_range(total_len: u64, nranks: c_int, rank: c_int, offset: *mut u64, len: *mut u64,
                          cv_bytes: *mut u64) -> c_int;
    pub fn sd_split_checksum_create(ctx: *mut sd_cas_ctx, total_len: u64, nranks: c_int, rank: c_int,
                                    out: *mut *mut sd_split_checksum) -> c_int;
    pub fn sd_split_checksum_destroy(split: *mut sd_split_checksum);
    pub fn sd_split_checksum_mgpu(ctx: *mut sd_cas_ctx, comm: *mut sd_comm, split: *mut sd_split_checksum,
                                  d_slice: *const u8, d_cvs: *mut u8, d_hash32: *mut u8, stream: *mut c_void) -> c_int;
    pub fn sd_cpu_split_leaves(slice: *const u8, total_len: u64, nranks: c_int, rank: c_int, cvs: *mut u8,
                               nthreads: c_int) -> c_int;
    pub fn sd_cpu_split_root(cvs: *const u8, total_len: u64, out_hash32: *mut u8) -> c_int;
}

/// One context per process on device 0 (the job system's 5 concurrent jobs, watcher and
/// non_indexed tasks all share it: every entry point is thread-safe).
pub struct Ctx(*mut sd_cas_ctx);
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

/// The process's GPU context, or the reason there is none (no gfx950 device, driver
/// error, ABI mismatch) -- callers then take the CPU path.  Never panics.
pub fn ctx() -> Result<&'static Ctx, io::Error> {
    static CTX: OnceLock<Result<Ctx, String>> = OnceLock::new();
    CTX.get_or_init(|| {
        let abi = unsafe { sd_cas_abi_version() };
        if abi != SD_CAS_ABI_VERSION {
            return Err(format!("libsdcas ABI {abi}, this binding expects {SD_CAS_ABI_VERSION}"));
        }
        let mut p = std::ptr::null_mut();
        match unsafe { sd_cas_ctx_create(0, &mut p) } {
            SD_OK => Ok(Ctx(p)),
            _ => Err(last_error()),
        }
    })
    .as_ref()
    .map_err(|e| io::Error::new(io::ErrorKind::Unsupported, e.clone()))
}

pub fn last_error() -> String {
    unsafe { CStr::from_ptr(sd_cas_last_error()) }.to_string_lossy().into_owned()
}

/// sd_file_status -> the io::Error the reference's reads would have produced.
pub fn status_to_io(st: i32) -> io::Error {
    match st & 0xFFFF {
        SD_FILE_SHORT_READ => io::ErrorKind::UnexpectedEof.into(), // read_exact (cas.rs:36,43,56)
        SD_FILE_IO_ERROR => io::Error::from_raw_os_error((st >> 16) & 0xFFFF),
        _ => io::Error::new(io::ErrorKind::Other, format!("sd_cas status {st}")),
    }
}

fn cpath(p: &Path) -> Result<CString, io::Error> {
    CString::new(p.as_os_str().as_bytes()).map_err(|e| io::Error::new(io::ErrorKind::InvalidInput, e))
}

fn hex_at(buf: &[c_char], i: usize, stride: usize, len: usize) -> String {
    buf[stride * i..stride * i + len].iter().map(|&b| b as u8 as char).collect()
}

fn per_file(rc: c_int, status: &[i32], hex: &[c_char], stride: usize, len: usize) -> Vec<Result<String, io::Error>> {
    (0..status.len())
        .map(|i| {
            if rc != SD_OK {
                Err(io::Error::new(io::ErrorKind::Other, last_error()))
            } else if status[i] != SD_FILE_OK {
                Err(status_to_io(status[i]))
            } else {
                Ok(hex_at(hex, i, stride, len))
            }
        })
        .collect()
}

/// Batched generate_cas_id (cas.rs:23-62): one result per (path, size), in order.  On the
/// GPU the library reads the windows on its stager pool and overlaps them with the
/// kernels; without a device, the CPU path on 16 host threads.
pub fn cas_ids_blocking(files: &[(&Path, u64)]) -> Vec<Result<String, io::Error>> {
    let n = files.len();
    let c: Vec<CString> = match files.iter().map(|f| cpath(f.0)).collect() {
        Ok(v) => v,
        Err(e) => return (0..n).map(|_| Err(io::Error::new(e.kind(), e.to_string()))).collect(),
    };
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let sizes: Vec<u64> = files.iter().map(|f| f.1).collect();
    let mut hex = vec![0 as c_char; 17 * n];
    let mut status = vec![0i32; n];
    let rc = unsafe {
        match ctx() {
            Ok(g) => sd_cas_ids_files(g.0, ptrs.as_ptr(), sizes.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr(), 16),
            Err(_) => sd_cpu_cas_ids_files(ptrs.as_ptr(), sizes.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr(), 16),
        }
    };
    per_file(rc, &status, &hex, 17, 16)
}

/// Single-file generate_cas_id for the latency callers (watcher, non_indexed).
pub fn cas_id_blocking(path: &Path, size: u64) -> Result<String, io::Error> {
    let c = cpath(path)?;
    let mut hex = [0 as c_char; 17];
    let mut st = 0i32;
    let rc = unsafe {
        match ctx() {
            Ok(g) => sd_cas_id_path(g.0, c.as_ptr(), size, hex.as_mut_ptr(), &mut st),
            Err(_) => sd_cpu_cas_id_path(c.as_ptr(), size, hex.as_mut_ptr(), &mut st),
        }
    };
    per_file(rc, &[st], &hex, 17, 16).pop().expect("one result")
}

/// Batched file_checksum (hash.rs:10-24).
pub fn checksums_blocking(paths: &[&Path]) -> Vec<Result<String, io::Error>> {
    let n = paths.len();
    let c: Vec<CString> = match paths.iter().map(|p| cpath(p)).collect() {
        Ok(v) => v,
        Err(e) => return (0..n).map(|_| Err(io::Error::new(e.kind(), e.to_string()))).collect(),
    };
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let mut hex = vec![0 as c_char; 65 * n];
    let mut status = vec![0i32; n];
    let rc = unsafe {
        match ctx() {
            Ok(g) => sd_file_checksums(g.0, ptrs.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr()),
            Err(_) => sd_cpu_file_checksums(ptrs.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr(), 16),
        }
    };
    per_file(rc, &status, &hex, 65, 64)
}

/// Single-file file_checksum (the watcher's recompute, watcher/utils.rs:438-446).
pub fn checksum_blocking(path: &Path) -> Result<String, io::Error> {
    let c = cpath(path)?;
    let mut hex = [0 as c_char; 65];
    let mut st = 0i32;
    let rc = unsafe {
        match ctx() {
            Ok(g) => sd_file_checksum_path(g.0, c.as_ptr(), hex.as_mut_ptr(), &mut st),
            Err(_) => sd_cpu_file_checksum_path(c.as_ptr(), hex.as_mut_ptr(), &mut st),
        }
    };
    per_file(rc, &[st], &hex, 65, 64).pop().expect("one result")
}

/// libsdcas's RCCL communicator for a multi-GPU library scan (one process per GPU).
/// A member of an in-process group holds a reference to the group, so the group is
/// destroyed only after its last member (sd_comm_destroy writes to the group).
pub struct Comm {
    raw: *mut sd_comm,
    _group: Option<Arc<GroupHandle>>,
}
unsafe impl Send for Comm {}

impl Comm {
    /// On rank 0: the 128-byte id every rank passes to [`Comm::join`] (out of band).
    pub fn unique_id() -> Result<[u8; SD_COMM_ID_BYTES], io::Error> {
        let mut id = [0u8; SD_COMM_ID_BYTES];
        match unsafe { sd_comm_id(id.as_mut_ptr()) } {
            SD_OK => Ok(id),
            _ => Err(io::Error::new(io::ErrorKind::Other, last_error())),
        }
    }
    /// Collective over all ranks (ncclCommInitRank on the context's device).
    pub fn join(id: &[u8; SD_COMM_ID_BYTES], nranks: i32, rank: i32) -> Result<Comm, io::Error> {
        let g = ctx()?;
        let mut p = std::ptr::null_mut();
        match unsafe { sd_comm_create(g.0, id.as_ptr(), nranks, rank, &mut p) } {
            SD_OK => Ok(Comm { raw: p, _group: None }),
            _ => Err(io::Error::new(io::ErrorKind::Other, last_error())),
        }
    }
    /// One rank of an in-process group: the ranks are threads of this process, each with its
    /// own context (`ctx`, e.g. one per device from sd_cas_ctx_create); every collective has
    /// the RCCL communicator's semantics.  The member keeps the group alive: dropping the
    /// `CommGroup` first only releases the caller's handle.
    pub fn join_local(group: &CommGroup, ctx: *mut sd_cas_ctx, rank: i32) -> Result<Comm, io::Error> {
        let mut p = std::ptr::null_mut();
        match unsafe { sd_comm_create_local(ctx, group.0.0, rank, &mut p) } {
            SD_OK => Ok(Comm { raw: p, _group: Some(Arc::clone(&group.0)) }),
            _ => Err(io::Error::new(io::ErrorKind::Other, last_error())),
        }
    }
    pub fn raw(&self) -> *mut sd_comm {
        self.raw
    }
}

impl Drop for Comm {
    fn drop(&mut self) {
        // the communicator first; then the field drops release the group reference
        unsafe { sd_comm_destroy(self.raw) }
    }
}

/// The owned sd_comm_group; destroyed when the group handle and every member are gone.
pub struct GroupHandle(*mut sd_comm_group);
unsafe impl Send for GroupHandle {}
unsafe impl Sync for GroupHandle {}

impl Drop for GroupHandle {
    fn drop(&mut self) {
        unsafe { sd_comm_group_destroy(self.0) }
    }
}

/// The rendezvous of an in-process group of `nranks` ranks (sd_comm_group_create).
pub struct CommGroup(Arc<GroupHandle>);

impl CommGroup {
    pub fn new(nranks: i32) -> Result<CommGroup, io::Error> {
        let mut p = std::ptr::null_mut();
        match unsafe { sd_comm_group_create(nranks, &mut p) } {
            SD_OK => Ok(CommGroup(Arc::new(GroupHandle(p)))),
            _ => Err(io::Error::new(io::ErrorKind::Other, last_error())),
        }
    }
}

