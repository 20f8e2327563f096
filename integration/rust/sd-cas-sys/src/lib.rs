//! Raw FFI mirror of `include/sd_cas.h` (ABI version 1) plus a small safe layer used by
//! `core/src/object/cas.rs` and `core/src/object/validation/hash.rs`.
//!
//! Conventions follow the reference's own FFI (`apps/mobile/modules/sd-core/ios/crate/
//! src/lib.rs:36-86`): plain pointers and sizes, no panics across the boundary.  Behind
//! the ABI, libsdcas catches every C++ exception and returns a negative `sd_rc`.
#![allow(non_camel_case_types)]
use std::ffi::{CStr, CString};
use std::io;
use std::os::raw::{c_char, c_int};
use std::os::unix::ffi::OsStrExt;
use std::path::Path;
use std::sync::OnceLock;

#[repr(C)]
pub struct sd_cas_ctx {
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

pub const SD_CAS_ABI_VERSION: c_int = 1;
pub const SD_OK: c_int = 0;
pub const SD_FILE_OK: i32 = 0;
pub const SD_FILE_SKIPPED_EMPTY: i32 = 1;
pub const SD_FILE_IO_ERROR: i32 = 2;
pub const SD_FILE_SHORT_READ: i32 = 3;

extern "C" {
    pub fn sd_cas_abi_version() -> c_int;
    pub fn sd_cas_last_error() -> *const c_char;
    pub fn sd_cas_ctx_create(device: c_int, out: *mut *mut sd_cas_ctx) -> c_int;
    pub fn sd_cas_ctx_destroy(ctx: *mut sd_cas_ctx);
    pub fn sd_cas_stage_plan(sizes: *const u64, n: usize, ext: *mut sd_extent, total: *mut u64) -> c_int;
    pub fn sd_cas_ids_files(ctx: *mut sd_cas_ctx, paths: *const *const c_char, sizes: *const u64, n: usize,
                            out_hex17: *mut c_char, status: *mut i32, nthreads: c_int) -> c_int;
    pub fn sd_cas_id_path(ctx: *mut sd_cas_ctx, path: *const c_char, size: u64, out_hex17: *mut c_char,
                          status: *mut i32) -> c_int;
    pub fn sd_file_checksums(ctx: *mut sd_cas_ctx, paths: *const *const c_char, n: usize,
                             out_hex65: *mut c_char, status: *mut i32) -> c_int;
    pub fn sd_file_checksum_path(ctx: *mut sd_cas_ctx, path: *const c_char, out_hex65: *mut c_char,
                                 status: *mut i32) -> c_int;
}

/// One context per process on device 0 (the job system's 5 concurrent jobs, watcher and
/// non_indexed tasks all share it: every entry point is thread-safe).
pub struct Ctx(*mut sd_cas_ctx);
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

pub fn ctx() -> &'static Ctx {
    static CTX: OnceLock<Ctx> = OnceLock::new();
    CTX.get_or_init(|| {
        assert_eq!(unsafe { sd_cas_abi_version() }, SD_CAS_ABI_VERSION, "libsdcas ABI mismatch");
        let mut p = std::ptr::null_mut();
        let rc = unsafe { sd_cas_ctx_create(0, &mut p) };
        // no gfx950 device => no fallback (the library has no CPU path)
        assert_eq!(rc, SD_OK, "libsdcas: {}", last_error());
        Ctx(p)
    })
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

fn cpath(p: &Path) -> CString {
    CString::new(p.as_os_str().as_bytes()).expect("path with NUL")
}

fn hex_at(buf: &[c_char], i: usize, stride: usize, len: usize) -> String {
    buf[stride * i..stride * i + len].iter().map(|&b| b as u8 as char).collect()
}

/// Batched generate_cas_id (cas.rs:23-62): one result per (path, size), in order.  The
/// library preads the windows on its stager pool and overlaps them with the GPU.
pub fn cas_ids_blocking(files: &[(&Path, u64)]) -> Vec<Result<String, io::Error>> {
    let n = files.len();
    let c: Vec<CString> = files.iter().map(|f| cpath(f.0)).collect();
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let sizes: Vec<u64> = files.iter().map(|f| f.1).collect();
    let mut hex = vec![0 as c_char; 17 * n];
    let mut status = vec![0i32; n];
    let rc = unsafe {
        sd_cas_ids_files(ctx().0, ptrs.as_ptr(), sizes.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr(), 16)
    };
    (0..n)
        .map(|i| {
            if rc != SD_OK {
                Err(io::Error::new(io::ErrorKind::Other, last_error()))
            } else if status[i] != SD_FILE_OK {
                Err(status_to_io(status[i]))
            } else {
                Ok(hex_at(&hex, i, 17, 16))
            }
        })
        .collect()
}

/// Single-file generate_cas_id for the latency callers (watcher, non_indexed): concurrent
/// calls are coalesced into GPU batches inside the library (sd_cas_id_path).
pub fn cas_id_blocking(path: &Path, size: u64) -> Result<String, io::Error> {
    let c = cpath(path);
    let mut hex = [0 as c_char; 17];
    let mut st = 0i32;
    let rc = unsafe { sd_cas_id_path(ctx().0, c.as_ptr(), size, hex.as_mut_ptr(), &mut st) };
    if rc != SD_OK {
        return Err(io::Error::new(io::ErrorKind::Other, last_error()));
    }
    if st != SD_FILE_OK {
        return Err(status_to_io(st));
    }
    Ok(hex_at(&hex, 0, 17, 16))
}

/// Batched file_checksum (hash.rs:10-24).
pub fn checksums_blocking(paths: &[&Path]) -> Vec<Result<String, io::Error>> {
    let n = paths.len();
    let c: Vec<CString> = paths.iter().map(|p| cpath(p)).collect();
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let mut hex = vec![0 as c_char; 65 * n];
    let mut status = vec![0i32; n];
    let rc = unsafe { sd_file_checksums(ctx().0, ptrs.as_ptr(), n, hex.as_mut_ptr(), status.as_mut_ptr()) };
    (0..n)
        .map(|i| {
            if rc != SD_OK {
                Err(io::Error::new(io::ErrorKind::Other, last_error()))
            } else if status[i] != SD_FILE_OK {
                Err(status_to_io(status[i]))
            } else {
                Ok(hex_at(&hex, i, 65, 64))
            }
        })
        .collect()
}

/// Single-file file_checksum, coalesced (sd_file_checksum_path).
pub fn checksum_blocking(path: &Path) -> Result<String, io::Error> {
    let c = cpath(path);
    let mut hex = [0 as c_char; 65];
    let mut st = 0i32;
    let rc = unsafe { sd_file_checksum_path(ctx().0, c.as_ptr(), hex.as_mut_ptr(), &mut st) };
    if rc != SD_OK {
        return Err(io::Error::new(io::ErrorKind::Other, last_error()));
    }
    if st != SD_FILE_OK {
        return Err(status_to_io(st));
    }
    Ok(hex_at(&hex, 0, 65, 64))
}
