// Replacement body of core/src/object/cas.rs (reference :1-62).  The signature of
// generate_cas_id and its 16-hex output stay.
use std::path::{Path, PathBuf};

use tokio::{io, task::spawn_blocking};

// The sampling layout (head, 4 samples, tail; whole files up to 100 KiB) is the library's
// contract now: SD_SAMPLE_COUNT / SD_SAMPLE_SIZE / SD_HEADER_OR_FOOTER_SIZE /
// SD_MINIMUM_FILE_SIZE in include/sd_cas.h, checked against cas.rs:10-21 by the oracle tests.

/// Unchanged signature (cas.rs:23).  One file (watcher, non_indexed): the library's
/// latency policy hashes it on the CPU while few calls are in flight and coalesces
/// concurrent callers into GPU batches beyond that; without a device, the CPU path.
pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) -> Result<String, io::Error> {
    let p: PathBuf = path.as_ref().to_path_buf();
    spawn_blocking(move || sd_cas_sys::cas_id_blocking(&p, size))
        .await
        .map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
}

/// Batched sibling for identifier_job_step (file_identifier/mod.rs:107-134): one GPU
/// call for the whole step instead of join_all over per-file futures.
pub async fn generate_cas_ids(files: Vec<(PathBuf, u64)>) -> Vec<Result<String, io::Error>> {
    let n = files.len();
    spawn_blocking(move || {
        let refs: Vec<(&Path, u64)> = files.iter().map(|(p, s)| (p.as_path(), *s)).collect();
        sd_cas_sys::cas_ids_blocking(&refs)
    })
    .await
    .unwrap_or_else(|e| (0..n).map(|_| Err(io::Error::new(io::ErrorKind::Other, e.to_string()))).collect())
}
