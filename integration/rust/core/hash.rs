// Replacement body of core/src/object/validation/hash.rs (reference :1-24): same
// signature and 64-hex output, the same reads (1 MiB read calls until a short one), hashed
// by libsdcas (sd_file_checksum_path; the CPU path when the node has no gfx950 device).
use std::path::{Path, PathBuf};

use tokio::{io, task::spawn_blocking};

pub async fn file_checksum(path: impl AsRef<Path>) -> Result<String, io::Error> {
    let p: PathBuf = path.as_ref().to_path_buf();
    spawn_blocking(move || sd_cas_sys::checksum_blocking(&p))
        .await
        .map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
}

/// Batched sibling for a batched validator step (validator_job.rs:126-168).
pub async fn file_checksums(paths: Vec<PathBuf>) -> Vec<Result<String, io::Error>> {
    let n = paths.len();
    spawn_blocking(move || {
        let refs: Vec<&Path> = paths.iter().map(|p| p.as_path()).collect();
        sd_cas_sys::checksums_blocking(&refs)
    })
    .await
    .unwrap_or_else(|e| (0..n).map(|_| Err(io::Error::new(io::ErrorKind::Other, e.to_string()))).collect())
}
