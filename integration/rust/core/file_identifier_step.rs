// Replacement excerpt of core/src/object/file_identifier/mod.rs:57-134: FileMetadata::new
// and the hashing half of identifier_job_step.  Everything from mod.rs:136 on (write_ops
// of the cas_ids, find_many of existing Objects, link / create_many) is unchanged.
//
// The reference awaits join_all over <= 100 per-file FileMetadata::new futures (mod.rs:
// 107-134), each hashing its own file on one task.  Here the step keeps the per-file stat
// and kind detection (out of scope, unchanged) and hashes the whole step with ONE
// generate_cas_ids call (integration/rust/core/cas.rs -> sd_cas_ids_files: the library's
// stager pool reads every file's windows into pinned memory, overlapped with the GPU).
// The 100-row CHUNK_SIZE stays: Object linking depends on it (duplicates inside one chunk
// each create their own Object, mod.rs:233-241), so a larger GPU batch must come from
// hashing more steps at once, never from changing the chunking.
use std::{collections::HashMap, path::{Path, PathBuf}};

use futures::future::join_all;
use tokio::fs;
use tracing::{error, trace};
use uuid::Uuid;

use crate::{
    location::file_path_helper::{file_path_for_file_identifier, IsolatedFilePathData},
    object::cas::generate_cas_ids,
    util::error::FileIOError,
};
use sd_file_ext::extensions::Extension;
use sd_prisma::prisma::location;

use super::{FileMetadata, ObjectKind};

impl FileMetadata {
    /// mod.rs:59-97 for every file of one identifier step: the per-file metadata and kind
    /// as before, then one batched hash for the non-empty files.  Results in input order;
    /// a file's error is its own (the caller logs and drops it, mod.rs:127-128).
    pub async fn new_batch(
        location_path: impl AsRef<Path>,
        iso_file_paths: &[&IsolatedFilePathData<'_>],
    ) -> Vec<Result<FileMetadata, FileIOError>> {
        let location_path = location_path.as_ref();
        // mod.rs:63-78: stat, the directory assert, the kind -- concurrently, as today
        let stats = join_all(iso_file_paths.iter().map(|iso| async move {
            let path = location_path.join(iso);
            let fs_metadata = fs::metadata(&path).await.map_err(|e| FileIOError::from((&path, e)))?;
            assert!(!fs_metadata.is_dir(), "We can't generate cas_id for directories");
            let kind = Extension::resolve_conflicting(&path, false)
                .await
                .map(Into::into)
                .unwrap_or(ObjectKind::Unknown);
            Ok::<_, FileIOError>((path, fs_metadata, kind))
        }))
        .await;

        // mod.rs:80-88: empty files get no cas_id and are not hashed
        let to_hash: Vec<(PathBuf, u64)> = stats
            .iter()
            .filter_map(|r| r.as_ref().ok())
            .filter(|(_, md, _)| md.len() != 0)
            .map(|(path, md, _)| (path.clone(), md.len()))
            .collect();
        let mut cas_ids = generate_cas_ids(to_hash).await.into_iter();

        stats
            .into_iter()
            .map(|r| {
                let (path, fs_metadata, kind) = r?;
                let cas_id = if fs_metadata.len() != 0 {
                    let id = cas_ids.next().expect("one result per hashed file");
                    Some(id.map_err(|e| FileIOError::from((&path, e)))?)
                } else {
                    None
                };
                trace!("Analyzed file: {path:?} {cas_id:?} {kind:?}");
                Ok(FileMetadata { cas_id, kind, fs_metadata })
            })
            .collect()
    }
}

/// The hashing half of identifier_job_step (mod.rs:100-134), batched.  Returns the same
/// map the reference builds, keyed by file_path.pub_id.
pub(super) async fn step_metadatas<'a>(
    location: &location::Data,
    location_path: &Path,
    file_paths: &'a [file_path_for_file_identifier::Data],
) -> HashMap<Uuid, (FileMetadata, &'a file_path_for_file_identifier::Data)> {
    // mod.rs:110-115
    let entries: Vec<(IsolatedFilePathData<'_>, &file_path_for_file_identifier::Data)> = file_paths
        .iter()
        .filter_map(|file_path| {
            IsolatedFilePathData::try_from((location.id, file_path))
                .map(|iso_file_path| (iso_file_path, file_path))
                .map_err(|e| error!("Failed to extract isolated file path data: {e:#?}"))
                .ok()
        })
        .collect();
    let isos: Vec<&IsolatedFilePathData<'_>> = entries.iter().map(|(iso, _)| iso).collect();
    let metadatas = FileMetadata::new_batch(location_path, &isos).await;

    // mod.rs:119-134
    entries
        .into_iter()
        .zip(metadatas)
        .filter_map(|((_, file_path), metadata)| {
            metadata
                .map(|metadata| {
                    (
                        // SAFETY: This should never happen
                        Uuid::from_slice(&file_path.pub_id).expect("file_path.pub_id is invalid!"),
                        (metadata, file_path),
                    )
                })
                .map_err(|e| error!("Failed to extract file metadata: {e:#?}"))
                .ok()
        })
        .collect()
}

// In identifier_job_step (mod.rs:100), lines 107-134 become:
//
//     let file_paths_metadatas = step_metadatas(location, location_path, file_paths).await;
//
// and the rest of the function (mod.rs:136-333) stays as it is.
