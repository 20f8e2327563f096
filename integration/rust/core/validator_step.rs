// Replacement excerpt of core/src/object/validation/validator_job.rs:100-168: the
// ObjectValidatorJob with batched steps.
//
// The reference makes one job step per file (init: `Ok(steps.into())`, validator_job.rs:
// 123) and hashes it with file_checksum inside execute_step (:147-149), aborting the step
// -- and the job -- with `?` on the first I/O error.  Here a step is a batch of up to
// VALIDATOR_BATCH file_paths hashed with ONE file_checksums call
// (integration/rust/core/hash.rs -> sd_file_checksums: parallel reads into pinned windows,
// overlapped with the GPU), and the per-file policy is kept: files are committed in order,
// and the first failing file aborts the step with the same ValidatorError it raises today,
// after every file before it has had its checksum written, exactly as the one-file steps
// before it would have.
use serde_json::json;

use crate::{
    job::{CurrentStep, JobError, JobStepOutput, WorkerContext},
    library::Library,
    location::file_path_helper::{file_path_for_object_validator, IsolatedFilePathData},
    prisma::file_path,
    sync,
    util::error::FileIOError,
};

use super::{hash::file_checksums, ValidatorError};

/// Files per validator step.  Each file is still hashed by itself (a full-file checksum);
/// the batch amortises the GPU round trip and overlaps the reads.
pub const VALIDATOR_BATCH: usize = 64;

// In `init` (validator_job.rs:100-123) the steps become chunks of the same query result:
//
//     let steps = db.file_path().find_many(...).select(file_path_for_object_validator::select()).exec().await?;
//     *data = Some(ObjectValidatorJobData { location_path, task_count: steps.len() });
//     Ok(steps.chunks(VALIDATOR_BATCH).map(<[_]>::to_vec).collect::<Vec<_>>().into())
//
// with `type Step = Vec<file_path_for_object_validator::Data>;`.

pub(super) async fn execute_batched_step(
    init: &super::ObjectValidatorJobInit,
    ctx: &WorkerContext,
    CurrentStep { step: file_paths, .. }: CurrentStep<'_, Vec<file_path_for_object_validator::Data>>,
    data: &super::ObjectValidatorJobData,
) -> Result<JobStepOutput<Vec<file_path_for_object_validator::Data>, ()>, JobError> {
    let Library { db, sync, .. } = &*ctx.library;

    // validator_job.rs:142: only files still lacking a checksum
    let todo: Vec<&file_path_for_object_validator::Data> =
        file_paths.iter().filter(|fp| fp.integrity_checksum.is_none()).collect();
    // :143-146, with the same `?` on a file path that cannot be made relative
    let full_paths = todo
        .iter()
        .map(|fp| Ok(data.location_path.join(IsolatedFilePathData::try_from((init.location.id, *fp))?)))
        .collect::<Result<Vec<_>, JobError>>()?;

    let checksums = file_checksums(full_paths.clone()).await;

    for ((file_path, full_path), checksum) in todo.into_iter().zip(full_paths).zip(checksums) {
        // :147-149: the first failing file aborts the step (and the job) as before
        let checksum = checksum.map_err(|e| ValidatorError::FileIO(FileIOError::from((full_path, e))))?;
        // :151-165 unchanged, one write per file
        sync.write_op(
            db,
            sync.shared_update(
                prisma_sync::file_path::SyncId { pub_id: file_path.pub_id.clone() },
                file_path::integrity_checksum::NAME,
                json!(&checksum),
            ),
            db.file_path().update(
                file_path::pub_id::equals(file_path.pub_id.clone()),
                vec![file_path::integrity_checksum::set(Some(checksum))],
            ),
        )
        .await?;
    }
    Ok(().into())
}
