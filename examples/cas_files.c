/* cas_files.c -- the drop-in boundary used from plain C: prints the cas_id (cas.rs:23-62)
 * and, with -c, the checksum (hash.rs:10-24) of every path on the command line, like the
 * per-file callers in the job system.  Uses the GPU when a gfx950 device is present and the
 * library's CPU path (sd_cpu_*) otherwise -- the routing the Rust shim's ctx() does.
 *
 *   gcc -O2 -Iinclude examples/cas_files.c -Lspacedrive_amd -lsdcas \
 *       -Wl,-rpath,$PWD/spacedrive_amd -o cas_files
 *   ./cas_files [-c] [--cpu] FILE...
 * Output: one line per file, "<cas_id or checksum>  <path>", or "error(<status>/<errno>)".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "sd_cas.h"

int main(int argc, char** argv) {
    int checksum = 0, force_cpu = 0, first = 1;
    for (; first < argc && argv[first][0] == '-'; first++) {
        if (!strcmp(argv[first], "-c")) checksum = 1;
        else if (!strcmp(argv[first], "--cpu")) force_cpu = 1;
        else {
            fprintf(stderr, "usage: %s [-c] [--cpu] FILE...\n", argv[0]);
            return 2;
        }
    }
    const size_t n = (size_t)(argc - first);
    if (n == 0) return 0;
    const char* const* paths = (const char* const*)(argv + first);
    if (sd_cas_abi_version() != SD_CAS_ABI_VERSION) {
        fprintf(stderr, "libsdcas ABI %d, header %d\n", sd_cas_abi_version(), SD_CAS_ABI_VERSION);
        return 2;
    }
    sd_cas_ctx* ctx = NULL;
    if (!force_cpu && sd_cas_ctx_create(0, &ctx) != SD_OK) ctx = NULL; /* no device: CPU path */
    const size_t width = checksum ? 65 : 17;
    char* out = calloc(n, width);
    int32_t* status = calloc(n, sizeof(int32_t));
    uint64_t* sizes = calloc(n, sizeof(uint64_t));
    if (!out || !status || !sizes) return 3;
    int rc;
    if (checksum) {
        rc = ctx ? sd_file_checksums(ctx, paths, n, out, status) : sd_cpu_file_checksums(paths, n, out, status, 16);
    } else {
        /* FileMetadata::new (file_identifier/mod.rs:65-88): the size comes from the metadata */
        for (size_t i = 0; i < n; i++) {
            struct stat st;
            sizes[i] = stat(paths[i], &st) == 0 ? (uint64_t)st.st_size : 0;
        }
        rc = ctx ? sd_cas_ids_files(ctx, paths, sizes, n, out, status, 16)
                 : sd_cpu_cas_ids_files(paths, sizes, n, out, status, 16);
    }
    if (rc != SD_OK) {
        fprintf(stderr, "libsdcas: %d %s\n", rc, sd_cas_last_error());
        return 1;
    }
    for (size_t i = 0; i < n; i++) {
        if (status[i] == SD_FILE_OK) printf("%s  %s\n", out + i * width, paths[i]);
        else printf("error(%d/%d)  %s\n", status[i] & 0xFFFF, status[i] >> 16, paths[i]);
    }
    if (ctx) sd_cas_ctx_destroy(ctx);
    free(out);
    free(status);
    free(sizes);
    return 0;
}
