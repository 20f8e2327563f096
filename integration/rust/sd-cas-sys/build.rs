// libsdcas.so is built by `make -C spacedrive_amd/csrc` (hipcc --offload-arch=gfx950).
fn main() {
    let dir = std::env::var("SD_CAS_LIB_DIR").unwrap_or_else(|_| "/opt/spacedrive/lib".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=sdcas");
    println!("cargo:rerun-if-env-changed=SD_CAS_LIB_DIR");
}
