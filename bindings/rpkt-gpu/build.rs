// Link librpkt_gpu.so (built in-tree by `python -m rpkt_amd.build`).  RPKT_GPU_LIB_DIR
// overrides the directory; the default is the repository's rpkt_amd/_build.
fn main() {
    let dir = std::env::var("RPKT_GPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::path::PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap());
        here.join("../../rpkt_amd/_build").display().to_string()
    });
    println!("cargo:rerun-if-env-changed=RPKT_GPU_LIB_DIR");
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=rpkt_gpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir);
}
