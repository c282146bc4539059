// build.rs for RustRayTrace with the HIP backend (integration/rust/src/hip/mod.rs).
// Links librrt_hip.so (built by `python -c "import __graft_entry__ as g; g.build()"`, i.e.
// hipcc --offload-arch=gfx950) only when the `hip` feature is on; the CPU/wgpu/CUDA builds are
// untouched. RRT_HIP_LIB_DIR = the directory holding librrt_hip.so.
fn main() {
    println!("cargo:rerun-if-env-changed=RRT_HIP_LIB_DIR");
    if std::env::var_os("CARGO_FEATURE_HIP").is_none() {
        return;
    }
    let dir = std::env::var("RRT_HIP_LIB_DIR").unwrap_or_else(|_| "../rrt-mi355x/rustraytrace_amd".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=rrt_hip");
    // Let `cargo run` find the .so without LD_LIBRARY_PATH.
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
}
