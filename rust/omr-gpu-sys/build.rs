// Links libomr_gpu.so (built in-tree by `make -C tfhe-omr_amd`) and the HIP runtime it uses.
// OMR_GPU_LIB_DIR overrides the library directory; ROCM_PATH the ROCm install (default /opt/rocm).
use std::env;
use std::path::PathBuf;

fn main() {
    let lib_dir = env::var("OMR_GPU_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../tfhe-omr_amd")
    });
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    println!("cargo:rerun-if-env-changed=OMR_GPU_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    println!("cargo:rerun-if-changed=../../include/omr_gpu.h");
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=omr_gpu");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib_dir.display());
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}/lib", rocm);
}
