// Builds libbote_hip.so with hipcc (gfx950) and links it.  Without ROCm the
// crate compiles to nothing and fantoch_bote keeps its CPU search.
use std::{env, process::Command};

fn main() {
    let hip = env::var("BOTE_HIP_DIR").unwrap_or_else(|_| "../bote_hip".into());
    if Command::new("hipcc").arg("--version").output().is_err() {
        return;
    }
    let status = Command::new("make")
        .args(&["-C", &format!("{}/fantoch_amd/csrc", hip), "ARCH=gfx950"])
        .status()
        .expect("make libbote_hip.so");
    assert!(status.success(), "libbote_hip.so build failed");
    println!("cargo:rustc-link-search=native={}/fantoch_amd/lib", hip);
    println!("cargo:rustc-link-lib=dylib=bote_hip");
    println!("cargo:rustc-cfg=bote_hip");
    println!("cargo:rerun-if-changed={}/fantoch_amd/csrc", hip);
    println!("cargo:rerun-if-changed={}/include/bote_hip.h", hip);
}
