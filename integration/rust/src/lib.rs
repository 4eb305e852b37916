//! fantoch_bote_hip: the MI355X (gfx950) search behind fantoch_bote's API.
//! build.rs sets `cfg(bote_hip)` only when hipcc built libbote_hip.so; without
//! ROCm the crate is empty and fantoch_bote keeps its CPU search.
#[cfg(bote_hip)]
pub mod hip;
#[cfg(bote_hip)]
pub mod hip_search;
