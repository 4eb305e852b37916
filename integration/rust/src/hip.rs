//! Raw FFI to libbote_hip.so, one item per declaration of include/bote_hip.h.
//! Sketch for fantoch_bote maintainers; not compiled here.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub const BOTE_OK: c_int = 0;
pub const BOTE_E_ARG: c_int = -1;
pub const BOTE_E_QUORUM_GT_N: c_int = -2;
pub const BOTE_E_DEVICE: c_int = -3;
pub const BOTE_E_RANGE: c_int = -4;
pub const BOTE_E_NOMEM: c_int = -5;
pub const BOTE_E_NODEV: c_int = -6;

pub const BOTE_FPAXOS: c_int = 0;
pub const BOTE_EPAXOS: c_int = 1;
pub const BOTE_ATLAS: c_int = 2;
pub const BOTE_TEMPO: c_int = 3;
pub const BOTE_TEMPO_TINY: c_int = 4;

pub const BOTE_KERNEL_AUTO: c_int = 0;
pub const BOTE_KERNEL_GENERIC: c_int = 1;
pub const BOTE_KERNEL_FAST: c_int = 2;
pub const BOTE_KERNEL_GROUP: c_int = 3;

pub const BOTE_FT_F1: i32 = 1;
pub const BOTE_FT_F1F2: i32 = 2;

pub const BOTE_STAT_MEAN: c_int = 0;
pub const BOTE_STAT_COV: c_int = 1;
pub const BOTE_STAT_MDTM: c_int = 2;

pub const BOTE_OBJ_SCORE: u32 = 0;
pub const BOTE_OBJ_MEAN: u32 = 1;
pub const BOTE_OBJ_COV: u32 = 2;

#[repr(C)]
pub struct bote_planet {
    _p: [u8; 0],
}
#[repr(C)]
pub struct bote_sweep {
    _p: [u8; 0],
}
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct bote_objective {
    pub kind: u32,
    pub slot: u32,
}
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct bote_ranking_params {
    pub min_mean_fpaxos_improv: f64,
    pub min_mean_epaxos_improv: f64,
    pub min_fairness_fpaxos_improv: f64,
    pub min_mean_decrease: f64,
    pub ft_metric: i32,
}
#[repr(C)]
#[derive(Clone, Copy, Debug, PartialEq, Eq, PartialOrd, Ord)]
pub struct bote_topk_record {
    pub key: u64,
    pub rank: u64,
}

extern "C" {
    pub fn bote_last_error() -> *const c_char;
    pub fn bote_device_count(out: *mut c_int) -> c_int;
    pub fn bote_planet_create(lat: *const u16, r: u32, device: c_int, out: *mut *mut bote_planet) -> c_int;
    pub fn bote_planet_destroy(p: *mut bote_planet) -> c_int;
    pub fn bote_planet_regions(p: *const bote_planet, out_r: *mut u32) -> c_int;
    pub fn bote_quorum_size(protocol: c_int, n: u32, f: u32) -> c_int;
    pub fn bote_max_f(n: u32) -> u32;
    pub fn bote_quorum_latencies(p: *const bote_planet, froms: *const u32, nf: u32, regions: *const u32,
                                 nr: u32, q: u32, out: *mut u64) -> c_int;
    pub fn bote_leaderless(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                           q: u32, out: *mut u64) -> c_int;
    pub fn bote_leader(p: *const bote_planet, leader: u32, servers: *const u32, ns: u32, clients: *const u32,
                       nc: u32, q: u32, out: *mut u64) -> c_int;
    pub fn bote_all_leaders(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                            q: u32, out: *mut u64) -> c_int;
    pub fn bote_best_leader(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                            q: u32, stat: c_int, out_pos: *mut u32, out_lat: *mut u64) -> c_int;
    pub fn bote_eval(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32, n: u32,
                     configs: *const u32, rank_begin: u64, ncfg: u64, rp: *const bote_ranking_params,
                     out_vals: *mut u32, out_leader: *mut u32, out_sum: *mut u64, out_sumsq: *mut u64,
                     out_mean: *mut f64, out_cov: *mut f64, out_score: *mut f64, out_valid: *mut u8) -> c_int;
    pub fn bote_sweep_create(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                             n: u32, objs: *const bote_objective, n_obj: u32, k: u32,
                             rp: *const bote_ranking_params, digest: c_int, out: *mut *mut bote_sweep) -> c_int;
    pub fn bote_sweep_create_ex(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                                n: u32, objs: *const bote_objective, n_obj: u32, k: u32,
                                rp: *const bote_ranking_params, digest: c_int, kernel: c_int,
                                out: *mut *mut bote_sweep) -> c_int;
    pub fn bote_sweep_launch(s: *mut bote_sweep, rank_begin: u64, rank_end: u64, stream: *mut c_void) -> c_int;
    pub fn bote_sweep_deferred(s: *mut bote_sweep, stream: *mut c_void, out: *mut u64) -> c_int;
    pub fn bote_sweep_split(s: *const bote_sweep, rank_begin: u64, rank_end: u64, parts: u32,
                            out_bounds: *mut u64) -> c_int;
    pub fn bote_eval_leaderless(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                                n: u32, configs: *const u32, rank_begin: u64, ncfg: u64, quorum_sizes: *const u32,
                                nq: u32, out_vals: *mut u32, out_sum: *mut u64, out_sumsq: *mut u64) -> c_int;
    pub fn bote_search_topk(planets: *const *const bote_planet, n_devices: u32, servers: *const u32, ns: u32,
                            clients: *const u32, nc: u32, n: u32, rank_begin: u64, rank_end: u64,
                            objs: *const bote_objective, n_obj: u32, k: u32, rp: *const bote_ranking_params,
                            digest: c_int, out: *mut bote_topk_record, out_count: *mut u32, out_valid: *mut u64,
                            out_digest: *mut u64) -> c_int;
    pub fn bote_search_create(planets: *const *const bote_planet, n_devices: u32, servers: *const u32, ns: u32,
                              clients: *const u32, nc: u32, n: u32, rank_begin: u64, rank_end: u64,
                              objs: *const bote_objective, n_obj: u32, k: u32, rp: *const bote_ranking_params,
                              digest: c_int, keys: u32, out: *mut *mut bote_search) -> c_int;
    pub fn bote_search_launch(h: *mut bote_search) -> c_int;
    pub fn bote_search_result(h: *mut bote_search, out: *mut bote_topk_record, out_count: *mut u32,
                              out_valid: *mut u64, out_digest: *mut u64) -> c_int;
    pub fn bote_search_bounds(h: *const bote_search, out_bounds: *mut u64) -> c_int;
    pub fn bote_search_destroy(h: *mut bote_search) -> c_int;
    pub fn bote_sweep_create_keys(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                                  n: u32, objs: *const bote_objective, n_obj: u32, k: u32,
                                  rp: *const bote_ranking_params, digest: c_int, kernel: c_int, keys: u32,
                                  out: *mut *mut bote_sweep) -> c_int;
    pub fn bote_eval_keys(p: *const bote_planet, servers: *const u32, ns: u32, clients: *const u32, nc: u32,
                          n: u32, configs: *const u32, rank_begin: u64, ncfg: u64, keys: u32, out_leader: *mut u32,
                          out_sum: *mut u64, out_sumsq: *mut u64, out_al_sum: *mut u64, out_al_sumsq: *mut u64)
        -> c_int;
    pub fn bote_evolving_chains(device: c_int, ns: u32, counts: *const u32, masks: *const *const u64,
                                scores: *const *const f64, means: *const *const f64, min_mean_decrease: f64,
                                ft_metric: c_int, max_out: u64, out_idx: *mut u32, out_score: *mut f64,
                                out_total: *mut u64) -> c_int;
    pub fn bote_sweep_result(s: *mut bote_sweep, stream: *mut c_void, out: *mut bote_topk_record,
                             out_count: *mut u32, out_valid: *mut u64, out_digest: *mut u64) -> c_int;
    pub fn bote_sweep_result_bytes(s: *const bote_sweep) -> u64;
    pub fn bote_sweep_result_device(s: *mut bote_sweep, dst: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn bote_merge_device(s: *const bote_sweep, src: *const c_void, n_shards: u32, dst: *mut c_void,
                             stream: *mut c_void) -> c_int;
    pub fn bote_sweep_last_kernel_ms(s: *mut bote_sweep, out_ms: *mut f32) -> c_int;
    pub fn bote_sweep_timing_reset(s: *mut bote_sweep) -> c_int;
    pub fn bote_sweep_timing(s: *mut bote_sweep, out_total_ms: *mut f32, out_launches: *mut u32) -> c_int;
    pub fn bote_sweep_is_fast(s: *const bote_sweep, out: *mut c_int) -> c_int;
    pub fn bote_sweep_grid(s: *const bote_sweep, out_grid: *mut u32, out_block: *mut u32, out_lds_bytes: *mut u32)
        -> c_int;
    pub fn bote_sweep_destroy(s: *mut bote_sweep) -> c_int;
    pub fn bote_colex_unrank(rank: u64, n: u32, ns: u32, out_positions: *mut u32) -> c_int;
    pub fn bote_binomial(ns: u32, n: u32) -> u64;
}

/// Turns a status code into the panic the reference raises at the same place
/// (fantoch_bote/src/lib.rs:84,178,184: `unwrap`/`expect`).
pub fn check(rc: c_int) {
    if rc != BOTE_OK {
        let msg = unsafe { std::ffi::CStr::from_ptr(bote_last_error()) };
        panic!("libbote_hip: {} (code {})", msg.to_string_lossy(), rc);
    }
}
