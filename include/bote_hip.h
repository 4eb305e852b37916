/*
 * bote_hip.h — C ABI of the MI355X (gfx950) implementation of fantoch_bote's
 * configuration search.  Plain pointers and sizes only; no exceptions or panics
 * cross this boundary.  Every entry point returns BOTE_OK (0) or a negative
 * BOTE_E_* code; bote_last_error() describes the last failure on this thread.
 *
 * Regions are integer ids in NAME ORDER (id == rank of the region's name), so
 * the reference's (latency, Region) distance order (fantoch/src/planet/mod.rs:
 * 122-140) is the (latency, id) order.  Latencies are row = from, column = to,
 * as Planet::ping_latency (planet/mod.rs:107-113).
 *
 * Each entry point names the reference interface it replaces.  The reference
 * is a Rust library without an FFI; INTEGRATION.md shows the `extern "C"`
 * binding a fantoch_bote maintainer would add on top of this header.
 */
#ifndef BOTE_HIP_H
#define BOTE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ status codes */
#define BOTE_OK 0
#define BOTE_E_ARG (-1)          /* bad argument (null pointer, size, id out of range) */
#define BOTE_E_QUORUM_GT_N (-2)  /* a quorum larger than the server set (reference: unwrap panic, lib.rs:178-184) */
#define BOTE_E_DEVICE (-3)       /* HIP runtime error */
#define BOTE_E_RANGE (-4)        /* value outside the supported range (latency > 16383, R > 128, n > 16, K > 128) */
#define BOTE_E_NOMEM (-5)        /* device allocation failed */
#define BOTE_E_NODEV (-6)        /* no HIP device */

/* ---------------------------------------------------------------- limits  */
#define BOTE_MAX_REGIONS 128
#define BOTE_MAX_N 16
#define BOTE_MAX_K 128
#define BOTE_MAX_OBJECTIVES 8
#define BOTE_MAX_LATENCY 16383
#define BOTE_MAX_CLIENTS 4096

/* --------------------------------------------------------------- enums    */
/* fantoch_bote/src/protocol.rs:5-9 (+ Tempo, fantoch/src/config.rs:317-329) */
#define BOTE_FPAXOS 0
#define BOTE_EPAXOS 1
#define BOTE_ATLAS 2
#define BOTE_TEMPO 3      /* Tempo fast quorum, non-tiny: n/2 + f */
#define BOTE_TEMPO_TINY 4 /* Tempo fast quorum, tiny: 2f */

/* fantoch/src/metrics/histogram.rs:7-11 */
#define BOTE_STAT_MEAN 0
#define BOTE_STAT_COV 1
#define BOTE_STAT_MDTM 2

/* Histogram key slots of ProtocolStats (fantoch_bote/src/protocol.rs:98-105):
 * slot = base + 5 * placement, placement 0 = Input, 1 = Colocated
 * (ClientPlacement, protocol.rs:38-55). */
#define BOTE_SLOT_AF1 0
#define BOTE_SLOT_FF1 1
#define BOTE_SLOT_AF2 2
#define BOTE_SLOT_FF2 3
#define BOTE_SLOT_E 4
#define BOTE_SLOT_COLOCATED 5
#define BOTE_NSLOTS 10

/* Key sets.  BOTE_KEYS_TEMPO_ALL_LEADERS (BASELINE config 5: "Tempo f=1,2 +
 * FPaxos all leaders") adds to the compute_stats keys, per config:
 *   * Tempo's tiny fast quorum 2f and write quorum f + 1
 *     (fantoch/src/config.rs:317-329) through Bote::leaderless, Input and
 *     Colocated: slot = 10 + 4 * placement + {TT1, TT2, TW1, TW2} offsets
 *     (Tempo's non-tiny fast quorum n/2 + f is the Atlas key af{f});
 *   * FPaxos with EVERY leader (Bote::all_leaders_stats, lib.rs:129-150) over
 *     the Input clients at q = f + 1, f = 1..max_f: the digest consumes every
 *     leader's moments, and slots FL1/FL2 hold the histogram of the best
 *     leader by Stats::Mean (Bote::best_leader, lib.rs:99-121, first minimum).
 * Slots with f = 2 exist only when max_f(n) >= 2. */
#define BOTE_KEYS_BASE 0
#define BOTE_KEYS_TEMPO_ALL_LEADERS 1
#define BOTE_SLOT_TT1 10 /* Tempo tiny, f = 1 (q = 2), Input; + 4 = Colocated */
#define BOTE_SLOT_TT2 11 /* Tempo tiny, f = 2 (q = 4) */
#define BOTE_SLOT_TW1 12 /* Tempo write, f = 1 (q = 2) */
#define BOTE_SLOT_TW2 13 /* Tempo write, f = 2 (q = 3) */
#define BOTE_SLOT_X_COLOCATED 4
#define BOTE_SLOT_FL1 18 /* FPaxos, best leader by mean, f = 1, Input */
#define BOTE_SLOT_FL2 19 /* FPaxos, best leader by mean, f = 2, Input */
#define BOTE_NSLOTS_X 20

/* Objectives of the streaming top-K (an extension: the reference stores every
 * config, search.rs:234-260; the MI355X build streams and keeps the best K). */
#define BOTE_OBJ_SCORE 0 /* max Search::compute_score among valid configs (search.rs:421-472) */
#define BOTE_OBJ_MEAN 1  /* min Histogram::mean of `slot` (exact sum order)          */
#define BOTE_OBJ_COV 2   /* min Histogram::cov of `slot`, keyed fl64(V / S1^2)        */

/* Sweep kernel paths (bote_sweep_create_ex); every path is exact. */
#define BOTE_KERNEL_AUTO 0    /* group kernel when eligible, else fast, else generic */
#define BOTE_KERNEL_GENERIC 1 /* eval_kernel (bote_kernels.hip): any planet */
#define BOTE_KERNEL_FAST 2    /* sweep_fast_kernel (bote_sweep.hip) */
#define BOTE_KERNEL_GROUP 3   /* sweep_group_kernel (bote_group.hip), n >= 4 */

#define BOTE_FT_F1 1   /* FTMetric::F1   (search.rs:652-666) */
#define BOTE_FT_F1F2 2 /* FTMetric::F1F2 */

typedef struct bote_planet bote_planet;
typedef struct bote_sweep bote_sweep;
typedef struct bote_search bote_search;

typedef struct {
  uint32_t kind; /* BOTE_OBJ_* */
  uint32_t slot; /* BOTE_SLOT_* (ignored for BOTE_OBJ_SCORE) */
} bote_objective;

/* RankingParams (search.rs:617-649); min_n/max_n are implied by the call. */
typedef struct {
  double min_mean_fpaxos_improv;
  double min_mean_epaxos_improv;
  double min_fairness_fpaxos_improv;
  double min_mean_decrease;
  int32_t ft_metric; /* BOTE_FT_F1 or BOTE_FT_F1F2 */
} bote_ranking_params;

/* One top-K record.  Records sort ascending by (key, rank).
 *   SCORE: key = ~orderable(score)  (higher score first)
 *   MEAN:  key = exact integer sum of the histogram (count is fixed per slot)
 *   COV:   key = IEEE bits of fl64(V / S1^2), V = count*sum(x^2) - S1^2;
 *          ~0 when the reference's COV is NaN (count <= 1 or S1 == 0)
 * rank = colex rank of the config: rank = sum_j C(p_j, j+1), p ascending
 * positions into the server list. */
typedef struct {
  uint64_t key;
  uint64_t rank;
} bote_topk_record;

/* -------------------------------------------------------------- errors --- */
const char* bote_last_error(void);
int bote_device_count(int* out);

/* -------------------------------------------------------------- planet --- */
/* Replaces Planet::from / from_latencies (fantoch/src/planet/mod.rs:38-54) as
 * the device-side planet: uploads the R x R matrix (uint16, row = from) to
 * `device`.  Ids must be in name order (id == name rank). */
int bote_planet_create(const uint16_t* lat, uint32_t R, int device, bote_planet** out);
int bote_planet_destroy(bote_planet* p);
int bote_planet_regions(const bote_planet* p, uint32_t* out_R);

/* ------------------------------------------------------------ protocol --- */
/* Protocol::quorum_size (protocol.rs:20-31); Tempo: config.rs:317-329.
 * Returns the quorum size (> 0) or a negative error. */
int bote_quorum_size(int protocol, uint32_t n, uint32_t f);
/* Search::max_f (search.rs:474-477) */
uint32_t bote_max_f(uint32_t n);

/* ---------------------------------------------- Bote, one configuration --- */
/* The per-call entry points below run stream-ordered on the planet's own
 * HIP stream with cached device workspaces and synchronise only that stream;
 * calls on one planet handle are serialised, distinct handles are independent. */
/* Bote::quorum_latency (lib.rs:155-163) for every `from` in `froms`. */
int bote_quorum_latencies(const bote_planet* p, const uint32_t* froms, uint32_t nf,
                          const uint32_t* regions, uint32_t nr, uint32_t q, uint64_t* out);
/* Bote::leaderless (lib.rs:38-59): per-client latency, client order. */
int bote_leaderless(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                    const uint32_t* clients, uint32_t nc, uint32_t q, uint64_t* out);
/* Bote::leader (lib.rs:67-89): per-client latency to `leader` plus its quorum. */
int bote_leader(const bote_planet* p, uint32_t leader, const uint32_t* servers, uint32_t ns,
                const uint32_t* clients, uint32_t nc, uint32_t q, uint64_t* out);
/* Bote::all_leaders_stats (lib.rs:129-150): out is ns x nc, leader-major. */
int bote_all_leaders(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                     const uint32_t* clients, uint32_t nc, uint32_t q, uint64_t* out);
/* Bote::best_leader (lib.rs:99-121): index into `servers` of the chosen leader
 * (first minimum under F64's total order) and, if out_lat != NULL, its nc
 * per-client latencies. */
int bote_best_leader(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                     const uint32_t* clients, uint32_t nc, uint32_t q, int stat,
                     uint32_t* out_pos, uint64_t* out_lat);

/* ---------------------------------------- compute_stats over many configs --- */
/* Search::compute_stats (search.rs:262-319) for a batch of configurations of
 * size n.  A configuration is n positions into `servers` (config order = the
 * given order; the FPaxos leader tie-break goes to the earliest).  Either
 * `configs` (ncfg x n positions) is given, or configs == NULL and the batch is
 * the colex ranks [rank_begin, rank_begin + ncfg).
 *
 * Outputs (host pointers; NULL to skip):
 *   out_vals   ncfg x (5*nc + 5*n) uint32: per-client latencies, slot-major —
 *              Input slots 0..4 (nc values each, client order), then Colocated
 *              slots 5..9 (n values each, config order).  Slots that do not
 *              exist for n (af2/ff2/af2C/ff2C when max_f(n) == 1) hold 0xFFFFFFFF.
 *   out_leader ncfg: position of the FPaxos leader inside the config
 *   out_sum, out_sumsq  ncfg x 10 uint64: exact sum and sum of squares per slot
 *   out_mean, out_cov   ncfg x 10 double: Histogram::mean (bit-exact) and
 *              Histogram::cov (from exact moments, within 1e-12 relative)
 *   out_score, out_valid ncfg: Search::compute_score under `rp` (may be NULL
 *              to skip; bit-exact score and validity). */
int bote_eval(const bote_planet* p, const uint32_t* servers, uint32_t ns,
              const uint32_t* clients, uint32_t nc, uint32_t n, const uint32_t* configs,
              uint64_t rank_begin, uint64_t ncfg, const bote_ranking_params* rp,
              uint32_t* out_vals, uint32_t* out_leader, uint64_t* out_sum, uint64_t* out_sumsq,
              double* out_mean, double* out_cov, double* out_score, uint8_t* out_valid);

/* bote_eval with a key set: exact moments of every slot of `keys`
 * (BOTE_KEYS_*), config-major: out_sum, out_sumsq ncfg x 20 (slots absent for
 * n hold ~0; with BOTE_KEYS_BASE only the first 10 of each row are written,
 * stride 10), out_leader as bote_eval, and with BOTE_KEYS_TEMPO_ALL_LEADERS
 * every leader's FPaxos moments out_al_sum, out_al_sumsq ncfg x 2 x n
 * (f = 1, 2; leaders in config order; ~0 when f > max_f(n)). */
int bote_eval_keys(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                   const uint32_t* clients, uint32_t nc, uint32_t n, const uint32_t* configs,
                   uint64_t rank_begin, uint64_t ncfg, uint32_t keys, uint32_t* out_leader,
                   uint64_t* out_sum, uint64_t* out_sumsq, uint64_t* out_al_sum, uint64_t* out_al_sumsq);

/* Bote::leaderless (lib.rs:38-59) for a batch of configurations (as in
 * bote_eval: `configs` or colex ranks) and nq quorum sizes (1..8, each <= n) at
 * once.  This carries Tempo (fantoch/src/config.rs:317-329): fast quorum
 * n/2 + f (tiny: 2f) and write quorum f + 1, which Search::compute_stats does
 * not key.  Per config and quorum size (config-major, then quorum order):
 *   out_vals   nc Input-client latencies (client order) then n Colocated
 *              latencies (config order): ncfg x nq x (nc + n) uint32
 *   out_sum, out_sumsq  exact sum / sum of squares, [Input, Colocated]:
 *              ncfg x nq x 2 uint64 */
int bote_eval_leaderless(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                         const uint32_t* clients, uint32_t nc, uint32_t n, const uint32_t* configs,
                         uint64_t rank_begin, uint64_t ncfg, const uint32_t* quorum_sizes, uint32_t nq,
                         uint32_t* out_vals, uint64_t* out_sum, uint64_t* out_sumsq);

/* -------------------------------------- superset chains (ranking product) --- */
/* Search::sorted_evolving_configs (search.rs:97-178; super_configs :378-401,
 * min_mean_decrease :403-419) for ONE client set, on `device`.  Level l = 0..5
 * holds the ranked (valid) configs of n = 3 + 2l in enumeration order:
 *   masks[l][i]    bitmask of the config's positions in the server list (ns <= 64)
 *   scores[l][i]   Search::compute_score
 *   means[l][2i], means[l][2i+1]  Histogram::mean of the Atlas Input key, f = 1, 2
 * A chain takes one config per level, each a superset of the previous whose
 * Atlas means decrease by >= min_mean_decrease for f in FTMetric::fs(n - 2).
 * Out: *out_total chains; the first max_out in the reference's order (score
 * descending, equal scores in enumeration order): out_idx (6 level indices
 * per chain) and out_score (s3 + s5 + ... + s13, summed in that order). */
int bote_evolving_chains(int device, uint32_t ns, const uint32_t* counts, const uint64_t* const* masks,
                         const double* const* scores, const double* const* means,
                         double min_mean_decrease, int ft_metric, uint64_t max_out,
                         uint32_t* out_idx, double* out_score, uint64_t* out_total);

/* ------------------------------------------------ streaming search (hot) --- */
/* The exhaustive sweep (search.rs:199-260 + compute_stats + compute_score)
 * over colex ranks [rank_begin, rank_end) of n-subsets of `servers`, keeping
 * the best K configurations per objective on the device.
 *
 * bote_sweep_create uploads the lists and allocates the device workspace;
 * bote_sweep_launch is asynchronous on `hip_stream` (NULL = the planet's
 * device default stream) and may be called repeatedly (each launch restarts
 * the top-K); bote_sweep_result synchronises the stream and copies out:
 *   out        n_obj x K records, ascending (key, rank) per objective
 *   out_count  n_obj: records filled
 *   out_valid  configs with a valid compute_score (only with a SCORE objective)
 *   out_digest wrapping sum over configs of a per-config digest,
 *              only when `digest` was set at creation. */
int bote_sweep_create(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                      const uint32_t* clients, uint32_t nc, uint32_t n,
                      const bote_objective* objs, uint32_t n_obj, uint32_t K,
                      const bote_ranking_params* rp, int digest, bote_sweep** out);
/* bote_sweep_create with an explicit kernel path (BOTE_KERNEL_*); a forced
 * fast/group path that the planet or lists do not qualify for is BOTE_E_ARG. */
int bote_sweep_create_ex(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                         const uint32_t* clients, uint32_t nc, uint32_t n,
                         const bote_objective* objs, uint32_t n_obj, uint32_t K,
                         const bote_ranking_params* rp, int digest, int kernel, bote_sweep** out);
/* bote_sweep_create_ex with a key set (BOTE_KEYS_*): objectives may name
 * every slot of the set, and the digest folds all of its moments (DESIGN.md
 * §7).  The extended set runs on the group kernel for n = 4..7 with config
 * 5's objectives (SCORE, MEAN af1, MEAN ff1, COV af1, MEAN e, MEAN TT1, MEAN
 * TW2, MEAN FL1, compiled in), otherwise on the generic kernel (any
 * objectives). */
int bote_sweep_create_keys(const bote_planet* p, const uint32_t* servers, uint32_t ns,
                           const uint32_t* clients, uint32_t nc, uint32_t n,
                           const bote_objective* objs, uint32_t n_obj, uint32_t K,
                           const bote_ranking_params* rp, int digest, int kernel, uint32_t keys,
                           bote_sweep** out);
/* Asynchronous on `hip_stream`: the sweep kernel, the exact fix-up of its
 * deferred near-tie configs, the (device-decided) overflow fallback and the
 * merge chain are all stream-ordered; no host synchronisation. */
int bote_sweep_launch(bote_sweep* s, uint64_t rank_begin, uint64_t rank_end, void* hip_stream);
int bote_sweep_result(bote_sweep* s, void* hip_stream, bote_topk_record* out, uint32_t* out_count,
                      uint64_t* out_valid, uint64_t* out_digest);
/* Device-side result block for collectives: `dst` (device memory, or pinned
 * host memory for a direct copy to the host; at least
 * bote_sweep_result_bytes()) receives [n_obj x 128 records, ascending, padded
 * with all-ones records][valid u64][digest u64], stream-ordered after the last
 * launch.  Only the first K records of each objective are meaningful. */
uint64_t bote_sweep_result_bytes(const bote_sweep* s);
int bote_sweep_result_device(bote_sweep* s, void* dst, void* hip_stream);
/* Deterministic merge of `n_shards` device result blocks laid out back to back
 * (e.g. an all-gather over ranks) into one block at `dst`, on the device. */
int bote_merge_device(const bote_sweep* s, const void* src, uint32_t n_shards, void* dst,
                      void* hip_stream);
/* Kernel-only timing of the most recent launch (HIP events around the sweep
 * kernel on its stream), in milliseconds; merge kernels excluded. */
int bote_sweep_last_kernel_ms(bote_sweep* s, float* out_ms);
/* Sum of the sweep-kernel durations (HIP events on the launch stream) of every
 * launch since the last bote_sweep_timing_reset; synchronises on the last. */
int bote_sweep_timing_reset(bote_sweep* s);
int bote_sweep_timing(bote_sweep* s, float* out_total_ms, uint32_t* out_launches);
/* Which sweep kernel runs: 0 the generic kernel (bote_kernels.hip), 1 the
 * packed fast-path kernel (bote_sweep.hip), 2 the group kernel
 * (bote_group.hip).  All are exact (DESIGN.md "Kernels"). */
int bote_sweep_is_fast(const bote_sweep* s, int* out);
/* Shard boundaries for `parts` devices over [rank_begin, rank_end): out[0] =
 * rank_begin, out[parts] = rank_end, ascending.  On the group kernel the
 * shards have equal estimated cost (a group of C(p, 3) configs costs
 * ceil(C(p, 3) / 64) wavefront steps plus its precompute; equal rank shares
 * of R=64 n=7 differ by up to 14 % over 8 devices), otherwise equal rank
 * counts.  Host only (no device work).  Replaces the reference's split of
 * work, a rayon fork-join over client sets (fantoch_bote/src/search.rs:209-231):
 * here one client set's rank space is split. */
int bote_sweep_split(const bote_sweep* s, uint64_t rank_begin, uint64_t rank_end, uint32_t parts,
                     uint64_t* out_bounds);
/* Configs the fast/group kernel deferred to the exact generic kernel in the
 * last launch (COV near-ties; more than 2^20 => the whole range was recomputed
 * on the generic path).  Synchronises `hip_stream`.  0 on the generic path. */
int bote_sweep_deferred(bote_sweep* s, void* hip_stream, uint64_t* out);
/* Launch geometry chosen at creation (persistent grid, block size, LDS bytes). */
int bote_sweep_grid(const bote_sweep* s, uint32_t* out_grid, uint32_t* out_block, uint32_t* out_lds_bytes);
int bote_sweep_destroy(bote_sweep* s);

/* ------------------------------------------------ multi-device search --- */
/* The exhaustive search over colex ranks [rank_begin, rank_end) sharded over
 * n_devices planets (planets[i] lives on the device that sweeps shard i; a
 * device may appear more than once).  Replaces the rayon fork-join of
 * Search::compute_all_configs (fantoch_bote/src/search.rs:199-232) for a
 * single client set, so its output is Search's streamed equivalent.  Every
 * planet must hold the same latency matrix.
 *
 * bote_search_create does all host work once: one sweep, stream and result
 * buffer per shard, the shard bounds (equal estimated cost, as
 * bote_sweep_split) and each shard's work-chunk table, from ONE host walk of
 * the rank space shared by all shards; it returns with the handle idle.  For
 * every shard on a device other than planets[0]'s it checks
 * hipDeviceCanAccessPeer and enables that device's access to planets[0]'s
 * ("already enabled" is success; a failure to enable returns BOTE_E_DEVICE),
 * so the shard writes its result block over xGMI; without peer capability the
 * runtime stages the copy through host memory.
 * bote_search_launch is device work only and asynchronous: every shard's
 * sweep on its own stream, a peer copy of its result block to planets[0]'s
 * device, and a (key, rank) merge tree there.  It may be called repeatedly
 * (each launch recomputes the whole range).  bote_search_result waits for the
 * last launch and copies out as bote_sweep_result; the result equals one
 * unsharded sweep.  `keys` selects the key set (BOTE_KEYS_*, as
 * bote_sweep_create_keys).  Calls on one handle must not overlap. */
int bote_search_create(const bote_planet* const* planets, uint32_t n_devices,
                       const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                       uint32_t n, uint64_t rank_begin, uint64_t rank_end,
                       const bote_objective* objs, uint32_t n_obj, uint32_t K,
                       const bote_ranking_params* rp, int digest, uint32_t keys, bote_search** out);
int bote_search_launch(bote_search* h);
int bote_search_result(bote_search* h, bote_topk_record* out, uint32_t* out_count,
                       uint64_t* out_valid, uint64_t* out_digest);
/* The shard bounds chosen at creation: n_devices + 1 ascending ranks. */
int bote_search_bounds(const bote_search* h, uint64_t* out_bounds);
int bote_search_destroy(bote_search* h);
/* One-shot form: create + launch + result + destroy. */
int bote_search_topk(const bote_planet* const* planets, uint32_t n_devices,
                     const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                     uint32_t n, uint64_t rank_begin, uint64_t rank_end,
                     const bote_objective* objs, uint32_t n_obj, uint32_t K,
                     const bote_ranking_params* rp, int digest, bote_topk_record* out,
                     uint32_t* out_count, uint64_t* out_valid, uint64_t* out_digest);

/* colex unrank helper (host): rank -> n ascending positions < ns. */
int bote_colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out_positions);
/* C(ns, n) as uint64 (0 on overflow or n > ns). */
uint64_t bote_binomial(uint32_t ns, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* BOTE_HIP_H */
