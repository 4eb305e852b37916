// bote_kernels.hpp — launch interface between the C ABI (bote_capi.hip) and
// the gfx950 kernels (bote_kernels.hip).
#pragma once
#include "bote_device.hpp"

namespace bote {

constexpr int NSLOT = 10;
constexpr int G_MERGE_LISTS = 8;  // lists merged per workgroup
enum { SLOT_AF1 = 0, SLOT_FF1 = 1, SLOT_AF2 = 2, SLOT_FF2 = 3, SLOT_E = 4 };
enum { OBJ_SCORE = 0, OBJ_MEAN = 1, OBJ_COV = 2 };

struct EvalArgs {
  // planet (device): latency << 4, row = from
  const uint32_t* mat;
  uint32_t R;
  // server list (region ids; positions index it) and client list
  const uint32_t* srv;
  uint32_t ns;
  const uint32_t* cli;
  uint32_t nc;
  int srv_sorted;  // srv ascending => colex positions are already in name order
  // work: explicit configs (positions, n per config) or colex ranks
  const uint32_t* cfgs;
  // or an explicit device list of colex ranks whose length is read on the
  // device (the fast sweep's deferred near-tie configs): [0, *rank_count)
  const uint64_t* rank_list;
  const unsigned long long* rank_count;
  uint64_t rb, re;  // [rb, re) ranks, or config indices when cfgs != null
  uint32_t runlen;  // consecutive ranks per lane job
  const uint64_t* binom;  // (ns+1) x (n+1)
  // ranking params (compute_score)
  int want_score;
  double p_fmean, p_emean, p_fair;
  int ft_metric;
  // key set: 0 compute_stats' 10 slots; 1 the extended key set (slots
  // 10..19 and every leader's FPaxos moments; include/bote_hip.h)
  uint32_t keys;
  // FULL outputs (moments: NSLOT or, with keys, NSLOT_X per config)
  uint32_t* out_vals;
  uint32_t* out_leader;
  uint64_t* out_s1;
  uint64_t* out_s2;
  double* out_mean;
  double* out_cov;
  double* out_score;
  uint8_t* out_valid;
  uint64_t* out_al_s1;  // keys: ncfg x 2 x n, all leaders (f = 1, 2; config order)
  uint64_t* out_al_s2;
  // TOP-K outputs
  int n_obj;
  uint32_t obj_kind[MAXOBJ];
  uint32_t obj_slot[MAXOBJ];
  uint32_t K;
  Rec* out_top;                      // [grid][n_obj][KP]
  unsigned long long* out_counters;  // [0] valid count, [1] digest
  int want_digest;
  // overflow fallback of the fast sweep: when set, every block exits at once
  // unless *run_if_over > over_cap (the deferred-rank queue overflowed), so the
  // fallback is stream-ordered with no host round trip
  const unsigned long long* run_if_over;
  uint64_t over_cap;
};

struct SingleArgs {
  const uint32_t* mat;  // latency << 4
  uint32_t R;
  const uint32_t* servers;
  uint32_t ns;
  const uint32_t* clients;
  uint32_t nc;
  const uint32_t* froms;
  uint32_t nf;
  uint32_t q;
  uint32_t leader;
  int stat;
  uint64_t* out;
  uint32_t* out_pos;
  int* err;
};

// ---- fast-path sweep (bote_sweep.hip)
constexpr uint32_t FAST_BD = 256;
struct FastArgs {
  const uint2* cqt;  // client quads, column-major, column stride cq_stride uint2 (quad_stride)
  const uint2* rqt;  // region quads (rows = all regions), used when rq_separate
  int rq_separate;
  uint32_t R, cq_quads, rq_quads;
  uint32_t cq_stride, rq_stride;  // quads per column (>= quads + 1; an odd number of 16-B units)
  const uint32_t* srv;
  uint32_t ns;
  int srv_identity;  // srv[p] == p
  uint32_t nc;
  const uint64_t* binom;
  uint64_t rb, re;
  uint32_t runlen;
  uint32_t s2_flush;  // quads per 32-bit sum-of-squares chunk
  uint32_t g_flush;   // group kernel: quads per flush of its 32-bit square sums and packed-u16 sums
  uint32_t k_flush;   // group kernel, extended keys: quads per flush of its 32-bit sum of squared keys
  uint32_t gbd;       // group kernel: workgroup size (multiple of 64, <= 1024)
  uint32_t gqsh;      // group kernel: log2 of the qtab plane stride in bytes (1 << gqsh >= gbd * 4)
  uint32_t gslots;    // group kernel, n <= 7: client lines per wave (0: none), see bote_group.hip
  uint32_t grx;       // group kernel, n <= 7: per-group position table (1) or per-lane row sorts (0)
  uint32_t keys;      // group kernel: 1 = the extended key set (n = 4..7, default objectives first)
  uint32_t gbins;     // group kernel, base key set: the member-binned client loop (bote_group.hip BN)
  uint32_t s32;       // every sum of squares of a slot fits 32 bits (nc (2 max)^2 < 2^32): the SI group kernels keep them in 32 bits
  uint32_t v32;       // and every V = cnt s2 - s1^2 (cnt^2 (2 max)^2 < 2^32)
  // group kernel work distribution: nwchunks > 0: waves take cost-balanced
  // rank chunks [wchunks[c], wchunks[c+1]) from ticket counters (zeroed
  // before each launch); 0: each wave sweeps an equal share of ranks.  The
  // counter is sharded wshards ways (one 128-B line each, wctr[32 * x]):
  // blocks b with b % wshards == x take chunks x, x + wshards, ... (one
  // device-scope word saturates near 90 tickets per us, MI355X_MICROARCH.md)
  const uint64_t* wchunks;
  uint32_t nwchunks;
  unsigned int* wctr;
  uint32_t wshards;
  // per chunk, 4 u64: the colex rank of its first group's fixed positions,
  // then those positions as bytes (16 at most); null: unranked on the device
  const uint64_t* wstate;
  // top-K seed (bote_capi.hip launch_fast_path): the sample launch (smin
  // non-null) takes nwchunks chunks of ssteps steps at wchunks[c] and records, per
  // objective o, the least key of chunk c at smin[o * nwchunks + c] (no lists,
  // counters or deferrals); seed_kernel turns those into tseed[o], the K-th
  // least, a bound on the launch's K-th key that the main launch starts its
  // thresholds at
  // With smin_wave, the slot is the wave's (o * waves + wave, the least key
  // of the chunks it took): as many slots as waves, not chunks, for the seed
  // kernel to select from (K slots <= x are still K distinct configs <= x).
  uint64_t* smin;
  const uint64_t* tseed;
  uint32_t ssteps;  // sample launch: steps (of 64 configs) per sample chunk
  uint32_t smin_wave;
  // kbound (non-null: the one-launch merge follows): per objective the least
  // K-th key over the blocks' full lists (atomicMin at the list dump, reset by
  // zero_ctl); a block then writes only its records with keys <= that bound,
  // then a rec_max terminator, instead of n_obj x KP records
  unsigned long long* kbound;
  int want_score, p_int;
  int64_t p1i, p2i;  // p_int: min_mean_{fpaxos,epaxos}_improv * nc as integers
  // group kernel mean tests on D = the integer difference of two sums: true
  // above hi, false below lo, the reference's f64 arithmetic in [lo, hi]
  // (lo = hi = p1i when p_int; otherwise floor/ceil of p * nc -/+ 1)
  int32_t m1_lo, m1_hi, m2_lo, m2_hi;
  double p_fmean, p_emean;
  int ft_metric;
  int n_obj;
  uint32_t obj_kind[MAXOBJ];
  uint32_t obj_slot[MAXOBJ];
  uint32_t K;
  Rec* out_top;
  unsigned long long* out_counters;
  int want_digest;
  // group kernel (bote_group.hip): packed (p0 | p1 << 8 | p2 << 16) of the
  // 3-subsets of positions in colex order (the low part of a group's ranks)
  const uint32_t* lowtab;
  uint64_t* queue;  // deferred near-tie configs (colex ranks)
  unsigned long long* queue_count;
  uint64_t queue_cap;
#ifdef BOTE_DEBUG
  // Device-assert builds only (scripts/build_variant.sh debug -DBOTE_DEBUG):
  // failed bounds checks set bits in *dbg_flag (soft asserts: no trap, the
  // kernel keeps running) and bote_sweep_result reports BOTE_E_DEVICE.
  unsigned int* dbg_flag;
  uint64_t lowtab_n;  // entries of lowtab
#endif
#ifdef BOTE_PATHSTATS
  // Path-statistics builds only (scripts/build_variant.sh pstats -DBOTE_PATHSTATS,
  // scripts/pathstats.py): per wave-step, how often each rare path of the group
  // kernel runs for the wavefront (any lane taking it), 64 counters
  unsigned long long* pstats;
#endif
#ifdef BOTE_ABLATION
  // Timing-diagnostics builds only (scripts/build_variant.sh NAME -DBOTE_ABLATION,
  // env BOTE_ABLATE; results are wrong when set).  The product library is
  // compiled without it: ABLATE() is the constant false there.
  // 1 skip client loop, 2 skip Q phase, 4 skip top-K step, 8 skip score, 16 skip digest;
  // group kernel: 32 skip variable-row sorts, 64 skip fixed-row insertions,
  // 128 skip leader selection, 256 skip validity, 512 skip colocated FPaxos
  uint32_t ablate;
#endif
};
#ifdef BOTE_DEBUG
// bit `code` of *dbg_flag when `cond` fails (codes: DESIGN.md §5, debug build)
#define GASSERT(a, cond, code)                                                    \
  do {                                                                            \
    if (!(cond)) atomicOr((a).dbg_flag, 1u << (code));                            \
  } while (0)
#else
#define GASSERT(a, cond, code) \
  do {                         \
  } while (0)
#endif
#ifdef BOTE_PATHSTATS
// counter k += 1 when any active lane of the wavefront has `cond` (one lane adds)
#define PSTAT(a, k, cond)                                                                        \
  do {                                                                                           \
    const unsigned long long pm_ = __ballot(cond), pa_ = __ballot(1);                            \
    if (pm_ && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(pa_)) atomicAdd(&(a).pstats[k], 1ull); \
  } while (0)
#else
#define PSTAT(a, k, cond) \
  do {                    \
  } while (0)
#endif
#ifdef BOTE_ABLATION
#define ABLATE(a, bit) (((a).ablate & (bit)) != 0)
#else
#define ABLATE(a, bit) false
#endif
size_t fast_smem_bytes(const FastArgs& a, uint32_t n);
int fast_occupancy(uint32_t n, size_t shm);
// (e0, e1: events carried by the dispatch itself, hipExtLaunchKernelGGL, for a timed launch)
hipError_t launch_fast(const FastArgs& a, uint32_t n, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0 = nullptr,
                       hipEvent_t e1 = nullptr);
size_t group_smem_bytes(const FastArgs& a, uint32_t n);
bool group_uses_lines(uint32_t n);  // n <= 7: client lines (FastArgs::gslots) and register lookups
// the extended key set's group kernels target BOTE_GROUP_WAVES_XK waves per
// SIMD and are bounded to workgroups of that many waves per SIMD
// (GROUP_XK_MAX_BD); the capi's eligibility probe and its geometry loop share
// it. 4 (128 VGPRs, 404 B/lane scratch) beats 3 (168 VGPRs, 252 B/lane) on
// config 5: 186.1 / 185.8 ms vs 198.3 / 197.9 ms kernel, same valid count and
// digest (profiles/r05r: DESIGN.md §5)
#ifndef BOTE_GROUP_WAVES_XK
#define BOTE_GROUP_WAVES_XK 4
#endif
constexpr uint32_t GROUP_XK_MAX_BD = 256 * BOTE_GROUP_WAVES_XK;
bool group_supports_keys(uint32_t n, uint32_t bd);  // the extended key set on the group kernel (n = 4..7, bd <= GROUP_XK_MAX_BD)
// workgroups per CU of the kernel instantiation launch_group runs for `a`
// (workgroup size a.gbd)
int group_occupancy(const FastArgs& a, uint32_t n, size_t shm, bool def_objectives);
hipError_t launch_group(const FastArgs& a, uint32_t n, bool def_objectives, uint32_t grid, size_t shm, hipStream_t st,
                        hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

size_t eval_smem_bytes(const EvalArgs& a, uint32_t n, uint32_t bd, bool topk);
int eval_occupancy(uint32_t n, bool full, uint32_t bd, size_t shm, bool keys = false);
hipError_t launch_eval(const EvalArgs& a, uint32_t n, bool full, uint32_t grid, uint32_t bd, size_t shm,
                       hipStream_t st);
hipError_t launch_merge(const Rec* src, uint32_t n_lists, uint64_t list_stride, Rec* dst, uint64_t out_stride,
                        uint32_t n_obj, hipStream_t st);
// Merge whose input is chosen on the device: `alt` (alt_lists lists) when
// *sel > cap, else `src` (n_lists lists).
constexpr uint32_t WIDE_MERGE_LISTS = 4096;
// one launch for a sweep's block lists (<= WIDE_MERGE_LISTS lists): the K least per
// objective into dst[o * KP] (sel/alt/cap: the overflow fallback's choice)
// csrc/calt/cdst: the counters (valid, digest) copied to cdst by the same
// device choice (sel) as the lists, as launch_pick_counters does
hipError_t launch_merge_wide(const Rec* src, uint32_t n_lists, const Rec* alt, uint32_t alt_lists, uint64_t list_stride,
                             const unsigned long long* sel, uint64_t cap, const unsigned long long* kbound, Rec* dst,
                             uint32_t n_obj, uint32_t K, const unsigned long long* csrc, const unsigned long long* calt,
                             uint64_t* cdst, hipStream_t st);
hipError_t launch_merge_sel(const Rec* src, uint32_t n_lists, const Rec* alt, uint32_t alt_lists, uint64_t list_stride,
                            const unsigned long long* sel, uint64_t cap, Rec* dst, uint64_t out_stride, uint32_t n_obj,
                            hipStream_t st);
// dst[0..1] = (*sel > cap ? alt : src)[0..1]
hipError_t launch_zero_ctl(unsigned long long* counters, unsigned long long* qcount, unsigned int* wctr,
                           unsigned long long* counters_alt, unsigned long long* kbound, hipStream_t st);
hipError_t launch_seed(const uint64_t* smin, uint32_t nsamp, uint32_t n_obj, uint32_t K, uint64_t* tseed,
                       hipStream_t st);
hipError_t launch_pick_counters(const unsigned long long* src, const unsigned long long* alt,
                                const unsigned long long* sel, uint64_t cap, uint64_t* dst, hipStream_t st);

hipError_t launch_sum_counters(const uint64_t* src, uint32_t n, uint64_t stride, uint64_t off, uint64_t* dst,
                               hipStream_t st);
// ---- leaderless latencies for several quorum sizes (bote_quorums.hip)
struct LqArgs {
  const uint32_t* mat;  // latency << 4
  uint32_t R;
  const uint32_t* srv;
  uint32_t ns;
  const uint32_t* cli;
  uint32_t nc;
  const uint32_t* cfgs;  // ncfg x n positions, or null (colex ranks from rank_begin)
  const uint64_t* binom;
  uint64_t rank_begin, ncfg;
  const uint32_t* qs;  // nq quorum sizes, each in [1, n]
  uint32_t nq;
  uint32_t* out_vals;   // ncfg x nq x (nc + n)
  uint64_t* out_sum;    // ncfg x nq x 2 (Input, Colocated)
  uint64_t* out_sumsq;  // ncfg x nq x 2
};
size_t lq_smem_bytes(const LqArgs& a, uint32_t n);
hipError_t launch_leaderless_q(const LqArgs& a, uint32_t n, uint32_t grid, size_t shm, hipStream_t st);

// ---- Search::sorted_evolving_configs on the device (bote_chain.hip)
struct ChainHostLevel {
  uint32_t cnt, n;
  const uint64_t* mask;
  const double* score;
  const double* mean;
};
hipError_t chain_search(const ChainHostLevel* lv, uint32_t ns, int ft_metric, double min_dec, uint64_t max_out,
                        uint32_t* out_idx, double* out_score, uint64_t* out_total, hipStream_t st, int* too_many);

hipError_t launch_single(const SingleArgs& a, int mode, hipStream_t st);
hipError_t launch_best_leader(const SingleArgs& a, const uint64_t* vals, double* stat, hipStream_t st);

}  // namespace bote
