// bote_capi.hip — C ABI (include/bote_hip.h) over the gfx950 kernels.
//
// Host responsibilities only: argument validation (the reference panics, we
// return BOTE_E_* codes), device buffers, launch geometry and the merge chain.
// Every computation of latencies, quorums, leaders, histograms moments, scores
// and top-K selection runs on the device (bote_kernels.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <map>
#include <memory>
#include <vector>

#include "../../include/bote_hip.h"
#include "bote_host.hpp"
#include "bote_kernels.hpp"

using bote::EvalArgs;
using bote::Rec;
using bote::SingleArgs;

using namespace bote::host;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return fail(BOTE_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// RAII device buffer; reserve() grows it (grow-only, for cached workspaces)
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) {
    cap = bytes ? bytes : 16;
    return hipMalloc(&p, cap);
  }
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    const size_t old = cap;  // grow geometrically: a slightly larger call does not reallocate again
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    return alloc(std::max(bytes, 2 * old));
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

int check_regions(const uint32_t* ids, uint32_t n, uint32_t R, bool distinct, const char* what) {
  if (n && !ids) return fail(BOTE_E_ARG, std::string(what) + " is null");
  std::vector<uint8_t> seen(R, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (ids[i] >= R) return fail(BOTE_E_ARG, std::string(what) + ": region id out of range");
    if (distinct && seen[ids[i]]++) return fail(BOTE_E_ARG, std::string(what) + ": duplicate region");
  }
  return BOTE_OK;
}

uint32_t distinct_count(const uint32_t* ids, uint32_t n, uint32_t R) {
  std::vector<uint8_t> seen(R, 0);
  uint32_t c = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!seen[ids[i]]++) ++c;
  return c;
}

int device_cus(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
  return prop.multiProcessorCount;
}

size_t device_max_lds(int dev) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || v <= 0)
    return 160 * 1024;
  return (size_t)std::max(v, 160 * 1024);
}

}  // namespace

// A planet resident on one device.  The per-call entry points (bote_eval,
// bote_leaderless, ...) run stream-ordered on the planet's own non-blocking
// stream with cached, grow-only device workspaces; calls on one handle are
// serialised by its mutex, calls on distinct handles are independent (no
// device-wide synchronisation anywhere).
struct bote_planet {
  int device;
  uint32_t R;
  std::vector<uint16_t> lat;
  uint32_t* d_mat = nullptr;
  hipStream_t stream = nullptr;
  mutable std::mutex mu;
  mutable DBuf ws[14];
};

struct bote_sweep {
  const bote_planet* p = nullptr;
  uint32_t n = 0, ns = 0, nc = 0, n_obj = 0, K = 0;
  EvalArgs args{};
  uint32_t grid = 0, bd = 0;
  size_t shm = 0;
  DBuf srv, cli, binom, top, tmp0, tmp1, result, counters;
  // overflow fallback of the fast path (generic kernel over the whole range,
  // run only when the deferred queue overflowed; chosen on the device)
  DBuf top_alt, counters_alt;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t last0 = nullptr, last1 = nullptr;  // the last launch's kernel events (ev0/ev1 or a timing slot)
  // recorded after the last work enqueued on the sweep's buffers (a launch's
  // merge chain, a result copy): destroy waits on it, not on the device
  hipEvent_t done = nullptr;
  // per-launch kernel timing since the last bote_sweep_timing_reset
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evpool;
  size_t ev_used = 0;
  bool launched = false;
  // fast path (bote_sweep.hip) + exact fixup of its deferred configs
  bool fast = false;
  bool group = false;  // fast path runs the group kernel (bote_group.hip)
  bool def_obj = false;  // the default objective set, compiled into the group kernel
  bote::FastArgs fargs{};
  uint32_t fgrid = 0;
  size_t fshm = 0;
  uint32_t xgrid = 0;  // generic fixup grid (deferred configs)
  DBuf cqt, rqt, queue, qcount, lowtab;
  DBuf dbg;  // BOTE_DEBUG builds: device-assert flag bits
  DBuf pstats;  // BOTE_PATHSTATS builds: 64 path counters (group kernel)
  // group kernel work chunks per launch range (cached: a bench or a shard
  // re-launches the same range), plus the ticket counter
  struct Chunks {
    std::vector<uint64_t> host;   // kept alive: the async upload reads it
    std::vector<uint64_t> state;  // per chunk: FastArgs::wstate (4 u64)
    DBuf dev, sdev;
    uint32_t n = 0;
  };
  std::map<std::pair<uint64_t, uint64_t>, std::unique_ptr<Chunks>> chunks;
  // top-K seed: the sample launch's one-step chunks per launch range (same
  // layout: starts in host/dev, FastArgs::wstate in state/sdev), its per-chunk
  // minima and the seed keys
  std::map<std::pair<uint64_t, uint64_t>, std::unique_ptr<Chunks>> samples;
  DBuf smin, tseed;
  DBuf kbound;  // group lists' K-th key bound (FastArgs::kbound)
  // host walks of the groups (bote_host.hpp): one walk serves the split and
  // the chunk tables of every sub-range it covers (bote_search_* shares one
  // walk across its shards' sweeps)
  mutable std::vector<std::shared_ptr<const GroupWalk>> walks;
  DBuf wctr;
  uint64_t last_rb = 0, last_re = 0;
  hipStream_t last_stream = nullptr;
  uint64_t result_bytes() const { return (uint64_t)n_obj * bote::KP * 16 + 16; }
};

namespace {
constexpr uint64_t QUEUE_CAP = 1ull << 20;  // deferred near-tie configs per launch

#ifndef BOTE_CHUNKS_PER_WAVE
#define BOTE_CHUNKS_PER_WAVE 32
#endif
}  // namespace

// Restores the calling thread's current HIP device when an entry returns:
// the entries switch to their planet's device, and the library must not
// leave the caller (a Rust or PyTorch host on another device) switched.
struct DevGuard {
  int dev = -1;
  DevGuard() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DevGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
  DevGuard(const DevGuard&) = delete;
  DevGuard& operator=(const DevGuard&) = delete;
};

extern "C" {

const char* bote_last_error(void) { return g_err.c_str(); }

int bote_device_count(int* out) {
  if (!out) return fail(BOTE_E_ARG, "out is null");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *out = c;
  return BOTE_OK;
}

// ------------------------------------------------------------------ planet
int bote_planet_create(const uint16_t* lat, uint32_t R, int device, bote_planet** out) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!lat || !out) return fail(BOTE_E_ARG, "null argument");
  if (R == 0 || R > BOTE_MAX_REGIONS) return fail(BOTE_E_RANGE, "R must be in [1, 128]");
  for (size_t i = 0; i < (size_t)R * R; ++i)
    if (lat[i] > BOTE_MAX_LATENCY) return fail(BOTE_E_RANGE, "latency above 16383");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(BOTE_E_NODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(BOTE_E_ARG, "device out of range");
  HIP_TRY(hipSetDevice(device));
  auto* p = new bote_planet();
  p->device = device;
  p->R = R;
  p->lat.assign(lat, lat + (size_t)R * R);
  std::vector<uint32_t> m((size_t)R * R);
  for (size_t i = 0; i < m.size(); ++i) m[i] = (uint32_t)lat[i] << bote::LAT_SHIFT;
  if (hipMalloc(&p->d_mat, m.size() * 4) != hipSuccess) {
    delete p;
    return fail(BOTE_E_NOMEM, "hipMalloc planet");
  }
  if (hipMemcpy(p->d_mat, m.data(), m.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipFree(p->d_mat);
    delete p;
    return fail(BOTE_E_DEVICE, "upload planet / create its stream");
  }
  *out = p;
  return BOTE_OK;
}

int bote_planet_destroy(bote_planet* p) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!p) return BOTE_OK;
  (void)hipSetDevice(p->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  if (p->d_mat) (void)hipFree(p->d_mat);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
  return BOTE_OK;
}

int bote_planet_regions(const bote_planet* p, uint32_t* out_R) {
  if (!p || !out_R) return fail(BOTE_E_ARG, "null argument");
  *out_R = p->R;
  return BOTE_OK;
}

// ---------------------------------------------------------------- protocol
int bote_quorum_size(int protocol, uint32_t n, uint32_t f) {
  switch (protocol) {
    case BOTE_FPAXOS: return (int)(f + 1);
    case BOTE_EPAXOS: { uint32_t m = n / 2; return (int)(m + (m + 1) / 2); }
    case BOTE_ATLAS: return (int)(n / 2 + f);
    case BOTE_TEMPO: return (int)(n / 2 + f);
    case BOTE_TEMPO_TINY: return (int)(2 * f);
    default: return fail(BOTE_E_ARG, "unknown protocol");
  }
}

uint32_t bote_max_f(uint32_t n) { return std::min(n / 2, 2u); }

uint64_t bote_binomial(uint32_t ns, uint32_t n) { return binom_u64(ns, n); }

int bote_colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out) {
  if (!out || n > ns) return fail(BOTE_E_ARG, "bad unrank arguments");
  if (!colex_unrank(rank, n, ns, out)) return fail(BOTE_E_ARG, "rank out of range");
  return BOTE_OK;
}

// --------------------------------------------------- single configuration
// least client count for the member-binned loop on the base key set (a build
// knob for A/B timing builds only; scripts/build_variant.sh)
#ifndef BOTE_GBINS_MIN_NC
#define BOTE_GBINS_MIN_NC 32
#endif

static int run_single(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                      const uint32_t* froms, uint32_t nf, uint32_t q, uint32_t leader, int mode, uint64_t* out,
                      size_t nout) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!p || !out) return fail(BOTE_E_ARG, "null argument");
  int rc;
  if ((rc = check_regions(servers, ns, p->R, false, "servers"))) return rc;
  if ((rc = check_regions(clients, nc, p->R, false, "clients"))) return rc;
  if ((rc = check_regions(froms, nf, p->R, false, "froms"))) return rc;
  if (mode == 2 && leader >= p->R) return fail(BOTE_E_ARG, "leader out of range");
  if (q == 0) return fail(BOTE_E_ARG, "quorum size 0");
  if (q > distinct_count(servers, ns, p->R)) return fail(BOTE_E_QUORUM_GT_N, "quorum larger than the server set");
  std::lock_guard<std::mutex> lk(p->mu);
  HIP_TRY(hipSetDevice(p->device));
  hipStream_t st = p->stream;
  DBuf &ds = p->ws[0], &dc = p->ws[1], &df = p->ws[2], &dout = p->ws[3];
  HIP_TRY(ds.reserve(ns * 4));
  HIP_TRY(dc.reserve(nc * 4));
  HIP_TRY(df.reserve(nf * 4));
  HIP_TRY(dout.reserve(nout * 8));
  if (ns) HIP_TRY(hipMemcpyAsync(ds.p, servers, ns * 4, hipMemcpyHostToDevice, st));
  if (nc) HIP_TRY(hipMemcpyAsync(dc.p, clients, nc * 4, hipMemcpyHostToDevice, st));
  if (nf) HIP_TRY(hipMemcpyAsync(df.p, froms, nf * 4, hipMemcpyHostToDevice, st));
  SingleArgs a{};
  a.mat = p->d_mat;
  a.R = p->R;
  a.servers = ds.as<uint32_t>();
  a.ns = ns;
  a.clients = dc.as<uint32_t>();
  a.nc = nc;
  a.froms = df.as<uint32_t>();
  a.nf = nf;
  a.q = q;
  a.leader = leader;
  a.out = dout.as<uint64_t>();
  HIP_TRY(bote::launch_single(a, mode, st));
  if (nout) HIP_TRY(hipMemcpyAsync(out, dout.p, nout * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return BOTE_OK;
}

int bote_quorum_latencies(const bote_planet* p, const uint32_t* froms, uint32_t nf, const uint32_t* regions,
                          uint32_t nr, uint32_t q, uint64_t* out) {
  return run_single(p, regions, nr, nullptr, 0, froms, nf, q, 0, 0, out, nf);
}

int bote_leaderless(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                    uint32_t q, uint64_t* out) {
  return run_single(p, servers, ns, clients, nc, nullptr, 0, q, 0, 1, out, nc);
}

int bote_leader(const bote_planet* p, uint32_t leader, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                uint32_t nc, uint32_t q, uint64_t* out) {
  return run_single(p, servers, ns, clients, nc, nullptr, 0, q, leader, 2, out, nc);
}

int bote_all_leaders(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                     uint32_t q, uint64_t* out) {
  return run_single(p, servers, ns, clients, nc, nullptr, 0, q, 0, 3, out, (size_t)ns * nc);
}

int bote_best_leader(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                     uint32_t q, int stat, uint32_t* out_pos, uint64_t* out_lat) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!p || !out_pos) return fail(BOTE_E_ARG, "null argument");
  if (ns == 0) return fail(BOTE_E_ARG, "the best leader should exist (empty server list)");
  if (stat < 0 || stat > 2) return fail(BOTE_E_ARG, "unknown stat");
  int rc;
  if ((rc = check_regions(servers, ns, p->R, false, "servers"))) return rc;
  if ((rc = check_regions(clients, nc, p->R, false, "clients"))) return rc;
  if (q == 0) return fail(BOTE_E_ARG, "quorum size 0");
  if (q > distinct_count(servers, ns, p->R)) return fail(BOTE_E_QUORUM_GT_N, "quorum larger than the server set");
  std::lock_guard<std::mutex> lk(p->mu);
  HIP_TRY(hipSetDevice(p->device));
  hipStream_t st = p->stream;
  DBuf &ds = p->ws[0], &dc = p->ws[1], &dv = p->ws[2], &dstat = p->ws[3], &dpos = p->ws[4];
  HIP_TRY(ds.reserve(ns * 4));
  HIP_TRY(dc.reserve(nc * 4));
  HIP_TRY(dv.reserve((size_t)ns * nc * 8));
  HIP_TRY(dstat.reserve(ns * 8));
  HIP_TRY(dpos.reserve(4));
  HIP_TRY(hipMemcpyAsync(ds.p, servers, ns * 4, hipMemcpyHostToDevice, st));
  if (nc) HIP_TRY(hipMemcpyAsync(dc.p, clients, nc * 4, hipMemcpyHostToDevice, st));
  SingleArgs a{};
  a.mat = p->d_mat;
  a.R = p->R;
  a.servers = ds.as<uint32_t>();
  a.ns = ns;
  a.clients = dc.as<uint32_t>();
  a.nc = nc;
  a.q = q;
  a.stat = stat;
  a.out = dv.as<uint64_t>();
  a.out_pos = dpos.as<uint32_t>();
  HIP_TRY(bote::launch_single(a, 3, st));
  HIP_TRY(bote::launch_best_leader(a, dv.as<uint64_t>(), dstat.as<double>(), st));
  HIP_TRY(hipMemcpyAsync(out_pos, dpos.p, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (out_lat && nc) {
    HIP_TRY(hipMemcpyAsync(out_lat, dv.as<uint64_t>() + (size_t)(*out_pos) * nc, nc * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  return BOTE_OK;
}

// ------------------------------------------------------- common validation
static int check_search_args(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                             uint32_t nc, uint32_t n) {
  if (!p) return fail(BOTE_E_ARG, "planet is null");
  if (n < 2) return fail(BOTE_E_QUORUM_GT_N, "config size must be >= 2 (FPaxos q = 2)");
  if (n > BOTE_MAX_N) return fail(BOTE_E_RANGE, "config size above 16");
  if (n > ns) return fail(BOTE_E_ARG, "config size larger than the server list");
  if (nc > BOTE_MAX_CLIENTS) return fail(BOTE_E_RANGE, "more than 4096 clients");
  int rc;
  if ((rc = check_regions(servers, ns, p->R, true, "servers"))) return rc;
  if ((rc = check_regions(clients, nc, p->R, false, "clients"))) return rc;
  return BOTE_OK;
}

static void fill_rank_params(EvalArgs& a, const bote_ranking_params* rp) {
  a.want_score = rp ? 1 : 0;
  if (rp) {
    a.p_fmean = rp->min_mean_fpaxos_improv;
    a.p_emean = rp->min_mean_epaxos_improv;
    a.p_fair = rp->min_fairness_fpaxos_improv;
    a.ft_metric = rp->ft_metric;
  }
}

// ------------------------------------------------------------------- eval
static int eval_impl(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                     uint32_t nc, uint32_t n, const uint32_t* configs, uint64_t rank_begin, uint64_t ncfg,
                     const bote_ranking_params* rp, uint32_t keys, uint32_t* out_vals, uint32_t* out_leader,
                     uint64_t* out_sum, uint64_t* out_sumsq, double* out_mean, double* out_cov, double* out_score,
                     uint8_t* out_valid, uint64_t* out_al_sum, uint64_t* out_al_sumsq) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  int rc;
  if (keys > BOTE_KEYS_TEMPO_ALL_LEADERS) return fail(BOTE_E_ARG, "unknown key set");
  if ((rc = check_search_args(p, servers, ns, clients, nc, n))) return rc;
  if (rp && rp->ft_metric != BOTE_FT_F1 && rp->ft_metric != BOTE_FT_F1F2) return fail(BOTE_E_ARG, "bad ft_metric");
  if (ncfg == 0) return BOTE_OK;
  if (configs) {
    for (uint64_t i = 0; i < ncfg; ++i) {
      uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t j = 0; j < n; ++j) {
        uint32_t x = configs[i * n + j];
        if (x >= ns) return fail(BOTE_E_ARG, "config position out of range");
        if (seen[x >> 5] & (1u << (x & 31))) return fail(BOTE_E_ARG, "duplicate position in config");
        seen[x >> 5] |= 1u << (x & 31);
      }
    }
  } else {
    uint64_t total = binom_u64(ns, n);
    if (rank_begin > total || ncfg > total - rank_begin) return fail(BOTE_E_ARG, "rank range out of bounds");
  }
  std::lock_guard<std::mutex> lk(p->mu);
  HIP_TRY(hipSetDevice(p->device));
  hipStream_t st = p->stream;
  const size_t stride = 5ull * nc + 5ull * n;
  const size_t NS = keys ? BOTE_NSLOTS_X : bote::NSLOT;
  DBuf &ds = p->ws[0], &dc = p->ws[1], &dcfg = p->ws[2], &dbin = p->ws[3], &dvals = p->ws[4], &dlead = p->ws[5],
       &ds1 = p->ws[6], &ds2 = p->ws[7], &dmean = p->ws[8], &dcov = p->ws[9], &dscore = p->ws[10],
       &dvalid = p->ws[11], &dal1 = p->ws[12], &dal2 = p->ws[13];
  HIP_TRY(ds.reserve(ns * 4));
  HIP_TRY(dc.reserve(nc * 4));
  HIP_TRY(hipMemcpyAsync(ds.p, servers, ns * 4, hipMemcpyHostToDevice, st));
  if (nc) HIP_TRY(hipMemcpyAsync(dc.p, clients, nc * 4, hipMemcpyHostToDevice, st));
  EvalArgs a{};
  a.mat = p->d_mat;
  a.R = p->R;
  a.srv = ds.as<uint32_t>();
  a.ns = ns;
  a.cli = dc.as<uint32_t>();
  a.nc = nc;
  a.srv_sorted = std::is_sorted(servers, servers + ns) ? 1 : 0;
  std::vector<uint64_t> t;
  if (configs) {
    HIP_TRY(dcfg.reserve(ncfg * n * 4));
    HIP_TRY(hipMemcpyAsync(dcfg.p, configs, ncfg * n * 4, hipMemcpyHostToDevice, st));
    a.cfgs = dcfg.as<uint32_t>();
    a.rb = 0;
    a.re = ncfg;
  } else {
    t = binom_table(ns, n);
    HIP_TRY(dbin.reserve(t.size() * 8));
    HIP_TRY(hipMemcpyAsync(dbin.p, t.data(), t.size() * 8, hipMemcpyHostToDevice, st));
    a.binom = dbin.as<uint64_t>();
    a.rb = rank_begin;
    a.re = rank_begin + ncfg;
  }
  a.runlen = 1;
  a.keys = keys;
  fill_rank_params(a, rp);
  if (out_vals) { HIP_TRY(dvals.reserve(ncfg * stride * 4)); a.out_vals = dvals.as<uint32_t>(); }
  if (out_leader) { HIP_TRY(dlead.reserve(ncfg * 4)); a.out_leader = dlead.as<uint32_t>(); }
  if (out_sum) { HIP_TRY(ds1.reserve(ncfg * NS * 8)); a.out_s1 = ds1.as<uint64_t>(); }
  if (out_sumsq) { HIP_TRY(ds2.reserve(ncfg * NS * 8)); a.out_s2 = ds2.as<uint64_t>(); }
  if (out_mean) { HIP_TRY(dmean.reserve(ncfg * NS * 8)); a.out_mean = dmean.as<double>(); }
  if (out_cov) { HIP_TRY(dcov.reserve(ncfg * NS * 8)); a.out_cov = dcov.as<double>(); }
  const size_t nal = (size_t)ncfg * 2 * n;
  if (keys && out_al_sum) { HIP_TRY(dal1.reserve(nal * 8)); a.out_al_s1 = dal1.as<uint64_t>(); }
  if (keys && out_al_sumsq) { HIP_TRY(dal2.reserve(nal * 8)); a.out_al_s2 = dal2.as<uint64_t>(); }
  if (out_score && rp) { HIP_TRY(dscore.reserve(ncfg * 8)); a.out_score = dscore.as<double>(); }
  if (out_valid && rp) { HIP_TRY(dvalid.reserve(ncfg)); a.out_valid = dvalid.as<uint8_t>(); }

  const uint32_t bd = 256;
  size_t shm = bote::eval_smem_bytes(a, n, bd, false);
  if (shm > device_max_lds(p->device)) return fail(BOTE_E_RANGE, "planet/client set too large for LDS");
  int nb = bote::eval_occupancy(n, true, bd, shm, keys != 0);
  uint64_t want = (ncfg + bd - 1) / bd;
  uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)device_cus(p->device) * nb);
  HIP_TRY(bote::launch_eval(a, n, true, grid, bd, shm, st));
  const hipMemcpyKind D2H = hipMemcpyDeviceToHost;
  if (out_vals) HIP_TRY(hipMemcpyAsync(out_vals, dvals.p, ncfg * stride * 4, D2H, st));
  if (out_leader) HIP_TRY(hipMemcpyAsync(out_leader, dlead.p, ncfg * 4, D2H, st));
  if (out_sum) HIP_TRY(hipMemcpyAsync(out_sum, ds1.p, ncfg * NS * 8, D2H, st));
  if (out_sumsq) HIP_TRY(hipMemcpyAsync(out_sumsq, ds2.p, ncfg * NS * 8, D2H, st));
  if (out_mean) HIP_TRY(hipMemcpyAsync(out_mean, dmean.p, ncfg * NS * 8, D2H, st));
  if (out_cov) HIP_TRY(hipMemcpyAsync(out_cov, dcov.p, ncfg * NS * 8, D2H, st));
  if (keys && out_al_sum) HIP_TRY(hipMemcpyAsync(out_al_sum, dal1.p, nal * 8, D2H, st));
  if (keys && out_al_sumsq) HIP_TRY(hipMemcpyAsync(out_al_sumsq, dal2.p, nal * 8, D2H, st));
  if (out_score && rp) HIP_TRY(hipMemcpyAsync(out_score, dscore.p, ncfg * 8, D2H, st));
  if (out_valid && rp) HIP_TRY(hipMemcpyAsync(out_valid, dvalid.p, ncfg, D2H, st));
  HIP_TRY(hipStreamSynchronize(st));
  return BOTE_OK;
}

int bote_eval(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
              uint32_t n, const uint32_t* configs, uint64_t rank_begin, uint64_t ncfg, const bote_ranking_params* rp,
              uint32_t* out_vals, uint32_t* out_leader, uint64_t* out_sum, uint64_t* out_sumsq, double* out_mean,
              double* out_cov, double* out_score, uint8_t* out_valid) {
  return eval_impl(p, servers, ns, clients, nc, n, configs, rank_begin, ncfg, rp, 0, out_vals, out_leader, out_sum,
                   out_sumsq, out_mean, out_cov, out_score, out_valid, nullptr, nullptr);
}

int bote_eval_keys(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                   uint32_t n, const uint32_t* configs, uint64_t rank_begin, uint64_t ncfg, uint32_t keys,
                   uint32_t* out_leader, uint64_t* out_sum, uint64_t* out_sumsq, uint64_t* out_al_sum,
                   uint64_t* out_al_sumsq) {
  return eval_impl(p, servers, ns, clients, nc, n, configs, rank_begin, ncfg, nullptr, keys, nullptr, out_leader,
                   out_sum, out_sumsq, nullptr, nullptr, nullptr, nullptr, out_al_sum, out_al_sumsq);
}

// ------------------------------------------ leaderless, many quorum sizes
// Bote::leaderless (lib.rs:38-59) over a batch of configurations for each of
// `nq` quorum sizes: Tempo's fast (n/2 + f; tiny 2f) and write (f + 1)
// quorums (fantoch/src/config.rs:317-329), which compute_stats does not key.
int bote_eval_leaderless(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                         uint32_t nc, uint32_t n, const uint32_t* configs, uint64_t rank_begin, uint64_t ncfg,
                         const uint32_t* quorum_sizes, uint32_t nq, uint32_t* out_vals, uint64_t* out_sum,
                         uint64_t* out_sumsq) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  int rc;
  if (!p) return fail(BOTE_E_ARG, "planet is null");
  if (n < 1 || n > BOTE_MAX_N) return fail(BOTE_E_RANGE, "config size must be in [1, 16]");
  if (n > ns) return fail(BOTE_E_ARG, "config size larger than the server list");
  if (nc > BOTE_MAX_CLIENTS) return fail(BOTE_E_RANGE, "more than 4096 clients");
  if (nq == 0 || nq > 8 || !quorum_sizes) return fail(BOTE_E_ARG, "1 to 8 quorum sizes");
  for (uint32_t i = 0; i < nq; ++i) {
    if (quorum_sizes[i] == 0) return fail(BOTE_E_ARG, "quorum size 0");
    if (quorum_sizes[i] > n) return fail(BOTE_E_QUORUM_GT_N, "quorum larger than the config");
  }
  if ((rc = check_regions(servers, ns, p->R, true, "servers"))) return rc;
  if ((rc = check_regions(clients, nc, p->R, false, "clients"))) return rc;
  if (ncfg == 0) return BOTE_OK;
  if (configs) {
    for (uint64_t i = 0; i < ncfg; ++i) {
      uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t j = 0; j < n; ++j) {
        uint32_t x = configs[i * n + j];
        if (x >= ns) return fail(BOTE_E_ARG, "config position out of range");
        if (seen[x >> 5] & (1u << (x & 31))) return fail(BOTE_E_ARG, "duplicate position in config");
        seen[x >> 5] |= 1u << (x & 31);
      }
    }
  } else {
    uint64_t total = binom_u64(ns, n);
    if (rank_begin > total || ncfg > total - rank_begin) return fail(BOTE_E_ARG, "rank range out of bounds");
  }
  std::lock_guard<std::mutex> lk(p->mu);
  HIP_TRY(hipSetDevice(p->device));
  hipStream_t st = p->stream;
  DBuf &ds = p->ws[0], &dc = p->ws[1], &dcfg = p->ws[2], &dbin = p->ws[3], &dq = p->ws[4], &dvals = p->ws[5],
       &ds1 = p->ws[6], &ds2 = p->ws[7];
  HIP_TRY(ds.reserve(ns * 4));
  HIP_TRY(dc.reserve(nc * 4));
  HIP_TRY(dq.reserve(nq * 4));
  HIP_TRY(hipMemcpyAsync(ds.p, servers, ns * 4, hipMemcpyHostToDevice, st));
  if (nc) HIP_TRY(hipMemcpyAsync(dc.p, clients, nc * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(dq.p, quorum_sizes, nq * 4, hipMemcpyHostToDevice, st));
  bote::LqArgs a{};
  a.mat = p->d_mat;
  a.R = p->R;
  a.srv = ds.as<uint32_t>();
  a.ns = ns;
  a.cli = dc.as<uint32_t>();
  a.nc = nc;
  a.qs = dq.as<uint32_t>();
  a.nq = nq;
  a.ncfg = ncfg;
  std::vector<uint64_t> t;
  if (configs) {
    HIP_TRY(dcfg.reserve(ncfg * n * 4));
    HIP_TRY(hipMemcpyAsync(dcfg.p, configs, ncfg * n * 4, hipMemcpyHostToDevice, st));
    a.cfgs = dcfg.as<uint32_t>();
  } else {
    t = binom_table(ns, n);
    HIP_TRY(dbin.reserve(t.size() * 8));
    HIP_TRY(hipMemcpyAsync(dbin.p, t.data(), t.size() * 8, hipMemcpyHostToDevice, st));
    a.binom = dbin.as<uint64_t>();
    a.rank_begin = rank_begin;
  }
  const size_t nv = (size_t)ncfg * nq * (nc + n), nm = (size_t)ncfg * nq * 2;
  if (out_vals) { HIP_TRY(dvals.reserve(nv * 4)); a.out_vals = dvals.as<uint32_t>(); }
  if (out_sum) { HIP_TRY(ds1.reserve(nm * 8)); a.out_sum = ds1.as<uint64_t>(); }
  if (out_sumsq) { HIP_TRY(ds2.reserve(nm * 8)); a.out_sumsq = ds2.as<uint64_t>(); }
  const size_t shm = bote::lq_smem_bytes(a, n);
  if (shm > device_max_lds(p->device)) return fail(BOTE_E_RANGE, "planet/client set too large for LDS");
  const uint32_t grid = (uint32_t)std::min<uint64_t>((ncfg + 255) / 256, (uint64_t)device_cus(p->device) * 4);
  HIP_TRY(bote::launch_leaderless_q(a, n, grid, shm, st));
  if (out_vals) HIP_TRY(hipMemcpyAsync(out_vals, dvals.p, nv * 4, hipMemcpyDeviceToHost, st));
  if (out_sum) HIP_TRY(hipMemcpyAsync(out_sum, ds1.p, nm * 8, hipMemcpyDeviceToHost, st));
  if (out_sumsq) HIP_TRY(hipMemcpyAsync(out_sumsq, ds2.p, nm * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return BOTE_OK;
}

// ---------------------------------------- superset chains (ranking product)
int bote_evolving_chains(int device, uint32_t ns, const uint32_t* counts, const uint64_t* const* masks,
                         const double* const* scores, const double* const* means, double min_mean_decrease,
                         int ft_metric, uint64_t max_out, uint32_t* out_idx, double* out_score, uint64_t* out_total) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!counts || !masks || !scores || !means || !out_total) return fail(BOTE_E_ARG, "null argument");
  if (ns == 0 || ns > 64) return fail(BOTE_E_RANGE, "the server list must hold 1 to 64 regions");
  if (ft_metric != BOTE_FT_F1 && ft_metric != BOTE_FT_F1F2) return fail(BOTE_E_ARG, "bad ft_metric");
  if (max_out && (!out_idx || !out_score)) return fail(BOTE_E_ARG, "null output");
  bote::ChainHostLevel lv[6];
  for (int l = 0; l < 6; ++l) {
    const uint32_t n = 3 + 2 * l;
    if (counts[l] && (!masks[l] || !scores[l] || !means[l])) return fail(BOTE_E_ARG, "null level array");
    for (uint32_t i = 0; i < counts[l]; ++i) {
      const uint64_t m = masks[l][i];
      if ((uint32_t)__builtin_popcountll(m) != n || (ns < 64 && (m >> ns)))
        return fail(BOTE_E_ARG, "level mask is not an n-subset of the server list");
    }
    lv[l] = bote::ChainHostLevel{counts[l], n, masks[l], scores[l], means[l]};
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(BOTE_E_NODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(BOTE_E_ARG, "device out of range");
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int too_many = 0;
  hipError_t e = bote::chain_search(lv, ns, ft_metric, min_mean_decrease, max_out, out_idx, out_score, out_total, st,
                                    &too_many);
  (void)hipStreamDestroy(st);
  if (e != hipSuccess) return fail(BOTE_E_DEVICE, std::string("chain search: ") + hipGetErrorString(e));
  if (too_many) return fail(BOTE_E_RANGE, "more than 2^31 chain prefixes at one level");
  return BOTE_OK;
}

// ------------------------------------------------------------------ sweep
int bote_sweep_create(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                      uint32_t nc, uint32_t n, const bote_objective* objs, uint32_t n_obj, uint32_t K,
                      const bote_ranking_params* rp, int digest, bote_sweep** out) {
  return bote_sweep_create_ex(p, servers, ns, clients, nc, n, objs, n_obj, K, rp, digest, BOTE_KERNEL_AUTO, out);
}

int bote_sweep_create_ex(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                         uint32_t nc, uint32_t n, const bote_objective* objs, uint32_t n_obj, uint32_t K,
                         const bote_ranking_params* rp, int digest, int kernel, bote_sweep** out) {
  return bote_sweep_create_keys(p, servers, ns, clients, nc, n, objs, n_obj, K, rp, digest, kernel, 0, out);
}

// slot s exists for config size n (f = 2 keys need max_f >= 2); slots >= 10
// only with the extended key set
static bool slot_exists_n(uint32_t n, uint32_t slot, uint32_t keys) {
  const bool f2 = bote_max_f(n) >= 2;
  if (slot < 10) {
    const uint32_t b = slot % 5;
    return !((b == BOTE_SLOT_AF2 || b == BOTE_SLOT_FF2) && !f2);
  }
  if (!keys || slot >= BOTE_NSLOTS_X) return false;
  if (slot < 18) return (slot - 10) % 2 == 0 || f2;
  return slot == 18 || f2;
}

int bote_sweep_create_keys(const bote_planet* p, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                           uint32_t nc, uint32_t n, const bote_objective* objs, uint32_t n_obj, uint32_t K,
                           const bote_ranking_params* rp, int digest, int kernel, uint32_t keys, bote_sweep** out) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  int rc;
  if (!out) return fail(BOTE_E_ARG, "out is null");
  if (keys > BOTE_KEYS_TEMPO_ALL_LEADERS) return fail(BOTE_E_ARG, "unknown key set");
  if (kernel < BOTE_KERNEL_AUTO || kernel > BOTE_KERNEL_GROUP) return fail(BOTE_E_ARG, "unknown kernel path");
  if ((rc = check_search_args(p, servers, ns, clients, nc, n))) return rc;
  if (n_obj > BOTE_MAX_OBJECTIVES) return fail(BOTE_E_RANGE, "more than 8 objectives");
  if (n_obj && !objs) return fail(BOTE_E_ARG, "objectives null");
  if (K == 0 || K > BOTE_MAX_K) return fail(BOTE_E_RANGE, "K must be in [1, 128]");
  bool has_score = false;
  for (uint32_t o = 0; o < n_obj; ++o) {
    if (objs[o].kind > BOTE_OBJ_COV) return fail(BOTE_E_ARG, "unknown objective kind");
    if (objs[o].kind == BOTE_OBJ_SCORE) {
      has_score = true;
      continue;
    }
    if (objs[o].slot >= (keys ? BOTE_NSLOTS_X : BOTE_NSLOTS)) return fail(BOTE_E_ARG, "slot out of range");
    if (!slot_exists_n(n, objs[o].slot, keys)) return fail(BOTE_E_ARG, "slot does not exist for this n (max_f < 2)");
  }
  if (has_score && !rp) return fail(BOTE_E_ARG, "SCORE objective needs ranking params");
  if (rp && rp->ft_metric != BOTE_FT_F1 && rp->ft_metric != BOTE_FT_F1F2) return fail(BOTE_E_ARG, "bad ft_metric");
  HIP_TRY(hipSetDevice(p->device));
  auto* s = new bote_sweep();
  auto cleanup = [&](int code) {
    bote_sweep_destroy(s);
    return code;
  };
  s->p = p;
  s->n = n;
  s->ns = ns;
  s->nc = nc;
  s->n_obj = n_obj;
  s->K = K;
  EvalArgs& a = s->args;
  a = EvalArgs{};
  auto t = binom_table(ns, n);
  if (s->srv.alloc(ns * 4) != hipSuccess || s->cli.alloc(nc * 4) != hipSuccess ||
      s->binom.alloc(t.size() * 8) != hipSuccess || s->counters.alloc(16) != hipSuccess)
    return cleanup(fail(BOTE_E_NOMEM, "hipMalloc sweep lists"));
  if (hipMemcpy(s->srv.p, servers, ns * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (nc && hipMemcpy(s->cli.p, clients, nc * 4, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(s->binom.p, t.data(), t.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(BOTE_E_DEVICE, "upload sweep lists"));
  a.mat = p->d_mat;
  a.R = p->R;
  a.srv = s->srv.as<uint32_t>();
  a.ns = ns;
  a.cli = s->cli.as<uint32_t>();
  a.nc = nc;
  a.srv_sorted = std::is_sorted(servers, servers + ns) ? 1 : 0;
  a.binom = s->binom.as<uint64_t>();
  fill_rank_params(a, has_score ? rp : nullptr);
  a.n_obj = (int)n_obj;
  for (uint32_t o = 0; o < n_obj; ++o) {
    a.obj_kind[o] = objs[o].kind;
    a.obj_slot[o] = objs[o].slot;
  }
  a.K = K;
  a.want_digest = digest ? 1 : 0;
  a.keys = keys;
  a.out_counters = s->counters.as<unsigned long long>();

  s->bd = 256;
  a.out_top = (Rec*)1;  // sizing with top-K structures
  s->shm = bote::eval_smem_bytes(a, n, s->bd, true);
  a.out_top = nullptr;
  if (s->shm > device_max_lds(p->device)) return cleanup(fail(BOTE_E_RANGE, "planet/client set too large for LDS"));
  int nb = bote::eval_occupancy(n, false, s->bd, s->shm, keys != 0);
  s->grid = (uint32_t)(device_cus(p->device) * nb);
  s->xgrid = 32;

  // ---- fast path: quad layouts, column sums are computed on the device.
  // `kernel` forces a path (tests, A/B timing; every path is exact); AUTO:
  // the group kernel when eligible and >= 90 % lane utilisation.
  const bool fair = has_score && rp && rp->min_fairness_fpaxos_improv != 0.0;
  s->fast = fast_eligible(p->lat.data(), p->R, servers, ns, nc, fair) && kernel != BOTE_KERNEL_GENERIC;
  if (kernel != BOTE_KERNEL_AUTO && kernel != BOTE_KERNEL_GENERIC && !s->fast)
    return cleanup(fail(BOTE_E_ARG, "the fast/group kernel is not eligible for this planet and lists"));
  // the extended key set runs on the group kernel (n = 4..7, the default
  // objectives first) or on the generic kernel
  // (config 5's objective set, compiled into the group kernel: bote.py
  // CONFIG5_OBJECTIVES = the default five, MEAN tt1, MEAN tw2, MEAN fl1)
  bool keys_def = n_obj == 8 && has_score;
  static const uint32_t dkk[8] = {BOTE_OBJ_SCORE, BOTE_OBJ_MEAN, BOTE_OBJ_MEAN, BOTE_OBJ_COV,
                                  BOTE_OBJ_MEAN,  BOTE_OBJ_MEAN, BOTE_OBJ_MEAN, BOTE_OBJ_MEAN};
  static const uint32_t dss[8] = {0, BOTE_SLOT_AF1, BOTE_SLOT_FF1, BOTE_SLOT_AF1,
                                  BOTE_SLOT_E, BOTE_SLOT_TT1, BOTE_SLOT_TW2, BOTE_SLOT_FL1};
  for (uint32_t o = 0; keys_def && o < 8; ++o)
    keys_def = objs[o].kind == dkk[o] && (dkk[o] == BOTE_OBJ_SCORE || objs[o].slot == dss[o]);
  // (the group kernel's extended keys use 32-bit moments: every sum of
  // squares nc * (2 max)^2 and 3 nc max must fit their 32/24 bits)
  uint64_t maxlat_all = 0;
  for (auto v : p->lat) maxlat_all = std::max<uint64_t>(maxlat_all, v);
  // (and its member bins: a client count below 2^8, a sum of nc keys
  // (latency << 4 | member) below 2^24 and two squared keys below 2^32,
  // bote_group.hip)
  const bool keys32 = (uint64_t)nc * (2 * maxlat_all) * (2 * maxlat_all) < (1ull << 32) &&
                      (uint64_t)nc * maxlat_all < (1ull << 16) &&  // (packed member-pair bins)
                      3ull * nc * maxlat_all < (1ull << 24) && nc < 256 &&
                      (uint64_t)nc * (16 * maxlat_all + 15) < (1ull << 24) &&
                      2 * (16 * maxlat_all + 15) * (16 * maxlat_all + 15) < (1ull << 32);
  if (keys && s->fast &&
      (!bote::group_supports_keys(n, bote::GROUP_XK_MAX_BD) || !keys_def || !keys32 || kernel == BOTE_KERNEL_FAST)) {
    if (kernel == BOTE_KERNEL_FAST || kernel == BOTE_KERNEL_GROUP)
      return cleanup(fail(BOTE_E_ARG, "the extended key set runs on the group kernel (n = 4..7, config 5's "
                                      "objectives) or the generic kernel"));
    s->fast = false;
  }
  if (s->fast) {
    bote::FastArgs& f = s->fargs;
    f = bote::FastArgs{};
    std::vector<uint32_t> ident(p->R);
    for (uint32_t i = 0; i < p->R; ++i) ident[i] = i;
    bool cli_ident = nc == p->R && std::equal(clients, clients + nc, ident.begin());
    uint32_t cq_quads = 0, rq_quads = 0, cq_stride = 0, rq_stride = 0;
    auto cq = quad_layout(p->lat.data(), p->R, clients, nc, bote::LAT_SHIFT, cq_quads, cq_stride);
    std::vector<uint16_t> rq;
    if (!cli_ident) rq = quad_layout(p->lat.data(), p->R, ident.data(), p->R, bote::LAT_SHIFT, rq_quads, rq_stride);
    if (s->cqt.alloc(cq.size() * 2) != hipSuccess || (!cli_ident && s->rqt.alloc(rq.size() * 2) != hipSuccess) ||
        s->queue.alloc(QUEUE_CAP * 8) != hipSuccess || s->qcount.alloc(16) != hipSuccess)
      return cleanup(fail(BOTE_E_NOMEM, "hipMalloc fast-path buffers"));
    if (hipMemcpy(s->cqt.p, cq.data(), cq.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        (!cli_ident && hipMemcpy(s->rqt.p, rq.data(), rq.size() * 2, hipMemcpyHostToDevice) != hipSuccess))
      return cleanup(fail(BOTE_E_DEVICE, "upload fast-path layouts"));
    f.cqt = s->cqt.as<uint2>();
    f.rqt = cli_ident ? s->cqt.as<uint2>() : s->rqt.as<uint2>();
    f.rq_separate = cli_ident ? 0 : 1;
    f.R = p->R;
    f.cq_quads = cq_quads;
    f.rq_quads = cli_ident ? cq_quads : rq_quads;
    f.cq_stride = cq_stride;
    f.rq_stride = cli_ident ? cq_stride : rq_stride;
    f.srv = s->srv.as<uint32_t>();
    f.ns = ns;
    f.keys = keys;
    f.srv_identity = 1;
    for (uint32_t i = 0; i < ns; ++i) f.srv_identity &= servers[i] == i;
    f.nc = nc;
    f.binom = s->binom.as<uint64_t>();
    uint32_t maxlat = 0;
    for (auto v : p->lat) maxlat = std::max<uint32_t>(maxlat, v);
    const uint64_t amax = 2ull * maxlat, per_quad = 4 * amax * amax;
    f.s2_flush = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, per_quad ? 0xFFFFFFFFull / per_quad : 1u << 20));
    // packed-u16 sums (group kernel): each half gains <= 2 * amax per quad
    const uint64_t s1_flush = amax ? 0xFFFFull / (2 * amax) : 1u << 20;
    f.g_flush = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(f.s2_flush, s1_flush));
    // extended keys: squares of the packed keys (latency << 4 | member), two
    // per dot2 into 32 bits (keys32 below requires 2 key^2 < 2^32)
    const uint64_t kmax = 16ull * maxlat + 15, kq = 4 * kmax * kmax;
    f.k_flush = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, 0xFFFFFFFFull / kq));
    // every slot's sum of squares below 2^32 (a value is at most a latency
    // plus a quorum latency, 2 max, over nc >= N clients): the bench-shaped
    // group kernels keep the moments in 32 bits (bote_group.hip S32)
    // (and the FPaxos moments' 24-bit multiplies: column sum + S1 <= 3 nc max < 2^24)
    f.s32 = (uint64_t)std::max(nc, n) * amax * amax < (1ull << 32) && 3ull * nc * maxlat < (1ull << 24) ? 1u : 0u;
    // and every V = cnt s2 - s1^2 in 32 bits: V = sum over pairs of
    // (x_i - x_j)^2 <= (cnt / 2)^2 (2 max)^2 = cnt^2 max^2 for values x in
    // [0, 2 max], so cnt max < 2^16 suffices (the kernels compute V mod 2^32
    // from 32-bit products: exact when V < 2^32).  Round 5 asked cnt^2 (2 max)^2
    // < 2^32, which config 5 (128 clients) missed.
    f.v32 = f.s32 && (uint64_t)std::max(nc, n) * maxlat < (1ull << 16) ? 1u : 0u;
    f.want_score = a.want_score;
    f.p_fmean = a.p_fmean;
    f.p_emean = a.p_emean;
    f.ft_metric = a.ft_metric;
    auto integral = [](double x) { return x == (double)(int64_t)x && x > -1e12 && x < 1e12; };
    f.p_int = integral(a.p_fmean) && integral(a.p_emean) ? 1 : 0;
    f.p1i = f.p_int ? (int64_t)a.p_fmean * (int64_t)nc : 0;
    f.p2i = f.p_int ? (int64_t)a.p_emean * (int64_t)nc : 0;
    auto band = [&](double p, int64_t pi, int32_t& lo, int32_t& hi) {
      const double t = p * (double)nc;
      const double l = f.p_int ? (double)pi : std::floor(t) - 1.0, h = f.p_int ? (double)pi : std::ceil(t) + 1.0;
      const double cap = 2147483647.0;  // D = a difference of two sums below 2^21
      lo = (int32_t)std::max(-cap, std::min(cap, l));
      hi = (int32_t)std::max(-cap, std::min(cap, h));
    };
    band(a.p_fmean, f.p1i, f.m1_lo, f.m1_hi);
    band(a.p_emean, f.p2i, f.m2_lo, f.m2_hi);
    f.n_obj = a.n_obj;
    for (int o = 0; o < bote::MAXOBJ; ++o) {
      f.obj_kind[o] = a.obj_kind[o];
      f.obj_slot[o] = a.obj_slot[o];
    }
    f.K = K;
    f.out_counters = a.out_counters;
    f.want_digest = a.want_digest;
    f.queue = s->queue.as<uint64_t>();
    f.queue_count = s->qcount.as<unsigned long long>();
    f.queue_cap = QUEUE_CAP;
#ifdef BOTE_DEBUG
    if (s->dbg.alloc(16) != hipSuccess || hipMemset(s->dbg.p, 0, 16) != hipSuccess)
      return cleanup(fail(BOTE_E_NOMEM, "debug flag"));
    f.dbg_flag = s->dbg.as<unsigned int>();
#endif
#ifdef BOTE_PATHSTATS
    if (s->pstats.alloc(64 * 8) != hipSuccess || hipMemset(s->pstats.p, 0, 64 * 8) != hipSuccess)
      return cleanup(fail(BOTE_E_NOMEM, "path counters"));
    f.pstats = s->pstats.as<unsigned long long>();
#endif
#ifdef BOTE_ABLATION
    const char* abl = getenv("BOTE_ABLATE");  // timing-diagnostics builds only
    f.ablate = abl ? (uint32_t)strtoul(abl, nullptr, 0) : 0u;
#endif
    s->fshm = bote::fast_smem_bytes(f, n);
    if (s->fshm > device_max_lds(p->device)) {
      s->fast = false;
    } else {
      s->fgrid = (uint32_t)(device_cus(p->device) * bote::fast_occupancy(n, s->fshm));
    }
    // group kernel: n >= 4, positions fit 8 bits, enough lane utilisation
    bool want_group = n >= 4 && ns <= 256 && group_utilisation(ns, n) >= 0.9;
    if (kernel != BOTE_KERNEL_AUTO) want_group = n >= 4 && ns <= 256 && kernel == BOTE_KERNEL_GROUP;
    if (kernel == BOTE_KERNEL_GROUP && !want_group) return cleanup(fail(BOTE_E_ARG, "group kernel needs n >= 4"));
    if (s->fast && want_group) {
      auto lt = low_table(ns - (n - 3));
#ifdef BOTE_DEBUG
      f.lowtab_n = lt.size();
#endif
      // (64 padding entries: a step's lanes read the table past a group's
      // last row without a clamp; those lanes hold no config)
      lt.resize(lt.size() + 64, 0u);
      if (s->lowtab.alloc(std::max<size_t>(lt.size(), 1) * 4) != hipSuccess)
        return cleanup(fail(BOTE_E_NOMEM, "hipMalloc group low table"));
      if (!lt.empty() && hipMemcpy(s->lowtab.p, lt.data(), lt.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return cleanup(fail(BOTE_E_DEVICE, "upload group low table"));
      f.lowtab = s->lowtab.as<uint32_t>();
      // workgroup size: 256 threads (4 waves).  Larger workgroups (which
      // share the client-quad matrix, so R = 128 fits more waves per CU) were
      // measured slower: R=128 n=6 at 640 threads, 5 waves/SIMD, 369 ms vs
      // 348 ms at 256 threads, 2 waves/SIMD.
      // bote.py DEFAULT_OBJECTIVES: SCORE, MEAN af1, MEAN ff1, COV af1, MEAN e
      static const uint32_t dk[5] = {BOTE_OBJ_SCORE, BOTE_OBJ_MEAN, BOTE_OBJ_MEAN, BOTE_OBJ_COV, BOTE_OBJ_MEAN};
      static const uint32_t ds[5] = {0, BOTE_SLOT_AF1, BOTE_SLOT_FF1, BOTE_SLOT_AF1, BOTE_SLOT_E};
      s->def_obj = (keys ? keys_def : n_obj == 5) && f.want_score;
      for (uint32_t o = 0; s->def_obj && o < 5; ++o)
        s->def_obj = objs[o].kind == dk[o] && (dk[o] == BOTE_OBJ_SCORE || objs[o].slot == ds[o]);
      // One geometry per candidate workgroup size: the position table (n <= 7)
      // unless its LDS lowers the workgroups per CU, then as many client
      // lines per wave (<= 16) as keep that occupancy.  A workgroup shares the
      // client-quad matrix (CQT) among its waves, so at R = 128 larger
      // workgroups leave LDS for the client lines that 256-thread ones cannot
      // hold (a step has 7.7 distinct (p1, p2) on average at R=64 n=7, 4.0 at
      // R=128 n=6).  pick_group_geometry keeps the best.
      // the member-binned client loop on the base key set: bench-shaped
      // sweeps (server identity, digest, F1F2: the SI kernels) with >= 32
      // clients, where the bin fields cannot overflow (R=64 n=7: 14.26 vs
      // 14.89 ms for the register lookups, profiles/r04c; R=128 n=6: 168 vs
      // 180 ms, round 3)
      f.gbins = !keys && s->def_obj && bote::group_uses_lines(n) && nc >= BOTE_GBINS_MIN_NC && nc < 256 && f.srv_identity &&
                f.want_digest && f.ft_metric == 2 && (uint64_t)nc * (16ull * maxlat + 15) < (1ull << 24) &&
                (uint64_t)nc * maxlat < (1ull << 16) &&  // (packed member-pair bins)
                2 * (16ull * maxlat + 15) * (16ull * maxlat + 15) < (1ull << 32);
      struct GGeo {
        uint32_t bd = 0, grx = 0, gslots = 0, gqsh = 10;
        int occ = 0;
        size_t shm = 0;
      };
      auto geometry = [&](uint32_t bd) {
        GGeo g;
        g.bd = bd;
        f.gbd = bd;
        // qtab member planes (non-PERM kernels): one u32 per thread, so the
        // plane stride 1 << gqsh must hold gbd * 4 bytes (bote_group.hip)
        f.gqsh = 10;
        while ((1u << f.gqsh) < f.gbd * 4) ++f.gqsh;
        f.gslots = 0;
        f.grx = 0;
        if (bote::group_uses_lines(n)) {
          const int occ_plain = bote::group_occupancy(f, n, bote::group_smem_bytes(f, n), s->def_obj);
          f.grx = 1;
          if (bote::group_occupancy(f, n, bote::group_smem_bytes(f, n), s->def_obj) < occ_plain) f.grx = 0;
          const int occ0 = bote::group_occupancy(f, n, bote::group_smem_bytes(f, n), s->def_obj);
          for (uint32_t sl = 16; sl >= 1; --sl) {
            f.gslots = sl;
            const size_t sh = bote::group_smem_bytes(f, n);
            if (sh <= device_max_lds(p->device) && bote::group_occupancy(f, n, sh, s->def_obj) >= occ0) break;
            f.gslots = 0;
          }
        }
        g.grx = f.grx;
        g.gslots = f.gslots;
        g.gqsh = f.gqsh;
        g.shm = bote::group_smem_bytes(f, n);
        g.occ = g.shm <= device_max_lds(p->device) ? bote::group_occupancy(f, n, g.shm, s->def_obj) : 0;
        return g;
      };
      // candidates: multiples of 256 threads up to 1024 (the extended key
      // set's kernels are bounded to bote::group_supports_keys' size).  Sizes
      // of 6 or 10 waves put unequal wave counts on the 4 SIMDs of a CU
      // (384 threads measured 16-21 % slower than both neighbours).
      // BOTE_GROUP_BD (env) forces one size (A/B timing).
      const char* bd_env = getenv("BOTE_GROUP_BD");
      const uint32_t bd_only = bd_env ? (uint32_t)strtoul(bd_env, nullptr, 0) : 0u;
      GGeo best;
      for (uint32_t bd = 256; bd <= 1024; bd += 128) {
        if (bd_only ? bd != bd_only : bd % 256 != 0) continue;
        if (keys && !bote::group_supports_keys(n, bd)) continue;
        const GGeo g = geometry(bd);
        if (g.occ > 0 && bote::host::pick_group_geometry(g.bd, g.occ, g.gslots, best.bd, best.occ, best.gslots)) best = g;
      }
      if (best.occ > 0 && (!keys || s->def_obj)) {
        f.gbd = best.bd;
        f.grx = best.grx;
        f.gslots = best.gslots;
        f.gqsh = best.gqsh;
        s->group = true;
        s->fshm = best.shm;
        s->fgrid = (uint32_t)(device_cus(p->device) * best.occ);
      }
    }
  }
  // the fast (non-group) kernel does not compute the extended key set
  if (keys && s->fast && !s->group) s->fast = false;
  // the generic path may also run on a fast sweep (overflow recompute)
  const uint32_t lists = s->fast ? std::max(s->grid, s->fgrid + s->xgrid) : s->grid;
  size_t top_bytes = (size_t)lists * std::max<uint32_t>(n_obj, 1) * bote::KP * 16;
  size_t tmp_bytes = (size_t)((lists + 7) / 8) * std::max<uint32_t>(n_obj, 1) * bote::KP * 16;
  if (s->top.alloc(top_bytes) != hipSuccess || s->tmp0.alloc(tmp_bytes) != hipSuccess ||
      s->tmp1.alloc(tmp_bytes) != hipSuccess || s->result.alloc(s->result_bytes()) != hipSuccess)
    return cleanup(fail(BOTE_E_NOMEM, "hipMalloc sweep workspace"));
  if (s->fast && (s->top_alt.alloc((size_t)s->grid * std::max<uint32_t>(n_obj, 1) * bote::KP * 16) != hipSuccess ||
                  s->counters_alt.alloc(16) != hipSuccess))
    return cleanup(fail(BOTE_E_NOMEM, "hipMalloc overflow fallback workspace"));
  a.out_top = n_obj ? s->top.as<Rec>() : nullptr;
  s->fargs.out_top = a.out_top;
  if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&s->done, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(BOTE_E_DEVICE, "hipEventCreate"));
  *out = s;
  return BOTE_OK;
}

int bote_sweep_is_fast(const bote_sweep* s, int* out) {
  if (!s || !out) return fail(BOTE_E_ARG, "null argument");
  *out = s->fast ? (s->group ? 2 : 1) : 0;
  return BOTE_OK;
}

// The cached group walk covering [rb, re) (walked on first use; a handful of
// walks are kept, the oldest dropped first).  Null off the group kernel or
// when the range has too many groups to walk.
static std::shared_ptr<const GroupWalk> walk_for(const bote_sweep* s, uint64_t rb, uint64_t re) {
  if (!s->fast || !s->group || re <= rb) return nullptr;
  for (const auto& w : s->walks)
    if (w->covers(rb, re)) return w;
  std::shared_ptr<const GroupWalk> w = walk_groups(s->ns, s->n, s->nc, rb, re);
  if (!w) return nullptr;
  if (s->walks.size() >= 8) s->walks.erase(s->walks.begin());
  s->walks.push_back(w);
  return w;
}

int bote_sweep_split(const bote_sweep* s, uint64_t rank_begin, uint64_t rank_end, uint32_t parts,
                     uint64_t* out_bounds) {
  if (!s || !out_bounds) return fail(BOTE_E_ARG, "null argument");
  if (parts == 0) return fail(BOTE_E_ARG, "parts must be >= 1");
  if (rank_begin > rank_end || rank_end > binom_u64(s->ns, s->n)) return fail(BOTE_E_ARG, "rank range out of bounds");
  std::vector<uint64_t> b;
  if (rank_end - rank_begin >= (uint64_t)parts * 64) {
    if (auto w = walk_for(s, rank_begin, rank_end)) b = cut_chunks(*w, rank_begin, rank_end, parts);
  }
  if (b.size() != (size_t)parts + 1) {
    b.resize((size_t)parts + 1);
    const uint64_t span = rank_end - rank_begin;
    for (uint32_t i = 0; i <= parts; ++i) b[i] = rank_begin + (uint64_t)(((unsigned __int128)span * i) / parts);
  }
  std::copy(b.begin(), b.end(), out_bounds);
  return BOTE_OK;
}

#ifndef BOTE_CHUNK_TAIL
#define BOTE_CHUNK_TAIL 3  // guided tail rounds of the chunk table (0: equal-cost chunks only)
#endif
// The group kernel's work-chunk table for [rb, re): cut from a cached walk
// and uploaded on `st` once per range (a bench or a shard re-launches the same
// range).  Null chunks (even rank split in the kernel) off the group kernel.
static int sweep_chunks(bote_sweep* s, uint64_t rb, uint64_t re, hipStream_t st, const bote_sweep::Chunks** out) {
  *out = nullptr;
  if (!s->fast || !s->group) return BOTE_OK;
  auto key = std::make_pair(rb, re);
  auto it = s->chunks.find(key);
  if (it == s->chunks.end()) {
    if (s->chunks.size() >= 16) {  // bounded cache: drain the last stream before freeing
      if (s->last_stream) HIP_TRY(hipStreamSynchronize(s->last_stream));
      HIP_TRY(hipStreamSynchronize(st));
      s->chunks.clear();
    }
    auto c = std::make_unique<bote_sweep::Chunks>();
    const uint32_t nwaves = s->fgrid * (s->fargs.gbd / 64);
    // (no chunk below ~4 wavefront steps of configs)
    const char* cpw_env = getenv("BOTE_CHUNKS_PER_WAVE");  // (A/B timing)
    const uint64_t cpw = cpw_env ? std::max(1ul, strtoul(cpw_env, nullptr, 0))
                                 : (uint64_t)chunks_per_wave(re - rb, nwaves, s->fargs.nc, BOTE_CHUNKS_PER_WAVE);
    const uint64_t want = std::min<uint64_t>((uint64_t)nwaves * cpw, (re - rb) / 256 + 1);
    // guided: the launch's last chunks shrink (BOTE_CHUNK_TAIL rounds of one
    // chunk per wave at 1/2, 1/4, ... of the base size), so the waves finish
    // within a small chunk of each other instead of a base chunk
    if (auto w = walk_for(s, rb, re)) c->host = cut_chunks_guided(*w, rb, re, (uint32_t)want, nwaves, BOTE_CHUNK_TAIL);
    if (!c->host.empty()) {
      c->n = (uint32_t)c->host.size() - 1;
      if (c->dev.alloc(c->host.size() * 8) != hipSuccess) return fail(BOTE_E_NOMEM, "hipMalloc work chunks");
      HIP_TRY(hipMemcpyAsync(c->dev.p, c->host.data(), c->host.size() * 8, hipMemcpyHostToDevice, st));
      // each chunk's first group (FastArgs::wstate): the kernel starts a
      // chunk with two loads instead of a device unrank
      const uint32_t F = s->n - 3;
      if (F <= 16) {
        c->state.assign((size_t)c->n * 4, 0);
        std::vector<uint32_t> p(s->n);
        for (uint32_t i = 0; i < c->n; ++i) {
          if (!colex_unrank(c->host[i], s->n, s->ns, p.data())) return fail(BOTE_E_ARG, "chunk rank out of range");
          uint64_t base = 0, b[2] = {0, 0};
          for (uint32_t k = 0; k < F; ++k) {
            base += binom_u64(p[3 + k], k + 4);
            b[k / 8] |= (uint64_t)p[3 + k] << (8 * (k % 8));
          }
          c->state[4 * (size_t)i] = base;
          c->state[4 * (size_t)i + 1] = b[0];
          c->state[4 * (size_t)i + 2] = b[1];
        }
        if (c->sdev.alloc(c->state.size() * 8) != hipSuccess) return fail(BOTE_E_NOMEM, "hipMalloc chunk states");
        HIP_TRY(hipMemcpyAsync(c->sdev.p, c->state.data(), c->state.size() * 8, hipMemcpyHostToDevice, st));
      }
    }
    it = s->chunks.emplace(key, std::move(c)).first;
  }
  *out = it->second.get();
  return BOTE_OK;
}

// Merge `lists` per-block lists into the result block and append the counters:
// one launch when the group kernel bounded its lists (kbound: few records per
// list), else the tree of 8-way merges (full lists).
// With `sel` (fast path), the first level reads the overflow fallback's
// `alt_lists` lists and counters instead when *sel > QUEUE_CAP (on the device).
static bool wide_merge(uint32_t lists, uint32_t alt_lists) {
  return lists <= bote::WIDE_MERGE_LISTS && alt_lists <= bote::WIDE_MERGE_LISTS;
}
static int merge_chain(bote_sweep* s, uint32_t lists, hipStream_t st, const unsigned long long* sel = nullptr,
                       uint32_t alt_lists = 0, const unsigned long long* kbound = nullptr) {
  const uint64_t lstride = (uint64_t)s->n_obj * bote::KP;
  Rec* rec_out = s->result.as<Rec>();
  uint64_t* cdst = (uint64_t*)((char*)s->result.p + lstride * 16);
  if (s->n_obj && kbound && sel && wide_merge(lists, alt_lists)) {
    // one launch: the lists' filled prefixes gathered and ranked in LDS, and
    // the counters picked by the same device choice
    HIP_TRY(bote::launch_merge_wide(s->top.as<Rec>(), lists, s->top_alt.as<Rec>(), alt_lists, lstride, sel, QUEUE_CAP,
                                    kbound, rec_out, s->n_obj, s->K, s->counters.as<unsigned long long>(),
                                    s->counters_alt.as<unsigned long long>(), cdst, st));
    return BOTE_OK;
  }
  if (s->n_obj) {
    const Rec* src = s->top.as<Rec>();
    Rec* bufs[2] = {s->tmp0.as<Rec>(), s->tmp1.as<Rec>()};
    int b = 0;
    if (sel) {
      Rec* dst = lists > bote::G_MERGE_LISTS || alt_lists > bote::G_MERGE_LISTS ? bufs[b] : rec_out;
      HIP_TRY(bote::launch_merge_sel(src, lists, s->top_alt.as<Rec>(), alt_lists, lstride, sel, QUEUE_CAP, dst, lstride,
                                     s->n_obj, st));
      lists = (std::max(lists, alt_lists) + bote::G_MERGE_LISTS - 1) / bote::G_MERGE_LISTS;
      src = dst;
      b ^= 1;
      if (dst == rec_out) lists = 0;
    }
    while (lists > bote::G_MERGE_LISTS) {
      HIP_TRY(bote::launch_merge(src, lists, lstride, bufs[b], lstride, s->n_obj, st));
      src = bufs[b];
      b ^= 1;
      lists = (lists + bote::G_MERGE_LISTS - 1) / bote::G_MERGE_LISTS;
    }
    if (lists) HIP_TRY(bote::launch_merge(src, lists, lstride, rec_out, lstride, s->n_obj, st));
  }
  if (sel) {
    HIP_TRY(bote::launch_pick_counters(s->counters.as<unsigned long long>(), s->counters_alt.as<unsigned long long>(),
                                       sel, QUEUE_CAP, cdst, st));
  } else {
    HIP_TRY(hipMemcpyAsync(cdst, s->counters.p, 16, hipMemcpyDeviceToDevice, st));
  }
  return BOTE_OK;
}

static int timing_slot(bote_sweep* s, hipEvent_t*& e0, hipEvent_t*& e1) {
  if (s->ev_used == s->evpool.size()) {
    hipEvent_t a0, a1;
    HIP_TRY(hipEventCreate(&a0));
    HIP_TRY(hipEventCreate(&a1));
    s->evpool.emplace_back(a0, a1);
  }
  auto& tp = s->evpool[s->ev_used++];
  e0 = &tp.first;
  e1 = &tp.second;
  return BOTE_OK;
}

// Generic kernel over [rb, re): the exact path for any planet.
static int launch_generic(bote_sweep* s, uint64_t rb, uint64_t re, hipStream_t st, bool timed) {
  EvalArgs a = s->args;
  a.rb = rb;
  a.re = re;
  const uint64_t count = re - rb;
  const uint64_t G = (uint64_t)s->grid * s->bd;
  a.runlen = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(32, count / (G * 8)));
  HIP_TRY(hipMemsetAsync(s->counters.p, 0, 16, st));
  hipEvent_t *e0 = nullptr, *e1 = nullptr;
  int rc;
  if (timed && (rc = timing_slot(s, e0, e1))) return rc;
  s->last0 = e0 ? *e0 : s->ev0;
  s->last1 = e1 ? *e1 : s->ev1;
  HIP_TRY(hipEventRecord(s->last0, st));
  HIP_TRY(bote::launch_eval(a, s->n, false, s->grid, s->bd, s->shm, st));
  HIP_TRY(hipEventRecord(s->last1, st));
  return merge_chain(s, s->grid, st);
}

// The top-K seed of a group launch over [rb, re) (launch_fast_path): sets
// f.tseed, or leaves it null when the range is too small to sample.
// sample steps per wave on a full range (r03v A/B: 8 vs 1, kernel -1.6 %, 1/8
// shard -5 %; r05g: 4 and 8 give the same R=64 n=7 step, 14.15-14.17 vs
// 14.16-14.25 ms, and 4 halves the sample launch: 0.14 vs 0.18 ms outside the kernel)
constexpr uint32_t SEED_STEPS = 4;
static int sample_seed(bote_sweep* s, bote::FastArgs& f, uint64_t rb, uint64_t re, hipStream_t st) {
  const uint32_t nwaves = s->fgrid * (s->fargs.gbd / 64);
  const uint32_t base = std::min<uint32_t>(4096, nwaves);
  // SEED_STEPS one-step chunks per wave, disjoint and at most 1/8 of the
  // range.  (Chunks of 8 consecutive steps, 4,096 of them, measured slower:
  // kernel 15.52 vs 15.35 ms, their K least minima are a looser bound, r03x.)
  const uint64_t fit = (re - rb) / (64 * 8);
  const uint32_t ssteps = 1;  // one step per sample chunk (one group precompute each)
  // sample steps per wave: SEED_STEPS on a full sweep; a shard's launch
  // scales them by sqrt(its share of the rank space), rounded up: the sample
  // costs ~ steps, the block merges it saves
  // ~ range / steps, so the best count grows as sqrt(range).  r05g, R=64 n=7
  // shards, 8 scaled (8 / 3 / 1 steps) against 8 fixed: 1/8 shard 2.089 vs
  // 2.125 ms per step, 1/64 0.492 vs 0.531 ms
  const double share = (double)(re - rb) / (double)binom_u64(s->ns, s->n);
  const uint32_t steps =
      (uint32_t)std::max(1.0, std::min((double)SEED_STEPS, std::ceil(SEED_STEPS * std::sqrt(share) - 1e-9)));
  const uint32_t nsamp = (uint32_t)std::min<uint64_t>(
      {(uint64_t)base * std::max<uint32_t>(1, steps), std::max<uint64_t>(base, fit / ssteps), 65536});
  if (nsamp < s->K || re - rb < (uint64_t)nsamp * ssteps * 64 * 8) return BOTE_OK;
  auto key = std::make_pair(rb, re);
  auto it = s->samples.find(key);
  if (it == s->samples.end()) {
    if (s->samples.size() >= 16) {
      if (s->last_stream) HIP_TRY(hipStreamSynchronize(s->last_stream));
      HIP_TRY(hipStreamSynchronize(st));
      s->samples.clear();
    }
    auto c = std::make_unique<bote_sweep::Chunks>();
    c->n = nsamp;
    c->host.resize(nsamp);
    c->state.assign((size_t)nsamp * 4, 0);
    std::vector<uint32_t> p(s->n);
    const uint32_t F = s->n - 3;
    if (F > 16) return BOTE_OK;
    for (uint32_t i = 0; i < nsamp; ++i) {
      const uint64_t b = rb + (uint64_t)(((unsigned __int128)(re - rb - 64) * i) / nsamp);
      c->host[i] = b;
      if (!colex_unrank(b, s->n, s->ns, p.data())) return fail(BOTE_E_ARG, "sample rank out of range");
      uint64_t base = 0, w[2] = {0, 0};
      for (uint32_t k = 0; k < F; ++k) {
        base += binom_u64(p[3 + k], k + 4);
        w[k / 8] |= (uint64_t)p[3 + k] << (8 * (k % 8));
      }
      c->state[4 * (size_t)i] = base;
      c->state[4 * (size_t)i + 1] = w[0];
      c->state[4 * (size_t)i + 2] = w[1];
    }
    if (c->dev.alloc(c->host.size() * 8) != hipSuccess || c->sdev.alloc(c->state.size() * 8) != hipSuccess)
      return fail(BOTE_E_NOMEM, "hipMalloc sample chunks");
    HIP_TRY(hipMemcpyAsync(c->dev.p, c->host.data(), c->host.size() * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->sdev.p, c->state.data(), c->state.size() * 8, hipMemcpyHostToDevice, st));
    it = s->samples.emplace(key, std::move(c)).first;
  }
  const bote_sweep::Chunks* c = it->second.get();
  // slots: one per wave (K slots at or below a key are K distinct configs: the
  // waves' chunks are disjoint), or one per chunk on grids of fewer than K waves
  const uint32_t slots = nwaves >= s->K ? nwaves : nsamp;
  if (s->smin.reserve((size_t)s->n_obj * slots * 8) != hipSuccess || s->tseed.reserve(bote::MAXOBJ * 8) != hipSuccess)
    return fail(BOTE_E_NOMEM, "hipMalloc top-K seed");
  // (per-wave slots: each wave clears its own at the sample launch's start)
  if (slots != nwaves || slots == nsamp) HIP_TRY(hipMemsetAsync(s->smin.p, 0xFF, (size_t)s->n_obj * slots * 8, st));
  bote::FastArgs fs = f;
  fs.smin = s->smin.as<uint64_t>();
  fs.tseed = nullptr;
  fs.wchunks = c->dev.as<uint64_t>();
  fs.wstate = c->sdev.as<uint64_t>();
  fs.nwchunks = nsamp;
  fs.ssteps = ssteps;
  fs.smin_wave = slots == nwaves && slots != nsamp ? 1u : 0u;
  fs.wctr = f.wctr + 256;  // the sample launch's ticket shards
  HIP_TRY(bote::launch_group(fs, s->n, s->def_obj, s->fgrid, s->fshm, st));
  HIP_TRY(bote::launch_seed(fs.smin, fs.smin_wave ? nwaves : nsamp, s->n_obj, s->K, s->tseed.as<uint64_t>(), st));
  f.tseed = s->tseed.as<uint64_t>();
  return BOTE_OK;
}

// Fast kernel over [rb, re), then the generic kernel over its deferred ranks.
static int launch_fast_path(bote_sweep* s, uint64_t rb, uint64_t re, hipStream_t st) {
  bote::FastArgs f = s->fargs;
  f.rb = rb;
  f.re = re;
  const uint64_t count = re - rb;
  const uint64_t G = (uint64_t)s->fgrid * bote::FAST_BD;
  f.runlen = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(32, count / (G * 8)));
  if (s->group) {
    // cost-balanced chunks (32 per wave), taken dynamically (bote_group.hip)
    const bote_sweep::Chunks* ch = nullptr;
    int crc = sweep_chunks(s, rb, re, st, &ch);
    if (crc) return crc;
    f.nwchunks = ch ? ch->n : 0;
    f.wchunks = ch ? ch->dev.as<uint64_t>() : nullptr;
    f.wstate = ch && !ch->state.empty() ? ch->sdev.as<uint64_t>() : nullptr;
    if (f.nwchunks) {
      // (8 shards of 128 B for the main launch, 8 for the sample launch)
      if (!s->wctr.p && s->wctr.alloc(16 * 128) != hipSuccess) return fail(BOTE_E_NOMEM, "hipMalloc work counters");
      f.wctr = s->wctr.as<unsigned int>();
      // 8 counter shards when the grid divides evenly (equal blocks per shard)
      f.wshards = s->fgrid % 8 == 0 ? 8u : 1u;
    }
  }
  // counters, deferred count, work tickets, fallback counters: one launch
  // the group blocks' lists shrink to the records within the least K-th key
  // of any block's list when the one-launch merge reads them
  f.kbound = nullptr;
  if (s->group && s->n_obj && s->K && wide_merge(s->fgrid + s->xgrid, s->grid)) {
    if (!s->kbound.p && s->kbound.alloc(bote::MAXOBJ * 8) != hipSuccess) return fail(BOTE_E_NOMEM, "hipMalloc K-th key bound");
    f.kbound = s->kbound.as<unsigned long long>();
  }
  HIP_TRY(bote::launch_zero_ctl(s->counters.as<unsigned long long>(), s->qcount.as<unsigned long long>(),
                                f.nwchunks ? f.wctr : nullptr, s->counters_alt.as<unsigned long long>(), f.kbound, st));
  // top-K seed: one step of 64 configs per wave at evenly spaced ranks, then
  // per objective the K-th least of the chunks' minimum keys (a bound on the
  // range's K-th key: K distinct configs of the range reach it), so that the
  // blocks' lists start with a threshold instead of filling from empty (the
  // fill costs about the same per block whatever the range: at 1/8 of R=64
  // n=7 it was 1/8 of the kernel)
  if (s->group && f.nwchunks && s->n_obj && s->K) {
    int src = sample_seed(s, f, rb, re, st);
    if (src) return src;
  }
  hipEvent_t *e0 = nullptr, *e1 = nullptr;
  int rc;
  if ((rc = timing_slot(s, e0, e1))) return rc;
  // the kernel's events ride on its dispatch (hipExtLaunchKernelGGL): a
  // separate hipEventRecord before and after the kernel left ~10 us of idle
  // GPU each (profiles/r05b trace)
  s->last0 = *e0;
  s->last1 = *e1;
  if (s->group) HIP_TRY(bote::launch_group(f, s->n, s->def_obj, s->fgrid, s->fshm, st, *e0, *e1));
  else HIP_TRY(bote::launch_fast(f, s->n, s->fgrid, s->fshm, st, *e0, *e1));
  // exact fixup of the deferred configs: generic kernel over the rank list
  EvalArgs a = s->args;
  a.rank_list = s->queue.as<uint64_t>();
  a.rank_count = s->qcount.as<unsigned long long>();
  a.rb = 0;
  a.re = QUEUE_CAP;
  a.runlen = 1;
  a.out_top = s->n_obj ? s->top.as<Rec>() + (size_t)s->fgrid * s->n_obj * bote::KP : nullptr;
  HIP_TRY(bote::launch_eval(a, s->n, false, s->xgrid, s->bd, s->shm, st));
  // overflow fallback: more deferred configs than the queue holds => the
  // generic kernel recomputes the whole range into its own lists/counters and
  // the merge picks those.  Decided on the device (every block of the fallback
  // exits at once otherwise): no host round trip per launch.
  EvalArgs g = s->args;
  g.rb = rb;
  g.re = re;
  const uint64_t GG = (uint64_t)s->grid * s->bd;
  g.runlen = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(32, count / (GG * 8)));
  g.out_top = s->n_obj ? s->top_alt.as<Rec>() : nullptr;
  g.out_counters = s->counters_alt.as<unsigned long long>();
  g.run_if_over = s->qcount.as<unsigned long long>();
  g.over_cap = QUEUE_CAP;
  HIP_TRY(bote::launch_eval(g, s->n, false, s->grid, s->bd, s->shm, st));
  return merge_chain(s, s->fgrid + s->xgrid, st, s->qcount.as<unsigned long long>(), s->grid, f.kbound);
}

int bote_sweep_launch(bote_sweep* s, uint64_t rank_begin, uint64_t rank_end, void* hip_stream) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s) return fail(BOTE_E_ARG, "sweep is null");
  uint64_t total = binom_u64(s->ns, s->n);
  if (rank_begin > rank_end || rank_end > total) return fail(BOTE_E_ARG, "rank range out of bounds");
  HIP_TRY(hipSetDevice(s->p->device));
  hipStream_t st = (hipStream_t)hip_stream;
  int rc = s->fast ? launch_fast_path(s, rank_begin, rank_end, st) : launch_generic(s, rank_begin, rank_end, st, true);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(s->done, st));
  s->last_rb = rank_begin;
  s->last_re = rank_end;
  s->last_stream = st;
  s->launched = true;
  return BOTE_OK;
}

uint64_t bote_sweep_result_bytes(const bote_sweep* s) { return s ? s->result_bytes() : 0; }

#ifdef BOTE_PATHSTATS
// Path-statistics builds only (not in include/bote_hip.h): the 64 group-kernel
// path counters since the last call (read, then reset; scripts/pathstats.py).
int bote_sweep_pathstats(bote_sweep* s, uint64_t* out) {
  DevGuard dev_guard;
  if (!s || !out || !s->pstats.p) return fail(BOTE_E_ARG, "no path counters");
  HIP_TRY(hipSetDevice(s->p->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, s->pstats.p, 64 * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(s->pstats.p, 0, 64 * 8));
  return BOTE_OK;
}
#endif

int bote_sweep_result_device(bote_sweep* s, void* dst, void* hip_stream) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s || !dst) return fail(BOTE_E_ARG, "null argument");
  if (!s->launched) return fail(BOTE_E_ARG, "sweep not launched");
  HIP_TRY(hipSetDevice(s->p->device));
  // (dst: device memory, or pinned host memory: the direct device-to-host copy)
  HIP_TRY(hipMemcpyAsync(dst, s->result.p, s->result_bytes(), hipMemcpyDefault, (hipStream_t)hip_stream));
  HIP_TRY(hipEventRecord(s->done, (hipStream_t)hip_stream));
  return BOTE_OK;
}

static void unpack_result(const bote_sweep* s, const std::vector<uint8_t>& blk, bote_topk_record* out,
                          uint32_t* out_count, uint64_t* out_valid, uint64_t* out_digest) {
  static_assert(sizeof(bote_topk_record) == sizeof(TopkRecord), "record layout");
  bote::host::unpack_result(blk.data(), s->n_obj, s->K, bote::KP, (TopkRecord*)out, out_count, out_valid, out_digest);
}

int bote_sweep_result(bote_sweep* s, void* hip_stream, bote_topk_record* out, uint32_t* out_count,
                      uint64_t* out_valid, uint64_t* out_digest) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s) return fail(BOTE_E_ARG, "sweep is null");
  if (!s->launched) return fail(BOTE_E_ARG, "sweep not launched");
  HIP_TRY(hipSetDevice(s->p->device));
  std::vector<uint8_t> blk(s->result_bytes());
  HIP_TRY(hipMemcpyAsync(blk.data(), s->result.p, blk.size(), hipMemcpyDeviceToHost, (hipStream_t)hip_stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)hip_stream));
#ifdef BOTE_DEBUG
  if (s->dbg.p) {
    unsigned int flag = 0;
    HIP_TRY(hipMemcpy(&flag, s->dbg.p, 4, hipMemcpyDeviceToHost));
    if (flag) return fail(BOTE_E_DEVICE, "device assert failed (BOTE_DEBUG), flag bits " + std::to_string(flag));
  }
#endif
  unpack_result(s, blk, out, out_count, out_valid, out_digest);
  return BOTE_OK;
}

int bote_merge_device(const bote_sweep* s, const void* src, uint32_t n_shards, void* dst, void* hip_stream) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s || !src || !dst || n_shards == 0) return fail(BOTE_E_ARG, "bad merge arguments");
  if (n_shards > bote::G_MERGE_LISTS) return fail(BOTE_E_RANGE, "at most 8 shards per merge call");
  HIP_TRY(hipSetDevice(s->p->device));
  hipStream_t st = (hipStream_t)hip_stream;
  const uint64_t bstride = s->result_bytes() / 16;  // records per block
  const uint64_t lstride = (uint64_t)s->n_obj * bote::KP;
  if (s->n_obj) HIP_TRY(bote::launch_merge((const Rec*)src, n_shards, bstride, (Rec*)dst, lstride, s->n_obj, st));
  HIP_TRY(bote::launch_sum_counters((const uint64_t*)src, n_shards, bstride * 2, lstride * 2,
                                    (uint64_t*)dst + lstride * 2, st));
  return BOTE_OK;
}

int bote_sweep_last_kernel_ms(bote_sweep* s, float* out_ms) {
  if (!s || !out_ms) return fail(BOTE_E_ARG, "null argument");
  if (!s->launched) return fail(BOTE_E_ARG, "sweep not launched");
  HIP_TRY(hipEventSynchronize(s->last1));
  HIP_TRY(hipEventElapsedTime(out_ms, s->last0, s->last1));
  return BOTE_OK;
}

int bote_sweep_timing_reset(bote_sweep* s) {
  if (!s) return fail(BOTE_E_ARG, "sweep is null");
  s->ev_used = 0;
  return BOTE_OK;
}

int bote_sweep_timing(bote_sweep* s, float* out_total_ms, uint32_t* out_launches) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s || !out_total_ms || !out_launches) return fail(BOTE_E_ARG, "null argument");
  HIP_TRY(hipSetDevice(s->p->device));
  float tot = 0.f;
  for (size_t i = 0; i < s->ev_used; ++i) {
    float ms = 0.f;
    HIP_TRY(hipEventSynchronize(s->evpool[i].second));
    HIP_TRY(hipEventElapsedTime(&ms, s->evpool[i].first, s->evpool[i].second));
    tot += ms;
  }
  *out_total_ms = tot;
  *out_launches = (uint32_t)s->ev_used;
  return BOTE_OK;
}

int bote_sweep_deferred(bote_sweep* s, void* hip_stream, uint64_t* out) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s || !out) return fail(BOTE_E_ARG, "null argument");
  *out = 0;
  if (!s->fast || !s->launched) return BOTE_OK;
  HIP_TRY(hipSetDevice(s->p->device));
  unsigned long long q = 0;
  HIP_TRY(hipMemcpyAsync(&q, s->qcount.p, 8, hipMemcpyDeviceToHost, (hipStream_t)hip_stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)hip_stream));
  *out = q;
  return BOTE_OK;
}

int bote_sweep_grid(const bote_sweep* s, uint32_t* out_grid, uint32_t* out_block, uint32_t* out_lds_bytes) {
  if (!s) return fail(BOTE_E_ARG, "sweep is null");
  if (out_grid) *out_grid = s->fast ? s->fgrid : s->grid;
  if (out_block) *out_block = s->fast ? (s->group ? s->fargs.gbd : bote::FAST_BD) : s->bd;
  if (out_lds_bytes) *out_lds_bytes = (uint32_t)(s->fast ? s->fshm : s->shm);
  return BOTE_OK;
}

int bote_sweep_destroy(bote_sweep* s) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!s) return BOTE_OK;
  (void)hipSetDevice(s->p ? s->p->device : 0);
  // work the last launch or result copy enqueued may still run (a launch
  // without a result call): wait for it before the buffers are freed and
  // handed to the next allocation.  An event, not the caller's stream (it may
  // be gone by now) and not the device (hipDeviceSynchronize would also wait
  // for other sweeps' and other threads' work: ADVICE r05)
  if (s->done) {
    if (s->launched) (void)hipEventSynchronize(s->done);
    (void)hipEventDestroy(s->done);
  }
  for (auto& e : s->evpool) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  delete s;
  return BOTE_OK;
}


// ------------------------------------------------- multi-device search ----
// the whole sharded search without PyTorch.  A bote_search
// holds, per shard i of [rank_begin, rank_end), a sweep on planets[i]'s device
// with a stream of its own, its rank bounds (equal estimated cost: one host
// walk of the groups, shared by every shard's sweep) and its uploaded
// work-chunk table; plus the gather and merge buffers on planets[0]'s device.
// A launch is then device work only: every shard's sweep and merge chain, a
// peer copy of its result block to the root device, and a deterministic
// (key, rank) merge tree there.  The result equals one unsharded sweep (the
// merge order does not depend on the number of shards).  Reference: the only
// parallelism of the reference search is rayon over client sets
// (search.rs:209-231); this replaces it for one client set over a node's GPUs.
struct bote_search {
  struct Shard {
    bote_sweep* sw = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    DBuf local;  // the shard's result block on its own device (remote shards)
    uint64_t b = 0, e = 0;
    int dev = 0;
    // (remote shards) peer access to the root device is enabled, so the
    // result block's copy goes device to device over xGMI; false: the
    // runtime stages hipMemcpyPeerAsync through host memory
    bool peer_direct = false;
  };
  std::vector<Shard> sh;
  int root = 0;
  hipStream_t rst = nullptr;
  // recorded on rst after a launch's last merge: the next launch's shard
  // streams wait on it before they overwrite `gathered` (a launch may follow
  // a launch without a result() between them)
  hipEvent_t merged_ev = nullptr;
  DBuf gathered, bufa, bufb, merged;
  uint64_t nb = 0;
  uint64_t rb = 0, re = 0;
  bool launched = false;
};

namespace {
// Drains every stream of the handle, then frees it (any state, error paths too).
void search_free(bote_search* h) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!h) return;
  for (auto& x : h->sh) {
    if (x.st) {
      (void)hipSetDevice(x.dev);
      (void)hipStreamSynchronize(x.st);
    }
  }
  if (h->rst) {
    (void)hipSetDevice(h->root);
    (void)hipStreamSynchronize(h->rst);
    (void)hipStreamDestroy(h->rst);
  }
  if (h->merged_ev) {
    (void)hipSetDevice(h->root);
    (void)hipEventDestroy(h->merged_ev);
  }
  for (auto& x : h->sh) {
    (void)hipSetDevice(x.dev);
    if (x.done) (void)hipEventDestroy(x.done);
    if (x.st) (void)hipStreamDestroy(x.st);
    if (x.sw) bote_sweep_destroy(x.sw);
    x.local.release();
  }
  (void)hipSetDevice(h->root);
  delete h;
}

// hipError_t -> BOTE_E_DEVICE with context (no early return past cleanup)
int hip_fail(hipError_t e, const char* what) {
  return fail(BOTE_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

int bote_search_create(const bote_planet* const* planets, uint32_t n_devices, const uint32_t* servers, uint32_t ns,
                       const uint32_t* clients, uint32_t nc, uint32_t n, uint64_t rank_begin, uint64_t rank_end,
                       const bote_objective* objs, uint32_t n_obj, uint32_t K, const bote_ranking_params* rp,
                       int digest, uint32_t keys, bote_search** out) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!out) return fail(BOTE_E_ARG, "out is null");
  *out = nullptr;
  if (!planets || n_devices == 0) return fail(BOTE_E_ARG, "no planets");
  if (n_devices > 1024) return fail(BOTE_E_RANGE, "at most 1024 shards");
  for (uint32_t i = 0; i < n_devices; ++i) {
    if (!planets[i]) return fail(BOTE_E_ARG, "planet is null");
    if (planets[i]->R != planets[0]->R || planets[i]->lat != planets[0]->lat)
      return fail(BOTE_E_ARG, "the shards' planets differ");
  }
  if (n > ns) return fail(BOTE_E_ARG, "config size larger than the server list");
  const uint64_t total = binom_u64(ns, n);
  if (rank_begin > rank_end || rank_end > total) return fail(BOTE_E_ARG, "rank range out of bounds");
  auto* h = new bote_search();
  h->sh = std::vector<bote_search::Shard>(n_devices);
  h->root = planets[0]->device;
  h->rb = rank_begin;
  h->re = rank_end;
  auto cleanup = [&](int code) {
    search_free(h);
    return code;
  };
  hipError_t e;
  int rc;
  for (uint32_t i = 0; i < n_devices; ++i) {
    auto& x = h->sh[i];
    x.dev = planets[i]->device;
    if ((rc = bote_sweep_create_keys(planets[i], servers, ns, clients, nc, n, objs, n_obj, K, rp, digest,
                                     BOTE_KERNEL_AUTO, keys, &x.sw)))
      return cleanup(rc);
    if ((e = hipSetDevice(x.dev)) != hipSuccess) return cleanup(hip_fail(e, "hipSetDevice (shard)"));
    if ((e = hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&x.done, hipEventDisableTiming)) != hipSuccess)
      return cleanup(hip_fail(e, "shard stream/event"));
  }
  // shards of equal estimated cost from one walk of the groups, shared by
  // every shard's sweep (their chunk tables are cut from it)
  std::vector<uint64_t> bnd((size_t)n_devices + 1);
  if ((rc = bote_sweep_split(h->sh[0].sw, rank_begin, rank_end, n_devices, bnd.data()))) return cleanup(rc);
  for (uint32_t i = 1; i < n_devices; ++i)
    for (const auto& w : h->sh[0].sw->walks) h->sh[i].sw->walks.push_back(w);
  for (uint32_t i = 0; i < n_devices; ++i) {
    auto& x = h->sh[i];
    x.b = bnd[i];
    x.e = bnd[i + 1];
    const bote_sweep::Chunks* ch = nullptr;
    if ((e = hipSetDevice(x.dev)) != hipSuccess) return cleanup(hip_fail(e, "hipSetDevice (shard)"));
    if ((rc = sweep_chunks(x.sw, x.b, x.e, x.st, &ch))) return cleanup(rc);
  }
  // gather + merge buffers on the root device
  h->nb = h->sh[0].sw->result_bytes();
  const size_t groups = (n_devices + bote::G_MERGE_LISTS - 1) / bote::G_MERGE_LISTS;
  if ((e = hipSetDevice(h->root)) != hipSuccess) return cleanup(hip_fail(e, "hipSetDevice (root)"));
  if ((e = hipStreamCreateWithFlags(&h->rst, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->merged_ev, hipEventDisableTiming)) != hipSuccess)
    return cleanup(hip_fail(e, "root stream/event"));
  if (h->gathered.alloc(h->nb * n_devices) != hipSuccess || h->bufa.alloc(h->nb * groups) != hipSuccess ||
      h->bufb.alloc(h->nb * groups) != hipSuccess || h->merged.alloc(h->nb) != hipSuccess)
    return cleanup(fail(BOTE_E_NOMEM, "gather buffers"));
  for (auto& x : h->sh) {
    if (x.dev == h->root) continue;
    if ((e = hipSetDevice(x.dev)) != hipSuccess) return cleanup(hip_fail(e, "hipSetDevice (shard)"));
    if (x.local.alloc(h->nb) != hipSuccess) return cleanup(fail(BOTE_E_NOMEM, "shard result block"));
    // the shard's device writes its block into the root's memory: enable its
    // peer access to the root (xGMI), "already enabled" (another handle, or
    // the caller) counting as success; without peer access the copy is still
    // correct, staged through the host by the runtime
    int can = 0;
    if ((e = hipDeviceCanAccessPeer(&can, x.dev, h->root)) != hipSuccess)
      return cleanup(hip_fail(e, "hipDeviceCanAccessPeer"));
    if (can) {
      e = hipDeviceEnablePeerAccess(h->root, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();  // (clear the sticky "already enabled")
        e = hipSuccess;
      }
      if (e != hipSuccess) return cleanup(hip_fail(e, "hipDeviceEnablePeerAccess (shard to root)"));
      x.peer_direct = true;
    }
  }
  // the chunk uploads are stream-ordered before the first launch; drain them
  // here so that create returns with the handle idle
  for (auto& x : h->sh) {
    (void)hipSetDevice(x.dev);
    if ((e = hipStreamSynchronize(x.st)) != hipSuccess) return cleanup(hip_fail(e, "shard setup"));
  }
  (void)hipSetDevice(h->root);
  *out = h;
  return BOTE_OK;
}

int bote_search_bounds(const bote_search* h, uint64_t* out_bounds) {
  if (!h || !out_bounds) return fail(BOTE_E_ARG, "null argument");
  for (size_t i = 0; i < h->sh.size(); ++i) out_bounds[i] = h->sh[i].b;
  out_bounds[h->sh.size()] = h->sh.empty() ? h->rb : h->sh.back().e;
  return BOTE_OK;
}

int bote_search_launch(bote_search* h) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!h) return fail(BOTE_E_ARG, "search is null");
  int rc;
  hipError_t e;
  const uint32_t nd = (uint32_t)h->sh.size();
  // every shard first (asynchronous, one stream each: no host work between)
  for (auto& x : h->sh)
    if ((rc = bote_sweep_launch(x.sw, x.b, x.e, x.st))) return rc;
  for (uint32_t i = 0; i < nd; ++i) {
    auto& x = h->sh[i];
    char* dst = h->gathered.as<char>() + h->nb * i;
    // (write-after-read: the previous launch's merge tree may still be reading `gathered`)
    if (h->launched) {
      if ((e = hipSetDevice(x.dev)) != hipSuccess || (e = hipStreamWaitEvent(x.st, h->merged_ev, 0)) != hipSuccess)
        return hip_fail(e, "wait for the previous merge");
    }
    if (x.dev == h->root) {
      if ((rc = bote_sweep_result_device(x.sw, dst, x.st))) return rc;
    } else {
      if ((rc = bote_sweep_result_device(x.sw, x.local.p, x.st))) return rc;
      if ((e = hipMemcpyPeerAsync(dst, h->root, x.local.p, x.dev, h->nb, x.st)) != hipSuccess)
        return hip_fail(e, "peer copy of a shard result");
    }
    if ((e = hipSetDevice(x.dev)) != hipSuccess || (e = hipEventRecord(x.done, x.st)) != hipSuccess)
      return hip_fail(e, "record shard event");
  }
  if ((e = hipSetDevice(h->root)) != hipSuccess) return hip_fail(e, "hipSetDevice (root)");
  for (auto& x : h->sh)
    if ((e = hipStreamWaitEvent(h->rst, x.done, 0)) != hipSuccess) return hip_fail(e, "wait shard");
  // merge tree, at most 8 blocks per merge
  const char* src = h->gathered.as<char>();
  uint32_t m = nd;
  char* bufs[2] = {h->bufa.as<char>(), h->bufb.as<char>()};
  int bsel = 0;
  const bote_sweep* s0 = h->sh[0].sw;
  while (m > (uint32_t)bote::G_MERGE_LISTS) {
    const uint32_t groups = (m + bote::G_MERGE_LISTS - 1) / bote::G_MERGE_LISTS;
    for (uint32_t g = 0; g < groups; ++g) {
      const uint32_t k = std::min<uint32_t>(bote::G_MERGE_LISTS, m - bote::G_MERGE_LISTS * g);
      if ((rc = bote_merge_device(s0, src + (size_t)h->nb * bote::G_MERGE_LISTS * g, k, bufs[bsel] + (size_t)h->nb * g,
                                  h->rst)))
        return rc;
    }
    src = bufs[bsel];
    bsel ^= 1;
    m = groups;
  }
  if ((rc = bote_merge_device(s0, src, m, h->merged.p, h->rst))) return rc;
  if ((e = hipEventRecord(h->merged_ev, h->rst)) != hipSuccess) return hip_fail(e, "record merge event");
  h->launched = true;
  return BOTE_OK;
}

int bote_search_result(bote_search* h, bote_topk_record* out, uint32_t* out_count, uint64_t* out_valid,
                       uint64_t* out_digest) {
  DevGuard dev_guard;  // the caller's current device is restored on return
  if (!h) return fail(BOTE_E_ARG, "search is null");
  if (!h->launched) return fail(BOTE_E_ARG, "search not launched");
  HIP_TRY(hipSetDevice(h->root));
  std::vector<uint8_t> blk(h->nb);
  HIP_TRY(hipMemcpyAsync(blk.data(), h->merged.p, h->nb, hipMemcpyDeviceToHost, h->rst));
  HIP_TRY(hipStreamSynchronize(h->rst));
  unpack_result(h->sh[0].sw, blk, out, out_count, out_valid, out_digest);
  return BOTE_OK;
}

int bote_search_destroy(bote_search* h) {
  search_free(h);
  return BOTE_OK;
}

int bote_search_topk(const bote_planet* const* planets, uint32_t n_devices, const uint32_t* servers, uint32_t ns,
                     const uint32_t* clients, uint32_t nc, uint32_t n, uint64_t rank_begin, uint64_t rank_end,
                     const bote_objective* objs, uint32_t n_obj, uint32_t K, const bote_ranking_params* rp,
                     int digest, bote_topk_record* out, uint32_t* out_count, uint64_t* out_valid,
                     uint64_t* out_digest) {
  bote_search* h = nullptr;
  int rc = bote_search_create(planets, n_devices, servers, ns, clients, nc, n, rank_begin, rank_end, objs, n_obj, K,
                              rp, digest, BOTE_KEYS_BASE, &h);
  if (rc) return rc;
  if (!(rc = bote_search_launch(h))) rc = bote_search_result(h, out, out_count, out_valid, out_digest);
  const std::string err = g_err;
  search_free(h);
  if (rc) g_err = err;
  return rc;
}

}  // extern "C"
