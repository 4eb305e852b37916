// =============================================================================
//  TEST INFRASTRUCTURE — NOT PRODUCT CODE.
//
//  CPU restatement of fantoch_bote's configuration search, used only as the
//  parity checker (tests/, __graft_entry__.smoke()) and as the CPU baseline leg
//  of bench.py.  Nothing in fantoch_amd/ links, loads or calls this file.
//
//  It restates the reference algorithm line for line, including its data
//  structures' observable behaviour:
//    * Planet rows sorted by (latency, Region name)     fantoch/src/planet/mod.rs:122-140
//    * nth_closest = linear filtered scan of the row     fantoch_bote/src/lib.rs:169-185
//    * quorum_latency / leaderless / leader             fantoch_bote/src/lib.rs:38-89,155-163
//    * all_leaders_stats / best_leader (first minimum;  fantoch_bote/src/lib.rs:99-150
//      Rust's sort_unstable_by is insertion sort for len <= 20, hence stable)
//    * Histogram as an ordered map u64 -> count, with   fantoch/src/metrics/histogram.rs:27-257
//      mean / ordered-sum variance / cov / mdtm /
//      percentile / Debug formatting
//    * F64 total order (NaN greatest), round() = {:.1}   fantoch/src/metrics/float.rs:22-24,62-89
//    * quorum sizes                                      fantoch_bote/src/protocol.rs:20-35
//    * compute_stats                                     fantoch_bote/src/search.rs:262-319
//    * compute_score / rank / super_configs /            fantoch_bote/src/search.rs:97-178,321-472
//      min_mean_decrease / sorted_evolving_configs
//    * FTMetric::fs, max_f                               fantoch_bote/src/search.rs:474-477,652-666
//    * Tempo quorum sizes (fast n/2+f, tiny 2f, write f+1) fantoch/src/config.rs:317-329 (through
//      Bote::leaderless, oracle_leaderless_batch)
//    * the extended key set (BOTE_KEYS_TEMPO_ALL_LEADERS, BASELINE config 5):
//      Tempo tiny/write leaderless keys and FPaxos all_leaders_stats per
//      config (compute_stats_x), as the GPU sweep computes them
//
//  Pinned against the reference's own known-answer tests (tests/test_oracle.py):
//  lib.rs:193-465, protocol.rs:118-154, search.rs:671-751, histogram.rs:390-463,
//  float.rs:109-177, planet/mod.rs:190-300, planet/dat.rs:115-154.
//
//  Extensions defined by this build (not in the reference, shared bit-for-bit
//  with the GPU path; see DESIGN.md "Objectives"):
//    * colex combination ranks  rank = sum_j C(p_j, j+1)
//    * streaming top-K objective keys (score, mean via exact sum, cov via
//      fl64(V / S1^2) with V = count*sum(x^2) - sum(x)^2)
// =============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Panic : std::runtime_error {
  explicit Panic(const std::string& s) : std::runtime_error(s) {}
};

// ---------------------------------------------------------------- Planet ----
struct Planet {
  uint32_t R = 0;
  std::vector<std::string> names;
  std::vector<std::vector<uint64_t>> lat;  // lat[from][to]
  // sorted[from] = (latency, region) sorted by (latency, name): planet/mod.rs:122-140
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sorted;

  void build_sorted() {
    sorted.assign(R, {});
    for (uint32_t f = 0; f < R; ++f) {
      auto& row = sorted[f];
      for (uint32_t t = 0; t < R; ++t) row.emplace_back(lat[f][t], t);
      std::sort(row.begin(), row.end(), [&](const auto& a, const auto& b) {
        if (a.first != b.first) return a.first < b.first;
        return names[a.second] < names[b.second];
      });
    }
  }
  uint64_t ping_latency(uint32_t from, uint32_t to) const { return lat[from][to]; }
};

// ------------------------------------------------------------------- F64 ----
// float.rs:62-79 — total order with NaN greatest, NaN == NaN.
int f64_cmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  if (a == b) return 0;
  bool an = std::isnan(a), bn = std::isnan(b);
  if (an && bn) return 0;
  return an ? 1 : -1;
}
// float.rs:22-24 — format!("{:.1}") (exact value, ties-to-even, like glibc).
std::string f64_round(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
  char buf[64];
  snprintf(buf, sizeof buf, "%.1f", x);
  return buf;
}

// ------------------------------------------------------------- Histogram ----
struct Histogram {
  std::map<uint64_t, uint64_t> values;  // histogram.rs:14-18 (BTreeMap<u64, usize>)

  template <class It>
  static Histogram from(It b, It e) {
    Histogram h;
    for (; b != e; ++b) h.values[*b] += 1;
    return h;
  }
  uint64_t count() const {
    uint64_t c = 0;
    for (auto& kv : values) c += kv.second;
    return c;
  }
  // histogram.rs:183-191 (u64 arithmetic, wrapping as in a release build)
  void sum_and_count(uint64_t& sum, uint64_t& count) const {
    sum = 0;
    count = 0;
    for (auto& kv : values) {
      sum += kv.first * kv.second;
      count += kv.second;
    }
  }
  uint64_t sumsq() const {
    uint64_t s = 0;
    for (auto& kv : values) s += kv.first * kv.first * kv.second;
    return s;
  }
  // histogram.rs:172-181
  void mean_and_count(double& mean, double& count) const {
    uint64_t s, c;
    sum_and_count(s, c);
    count = (double)c;
    mean = (double)s / count;
  }
  double mean() const {
    double m, c;
    mean_and_count(m, c);
    return m;
  }
  // histogram.rs:204-219 — ordered sum over distinct values ascending.
  double variance(double mean, double count) const {
    double sum = 0.0;
    for (auto& kv : values) {
      double x = (double)kv.first, xc = (double)kv.second;
      double diff = mean - x;
      double t = diff * diff;
      t = t * xc;
      sum = sum + t;
    }
    return sum / (count - 1.0);
  }
  double stddev() const {
    double m, c;
    mean_and_count(m, c);
    return std::sqrt(variance(m, c));
  }
  double cov() const {
    double m, c;
    mean_and_count(m, c);
    double s = std::sqrt(variance(m, c));
    return s / m;
  }
  double mdtm() const {
    double m, c;
    mean_and_count(m, c);
    double sum = 0.0;
    for (auto& kv : values) {
      double x = (double)kv.first, xc = (double)kv.second;
      double diff = m - x;
      sum = sum + std::fabs(diff) * xc;
    }
    return sum / c;
  }
  double min() const { return values.empty() ? NAN : (double)values.begin()->first; }
  double max() const { return values.empty() ? NAN : (double)values.rbegin()->first; }
  // histogram.rs:111-170
  double percentile(double p) const {
    if (!(p >= 0.0 && p <= 1.0)) throw Panic("percentile out of range");
    if (values.empty()) return 0.0;
    double count = (double)this->count();
    double index = p * count;
    double index_rounded = std::round(index);
    bool is_whole = std::fabs(index - index_rounded) == 0.0;
    uint64_t idx = (uint64_t)index_rounded;
    auto it = values.begin();
    double left, right;
    bool has_right;
    for (;;) {
      if (it == values.end()) throw Panic("there should a next histogram value");
      uint64_t v = it->first, c = it->second;
      if (idx == c) {
        left = (double)v;
        auto nx = std::next(it);
        has_right = nx != values.end();
        right = has_right ? (double)nx->first : 0.0;
        break;
      } else if (idx < c) {
        left = (double)v;
        right = left;
        has_right = true;
        break;
      } else {
        idx -= c;
        ++it;
      }
    }
    if (is_whole) {
      if (!has_right) throw Panic("there should be a right value");
      return (left + right) / 2.0;
    }
    return left;
  }
  // histogram.rs:238-257 — f64::round (half away from zero), Display, {:<5}.
  static std::string disp_round(double x) {
    double r = std::round(x);
    char buf[64];
    if (std::isnan(r))
      snprintf(buf, sizeof buf, "NaN");
    else if (std::isinf(r))
      snprintf(buf, sizeof buf, r > 0 ? "inf" : "-inf");
    else
      snprintf(buf, sizeof buf, "%.0f", r);
    std::string s(buf);
    while (s.size() < 5) s.push_back(' ');
    return s;
  }
  std::string debug_fmt() const {
    if (values.empty()) return "(empty)";
    std::string s;
    s += "avg=" + disp_round(mean());
    s += " std=" + disp_round(stddev());
    s += " p95=" + disp_round(percentile(0.95));
    s += " p99=" + disp_round(percentile(0.99));
    s += " p99.9=" + disp_round(percentile(0.999));
    s += " p99.99=" + disp_round(percentile(0.9999));
    s += " min=" + disp_round(min());
    s += " max=" + disp_round(max());
    return s;
  }
};

// -------------------------------------------------------------- Protocol ----
// protocol.rs:20-35
enum Proto { FPAXOS = 0, EPAXOS = 1, ATLAS = 2 };
size_t minority(size_t n) { return n / 2; }
size_t quorum_size(int p, size_t n, size_t f) {
  switch (p) {
    case FPAXOS: return f + 1;
    case EPAXOS: { size_t m = minority(n); return m + (m + 1) / 2; }
    default: return minority(n) + f;
  }
}
// search.rs:474-477
size_t max_f(size_t n) { return std::min(n / 2, (size_t)2); }

// Key slots shared with the GPU path: slot = base + 5 * placement,
// base: 0 af1, 1 ff1, 2 af2, 3 ff2, 4 e; placement 0 Input, 1 Colocated.
enum { K_AF1 = 0, K_FF1 = 1, K_AF2 = 2, K_FF2 = 3, K_E = 4, NKEYS = 10 };
// Extended key set (an extension of compute_stats for BASELINE config 5;
// include/bote_hip.h): Tempo tiny fast (q = 2f) and write (q = f + 1)
// leaderless keys, slot 10 + 4 * placement + {tt1, tt2, tw1, tw2}; FPaxos
// under the best-by-MEAN leader (best_leader with Stats::Mean), Input, slots
// 18 (f = 1) and 19 (f = 2); plus every leader's FPaxos histogram (Input,
// f = 1..max_f), which only feeds the digest.
enum { K_TT1 = 10, K_TT2 = 11, K_TW1 = 12, K_TW2 = 13, K_FL1 = 18, K_FL2 = 19, NKEYS_X = 20 };
int slot_atlas(size_t f) { return f == 1 ? K_AF1 : K_AF2; }
int slot_fpaxos(size_t f) { return f == 1 ? K_FF1 : K_FF2; }

// ------------------------------------------------------------------ Bote ----
struct Bote {
  const Planet* planet;

  static bool contains(const std::vector<uint32_t>& regions, uint32_t r) {
    for (uint32_t x : regions)
      if (x == r) return true;
    return false;
  }
  // lib.rs:169-185
  std::pair<uint64_t, uint32_t> nth_closest(size_t nth, uint32_t from,
                                            const std::vector<uint32_t>& regions) const {
    if (nth == 0) throw Panic("nth_closest(0)");
    size_t seen = 0;
    for (auto& e : planet->sorted[from]) {
      if (!contains(regions, e.second)) continue;
      if (++seen == nth) return e;
    }
    throw Panic("nth_closest: not enough regions");
  }
  // lib.rs:155-163
  uint64_t quorum_latency(uint32_t from, const std::vector<uint32_t>& regions, size_t q) const {
    return nth_closest(q, from, regions).first;
  }
  // lib.rs:38-59
  std::vector<uint64_t> leaderless(const std::vector<uint32_t>& servers,
                                   const std::vector<uint32_t>& clients, size_t q) const {
    std::vector<uint64_t> out;
    out.reserve(clients.size());
    for (uint32_t c : clients) {
      auto cl = nth_closest(1, c, servers);
      uint64_t ql = quorum_latency(cl.second, servers, q);
      out.push_back(cl.first + ql);
    }
    return out;
  }
  // lib.rs:67-89
  std::vector<uint64_t> leader(uint32_t l, const std::vector<uint32_t>& servers,
                               const std::vector<uint32_t>& clients, size_t q) const {
    uint64_t lq = quorum_latency(l, servers, q);
    std::vector<uint64_t> out;
    out.reserve(clients.size());
    for (uint32_t c : clients) out.push_back(planet->ping_latency(c, l) + lq);
    return out;
  }
  // lib.rs:129-150
  std::vector<std::pair<uint32_t, Histogram>> all_leaders_stats(
      const std::vector<uint32_t>& servers, const std::vector<uint32_t>& clients, size_t q) const {
    std::vector<std::pair<uint32_t, Histogram>> v;
    for (uint32_t l : servers) {
      auto lat = leader(l, servers, clients, q);
      v.emplace_back(l, Histogram::from(lat.begin(), lat.end()));
    }
    return v;
  }
  // lib.rs:99-121; stat: 0 Mean, 1 COV, 2 MDTM.  Insertion sort => first minimum.
  // Returns the index into `servers` of the chosen leader.
  size_t best_leader(const std::vector<uint32_t>& servers, const std::vector<uint32_t>& clients,
                     size_t q, int stat, Histogram* out_hist) const {
    auto stats = all_leaders_stats(servers, clients, q);
    if (stats.empty()) throw Panic("the best leader should exist");
    std::vector<double> key(stats.size());
    for (size_t i = 0; i < stats.size(); ++i)
      key[i] = stat == 0 ? stats[i].second.mean()
                         : stat == 1 ? stats[i].second.cov() : stats[i].second.mdtm();
    size_t best = 0;
    for (size_t i = 1; i < stats.size(); ++i)
      if (f64_cmp(key[i], key[best]) < 0) best = i;
    if (out_hist) *out_hist = stats[best].second;
    return best;
  }
};

// ------------------------------------------------------------ Stats (10) ----
struct ProtocolStats {
  bool has[NKEYS_X] = {};
  Histogram h[NKEYS_X];
  std::vector<uint64_t> raw[NKEYS_X];  // per-client values, client order
  uint32_t leader = 0;                 // region id of the FPaxos leader
  size_t leader_pos = 0;               // index of the leader inside `config`
  // extended key set: all_leaders_stats per f = 1..max_f, leaders in config order
  std::vector<Histogram> all_leaders[2];
};

// search.rs:262-319
void compute_stats(const Bote& bote, const std::vector<uint32_t>& config,
                   const std::vector<uint32_t>& all_clients, ProtocolStats& st) {
  size_t n = config.size();
  size_t q = quorum_size(FPAXOS, n, 1);
  size_t lpos = bote.best_leader(config, all_clients, q, 1, nullptr);
  uint32_t leader = config[lpos];
  st.leader = leader;
  st.leader_pos = lpos;
  for (int p = 0; p < 2; ++p) {
    const std::vector<uint32_t>& clients = p == 0 ? all_clients : config;
    for (size_t f = 1; f <= max_f(n); ++f) {
      auto a = bote.leaderless(config, clients, quorum_size(ATLAS, n, f));
      int sa = slot_atlas(f) + 5 * p;
      st.h[sa] = Histogram::from(a.begin(), a.end());
      st.raw[sa] = std::move(a);
      st.has[sa] = true;
      auto fp = bote.leader(leader, config, clients, quorum_size(FPAXOS, n, f));
      int sf = slot_fpaxos(f) + 5 * p;
      st.h[sf] = Histogram::from(fp.begin(), fp.end());
      st.raw[sf] = std::move(fp);
      st.has[sf] = true;
    }
    auto e = bote.leaderless(config, clients, quorum_size(EPAXOS, n, 0));
    int se = K_E + 5 * p;
    st.h[se] = Histogram::from(e.begin(), e.end());
    st.raw[se] = std::move(e);
    st.has[se] = true;
  }
}

// The extended key set (BASELINE config 5: "Tempo f=1,2 + FPaxos all
// leaders"): compute_stats plus, per placement and f = 1..max_f, Tempo's
// tiny fast quorum 2f and write quorum f + 1 through Bote::leaderless
// (fantoch/src/config.rs:317-329; the non-tiny fast quorum n/2 + f is the
// Atlas key already), and over the Input clients all_leaders_stats at
// q = f + 1 (lib.rs:129-150) with its best leader by Stats::Mean (lib.rs:99-121).
void compute_stats_x(const Bote& bote, const std::vector<uint32_t>& config,
                     const std::vector<uint32_t>& all_clients, ProtocolStats& st) {
  compute_stats(bote, config, all_clients, st);
  const size_t n = config.size();
  for (int p = 0; p < 2; ++p) {
    const std::vector<uint32_t>& clients = p == 0 ? all_clients : config;
    for (size_t f = 1; f <= max_f(n); ++f) {
      const int tt = K_TT1 + (int)(f - 1) + 4 * p, tw = K_TW1 + (int)(f - 1) + 4 * p;
      auto a = bote.leaderless(config, clients, 2 * f);
      st.h[tt] = Histogram::from(a.begin(), a.end());
      st.raw[tt] = std::move(a);
      st.has[tt] = true;
      auto w = bote.leaderless(config, clients, f + 1);
      st.h[tw] = Histogram::from(w.begin(), w.end());
      st.raw[tw] = std::move(w);
      st.has[tw] = true;
    }
  }
  for (size_t f = 1; f <= max_f(n); ++f) {
    auto al = bote.all_leaders_stats(config, all_clients, quorum_size(FPAXOS, n, f));
    st.all_leaders[f - 1].clear();
    for (auto& e : al) st.all_leaders[f - 1].push_back(e.second);
    Histogram best;
    const size_t b = bote.best_leader(config, all_clients, quorum_size(FPAXOS, n, f), 0, &best);
    (void)b;
    const int fl = K_FL1 + (int)(f - 1);
    st.h[fl] = best;
    st.has[fl] = true;
  }
}

// ------------------------------------------------------- Ranking params ----
struct RankingParams {
  double min_mean_fpaxos_improv, min_mean_epaxos_improv, min_fairness_fpaxos_improv,
      min_mean_decrease;
  size_t min_n, max_n;
  int ft_metric;  // 1 = F1, 2 = F1F2
};
// search.rs:657-665
std::vector<size_t> fs(int ft_metric, size_t n) {
  size_t m = std::min(n / 2, (size_t)ft_metric);
  std::vector<size_t> v;
  for (size_t f = 1; f <= m; ++f) v.push_back(f);
  return v;
}
const Histogram& get(const ProtocolStats& st, int slot) {
  if (!st.has[slot]) throw Panic("stats with key not found");
  return st.h[slot];
}
// search.rs:421-472
bool compute_score(size_t n, const ProtocolStats& st, const RankingParams& p, double& score) {
  bool valid = true;
  score = 0.0;
  for (size_t f : fs(p.ft_metric, n)) {
    const Histogram& atlas = get(st, slot_atlas(f));
    const Histogram& fpaxos = get(st, slot_fpaxos(f));
    double fmi = fpaxos.mean() - atlas.mean();
    double ffi = fpaxos.cov() - atlas.cov();
    valid = valid && fmi >= p.min_mean_fpaxos_improv && ffi >= p.min_fairness_fpaxos_improv;
    const Histogram& epaxos = get(st, K_E);
    double emi = epaxos.mean() - atlas.mean();
    if (n == 11 || n == 13) valid = valid && emi >= p.min_mean_epaxos_improv;
    double w = 30.0;
    double t = w * emi;
    t = fmi + t;
    score = score + t;
  }
  return valid;
}
// search.rs:403-419
bool min_mean_decrease(const ProtocolStats& st, const ProtocolStats& prev, size_t n,
                       const RankingParams& p) {
  size_t m = n - 2;
  for (size_t f : fs(p.ft_metric, m)) {
    const Histogram& a = get(st, slot_atlas(f));
    const Histogram& pa = get(prev, slot_atlas(f));
    if (!(pa.mean() - a.mean() >= p.min_mean_decrease)) return false;
  }
  return true;
}

// ------------------------------------------------------------- Binomials ----
struct Binom {
  std::vector<std::vector<uint64_t>> c;  // c[m][k]
  explicit Binom(uint32_t M, uint32_t K) : c(M + 1, std::vector<uint64_t>(K + 1, 0)) {
    for (uint32_t m = 0; m <= M; ++m) {
      c[m][0] = 1;
      for (uint32_t k = 1; k <= K && k <= m; ++k)
        c[m][k] = (k == m) ? 1 : c[m - 1][k - 1] + c[m - 1][k];
    }
  }
  uint64_t operator()(uint32_t m, uint32_t k) const {
    if (k > m) return 0;
    return c[m][k];
  }
};
// colex unrank: rank = sum_j C(p_j, j+1), p ascending.
void colex_unrank(const Binom& B, uint64_t rank, uint32_t n, uint32_t ns, uint32_t* p) {
  uint64_t r = rank;
  uint32_t hi = ns;  // exclusive bound for p_j
  for (int j = (int)n - 1; j >= 0; --j) {
    uint32_t k = (uint32_t)j + 1;
    uint32_t lo = (uint32_t)j, x = hi - 1;
    // largest x in [j, hi) with C(x, k) <= r
    while (x > lo && B(x, k) > r) --x;
    p[j] = x;
    r -= B(x, k);
    hi = x;
  }
}

// ---------------------------------------------------- Objectives (top-K) ----
// kinds shared with the GPU path (include/bote_hip.h).
enum { OBJ_SCORE = 0, OBJ_MEAN = 1, OBJ_COV = 2 };
struct Objective { uint32_t kind, slot; };

uint64_t orderable_f64(double x) {
  if (std::isnan(x)) x = NAN;  // canonical positive quiet NaN
  uint64_t b;
  memcpy(&b, &x, 8);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// Returns false when the config does not enter this objective (invalid score).
bool objective_key(const Objective& o, size_t n, const ProtocolStats& st, const RankingParams& rp,
                   uint64_t& key) {
  if (o.kind == OBJ_SCORE) {
    double score;
    if (!compute_score(n, st, rp, score)) return false;
    key = ~orderable_f64(score);
    return true;
  }
  const Histogram& h = get(st, (int)o.slot);
  uint64_t s1, c;
  h.sum_and_count(s1, c);
  if (o.kind == OBJ_MEAN) {
    key = s1;
    return true;
  }
  if (c <= 1 || s1 == 0) {
    key = ~0ull;
    return true;
  }
  uint64_t v = c * h.sumsq() - s1 * s1;
  double r = (double)v / ((double)s1 * (double)s1);
  memcpy(&key, &r, 8);
  return true;
}

struct TopK {
  size_t K;
  std::vector<std::pair<uint64_t, uint64_t>> v;  // (key, rank), kept sorted
  void push(uint64_t key, uint64_t rank) {
    std::pair<uint64_t, uint64_t> e(key, rank);
    if (v.size() == K && !(e < v.back())) return;
    auto it = std::lower_bound(v.begin(), v.end(), e);
    v.insert(it, e);
    if (v.size() > K) v.pop_back();
  }
};

uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Order-independent per-config digest shared with the GPU path (DESIGN.md §7,
// fantoch_amd/csrc/bote_device.hpp digest_*), summed over configs mod 2^64:
// a linear fold of 32-bit words, word w times its constant K_w as two 16-bit
// halves (mod 2^32) -- slot s's exact sum (w = 2s) and sum of squares (w =
// 2s + 1, folded to 32 bits as lo32(S2 ^ S2 >> 32)); with the extended key
// set (compute_stats_x) also slots 10..19 and every leader's FPaxos
// histogram (leader l at f: w = 40 + 2 (16 f + l)) -- then the rank and the
// leader position, through the murmur3 32-bit finaliser.
uint32_t digest_key(uint32_t w) {
  uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(w + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)z | 0x00010001u;
}
uint32_t digest_word(uint32_t h, uint32_t x, uint32_t k) {
  return h + (x & 0xFFFFu) * (k & 0xFFFFu) + (x >> 16) * (k >> 16);
}
uint64_t config_digest(uint64_t rank, const ProtocolStats& st) {
  auto fold = [](uint32_t h, uint32_t s, const Histogram& hh) {
    uint64_t s1, c;
    hh.sum_and_count(s1, c);
    uint64_t s2 = hh.sumsq();
    h = digest_word(h, (uint32_t)s1, digest_key(2 * s));
    return digest_word(h, (uint32_t)(s2 ^ (s2 >> 32)), digest_key(2 * s + 1));
  };
  uint32_t h = 0;
  for (int s = 0; s < NKEYS_X; ++s)
    if (st.has[s]) h = fold(h, (uint32_t)s, st.h[s]);
  for (int f = 0; f < 2; ++f)  // (empty unless the extended key set)
    for (size_t l = 0; l < st.all_leaders[f].size(); ++l) h = fold(h, 20 + 16 * f + (uint32_t)l, st.all_leaders[f][l]);
  uint32_t x = h + (uint32_t)rank * 0x9E3779B1u + (uint32_t)(rank >> 32) * 0xEBCA77u +
               (uint32_t)st.leader_pos * 0xB2AE3Du;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

thread_local std::string g_err;

}  // namespace

// =============================================================== C ABI ======
extern "C" {

const char* oracle_last_error() { return g_err.c_str(); }

// names: R NUL-terminated strings back to back.
void* oracle_planet_new(const uint16_t* lat, uint32_t R, const char* names) {
  auto* p = new Planet();
  p->R = R;
  const char* s = names;
  for (uint32_t i = 0; i < R; ++i) {
    p->names.emplace_back(s);
    s += strlen(s) + 1;
  }
  p->lat.assign(R, std::vector<uint64_t>(R));
  for (uint32_t f = 0; f < R; ++f)
    for (uint32_t t = 0; t < R; ++t) p->lat[f][t] = lat[(size_t)f * R + t];
  p->build_sorted();
  return p;
}
void oracle_planet_free(void* h) { delete (Planet*)h; }

// Planet::sorted(from) -> region ids in (latency, name) order.
int oracle_planet_sorted(void* h, uint32_t from, uint32_t* out_regions, uint64_t* out_lat) {
  auto* p = (Planet*)h;
  if (from >= p->R) return -1;
  for (uint32_t i = 0; i < p->R; ++i) {
    out_regions[i] = p->sorted[from][i].second;
    out_lat[i] = p->sorted[from][i].first;
  }
  return 0;
}

#define ORACLE_TRY try {
#define ORACLE_CATCH                 \
  }                                  \
  catch (const std::exception& e) {  \
    g_err = e.what();                \
    return -1;                       \
  }                                  \
  return 0;

int oracle_quorum_latency(void* h, uint32_t from, const uint32_t* regions, uint32_t nr, uint32_t q,
                          uint64_t* out) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> r(regions, regions + nr);
  *out = b.quorum_latency(from, r, q);
  ORACLE_CATCH
}
int oracle_leaderless(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                      uint32_t nc, uint32_t q, uint64_t* out) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> s(servers, servers + ns), c(clients, clients + nc);
  auto v = b.leaderless(s, c, q);
  std::copy(v.begin(), v.end(), out);
  ORACLE_CATCH
}
int oracle_leader(void* h, uint32_t leader, const uint32_t* servers, uint32_t ns,
                  const uint32_t* clients, uint32_t nc, uint32_t q, uint64_t* out) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> s(servers, servers + ns), c(clients, clients + nc);
  auto v = b.leader(leader, s, c, q);
  std::copy(v.begin(), v.end(), out);
  ORACLE_CATCH
}
int oracle_best_leader(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                       uint32_t nc, uint32_t q, int stat, uint32_t* out_pos) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> s(servers, servers + ns), c(clients, clients + nc);
  *out_pos = (uint32_t)b.best_leader(s, c, q, stat, nullptr);
  ORACLE_CATCH
}

// Bote::leaderless (lib.rs:38-59) for a batch of configs (region ids, config
// order) and nq quorum sizes: Input clients, then Colocated (the config).
//   out_vals: ncfg x nq x (nc + n) u64
int oracle_leaderless_batch(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n, const uint32_t* clients,
                            uint32_t nc, const uint32_t* qs, uint32_t nq, uint32_t threads, uint64_t* out_vals) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> cl(clients, clients + nc);
  if (threads == 0) threads = 1;
  std::vector<std::string> errs(threads);
  auto work = [&](uint32_t t) {
    try {
      for (uint64_t i = (uint64_t)ncfg * t / threads; i < (uint64_t)ncfg * (t + 1) / threads; ++i) {
        std::vector<uint32_t> cfg(configs + i * n, configs + (i + 1) * n);
        for (uint32_t qi = 0; qi < nq; ++qi) {
          uint64_t* o = out_vals + (i * nq + qi) * (nc + n);
          auto a = b.leaderless(cfg, cl, qs[qi]);
          auto c = b.leaderless(cfg, cfg, qs[qi]);
          std::copy(a.begin(), a.end(), o);
          std::copy(c.begin(), c.end(), o + nc);
        }
      }
    } catch (const std::exception& ex) {
      errs[t] = ex.what();
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Panic(e);
  ORACLE_CATCH
}

// Histogram statistics over a value list.  out: mean, stddev, cov, mdtm, min, max.
int oracle_hist_stats(const uint64_t* v, uint32_t n, double* out) {
  ORACLE_TRY
  Histogram hh = Histogram::from(v, v + n);
  out[0] = hh.mean();
  out[1] = hh.stddev();
  out[2] = hh.cov();
  out[3] = hh.mdtm();
  out[4] = hh.min();
  out[5] = hh.max();
  ORACLE_CATCH
}
int oracle_hist_percentile(const uint64_t* v, uint32_t n, double p, double* out) {
  ORACLE_TRY
  Histogram hh = Histogram::from(v, v + n);
  *out = hh.percentile(p);
  ORACLE_CATCH
}
int oracle_hist_fmt(const uint64_t* v, uint32_t n, char* buf, uint32_t cap) {
  ORACLE_TRY
  Histogram hh = Histogram::from(v, v + n);
  std::string s = hh.debug_fmt();
  if (s.size() + 1 > cap) throw Panic("buffer too small");
  memcpy(buf, s.c_str(), s.size() + 1);
  ORACLE_CATCH
}
int oracle_f64_round(double x, char* buf, uint32_t cap) {
  std::string s = f64_round(x);
  if (s.size() + 1 > cap) return -1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return 0;
}
int oracle_f64_cmp(double a, double b) { return f64_cmp(a, b); }
uint32_t oracle_quorum_size(int proto, uint32_t n, uint32_t f) {
  return (uint32_t)quorum_size(proto, n, f);
}

// compute_stats for a batch of explicit configs (region ids, config order).
//   configs:    ncfg x n region ids
//   out_vals:   ncfg x (5*nc + 5*n) u64 (slot-major: Input slots 0..4 each nc
//               values, then Colocated slots 5..9 each n values); missing
//               slots (n < 4: af2/ff2) are filled with ~0.
//   out_leader: ncfg leader positions inside the config
//   threads:    std::thread workers over contiguous config chunks
int oracle_compute_stats_mt(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n,
                            const uint32_t* clients, uint32_t nc, uint64_t* out_vals,
                            uint32_t* out_leader, uint32_t threads) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> cl(clients, clients + nc);
  size_t stride = 5 * (size_t)nc + 5 * (size_t)n;
  if (threads == 0) threads = 1;
  std::vector<std::string> errs(threads);
  auto work = [&](uint32_t t) {
    try {
      for (uint64_t i = (uint64_t)ncfg * t / threads; i < (uint64_t)ncfg * (t + 1) / threads; ++i) {
        std::vector<uint32_t> cfg(configs + i * n, configs + (i + 1) * n);
        ProtocolStats st;
        compute_stats(b, cfg, cl, st);
        uint64_t* o = out_vals + stride * i;
        for (int s = 0; s < NKEYS; ++s) {
          size_t len = s < 5 ? nc : n;
          size_t off = s < 5 ? (size_t)s * nc : 5 * (size_t)nc + (size_t)(s - 5) * n;
          for (size_t k = 0; k < len; ++k) o[off + k] = st.has[s] ? st.raw[s][k] : ~0ull;
        }
        out_leader[i] = (uint32_t)st.leader_pos;
      }
    } catch (const std::exception& ex) {
      errs[t] = ex.what();
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Panic(e);
  ORACLE_CATCH
}

int oracle_compute_stats(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n,
                         const uint32_t* clients, uint32_t nc, uint64_t* out_vals,
                         uint32_t* out_leader) {
  return oracle_compute_stats_mt(h, configs, ncfg, n, clients, nc, out_vals, out_leader, 1);
}

// compute_score (search.rs:421-472) for a batch of explicit configs.
int oracle_scores(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n, const uint32_t* clients,
                  uint32_t nc, const double* rparams, int ft_metric, double* out_score, uint8_t* out_valid) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> cl(clients, clients + nc);
  RankingParams rp{rparams[0], rparams[1], rparams[2], rparams[3], 3, 13, ft_metric};
  for (uint32_t i = 0; i < ncfg; ++i) {
    std::vector<uint32_t> cfg(configs + (size_t)i * n, configs + (size_t)(i + 1) * n);
    ProtocolStats st;
    compute_stats(b, cfg, cl, st);
    double score;
    out_valid[i] = compute_score(n, st, rp, score) ? 1 : 0;
    out_score[i] = score;
  }
  ORACLE_CATCH
}

void oracle_colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out) {
  Binom B(ns, n);
  colex_unrank(B, rank, n, ns, out);
}

// Streaming sweep over colex ranks [rb, re) of n-subsets of `servers`
// (positions index `servers`), with the reference's compute_stats per config.
//   objs:       n_obj objectives (kind, slot pairs)
//   out_key/out_rank: n_obj x K records sorted by (key, rank); out_cnt[o] = filled
//   out_valid:  number of configs with a valid compute_score
//   out_digest: wrapping sum of per-config digests
//   threads:    std::thread workers over contiguous rank chunks
//   keys:       0 the compute_stats keys; 1 the extended key set (compute_stats_x)
int oracle_sweep_x(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                   uint32_t nc, uint32_t n, uint64_t rb, uint64_t re, const uint32_t* objs,
                   uint32_t n_obj, uint32_t K, const double* rparams, int ft_metric, uint32_t keys,
                   uint32_t threads, uint64_t* out_key, uint64_t* out_rank, uint32_t* out_cnt,
                   uint64_t* out_valid, uint64_t* out_digest) {
  ORACLE_TRY
  const Planet* P = (Planet*)h;
  Bote b{P};
  std::vector<uint32_t> cl(clients, clients + nc);
  std::vector<Objective> ob(n_obj);
  for (uint32_t o = 0; o < n_obj; ++o) ob[o] = {objs[2 * o], objs[2 * o + 1]};
  RankingParams rp{rparams[0], rparams[1], rparams[2], rparams[3], 3, 13, ft_metric};
  Binom B(ns, n);
  if (threads == 0) threads = 1;
  uint64_t total = re > rb ? re - rb : 0;
  std::vector<std::vector<TopK>> tops(threads, std::vector<TopK>(n_obj, TopK{K, {}}));
  std::vector<uint64_t> valid(threads, 0), digest(threads, 0);
  std::vector<std::string> errs(threads);
  auto work = [&](uint32_t t) {
    try {
      uint64_t a = rb + total * t / threads, e = rb + total * (t + 1) / threads;
      std::vector<uint32_t> pos(n), cfg(n);
      for (uint64_t r = a; r < e; ++r) {
        colex_unrank(B, r, n, ns, pos.data());
        for (uint32_t j = 0; j < n; ++j) cfg[j] = servers[pos[j]];
        ProtocolStats st;
        if (keys) compute_stats_x(b, cfg, cl, st);
        else compute_stats(b, cfg, cl, st);
        double score;
        if (compute_score(n, st, rp, score)) valid[t]++;
        digest[t] += config_digest(r, st);
        for (uint32_t o = 0; o < n_obj; ++o) {
          uint64_t key;
          if (objective_key(ob[o], n, st, rp, key)) tops[t][o].push(key, r);
        }
      }
    } catch (const std::exception& ex) {
      errs[t] = ex.what();
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Panic(e);
  *out_valid = 0;
  *out_digest = 0;
  for (uint32_t t = 0; t < threads; ++t) {
    *out_valid += valid[t];
    *out_digest += digest[t];
  }
  for (uint32_t o = 0; o < n_obj; ++o) {
    TopK m{K, {}};
    for (uint32_t t = 0; t < threads; ++t)
      for (auto& e : tops[t][o].v) m.push(e.first, e.second);
    out_cnt[o] = (uint32_t)m.v.size();
    for (size_t i = 0; i < m.v.size(); ++i) {
      out_key[(size_t)o * K + i] = m.v[i].first;
      out_rank[(size_t)o * K + i] = m.v[i].second;
    }
  }
  ORACLE_CATCH
}

// oracle_sweep_x over an explicit list of colex ranks (any order, repeats
// counted again): the CPU baseline's seeded uniform sample (bench.py).  Same
// per-config work: unrank, compute_stats[_x], compute_score, digest, the
// objectives' top-K.
int oracle_sweep_ranks(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                       uint32_t n, const uint64_t* ranks, uint64_t nranks, const uint32_t* objs, uint32_t n_obj,
                       uint32_t K, const double* rparams, int ft_metric, uint32_t keys, uint32_t threads,
                       uint64_t* out_key, uint64_t* out_rank, uint32_t* out_cnt, uint64_t* out_valid,
                       uint64_t* out_digest) {
  ORACLE_TRY
  const Planet* P = (Planet*)h;
  Bote b{P};
  std::vector<uint32_t> cl(clients, clients + nc);
  std::vector<Objective> ob(n_obj);
  for (uint32_t o = 0; o < n_obj; ++o) ob[o] = {objs[2 * o], objs[2 * o + 1]};
  RankingParams rp{rparams[0], rparams[1], rparams[2], rparams[3], 3, 13, ft_metric};
  Binom B(ns, n);
  const uint64_t total = B(ns, n);
  for (uint64_t i = 0; i < nranks; ++i)
    if (ranks[i] >= total) throw Panic("rank out of range");
  if (threads == 0) threads = 1;
  std::vector<std::vector<TopK>> tops(threads, std::vector<TopK>(n_obj, TopK{K, {}}));
  std::vector<uint64_t> valid(threads, 0), digest(threads, 0);
  std::vector<std::string> errs(threads);
  auto work = [&](uint32_t t) {
    try {
      std::vector<uint32_t> pos(n), cfg(n);
      for (uint64_t i = nranks * t / threads; i < nranks * (t + 1) / threads; ++i) {
        const uint64_t r = ranks[i];
        colex_unrank(B, r, n, ns, pos.data());
        for (uint32_t j = 0; j < n; ++j) cfg[j] = servers[pos[j]];
        ProtocolStats st;
        if (keys) compute_stats_x(b, cfg, cl, st);
        else compute_stats(b, cfg, cl, st);
        double score;
        if (compute_score(n, st, rp, score)) valid[t]++;
        digest[t] += config_digest(r, st);
        for (uint32_t o = 0; o < n_obj; ++o) {
          uint64_t key;
          if (objective_key(ob[o], n, st, rp, key)) tops[t][o].push(key, r);
        }
      }
    } catch (const std::exception& ex) {
      errs[t] = ex.what();
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Panic(e);
  *out_valid = 0;
  *out_digest = 0;
  for (uint32_t t = 0; t < threads; ++t) {
    *out_valid += valid[t];
    *out_digest += digest[t];
  }
  for (uint32_t o = 0; o < n_obj; ++o) {
    TopK m{K, {}};
    for (uint32_t t = 0; t < threads; ++t)
      for (auto& e : tops[t][o].v) m.push(e.first, e.second);
    out_cnt[o] = (uint32_t)m.v.size();
    for (size_t i = 0; i < m.v.size(); ++i) {
      out_key[(size_t)o * K + i] = m.v[i].first;
      out_rank[(size_t)o * K + i] = m.v[i].second;
    }
  }
  ORACLE_CATCH
}

int oracle_sweep(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                 uint32_t nc, uint32_t n, uint64_t rb, uint64_t re, const uint32_t* objs,
                 uint32_t n_obj, uint32_t K, const double* rparams, int ft_metric,
                 uint32_t threads, uint64_t* out_key, uint64_t* out_rank, uint32_t* out_cnt,
                 uint64_t* out_valid, uint64_t* out_digest) {
  return oracle_sweep_x(h, servers, ns, clients, nc, n, rb, re, objs, n_obj, K, rparams, ft_metric, 0, threads,
                        out_key, out_rank, out_cnt, out_valid, out_digest);
}

// compute_stats_x (the extended key set) for a batch of explicit configs
// (region ids, config order): exact moments per slot and per leader.
//   out_s1, out_s2:   ncfg x 20 (slots 0..19; ~0 where a slot is absent)
//   out_al1, out_al2: ncfg x 2 x n (all leaders, f = 1, 2, config order; ~0 when f > max_f)
//   out_leader:       ncfg COV-best leader positions (compute_stats)
int oracle_moments_x(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n, const uint32_t* clients,
                     uint32_t nc, uint32_t threads, uint64_t* out_s1, uint64_t* out_s2, uint64_t* out_al1,
                     uint64_t* out_al2, uint32_t* out_leader) {
  ORACLE_TRY
  Bote b{(Planet*)h};
  std::vector<uint32_t> cl(clients, clients + nc);
  if (threads == 0) threads = 1;
  std::vector<std::string> errs(threads);
  auto work = [&](uint32_t t) {
    try {
      for (uint64_t i = (uint64_t)ncfg * t / threads; i < (uint64_t)ncfg * (t + 1) / threads; ++i) {
        std::vector<uint32_t> cfg(configs + i * n, configs + (i + 1) * n);
        ProtocolStats st;
        compute_stats_x(b, cfg, cl, st);
        for (int s = 0; s < NKEYS_X; ++s) {
          uint64_t s1 = ~0ull, c = 0, s2 = ~0ull;
          if (st.has[s]) {
            st.h[s].sum_and_count(s1, c);
            s2 = st.h[s].sumsq();
          }
          out_s1[i * NKEYS_X + s] = s1;
          out_s2[i * NKEYS_X + s] = s2;
        }
        for (int f = 0; f < 2; ++f)
          for (uint32_t l = 0; l < n; ++l) {
            uint64_t s1 = ~0ull, c = 0, s2 = ~0ull;
            if (l < st.all_leaders[f].size()) {
              st.all_leaders[f][l].sum_and_count(s1, c);
              s2 = st.all_leaders[f][l].sumsq();
            }
            out_al1[(i * 2 + f) * n + l] = s1;
            out_al2[(i * 2 + f) * n + l] = s2;
          }
        out_leader[i] = (uint32_t)st.leader_pos;
      }
    } catch (const std::exception& ex) {
      errs[t] = ex.what();
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw Panic(e);
  ORACLE_CATCH
}

// Search::new + sorted_evolving_configs (search.rs:47-178) for a single client
// set (R13C13 / R17C17 / R20C20), configs enumerated in lexicographic order of
// positions in `servers` (permutator order is not pinned).
// Chains in the reference's order: score descending (BTreeMap<F64, Vec<_>>
// iterated in reverse), equal scores in nested-loop insertion order.
struct ChainSearch {
  struct CS {
    std::vector<uint32_t> set;  // sorted by name
    std::vector<bool> mask;
    ProtocolStats st;
  };
  struct F64Less {
    bool operator()(double a, double b) const { return f64_cmp(a, b) < 0; }
  };
  std::map<size_t, std::vector<CS>> configs;
  std::map<double, std::vector<std::vector<const CS*>>, F64Less> chains;
  uint64_t nchains = 0;

  ChainSearch(const Planet* P, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
              const RankingParams& rp) {
    Bote b{P};
    std::vector<uint32_t> cl(clients, clients + nc);
    for (size_t n = 3; n <= 13; n += 2) {
      auto& vec = configs[n];
      if (n > ns) continue;
      std::vector<uint32_t> idx(n);
      for (size_t j = 0; j < n; ++j) idx[j] = (uint32_t)j;
      for (;;) {
        CS cs;
        std::vector<uint32_t> cfg(n);
        for (size_t j = 0; j < n; ++j) cfg[j] = servers[idx[j]];
        compute_stats(b, cfg, cl, cs.st);
        cs.set = cfg;
        std::sort(cs.set.begin(), cs.set.end(),
                  [&](uint32_t a, uint32_t c) { return P->names[a] < P->names[c]; });
        cs.mask.assign(P->R, false);
        for (auto r : cfg) cs.mask[r] = true;
        vec.push_back(std::move(cs));
        // lexicographic successor
        int j = (int)n - 1;
        while (j >= 0 && idx[j] == ns - n + j) --j;
        if (j < 0) break;
        ++idx[j];
        for (size_t k = j + 1; k < n; ++k) idx[k] = idx[k - 1] + 1;
      }
    }
    // rank (search.rs:329-354)
    std::map<size_t, std::vector<std::pair<double, const CS*>>> ranked;
    for (auto& kv : configs) {
      auto& out = ranked[kv.first];
      for (auto& cs : kv.second) {
        double score;
        if (compute_score(kv.first, cs.st, rp, score)) out.emplace_back(score, &cs);
      }
    }
    auto superset = [&](const CS& big, const CS& small) {
      for (auto r : small.set)
        if (!big.mask[r]) return false;
      return true;
    };
    auto supers = [&](size_t n, const CS& prev) {
      std::vector<std::pair<double, const CS*>> v;
      for (auto& e : ranked[n])
        if (superset(*e.second, prev) && min_mean_decrease(e.second->st, prev.st, n, rp)) v.push_back(e);
      return v;
    };
    for (auto& e3 : ranked[3])
      for (auto& e5 : supers(5, *e3.second))
        for (auto& e7 : supers(7, *e5.second))
          for (auto& e9 : supers(9, *e7.second))
            for (auto& e11 : supers(11, *e9.second))
              for (auto& e13 : supers(13, *e11.second)) {
                double sc = e3.first + e5.first;
                sc = sc + e7.first;
                sc = sc + e9.first;
                sc = sc + e11.first;
                sc = sc + e13.first;
                chains[sc].push_back({e3.second, e5.second, e7.second, e9.second, e11.second, e13.second});
                ++nchains;
              }
  }
};

int oracle_search_best(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients,
                       uint32_t nc, const double* rparams, int ft_metric, double* out_score,
                       uint32_t* out_chain, char* out_fmt, uint32_t fmt_cap,
                       uint64_t* out_nchains) {
  ORACLE_TRY
  const Planet* P = (Planet*)h;
  RankingParams rp{rparams[0], rparams[1], rparams[2], rparams[3], 3, 13, ft_metric};
  ChainSearch cs(P, servers, ns, clients, nc, rp);
  *out_nchains = cs.nchains;
  if (cs.chains.empty()) throw Panic("no chain");
  auto& best = *cs.chains.rbegin();
  *out_score = best.first;
  const auto& css = best.second.front();
  std::string fmt;
  for (size_t i = 0; i < 6; ++i) {
    for (size_t j = 0; j < 13; ++j)
      out_chain[i * 13 + j] = j < css[i]->set.size() ? css[i]->set[j] : ~0u;
    size_t n = css[i]->set.size();
    // search.rs:180-197 stats_fmt
    std::string line;
    for (int p = 0; p < 2; ++p) {
      const char* suf = p == 0 ? "" : "C";
      for (size_t f = 1; f <= max_f(n); ++f) {
        line += "af" + std::to_string(f) + suf + "=" + get(css[i]->st, slot_atlas(f) + 5 * p).debug_fmt() + " ";
        line += "ff" + std::to_string(f) + suf + "=" + get(css[i]->st, slot_fpaxos(f) + 5 * p).debug_fmt() + " ";
      }
      line += std::string("e") + suf + "=" + get(css[i]->st, K_E + 5 * p).debug_fmt() + " ";
    }
    fmt += line;
    fmt += "\n";
  }
  if (fmt.size() + 1 > fmt_cap) throw Panic("fmt buffer too small");
  memcpy(out_fmt, fmt.c_str(), fmt.size() + 1);
  ORACLE_CATCH
}

// The first K chains of sorted_evolving_configs in the reference's order:
//   out_score[k], out_chain[k][6][13] (region ids by name, ~0 padded); out_nchains = all chains.
//   out_digest: order-dependent digest of ALL chains (tests/test_gpu_chains.py):
//     h_k = bits(score_k); h_k = mix64(h_k ^ mask_l) for l = 0..5 (region-id bitmask, R <= 64);
//     digest = sum_k mix64(h_k + k) mod 2^64
int oracle_search_chains(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                         const double* rparams, int ft_metric, uint32_t K, double* out_score, uint32_t* out_chain,
                         uint64_t* out_nchains, uint64_t* out_digest) {
  ORACLE_TRY
  const Planet* P = (Planet*)h;
  if (P->R > 64) throw Panic("chain digest needs R <= 64");
  RankingParams rp{rparams[0], rparams[1], rparams[2], rparams[3], 3, 13, ft_metric};
  ChainSearch cs(P, servers, ns, clients, nc, rp);
  *out_nchains = cs.nchains;
  uint64_t k = 0, dig = 0;
  for (auto it = cs.chains.rbegin(); it != cs.chains.rend(); ++it)
    for (auto& ch : it->second) {
      if (k < K) {
        out_score[k] = it->first;
        for (size_t i = 0; i < 6; ++i)
          for (size_t j = 0; j < 13; ++j)
            out_chain[((size_t)k * 6 + i) * 13 + j] = j < ch[i]->set.size() ? ch[i]->set[j] : ~0u;
      }
      double sc = it->first;
      uint64_t hk;
      memcpy(&hk, &sc, 8);
      for (size_t i = 0; i < 6; ++i) {
        uint64_t m = 0;
        for (auto r : ch[i]->set) m |= 1ull << r;
        hk = mix64(hk ^ m);
      }
      dig += mix64(hk + k);
      ++k;
    }
  *out_digest = dig;
  ORACLE_CATCH
}

}  // extern "C"
