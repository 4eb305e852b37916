// bote_host.cpp — host-only pieces of libbote_hip.so (see bote_host.hpp).
// Plain C++ (g++), no HIP: sanitizer builds run it on any CPU.
#include "bote_host.hpp"

#include <algorithm>
#include <cmath>

namespace bote {
namespace host {

uint64_t binom_u64(uint32_t m, uint32_t k) {
  if (k > m) return 0;
  k = std::min(k, m - k);
  unsigned __int128 r = 1;
  for (uint32_t i = 1; i <= k; ++i) {
    r = r * (m - k + i) / i;
    if (r > (unsigned __int128)UINT64_MAX) return 0;
  }
  return (uint64_t)r;
}

std::vector<uint64_t> binom_table(uint32_t ns, uint32_t n) {
  // Pascal's rule, saturating at 0 (= overflow, as binom_u64) from the first
  // overflowing entry of a row on
  std::vector<uint64_t> t((size_t)(ns + 1) * (n + 1), 0);
  for (uint32_t m = 0; m <= ns; ++m) {
    t[(size_t)m * (n + 1)] = 1;
    for (uint32_t k = 1; k <= n && k <= m; ++k) {
      const uint64_t a = t[(size_t)(m - 1) * (n + 1) + k - 1];
      const uint64_t b = k <= m - 1 ? t[(size_t)(m - 1) * (n + 1) + k] : 0;
      const bool ovf = (a == 0) || (k <= m - 1 && b == 0) || b > UINT64_MAX - a;
      t[(size_t)m * (n + 1) + k] = ovf ? 0 : a + b;
    }
  }
  return t;
}

bool colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out) {
  if (n > ns) return false;
  const uint64_t total = binom_u64(ns, n);
  if (rank >= total) return false;
  uint64_t r = rank;
  uint32_t hi = ns;
  for (int j = (int)n - 1; j >= 0; --j) {
    const uint32_t k = (uint32_t)j + 1;
    uint32_t x = hi - 1;
    while (x > (uint32_t)j && binom_u64(x, k) > r) --x;
    out[j] = x;
    r -= binom_u64(x, k);
    hi = x;
  }
  return true;
}

uint64_t colex_rank(const uint32_t* pos, uint32_t n) {
  uint64_t r = 0;
  for (uint32_t j = 0; j < n; ++j) r += binom_u64(pos[j], j + 1);
  return r;
}

// Fitted per-group precompute, in wavefront steps: least squares over the
// per-shard kernel times of scripts/shard_balance.py (profiles/r02h_*): 0.64
// at 64 clients (n=7), 3.7 at 128 clients (n=6); a power of the client count
// in between, clamped outside.
#ifndef BOTE_GROUP_COST
#define BOTE_GROUP_COST 0.0  // 0: fitted per client count
#endif
double group_cost(uint32_t nc) {
  if (BOTE_GROUP_COST > 0) return BOTE_GROUP_COST;
  const double c = 0.64 * std::pow((double)nc / 64.0, 2.53);
  return std::min(8.0, std::max(0.25, c));
}

uint32_t chunks_per_wave(uint64_t ranks, uint32_t nwaves, uint32_t nc, uint32_t cap) {
  const uint32_t lo = std::min<uint32_t>(4, cap);
  if (nwaves == 0) return lo;
  const double T = (double)ranks / 64.0 / (double)nwaves;
  const double c = std::sqrt(T / group_cost(nc));
  return (uint32_t)std::max<double>(lo, std::min<double>(cap, std::floor(c + 0.5)));
}

std::shared_ptr<GroupWalk> walk_groups(uint32_t ns, uint32_t n, uint32_t nc, uint64_t rb, uint64_t re,
                                       uint64_t max_groups) {
  if (re <= rb || n < 4 || n > ns) return nullptr;
  const uint64_t total = binom_u64(ns, n);
  if (total == 0 || re > total) return nullptr;
  const uint32_t F = n - 3;
  const uint64_t all_groups = binom_u64(ns - 3, F);
  // too many groups to walk (each group holds at least one config)
  if ((all_groups == 0 || all_groups > max_groups) && re - rb > max_groups) return nullptr;
  const std::vector<uint64_t> T = binom_table(ns, n);
  auto C = [&](uint32_t m, uint32_t k) { return T[(size_t)m * (n + 1) + k]; };
  std::vector<uint32_t> p(n);
  if (!colex_unrank(rb, n, ns, p.data())) return nullptr;
  std::vector<uint32_t> q(p.begin() + 3, p.end());  // the fixed positions, a combination of {3 .. ns-1}
  auto w = std::make_shared<GroupWalk>();
  w->ns = ns;
  w->n = n;
  w->nc = nc;
  w->rb = rb;
  w->re = re;
  w->group_cost = group_cost(nc);
  const uint64_t expect = std::min<uint64_t>({all_groups ? all_groups : max_groups, re - rb, 1ull << 22});
  w->start.reserve(expect);
  w->len.reserve(expect);
  for (;;) {
    uint64_t base = 0;
    for (uint32_t k = 0; k < F; ++k) base += C(q[k], k + 4);
    const uint64_t g = C(q[0], 3);
    const uint64_t b = std::max(base, rb), e = std::min(base + g, re);
    if (b >= re) break;
    if (e > b) {
      w->start.push_back(b);
      w->len.push_back(e - b);
      if (w->start.size() > max_groups) return nullptr;
    }
    if (e >= re) break;
    // colex successor of the fixed positions
    uint32_t k = 0;
    while (k < F && q[k] + 1 >= (k + 1 < F ? q[k + 1] : ns)) ++k;
    if (k == F) break;
    ++q[k];
    for (uint32_t j = 0; j < k; ++j) q[j] = 3 + j;
  }
  return w;
}

// Boundaries of [b, e) at the given cumulative estimated costs (ascending,
// in wavefront steps; the first chunk starts at b, the last ends at e).
static std::vector<uint64_t> cut_at(const GroupWalk& w, uint64_t b, uint64_t e, const std::vector<double>& targets);

// The total estimated cost of [b, e) (ceil(len / 64) steps + the group cost
// per part of a group), the measure the chunk cuts divide.
static double range_cost(const GroupWalk& w, uint64_t b, uint64_t e) {
  const size_t i0 = (size_t)(std::upper_bound(w.start.begin(), w.start.end(), b) - w.start.begin()) - 1;
  const size_t i1 = (size_t)(std::lower_bound(w.start.begin(), w.start.end(), e) - w.start.begin());
  double total = 0;
  for (size_t i = i0; i < i1; ++i) {
    const uint64_t pb = std::max(w.start[i], b), pl = std::min(w.start[i] + w.len[i], e) - pb;
    total += (double)((pl + 63) / 64) + w.group_cost;
  }
  return total;
}

std::vector<uint64_t> cut_chunks_guided(const GroupWalk& w, uint64_t b, uint64_t e, uint32_t nchunks,
                                        uint32_t tail_waves, uint32_t levels) {
  if (e <= b || nchunks == 0 || !w.covers(b, e) || w.start.empty()) return {};
  // no tail unless the launch has at least 16 base chunks per wave (the tail
  // holds at most 1/16 of the work; on small shards, 8 chunks per wave, the
  // extra chunk-start precomputes cost more than the tail saves: r05q, 1/64
  // of R=64 n=7 0.496 vs 0.481 ms per step)
  if (tail_waves == 0 || levels == 0 || (uint64_t)nchunks < 16ull * tail_waves) return cut_chunks(w, b, e, nchunks);
  const double total = range_cost(w, b, e), c0 = total / nchunks;
  double tail = 0;
  for (uint32_t l = 1; l <= levels; ++l) tail += tail_waves * c0 / (double)(1u << l);
  const double head = total - tail;
  const uint32_t nh = (uint32_t)std::max(1.0, std::floor(head / c0 + 0.5));
  std::vector<double> t;
  t.reserve(nh + (size_t)levels * tail_waves);
  for (uint32_t i = 1; i <= nh; ++i) t.push_back(head * i / nh);
  double at = head;
  for (uint32_t l = 1; l <= levels; ++l)
    for (uint32_t k = 0; k < tail_waves; ++k) {
      at += c0 / (double)(1u << l);
      t.push_back(at);
    }
  t.back() = total;  // (rounding: the last chunk ends at e)
  return cut_at(w, b, e, t);
}

std::vector<uint64_t> cut_chunks(const GroupWalk& w, uint64_t b, uint64_t e, uint32_t nchunks) {
  std::vector<uint64_t> out;
  if (e <= b || nchunks == 0 || !w.covers(b, e) || w.start.empty()) return out;
  // the groups touching [b, e): the walk's clipped groups tile [rb, re)
  const size_t i0 = (size_t)(std::upper_bound(w.start.begin(), w.start.end(), b) - w.start.begin()) - 1;
  const size_t i1 = (size_t)(std::lower_bound(w.start.begin(), w.start.end(), e) - w.start.begin());  // one past
  auto part = [&](size_t i, uint64_t& pb, uint64_t& pl) {
    pb = std::max(w.start[i], b);
    pl = std::min(w.start[i] + w.len[i], e) - pb;
  };
  auto cost = [&](uint64_t pl) { return (double)((pl + 63) / 64) + w.group_cost; };
  double total = 0;
  for (size_t i = i0; i < i1; ++i) {
    uint64_t pb, pl;
    part(i, pb, pl);
    total += cost(pl);
  }
  out.reserve((size_t)nchunks + 1);
  out.push_back(b);
  double cum = 0;
  size_t i = i0;
  for (uint32_t c = 1; c < nchunks; ++c) {
    const double tgt = total * c / nchunks;
    uint64_t pb = 0, pl = 0;
    while (i < i1) {
      part(i, pb, pl);
      if (cum + cost(pl) > tgt) break;
      cum += cost(pl);
      ++i;
    }
    uint64_t bnd = e;
    if (i < i1) bnd = pb + (uint64_t)((tgt - cum) / cost(pl) * (double)pl);
    out.push_back(std::max(out.back(), std::min(bnd, e)));
  }
  out.push_back(e);
  return out;
}

static std::vector<uint64_t> cut_at(const GroupWalk& w, uint64_t b, uint64_t e, const std::vector<double>& targets) {
  std::vector<uint64_t> out;
  const size_t i0 = (size_t)(std::upper_bound(w.start.begin(), w.start.end(), b) - w.start.begin()) - 1;
  const size_t i1 = (size_t)(std::lower_bound(w.start.begin(), w.start.end(), e) - w.start.begin());
  auto part = [&](size_t i, uint64_t& pb, uint64_t& pl) {
    pb = std::max(w.start[i], b);
    pl = std::min(w.start[i] + w.len[i], e) - pb;
  };
  auto cost = [&](uint64_t pl) { return (double)((pl + 63) / 64) + w.group_cost; };
  out.reserve(targets.size() + 1);
  out.push_back(b);
  double cum = 0;
  size_t i = i0;
  for (size_t c = 0; c + 1 < targets.size(); ++c) {
    const double tgt = targets[c];
    uint64_t pb = 0, pl = 0;
    while (i < i1) {
      part(i, pb, pl);
      if (cum + cost(pl) > tgt) break;
      cum += cost(pl);
      ++i;
    }
    uint64_t bnd = e;
    if (i < i1) bnd = pb + (uint64_t)((tgt - cum) / cost(pl) * (double)pl);
    out.push_back(std::max(out.back(), std::min(bnd, e)));
  }
  out.push_back(e);
  return out;
}

// groups with smallest fixed position k hold C(k, 3) configs and run in
// ceil(C(k, 3) / 64) wavefront steps
double group_utilisation(uint32_t ns, uint32_t n) {
  if (n < 4 || n > ns) return 0.0;
  const uint32_t F = n - 3;
  long double cfg = 0, steps = 0;
  for (uint32_t k = 3; k + F <= ns; ++k) {
    const long double groups = (long double)binom_u64(ns - 1 - k, F - 1);
    const uint64_t g = binom_u64(k, 3);
    cfg += groups * g;
    steps += groups * (long double)((g + 63) / 64);
  }
  return steps > 0 ? (double)(cfg / (64 * steps)) : 0.0;
}

bool pick_group_geometry(uint32_t bd, int occ, uint32_t gslots, uint32_t best_bd, int best_occ,
                         uint32_t best_gslots) {
  if (occ <= 0) return false;
  if (best_occ <= 0) return true;
  // client lines for most steps first (up to 8 per wave: a step has 7.7
  // distinct (p1, p2) on average at R=64 n=7, 4.0 at R=128 n=6), then more
  // waves per CU, more client lines, the smaller size.  Measured at R=128
  // n=6: 10 keys 203.4 ms at 256 threads (3 workgroups per
  // CU, 4 lines) vs 183.3 ms at 512 (2 per CU, 16 lines); extended keys
  // 389.2 ms at 256 (no lines) vs 351.5 ms at 512 (1 per CU, 16 lines)
  const uint32_t c = std::min<uint32_t>(gslots, 8), bc = std::min<uint32_t>(best_gslots, 8);
  if (c != bc) return c > bc;
  const uint32_t w = (uint32_t)occ * (bd / 64), bw = (uint32_t)best_occ * (best_bd / 64);
  if (w != bw) return w > bw;
  if (gslots != best_gslots) return gslots > best_gslots;
  return bd < best_bd;
}

uint32_t quad_stride(uint32_t quads) {
  uint32_t s = quads + 1;
  if (s & 1) ++s;
  if ((s / 2) % 2 == 0) s += 2;
  return s;
}

std::vector<uint16_t> quad_layout(const uint16_t* lat, uint32_t R, const uint32_t* rows, uint32_t nrows,
                                  uint32_t shift, uint32_t& quads, uint32_t& stride) {
  quads = (nrows + 3) / 4;
  stride = quad_stride(quads);
  const uint32_t su16 = stride * 4;  // u16 per column
  std::vector<uint16_t> m((size_t)R * su16, 0);
  for (uint32_t t = 0; t < R; ++t)
    for (uint32_t c = 0; c < nrows; ++c) m[(size_t)t * su16 + c] = (uint16_t)(lat[(size_t)rows[c] * R + t] << shift);
  return m;
}

std::vector<uint32_t> low_table(uint32_t m) {
  std::vector<uint32_t> t;
  t.reserve(binom_u64(m, 3));
  for (uint32_t p2 = 2; p2 < m; ++p2)
    for (uint32_t p1 = 1; p1 < p2; ++p1)
      for (uint32_t p0 = 0; p0 < p1; ++p0) t.push_back(p0 | (p1 << 8) | (p2 << 16));
  return t;
}

bool fast_eligible(const uint16_t* lat, uint32_t R, const uint32_t* servers, uint32_t ns, uint32_t nc,
                   bool fairness_threshold) {
  if (nc < 2) return false;
  if (!std::is_sorted(servers, servers + ns)) return false;
  if (fairness_threshold) return false;
  for (size_t i = 0; i < (size_t)R * R; ++i)
    if (lat[i] > 4095) return false;
  for (uint32_t i = 0; i < ns; ++i)
    for (uint32_t j = 0; j < ns; ++j) {
      const uint16_t v = lat[(size_t)servers[i] * R + servers[j]];
      if (i == j ? v != 0 : v == 0) return false;
    }
  return true;
}

void unpack_result(const uint8_t* blk, uint32_t n_obj, uint32_t K, uint32_t kp, TopkRecord* out, uint32_t* out_count,
                   uint64_t* out_valid, uint64_t* out_digest) {
  const TopkRecord* r = (const TopkRecord*)blk;
  for (uint32_t o = 0; o < n_obj; ++o) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < K && i < kp; ++i) {
      const TopkRecord x = r[(size_t)o * kp + i];
      if (x.key == ~0ull && x.rank == ~0ull) break;
      if (out) out[(size_t)o * K + i] = x;
      ++c;
    }
    for (uint32_t i = c; out && i < K; ++i) out[(size_t)o * K + i] = TopkRecord{~0ull, ~0ull};
    if (out_count) out_count[o] = c;
  }
  const uint64_t* cnt = (const uint64_t*)(blk + (size_t)n_obj * kp * 16);
  if (out_valid) *out_valid = cnt[0];
  if (out_digest) *out_digest = cnt[1];
}

}  // namespace host
}  // namespace bote
