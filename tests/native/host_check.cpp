// Host-code checker for libbote_hip.so's host-only translation unit
// (fantoch_amd/csrc/bote_host.cpp), built with ASan + UBSan by
// tests/test_sanitize.py: colex ranks, the binomial table, the group walk and
// its chunk/shard cuts, quad layouts, the low table, fast-path eligibility and
// result-block unpacking, each against a direct restatement.  Prints
// "host ok" on success; any failed check exits 1.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../fantoch_amd/csrc/bote_host.hpp"

using namespace bote::host;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                 \
    }                                                             \
  } while (0)

// Direct restatement of a cost-balanced cut: walk every group of [rb, re)
// with per-group binomials (no table, no cache), cost ceil(len / 64) + gc.
static std::vector<uint64_t> direct_chunks(uint32_t ns, uint32_t n, uint32_t nc, uint64_t rb, uint64_t re,
                                           uint32_t nchunks) {
  std::vector<uint64_t> out;
  const uint32_t F = n - 3;
  std::vector<uint32_t> p(n);
  colex_unrank(rb, n, ns, p.data());
  std::vector<uint32_t> q(p.begin() + 3, p.end());
  std::vector<uint64_t> gb, gl;
  std::vector<double> gc;
  double total = 0;
  const double G = group_cost(nc);
  for (;;) {
    uint64_t base = 0;
    for (uint32_t k = 0; k < F; ++k) base += binom_u64(q[k], k + 4);
    const uint64_t g = binom_u64(q[0], 3);
    const uint64_t b = std::max(base, rb), e = std::min(base + g, re);
    if (b >= re) break;
    if (e > b) {
      gb.push_back(b);
      gl.push_back(e - b);
      gc.push_back((double)((e - b + 63) / 64) + G);
      total += gc.back();
    }
    if (e >= re) break;
    uint32_t k = 0;
    while (k < F && q[k] + 1 >= (k + 1 < F ? q[k + 1] : ns)) ++k;
    if (k == F) break;
    ++q[k];
    for (uint32_t j = 0; j < k; ++j) q[j] = 3 + j;
  }
  out.push_back(rb);
  double cum = 0;
  size_t i = 0;
  for (uint32_t c = 1; c < nchunks; ++c) {
    const double tgt = total * c / nchunks;
    while (i < gc.size() && cum + gc[i] <= tgt) cum += gc[i++];
    uint64_t bnd = re;
    if (i < gc.size()) bnd = gb[i] + (uint64_t)((tgt - cum) / gc[i] * (double)gl[i]);
    out.push_back(std::max(out.back(), std::min(bnd, re)));
  }
  out.push_back(re);
  return out;
}

static void check_binomials() {
  for (uint32_t ns : {1u, 5u, 20u, 64u, 128u, 130u, 256u}) {
    const uint32_t n = 16;
    const auto t = binom_table(ns, n);
    for (uint32_t m = 0; m <= ns; ++m)
      for (uint32_t k = 0; k <= n; ++k) CHECK(t[(size_t)m * (n + 1) + k] == binom_u64(m, k));
  }
  CHECK(binom_u64(64, 7) == 621216192ull);
  CHECK(binom_u64(128, 6) == 5423611200ull);
  CHECK(binom_u64(256, 16) == 0);  // overflow is 0
}

static void check_unrank() {
  std::mt19937_64 rng(7);
  const uint32_t shapes[][2] = {{20, 5}, {64, 7}, {128, 6}, {17, 13}, {5, 5}};
  for (auto& sh : shapes) {
    const uint32_t ns = sh[0], n = sh[1];
    const uint64_t total = binom_u64(ns, n);
    std::vector<uint32_t> p(n);
    for (int i = 0; i < 2000; ++i) {
      const uint64_t r = i < 2 ? (i == 0 ? 0 : total - 1) : rng() % total;
      CHECK(colex_unrank(r, n, ns, p.data()));
      for (uint32_t j = 1; j < n; ++j) CHECK(p[j - 1] < p[j]);
      CHECK(p[n - 1] < ns);
      CHECK(colex_rank(p.data(), n) == r);
    }
    CHECK(!colex_unrank(total, n, ns, p.data()));
  }
}

static void check_walk() {
  // the bench workload: R=64 n=7, every group of the rank space
  const uint32_t ns = 64, n = 7, nc = 64;
  const uint64_t total = binom_u64(ns, n);
  const auto t0 = std::chrono::steady_clock::now();
  auto w = walk_groups(ns, n, nc, 0, total);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  CHECK(w != nullptr);
  if (!w) return;
  std::printf("walk R=64 n=7: %zu groups in %.1f ms\n", w->start.size(), ms);
  CHECK(w->start.size() == binom_u64(ns - 3, n - 3));
  uint64_t at = 0;
  for (size_t i = 0; i < w->start.size(); ++i) {
    CHECK(w->start[i] == at);
    CHECK(w->len[i] > 0);
    at += w->len[i];
  }
  CHECK(at == total);
  // cuts: against the direct restatement, over the full range and sub-ranges
  // (a shard's chunk table cut from the shared full-range walk)
  for (uint32_t parts : {1u, 2u, 3u, 8u, 9u}) {
    const auto a = cut_chunks(*w, 0, total, parts), b = direct_chunks(ns, n, nc, 0, total, parts);
    CHECK(a == b);
    CHECK(a.size() == parts + 1 && a.front() == 0 && a.back() == total);
    for (size_t i = 1; i < a.size(); ++i) CHECK(a[i - 1] <= a[i]);
  }
  const auto sh = cut_chunks(*w, 0, total, 8);
  for (size_t i = 0; i + 1 < sh.size(); ++i) {
    const auto a = cut_chunks(*w, sh[i], sh[i + 1], 256);
    const auto b = direct_chunks(ns, n, nc, sh[i], sh[i + 1], 256);
    CHECK(a == b);
    auto ws = walk_groups(ns, n, nc, sh[i], sh[i + 1]);
    CHECK(ws && cut_chunks(*ws, sh[i], sh[i + 1], 256) == a);
  }
  // ranges that split a group, tiny ranges, one-config ranges
  std::mt19937_64 rng(11);
  for (int i = 0; i < 200; ++i) {
    uint64_t b = rng() % total, e = std::min(total, b + 1 + rng() % 5000);
    const auto a = cut_chunks(*w, b, e, 1 + rng() % 40);
    const uint32_t k = (uint32_t)a.size() - 1;
    CHECK(a == direct_chunks(ns, n, nc, b, e, k));
  }
  CHECK(cut_chunks(*w, 5, 5, 4).empty());
  // the guided table of a full launch (4,096 waves, 32 chunks per wave, 3
  // tail rounds): ascending, covering [0, total), the base-size chunks then
  // 3 rounds of 4,096 chunks of 1/2, 1/4, 1/8 of the base size
  {
    const uint32_t nw = 4096, cpw = 32;
    const auto g = cut_chunks_guided(*w, 0, total, nw * cpw, nw, 3);
    CHECK(g.front() == 0 && g.back() == total);
    for (size_t i = 1; i < g.size(); ++i) CHECK(g[i - 1] <= g[i]);
    const size_t nch = g.size() - 1;
    CHECK(nch > 3 * (size_t)nw && nch < (size_t)nw * cpw + 3 * nw);
    auto span = [&](size_t i) { return (double)(g[i + 1] - g[i]); };
    double head = 0, t1 = 0, t3 = 0;
    for (size_t i = 0; i < nch - 3 * nw; ++i) head += span(i);
    for (size_t i = nch - 3 * nw; i < nch - 2 * nw; ++i) t1 += span(i);
    for (size_t i = nch - nw; i < nch; ++i) t3 += span(i);
    head /= (double)(nch - 3 * nw);
    t1 /= nw;
    t3 /= nw;
    std::printf("guided chunks: %zu, mean ranks per chunk: base %.0f, tail 1/2 %.0f, tail 1/8 %.0f\n", nch, head, t1, t3);
    CHECK(t1 < 0.7 * head && t3 < 0.25 * head);
    // no tail: the equal-cost table; too few chunks per wave for a tail: the same
    CHECK(cut_chunks_guided(*w, 0, total, nw * cpw, 0, 3) == cut_chunks(*w, 0, total, nw * cpw));
    CHECK(cut_chunks_guided(*w, 0, total, nw * 8, nw, 3) == cut_chunks(*w, 0, total, nw * 8));
    // a shard's table
    const auto sg = cut_chunks_guided(*w, sh[3], sh[4], nw * 22, nw, 3);
    CHECK(sg.front() == sh[3] && sg.back() == sh[4]);
    for (size_t i = 1; i < sg.size(); ++i) CHECK(sg[i - 1] <= sg[i]);
  }
  // a walk does not serve a range it does not cover
  auto part = walk_groups(ns, n, nc, 1000, 2000);
  CHECK(part && part->covers(1000, 2000) && !part->covers(999, 2000));
  CHECK(cut_chunks(*part, 0, 2000, 4).empty());
  // R=128 n=6 (config 5) walk
  auto w2 = walk_groups(128, 6, 128, 0, binom_u64(128, 6));
  CHECK(w2 && w2->start.size() == binom_u64(125, 3));
  CHECK(walk_groups(64, 3, 64, 0, 10) == nullptr);  // n < 4: no groups
  CHECK(group_utilisation(64, 7) > 0.9);
}

static void check_layouts() {
  const uint32_t R = 9;
  std::vector<uint16_t> lat(R * R);
  for (uint32_t i = 0; i < R; ++i)
    for (uint32_t j = 0; j < R; ++j) lat[i * R + j] = i == j ? 0 : (uint16_t)(10 + 3 * i + j);
  const uint32_t rows[] = {4, 1, 7, 0, 8};
  uint32_t quads = 0, stride = 0;
  const auto m = quad_layout(lat.data(), R, rows, 5, 4, quads, stride);
  CHECK(quads == 2);
  CHECK(stride == 6);  // >= quads + 1, an odd number of 16-B units
  CHECK(m.size() == (size_t)R * stride * 4);
  for (uint32_t t = 0; t < R; ++t)
    for (uint32_t c = 0; c < stride * 4; ++c)
      CHECK(m[t * stride * 4 + c] == (c < 5 ? (uint16_t)(lat[rows[c] * R + t] << 4) : 0));
  for (uint32_t q = 0; q < 300; ++q) {
    const uint32_t s = quad_stride(q);
    CHECK(s >= q + 1 && s % 2 == 0 && (s / 2) % 2 == 1 && s <= q + 4);
  }
  CHECK(quad_stride(16) == 18 && quad_stride(32) == 34);
  const auto lt = low_table(10);
  CHECK(lt.size() == binom_u64(10, 3));
  for (size_t i = 0; i < lt.size(); ++i) {
    const uint32_t p[3] = {lt[i] & 0xFF, (lt[i] >> 8) & 0xFF, lt[i] >> 16};
    CHECK(colex_rank(p, 3) == i);
  }
  std::vector<uint32_t> srv(R);
  for (uint32_t i = 0; i < R; ++i) srv[i] = i;
  CHECK(fast_eligible(lat.data(), R, srv.data(), R, R, false));
  CHECK(!fast_eligible(lat.data(), R, srv.data(), R, R, true));
  CHECK(!fast_eligible(lat.data(), R, srv.data(), R, 1, false));
  std::swap(srv[0], srv[1]);
  CHECK(!fast_eligible(lat.data(), R, srv.data(), R, R, false));
  std::swap(srv[0], srv[1]);
  lat[2 * R + 3] = 0;  // a zero server-server latency
  CHECK(!fast_eligible(lat.data(), R, srv.data(), R, R, false));
  lat[2 * R + 3] = 4096;  // above the packed range
  CHECK(!fast_eligible(lat.data(), R, srv.data(), R, R, false));
}

static void check_unpack() {
  const uint32_t n_obj = 3, kp = 128, K = 5;
  std::vector<uint8_t> blk((size_t)n_obj * kp * 16 + 16, 0xFF);
  auto* r = (TopkRecord*)blk.data();
  for (uint32_t o = 0; o < n_obj; ++o)
    for (uint32_t i = 0; i < o + 3; ++i) r[o * kp + i] = TopkRecord{100u * o + i, 7u * i};
  uint64_t* cnt = (uint64_t*)(blk.data() + (size_t)n_obj * kp * 16);
  cnt[0] = 42;
  cnt[1] = 0xABCDEF;
  std::vector<TopkRecord> out(n_obj * K);
  uint32_t c[3];
  uint64_t valid = 0, dig = 0;
  unpack_result(blk.data(), n_obj, K, kp, out.data(), c, &valid, &dig);
  CHECK(valid == 42 && dig == 0xABCDEF);
  for (uint32_t o = 0; o < n_obj; ++o) {
    CHECK(c[o] == std::min(K, o + 3));
    for (uint32_t i = 0; i < K; ++i)
      CHECK(i < c[o] ? (out[o * K + i].key == 100u * o + i && out[o * K + i].rank == 7u * i)
                     : (out[o * K + i].key == ~0ull && out[o * K + i].rank == ~0ull));
  }
  unpack_result(blk.data(), n_obj, K, kp, nullptr, nullptr, nullptr, nullptr);  // all outputs optional
}

// The group geometry choice (bote_capi.hip): client-line coverage up to 8
// per wave first, then waves per CU, then more lines, then the smaller size;
// checked on the three measured R=128/R=64 cases.
static void check_geometry() {
  // R=64 n=7: 256 x 4 per CU vs 512 x 2, both 16 lines -> 256
  CHECK(pick_group_geometry(256, 4, 16, 0, 0, 0));
  CHECK(!pick_group_geometry(512, 2, 16, 256, 4, 16));
  // R=128 10 keys: 256 x 3 with 4 lines vs 512 x 2 with 16 -> 512
  CHECK(pick_group_geometry(512, 2, 16, 256, 3, 4));
  // extended keys: 256 x 3 without lines, 512 x 1, 768 x 1 (16 lines) -> 768
  CHECK(pick_group_geometry(512, 1, 16, 256, 3, 0));
  CHECK(pick_group_geometry(768, 1, 16, 512, 1, 16));
  CHECK(!pick_group_geometry(1024, 0, 16, 768, 1, 16));  // does not fit
  CHECK(!pick_group_geometry(256, 0, 0, 0, 0, 0));
}

// Chunks per wave (sweep_chunks): the cap on full sweeps, fewer on shards.
static void check_chunks_per_wave() {
  // R=64 n=7 on 4096 waves, 64 clients (group cost 0.64 steps)
  CHECK(chunks_per_wave(621216192ull, 4096, 64, 32) == 32);
  CHECK(chunks_per_wave(621216192ull / 8, 4096, 64, 32) == 22);
  CHECK(chunks_per_wave(621216192ull / 64, 4096, 64, 32) == 8);
  CHECK(chunks_per_wave(1000, 4096, 64, 32) == 4);
  CHECK(chunks_per_wave(5423611200ull, 4096, 128, 32) == 32);
  CHECK(chunks_per_wave(1ull << 40, 0, 64, 32) == 4);
  CHECK(chunks_per_wave(1ull << 40, 4096, 64, 2) == 2);
}

int main() {
  check_chunks_per_wave();
  check_geometry();
  check_binomials();
  check_unrank();
  check_walk();
  check_layouts();
  check_unpack();
  if (failures) {
    std::printf("%d host checks failed\n", failures);
    return 1;
  }
  std::printf("host ok\n");
  return 0;
}
