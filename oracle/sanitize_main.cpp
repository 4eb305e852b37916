// TEST INFRASTRUCTURE: host sanitizer driver for the CPU oracle.  Built with
// -fsanitize=address,undefined together with bote_oracle.cpp (oracle/Makefile
// target build/oracle_sanitize) and run by tests/test_sanitize.py.  It drives
// every oracle entry point the parity tests use over a small deterministic
// planet with ties, multiple threads included, plus the documented error paths.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
const char* oracle_last_error();
void* oracle_planet_new(const uint16_t* lat, uint32_t R, const char* names);
void oracle_planet_free(void* h);
int oracle_planet_sorted(void* h, uint32_t from, uint32_t* out_regions, uint64_t* out_lat);
int oracle_quorum_latency(void* h, uint32_t from, const uint32_t* regions, uint32_t nr, uint32_t q, uint64_t* out);
int oracle_leaderless(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                      uint32_t q, uint64_t* out);
int oracle_best_leader(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                       uint32_t q, int stat, uint32_t* out);
int oracle_hist_stats(const uint64_t* v, uint32_t n, double* out);
int oracle_hist_fmt(const uint64_t* v, uint32_t n, char* buf, uint32_t cap);
int oracle_compute_stats(void* h, const uint32_t* configs, uint32_t ncfg, uint32_t n, const uint32_t* clients,
                         uint32_t nc, uint64_t* out_vals, uint32_t* out_leader);
void oracle_colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out);
int oracle_sweep(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc, uint32_t n,
                 uint64_t rb, uint64_t re, const uint32_t* objs, uint32_t n_obj, uint32_t K, const double* rparams,
                 int ft_metric, uint32_t threads, uint64_t* out_key, uint64_t* out_rank, uint32_t* out_cnt,
                 uint64_t* out_valid, uint64_t* out_digest);
int oracle_search_best(void* h, const uint32_t* servers, uint32_t ns, const uint32_t* clients, uint32_t nc,
                       const double* rparams, int ft_metric, double* out_score, uint32_t* out_chain, char* out_fmt,
                       uint32_t fmt_cap, uint64_t* out_nchains);
}

int main() {
  const uint32_t R = 14;
  std::vector<uint16_t> lat(R * R);
  uint64_t z = 0x5EED;
  for (uint32_t i = 0; i < R; ++i)
    for (uint32_t j = 0; j < R; ++j) {
      z = z * 6364136223846793005ull + 1442695040888963407ull;
      lat[i * R + j] = i == j ? 0 : (uint16_t)(5 + (z >> 33) % 40);  // small range: many ties
    }
  std::string names;
  for (uint32_t i = 0; i < R; ++i) {
    char b[8];
    snprintf(b, sizeof b, "r%02u", i);
    names += b;
    names.push_back('\0');
  }
  void* p = oracle_planet_new(lat.data(), R, names.data());
  std::vector<uint32_t> all(R), regs(R);
  std::vector<uint64_t> l64(R);
  for (uint32_t i = 0; i < R; ++i) all[i] = i;
  int bad = 0;
  bad |= oracle_planet_sorted(p, 3, regs.data(), l64.data());
  uint64_t q = 0;
  bad |= oracle_quorum_latency(p, 2, all.data(), 5, 3, &q);
  bad |= oracle_leaderless(p, all.data(), 5, all.data(), R, 3, l64.data());
  uint32_t pos = 0;
  bad |= oracle_best_leader(p, all.data(), 7, all.data(), R, 2, 1, &pos);
  std::vector<uint64_t> h = {3, 3, 7, 1, 9};
  double st[6];
  char buf[1024];
  bad |= oracle_hist_stats(h.data(), (uint32_t)h.size(), st);
  bad |= oracle_hist_fmt(h.data(), (uint32_t)h.size(), buf, sizeof buf);
  const uint32_t n = 5, ncfg = 200;
  std::vector<uint32_t> cfg(ncfg * n);
  for (uint32_t r = 0; r < ncfg; ++r) oracle_colex_unrank(r * 9, n, R, &cfg[r * n]);
  std::vector<uint64_t> vals((size_t)ncfg * (5 * R + 5 * n));
  std::vector<uint32_t> lead(ncfg);
  bad |= oracle_compute_stats(p, cfg.data(), ncfg, n, all.data(), R, vals.data(), lead.data());
  const uint32_t objs[10] = {0, 0, 1, 0, 1, 1, 2, 0, 1, 4};
  const double rp[4] = {1.0, 0.0, 0.0, 0.0};
  std::vector<uint64_t> keys(5 * 16), ranks(5 * 16);
  std::vector<uint32_t> cnt(5);
  uint64_t valid = 0, digest = 0;
  bad |= oracle_sweep(p, all.data(), R, all.data(), R, 6, 0, 3003, objs, 5, 16, rp, 2, 3, keys.data(), ranks.data(),
                      cnt.data(), &valid, &digest);
  double score = 0;
  std::vector<uint32_t> chain(6 * 13);
  uint64_t nch = 0;
  std::vector<char> fmt(1 << 16);
  const double rp2[4] = {0.0, 0.0, 0.0, 0.0};
  int rc = oracle_search_best(p, all.data(), 13, all.data(), 13, rp2, 2, &score, chain.data(), fmt.data(),
                              (uint32_t)fmt.size(), &nch);
  // error paths: a quorum larger than the server set must fail cleanly
  const int err = oracle_quorum_latency(p, 0, all.data(), 2, 3, &q);
  oracle_planet_free(p);
  printf("sanitize: calls %s, search rc=%d, error path %s (%s), valid=%llu digest=%llu\n", bad ? "FAILED" : "ok", rc,
         err ? "ok" : "MISSING", oracle_last_error(), (unsigned long long)valid, (unsigned long long)digest);
  return bad || !err ? 1 : 0;
}
