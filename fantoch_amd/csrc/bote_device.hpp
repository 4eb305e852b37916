// bote_device.hpp — device-side building blocks for the gfx950 configuration
// search.  Integer min/select work on VALU; no MFMA (DESIGN.md "Roofline").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace bote {

constexpr int MAXN = 16;
constexpr int KP = 128;      // top-K list capacity per objective (K <= KP)
constexpr int MAXOBJ = 8;
constexpr uint32_t LAT_SHIFT = 4;  // LDS matrix holds latency << 4; low 4 bits = member index

// ------------------------------------------------------- compile-time config
// Quorum sizes for a config of size N (fantoch_bote/src/protocol.rs:20-35,
// search.rs:474-477).  Leaderless keys af1/af2/e need the q-th closest server
// of the client's nearest server; those q's (deduplicated) are "LQ".
template <int N>
struct QCfg {
  static constexpr int maxf = (N / 2 < 2) ? N / 2 : 2;
  static constexpr int m = N / 2;
  static constexpr int qa1 = m + 1;
  static constexpr int qa2 = m + 2;
  static constexpr int qe = m + (m + 1) / 2;
  static constexpr int qf1 = 2;
  static constexpr int qf2 = 3;
  // leaderless distinct q list
  static constexpr int lq0 = qa1;
  static constexpr bool a2_new = (maxf >= 2) && (qa2 != qa1);
  static constexpr int lq1 = a2_new ? qa2 : qe;
  static constexpr bool e_new = (qe != qa1) && !(maxf >= 2 && qe == qa2);
  static constexpr int NL = 1 + (a2_new ? 1 : 0) + (e_new ? 1 : 0);
  static constexpr int lq2 = qe;
  static constexpr int idx_a1 = 0;
  static constexpr int idx_a2 = a2_new ? 1 : 0;
  static constexpr int idx_e = (qe == qa1) ? 0 : ((maxf >= 2 && qe == qa2) ? 1 : (a2_new ? 2 : 1));
  __host__ __device__ static constexpr int lq(int i) { return i == 0 ? lq0 : (i == 1 ? (a2_new ? qa2 : qe) : qe); }
};

// Leaderless quorum tables of a config of size N: the compute_stats q's
// (QCfg::lq, tables 0 .. NL-1) and, with the extended key set (X: BASELINE
// config 5, include/bote_hip.h BOTE_KEYS_TEMPO_ALL_LEADERS), Tempo's tiny fast
// quorum 2f and write quorum f + 1 (fantoch/src/config.rs:317-329) where not
// already among them, ascending (tables NL .. NT-1).
template <int N, bool X>
struct QTab {
  using QC = QCfg<N>;
  static constexpr bool base_has(int q) {
    for (int t = 0; t < QC::NL; ++t)
      if (QC::lq(t) == q) return true;
    return false;
  }
  // Tempo's q's: f = 1: tiny 2, write 2; f = 2: tiny 4, write 3
  static constexpr bool ext(int q) { return X && (q == 2 || (QC::maxf >= 2 && (q == 3 || q == 4))) && !base_has(q); }
  static constexpr int NX = (ext(2) ? 1 : 0) + (ext(3) ? 1 : 0) + (ext(4) ? 1 : 0);
  static constexpr int NT = QC::NL + NX;
  __host__ __device__ static constexpr int q(int t) {
    if (t < QC::NL) return QC::lq(t);
    int k = t - QC::NL;
    for (int qq = 2; qq <= 4; ++qq)
      if (ext(qq)) {
        if (k == 0) return qq;
        --k;
      }
    return 0;
  }
  // table holding quorum size qq (-1: none)
  __host__ __device__ static constexpr int idx(int qq) {
    for (int t = 0; t < NT; ++t)
      if (q(t) == qq) return t;
    return -1;
  }
};

// Slots of the extended key set (include/bote_hip.h): 10 + 4 * placement +
// {tt1, tt2, tw1, tw2}; 18, 19 FPaxos under the best-by-mean leader (Input).
constexpr int NSLOT_X = 20;
enum { SLOT_TT1 = 10, SLOT_TT2 = 11, SLOT_TW1 = 12, SLOT_TW2 = 13, SLOT_FL1 = 18, SLOT_FL2 = 19 };
// slot s exists for config size N (f = 2 keys need max_f >= 2)
template <int N>
__host__ __device__ constexpr bool slot_exists(int s) {
  if (s < 10) {
    const int b = s % 5;
    return !((b == 2 || b == 3) && QCfg<N>::maxf < 2);
  }
  if (s < 18) return (s - 10) % 2 == 0 || QCfg<N>::maxf >= 2;  // tt2/tw2 (odd offsets) need f = 2
  return s == 18 || QCfg<N>::maxf >= 2;
}

// ----------------------------------------------------------- small helpers
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t orderable_f64(double x) {
  if (x != x) x = __longlong_as_double(0x7FF8000000000000ll);
  uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// F64 total order (fantoch/src/metrics/float.rs:62-79): NaN greatest.
__device__ __forceinline__ int f64_cmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  if (a == b) return 0;
  bool an = a != a, bn = b != b;
  if (an && bn) return 0;
  return an ? 1 : -1;
}

// Batcher odd-even merge sort network over a[0..P), P a power of two,
// fully unrolled (all indices are compile-time constants).
template <int P, typename T>
__device__ __forceinline__ void sort_network(T* a) {
#pragma unroll
  for (int p = 1; p < P; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < P; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          if (i + j + k < P && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            T x = a[i + j], y = a[i + j + k];
            a[i + j] = x < y ? x : y;
            a[i + j + k] = x < y ? y : x;
          }
        }
      }
    }
  }
}

template <int N>
struct Pow2 {
  static constexpr int v = N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : 16;
};

// --------------------------------------------- exact moment comparisons ----
// Moments of one histogram: count, exact sum and sum of squares.
struct Mom {
  uint64_t s1, s2;
  uint32_t cnt;
};

struct U128 {
  uint64_t hi, lo;
};
__device__ __forceinline__ U128 mul64(uint64_t a, uint64_t b) { return U128{__umul64hi(a, b), a * b}; }
__device__ __forceinline__ bool lt128(U128 a, U128 b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
__device__ __forceinline__ U128 sub128(U128 a, U128 b) {
  return U128{a.hi - b.hi - (a.lo < b.lo ? 1ull : 0ull), a.lo - b.lo};
}
__device__ __forceinline__ U128 shr128(U128 a, int s) {
  return U128{a.hi >> s, (a.lo >> s) | (a.hi << (64 - s))};
}

// V = count * sum(x^2) - sum(x)^2 = count * (count-1) * variance (exact).
__device__ __forceinline__ uint64_t mom_v(const Mom& m) { return (uint64_t)m.cnt * m.s2 - m.s1 * m.s1; }
// Histogram::cov (histogram.rs:193-197) is NaN when count <= 1 (0/0 variance)
// or when the mean is 0 (0/0).
__device__ __forceinline__ bool cov_nan(const Mom& m) { return m.cnt <= 1 || m.s1 == 0; }

enum { CMP_LT = -1, CMP_EQ = 0, CMP_GT = 1, CMP_AMBIG = 2 };

// Compare the reference's f64 COV of two histograms from exact moments.
// The reference's computed COV carries a relative error below ~1e-14
// (DESIGN.md "Exactness"); exact COV^2 ratios that differ by more than 2^-30
// relative therefore order the same way in f64.  Closer calls return
// CMP_AMBIG and the caller replays the reference arithmetic.
__device__ __forceinline__ int cov_cmp(const Mom& a, const Mom& b) {
  bool an = cov_nan(a), bn = cov_nan(b);
  if (an || bn) return (an && bn) ? CMP_EQ : (an ? CMP_GT : CMP_LT);
  uint64_t va = mom_v(a), vb = mom_v(b);
  if (va == 0 && vb == 0) return CMP_EQ;  // both exactly 0.0
  U128 x = mul64(va, b.s1 * b.s1), y = mul64(vb, a.s1 * a.s1);
  bool xl = lt128(x, y);
  U128 big = xl ? y : x, diff = xl ? sub128(y, x) : sub128(x, y);
  U128 tol = shr128(big, 30);
  if (!lt128(tol, diff)) return CMP_AMBIG;
  return xl ? CMP_LT : CMP_GT;
}

// Histogram::mean (histogram.rs:172-181): exact sum / count, one rounding.
__device__ __forceinline__ double mom_mean(const Mom& m) { return (double)m.s1 / (double)m.cnt; }
// COV from exact moments (sqrt(V / (c (c-1))) / mean): within a few ulp of the
// reference value; used for outputs, not for decisions.
__device__ __forceinline__ double mom_cov(const Mom& m) {
  double c = (double)m.cnt;
  double var = (double)mom_v(m) / (c * (c - 1.0));
  double mean = (double)m.s1 / c;
  return sqrt(var) / mean;
}

// ------------------------------------------- reference-exact f64 replay ----
// The reference computes variance as an ordered sum over DISTINCT values
// ascending of ((mean - x)^2 * count) (histogram.rs:204-219).  `gen(i)`
// yields the i-th of `cnt` values; distinct values are visited by repeated
// min-above scans (O(cnt * distinct)); only near-tie decisions come here.
template <class Gen>
__device__ __forceinline__ double ref_variance_sum(const Gen& gen, uint32_t cnt, double mean) {
  double sum = 0.0;
  uint32_t lo = 0;
  bool first = true;
  for (;;) {
    uint32_t x = 0xFFFFFFFFu, c = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t v = gen(i);
      if (!first && v < lo) continue;
      if (v < x) {
        x = v;
        c = 1;
      } else if (v == x) {
        ++c;
      }
    }
    if (c == 0) break;
    double d = mean - (double)x;
    double t = d * d;
    t = t * (double)c;
    sum = sum + t;
    if (x == 0xFFFFFFFFu) break;
    lo = x + 1;
    first = false;
  }
  return sum;
}

template <class Gen>
__device__ __forceinline__ double ref_cov(const Gen& gen, uint32_t cnt, uint64_t s1) {
  double c = (double)cnt;
  double mean = (double)s1 / c;
  double var = ref_variance_sum(gen, cnt, mean) / (c - 1.0);
  return sqrt(var) / mean;
}

template <class Gen>
__device__ __forceinline__ double ref_mdtm(const Gen& gen, uint32_t cnt, uint64_t s1) {
  double c = (double)cnt;
  double mean = (double)s1 / c;
  double sum = 0.0;
  uint32_t lo = 0;
  bool first = true;
  for (;;) {
    uint32_t x = 0xFFFFFFFFu, k = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t v = gen(i);
      if (!first && v < lo) continue;
      if (v < x) {
        x = v;
        k = 1;
      } else if (v == x) {
        ++k;
      }
    }
    if (k == 0) break;
    double d = mean - (double)x;
    sum = sum + fabs(d) * (double)k;
    if (x == 0xFFFFFFFFu) break;
    lo = x + 1;
    first = false;
  }
  return sum / c;
}

// --------------------------------------------------------- top-K records --
struct Rec {
  uint64_t key, rank;
};
__device__ __forceinline__ bool rec_lt(const Rec& a, const Rec& b) {
  return a.key < b.key || (a.key == b.key && a.rank < b.rank);
}
__device__ __forceinline__ Rec rec_max() { return Rec{~0ull, ~0ull}; }

// COV objective key (BOTE_OBJ_COV): bits of fl64(V / S1^2); all-ones when the
// reference's COV is NaN.  Monotone in the true COV.
__device__ __forceinline__ uint64_t cov_key(const Mom& m) {
  if (cov_nan(m)) return ~0ull;
  double rr = (double)mom_v(m) / ((double)m.s1 * (double)m.s1);
  return (uint64_t)__double_as_longlong(rr);
}

// Per-config digest, summed over configs mod 2^64.  A linear
// fold of 32-bit words, each times its own constant as two 16-bit halves (one
// v_dot2_u32_u16 per word, in any order), then the rank and the leader, then
// the murmur3 32-bit finaliser (a bijection: a config whose fold differs
// changes its term):
//   h = sum over the present words w:  lo16(x_w) lo16(K_w) + hi16(x_w) hi16(K_w)   (mod 2^32)
//     slot s (0..19):     x_{2s} = lo32(S1_s),  x_{2s+1} = lo32(S2_s ^ (S2_s >> 32))
//     leader l, f (XK):   w = 40 + 2 (16 f + l) (+1 for the sum of squares)
//   x = h + lo32(rank) 0x9E3779B1 + hi32(rank) 0xEBCA77 + leader_pos 0xB2AE3D   (mod 2^32)
//   d = fmix32(x)
// (oracle/bote_oracle.cpp config_digest restates it)
__host__ __device__ constexpr uint32_t digest_key(uint32_t w) {
  uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(w + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)z | 0x00010001u;
}
constexpr uint32_t DIGEST_WORD_LEADER = 40;  // first leader word (XK)
typedef unsigned short dg_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t digest_word(uint32_t h, uint32_t x, uint32_t k) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(dg_u16x2, x), __builtin_bit_cast(dg_u16x2, k), h, false);
}
// slot s's two words (s compile-time in every caller: the constants fold)
__device__ __forceinline__ uint32_t digest_fold(uint32_t h, uint32_t s, uint64_t s1, uint64_t s2) {
  h = digest_word(h, (uint32_t)s1, digest_key(2 * s));
  return digest_word(h, (uint32_t)(s2 ^ (s2 >> 32)), digest_key(2 * s + 1));
}
// leader l's FPaxos moments at f (0: f = 1, 1: f = 2), the extended key set
__device__ __forceinline__ uint32_t digest_fold_leader(uint32_t h, uint32_t f, uint32_t l, uint64_t s1, uint64_t s2) {
  return digest_fold(h, DIGEST_WORD_LEADER / 2 + 16 * f + l, s1, s2);
}
__device__ __forceinline__ uint64_t digest_final(uint64_t rank, uint32_t lead, uint32_t h) {
  uint32_t x = h + (uint32_t)rank * 0x9E3779B1u + __umul24((uint32_t)(rank >> 32), 0xEBCA77u) + __umul24(lead, 0xB2AE3Du);
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

// In-LDS bitonic sort of a[0..n), n a power of two, by the whole block.
__device__ inline void block_bitonic(Rec* a, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int l = i ^ j;
        if (l > i) {
          Rec x = a[i], y = a[l];
          bool up = (i & k) == 0;
          if (up ? rec_lt(y, x) : rec_lt(x, y)) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace bote

namespace bote {

// ----------------------------------------------- block-level top-K in LDS --
// Each objective keeps a sorted list of KP records; `thr[o]` is its K-th
// record.  A config enters the candidate buffer only if it beats thr[o]; the
// block merges candidates one objective at a time (bitonic sort + merge path).
struct TopkLds {
  Rec* top;   // n_obj * KP
  Rec* cand;  // blockDim.x (warm-up buffer, or MAXOBJ segments of SEG in batched mode)
  Rec* tmp;   // KP
  Rec* thr;   // MAXOBJ
  int* cnt;   // 1 + MAXOBJ counters (48 bytes reserved)
};

__device__ inline int lower_bound_rec(const Rec* a, int n, const Rec& x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (rec_lt(a[mid], x)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ inline int upper_bound_rec(const Rec* a, int n, const Rec& x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (!rec_lt(x, a[mid])) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ inline void topk_init(const TopkLds& t, int n_obj) {
  for (uint32_t i = threadIdx.x; i < (uint32_t)n_obj * KP; i += blockDim.x) t.top[i] = rec_max();
  if (threadIdx.x < MAXOBJ) t.thr[threadIdx.x] = rec_max();
  if (threadIdx.x <= MAXOBJ) t.cnt[threadIdx.x] = 0;  // [0] warm-up buffer, [1+o] segments
}

// Merge the candidate buffer (*t.cnt unsorted entries) into objective o's
// list by ranks: every record's output slot is the number of records of the
// other sequence below it plus its rank in its own.  Records are unique (one
// per config and objective), padding records only fill the tail.  O(n) per
// thread; after warm-up n is a handful, so this beats sorting the buffer.
__device__ inline void topk_merge(const TopkLds& t, int o, uint32_t K) {
  const int tid = threadIdx.x;
  const int n = *t.cnt;  // read after the caller's barrier: uniform
  Rec* top = t.top + o * KP;
  if (tid < KP) {
    const Rec x = top[tid];
    int r = tid;
    for (int j = 0; j < n; ++j) r += rec_lt(t.cand[j], x);
    if (r < KP) t.tmp[r] = x;
  }
  if (tid < n) {
    const Rec y = t.cand[tid];
    int r = lower_bound_rec(top, KP, y);
    for (int j = 0; j < n; ++j) r += rec_lt(t.cand[j], y);
    if (r < KP) t.tmp[r] = y;
  }
  __syncthreads();
  if (tid < KP) top[tid] = t.tmp[tid];
  __syncthreads();
  if (tid == 0) {
    t.thr[o] = top[K - 1];
    *t.cnt = 0;
  }
  __syncthreads();
}

// One block-synchronous step: every thread of the block must call it.
// ok[o] false = this lane offers nothing for objective o.
__device__ __forceinline__ void topk_step(const TopkLds& t, int n_obj, uint32_t K, const uint64_t (&key)[MAXOBJ],
                                          const bool (&ok)[MAXOBJ], uint64_t rank) {
  bool pass[MAXOBJ];
  bool any = false;
#pragma unroll
  for (int o = 0; o < MAXOBJ; ++o) {
    pass[o] = o < n_obj && ok[o] && rec_lt(Rec{key[o], rank}, t.thr[o]);
    any = any || pass[o];
  }
  if (__syncthreads_or(any)) {
#pragma unroll
    for (int o = 0; o < MAXOBJ; ++o) {
      if (o >= n_obj) break;
      if (pass[o] && rec_lt(Rec{key[o], rank}, t.thr[o])) {
        int i = atomicAdd(t.cnt, 1);
        t.cand[i] = Rec{key[o], rank};
      }
      __syncthreads();
      // every wave reads the count before any wave adds the next objective's
      // candidates: without the second barrier a wave that found no
      // candidate could run ahead into objective o + 1's atomicAdd while a
      // slower wave still reads the count for objective o, which then enters
      // the merge alone and merges unwritten candidate slots
      const int n = *t.cnt;
      __syncthreads();
      if (n > 0) topk_merge(t, o, K);
    }
  }
}

// ----------------------------------------------------- colex enumeration --
// rank = sum_j C(p_j, j+1) with p ascending (an extension: the reference's
// permutator order is not pinned).
template <int N>
__device__ __forceinline__ void colex_unrank(const uint64_t* binom, uint32_t ns, uint64_t rank, uint32_t (&p)[N]) {
  uint64_t r = rank;
  uint32_t hi = ns;
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    const uint32_t k = j + 1;
    uint32_t lo = j, up = hi;  // answer in [lo, up)
    while (up - lo > 1) {
      uint32_t mid = (lo + up) >> 1;
      if (binom[mid * (N + 1) + k] <= r) lo = mid; else up = mid;
    }
    p[j] = lo;
    r -= binom[lo * (N + 1) + k];
    hi = lo;
  }
}

template <int N>
__device__ __forceinline__ void colex_next(uint32_t ns, uint32_t (&p)[N]) {
  uint32_t js = N;  // first j with p[j] + 1 < p[j+1]
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    uint32_t nxt = (j == N - 1) ? ns : p[j + 1];
    if (p[j] + 1 < nxt) js = j;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) p[j] = (uint32_t)j < js ? (uint32_t)j : ((uint32_t)j == js ? p[j] + 1 : p[j]);
}

}  // namespace bote
