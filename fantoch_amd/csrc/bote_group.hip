// bote_group.hip — the group-structured sweep kernel (gfx950), the hot path
// for fast-path planets with config size N >= 4.
//
// Colex ranks of n-subsets are grouped by their N-3 LARGEST members: every
// rank sum_j C(p_j, j+1) with the same (p_3 .. p_{N-1}) lies in one contiguous
// range of C(p_3, 3) ranks (a "group"), and inside it only (p_0, p_1, p_2)
// vary.  A wavefront walks its contiguous share of the rank space group by
// group, 64 configs (one per lane) at a time.  Everything that depends only on
// the fixed members is computed once per group and is wave-uniform, kept in a
// per-wave LDS line (broadcast reads, no SGPR pressure):
//   * each client's nearest fixed member (packed latency << 4 | member), so
//     the hot loop reads 3 lane columns + 1 broadcast line instead of N
//     columns;
//   * the fixed members' sorted distances to each other, packed two rows per
//     word, so a fixed member's quorum latencies need only the 3 lane members
//     inserted (v_pk_min_u16 / v_pk_max_u16 on two rows at once);
//   * the fixed members' column statistics.
// Per lane: the 3 variable rows are sorted in full (two of them packed), the
// fixed rows get 3 insertions each, then leader selection, moments, validity,
// digest and objective keys.  COV decisions are screened in f32 and fall back
// to f64, then to deferral (the exact generic kernel), only inside their
// ambiguity bands.
//
// The block top-K is merged wave by wave under an LDS lock (no block
// barriers in the sweep): a wave whose configs may enter a list (key <= the
// list's K-th key, read lock-free) takes the lock and merges exactly.
//
// LDS is addressed with absolute 32-bit addresses (lds_* helpers) so that the
// per-client address arithmetic is one shift-add and constant offsets fold
// into the ds_read offset fields.
//
// Reference map: see bote_kernels.hip's header (Search::compute_stats,
// search.rs:262-319, and the Bote functions it calls, lib.rs:38-185).
#include "bote_fast.hpp"

#define AS3 __attribute__((address_space(3)))

namespace bote {

// Workgroup size: a.gbd threads (a multiple of 64, <= GROUP_MAX_BD), chosen on
// the host so that LDS does not cap the waves per SIMD (R = 128 needs larger
// workgroups than R = 64: the client-quad matrix is shared per workgroup).
constexpr int GROUP_MAX_BD = 1024;
// waves per SIMD the register allocation targets (5: <= 96 VGPRs; LDS per
// workgroup stays under 32 KB at R = 64, so 5 workgroups fit a CU)
#ifndef BOTE_GROUP_WAVES
#define BOTE_GROUP_WAVES 5
#endif
// PERM kernels (n <= 7) keep 8 more registers live through the client loop
// (the byte planes): at <= 96 VGPRs they spill, so they target 4 waves per
// SIMD (<= 128 VGPRs; measured faster than 5 waves with spills)
#ifndef BOTE_GROUP_WAVES_PERM
#define BOTE_GROUP_WAVES_PERM 4
#endif
// qtab member planes are 1 << a.gqsh bytes apart (>= gbd * 4, a power of two)

__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

template <int N>
struct GCfg {
  using QC = QCfg<N>;
  static constexpr int F = N - 3;         // wave-uniform (fixed) members
  static constexpr int FP = (F + 1) / 2;  // fixed rows, packed in pairs
  // a row's smallest off-diagonal distances that any quorum reads (ranks 0 .. KQ-1)
  static constexpr int KQ = cmax(cmax(QC::qa1, QC::maxf >= 2 ? QC::qa2 : 0), cmax(QC::qe, 3)) - 1;
  static_assert(KQ <= N - 1, "quorum larger than the config");
  // Register lookup of the members' quorum latencies (n <= 7, two tables):
  // member m's latency in table t is split into a low and a high byte, kept
  // in byte m of two 8-byte register planes per table, and a client's value
  // is picked by v_perm with the nearest member's tag (its index, the low 4
  // bits of the packed minimum) as the byte selector.  No per-lane LDS
  // table; larger n gathers from the LDS qtab instead.
  static constexpr bool PERM = N <= 7 && QC::NL == 2;
  // Per-position table (n <= 7, at most 4 fixed members): for every position
  // x below the group's smallest fixed position, 16 bytes computed once per
  // group: x's distances to the fixed members, sorted (row part), and the
  // fixed members' distances to x, packed in the fixed-row pairs (column
  // part).  A lane's three variable rows then start from their sorted fixed
  // parts and merge in the two distances to the other variable members, and
  // the fixed rows' inserts come packed: 3 LDS reads instead of 24 u16 reads
  // and two full row sorts.
  // (a launch argument, FastArgs::grx: the table costs ns x 16 B of LDS per
  // wave, which at R = 128 lowers the workgroups per CU, so the host enables
  // it only where the occupancy stays)
  static constexpr bool RX = N <= 7;
  static_assert(!RX || (F <= 4 && KQ <= 4), "position table holds 4 fixed members");
};

// per-wave group line: [rx: ns x 16 B (n <= 7)][mF: cq_stride uint2][Upk: FP*KQ u32][fS1: F u32][fV: F f32],
// padded to 16 bytes
__host__ __device__ inline uint32_t gline_rx_bytes(const FastArgs& a, int N) { return N <= 7 && a.grx ? a.ns * 16 : 0u; }
__host__ __device__ inline uint32_t gline_bytes(const FastArgs& a, int N, int KQ) {
  const int F = N - 3, FP = (F + 1) / 2;
  return (gline_rx_bytes(a, N) + a.cq_stride * 8 + (uint32_t)(FP * KQ + 2 * F) * 4 + 15) & ~15u;
}

// one wave's client lines (gslots lines of cq_stride quads, then the slots'
// keys), rounded to 16 B: the lines are read 16 B at a time (ds_read_b128)
__host__ __device__ inline uint32_t lines_wave_bytes(const FastArgs& a) {
  return (a.gslots * (a.cq_stride * 8 + 4) + 15) & ~15u;
}

// region 0: PERM kernels: per wave, gslots client lines of cq_stride
// quads; otherwise the qtab (N * NLW member planes of 1 << gqsh bytes)
__host__ __device__ inline size_t group_layout(const FastArgs& a, int N, int NLW, int KQ, bool perm, size_t* off) {
  size_t o = 0;
  off[0] = o;
  o += perm ? (size_t)(a.gbd / 64) * lines_wave_bytes(a) : ((size_t)N * NLW) << a.gqsh;
  o = (o + 15) & ~(size_t)15;
  off[1] = o; o += (size_t)a.R * a.cq_stride * 8;
  off[2] = o; o += a.rq_separate ? (size_t)a.R * a.rq_stride * 8 : 0;
  off[3] = o; o += (size_t)a.ns * 4;  // srv
  o = (o + 7) & ~(size_t)7;
  off[4] = o; o += (size_t)a.ns * 8;  // lrec: (cs1, f32 vcol) per position
  o = (o + 15) & ~(size_t)15;
  off[5] = o; o += (size_t)a.ns * 8;                   // cs2
  off[6] = o; o += (size_t)a.ns * 8;                   // vcol (f64)
  off[7] = o; o += (size_t)a.ns * 4;                   // vcol32: V as f32 (the screens' leader V)
  // (binomials stay in global memory: uniform scalar loads, once per group)
  o = (o + 15) & ~(size_t)15;
  off[8] = o; o += (size_t)(a.gbd / 64) * gline_bytes(a, N, KQ);  // per-wave group lines
  o = (o + 15) & ~(size_t)15;
  off[9] = o; o += (size_t)a.n_obj * a.K * 16;  // top: n_obj lists of K records
  off[10] = o; o += (size_t)64 * 16;           // cand (one wave's candidates)
  off[11] = o; o += (size_t)a.K * 16;          // tmp
  off[12] = o; o += (size_t)MAXOBJ * 16;      // thr
  off[13] = o; o += 48;                       // lock
  // extended key set (PERM kernels): per wave, N member bins of 64 lanes' u32
  // (the client loop's binned sums, sweep_group_kernel)
  o = (o + 15) & ~(size_t)15;
  off[14] = o; o += perm && (a.keys || a.gbins) ? (size_t)(a.gbd / 64) * N * 256 : 0;
  // per thread, its running digest (u64): an LDS add per step instead of a
  // 64-bit accumulator held in registers across the step loop, which the
  // register-bound kernels spilled to scratch and reloaded, added and stored
  // back every step (config 5: the bulk of its scratch write traffic)
  o = (o + 15) & ~(size_t)15;
  off[15] = o; o += (size_t)a.gbd * 8;
  return o;
}

template <int N>
static size_t group_smem_n(const FastArgs& a) {
  size_t off[16];
  return group_layout(a, N, QCfg<N>::NL <= 2 ? 1 : 2, GCfg<N>::KQ, GCfg<N>::PERM, off);
}

bool group_uses_lines(uint32_t n) {
  switch (n) {
#define PL_CASE(NN) case NN: return GCfg<NN>::PERM;
    PL_CASE(4) PL_CASE(5) PL_CASE(6) PL_CASE(7)
#undef PL_CASE
    default: return false;
  }
}

size_t group_smem_bytes(const FastArgs& a, uint32_t n) {
  switch (n) {
#define SM_CASE(NN) case NN: return group_smem_n<NN>(a);
    SM_CASE(4) SM_CASE(5) SM_CASE(6) SM_CASE(7) SM_CASE(8) SM_CASE(9) SM_CASE(10) SM_CASE(11) SM_CASE(12)
    SM_CASE(13) SM_CASE(14) SM_CASE(15) SM_CASE(16)
#undef SM_CASE
    default: return 0;
  }
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

// absolute-address LDS access
__device__ __forceinline__ uint32_t lds_base(const void* p) { return (uint32_t)(uintptr_t)(const AS3 void*)p; }
__device__ __forceinline__ uint32_t l16(uint32_t a) { return *(const AS3 uint16_t*)(uintptr_t)a; }
__device__ __forceinline__ uint32_t l32(uint32_t a) { return *(const AS3 uint32_t*)(uintptr_t)a; }
__device__ __forceinline__ uint2 l64(uint32_t a) {
  const uint64_t v = *(const AS3 uint64_t*)(uintptr_t)a;
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 l128(uint32_t a) {
  const u32x4 v = *(const AS3 u32x4*)(uintptr_t)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float lf32(uint32_t a) { return *(const AS3 float*)(uintptr_t)a; }
__device__ __forceinline__ void s16(uint32_t a, uint32_t v) { *(AS3 uint16_t*)(uintptr_t)a = (uint16_t)v; }
__device__ __forceinline__ void s32(uint32_t a, uint32_t v) { *(AS3 uint32_t*)(uintptr_t)a = v; }
__device__ __forceinline__ void s64(uint32_t a, uint32_t lo, uint32_t hi) {
  *(AS3 uint64_t*)(uintptr_t)a = (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void s128(uint32_t a, uint4 v) {
  u32x4 w;
  w.x = v.x;
  w.y = v.y;
  w.z = v.z;
  w.w = v.w;
  *(AS3 u32x4*)(uintptr_t)a = w;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ us2 ld_pair(uint32_t a, uint32_t b) {
  us2 r;
  r.x = *(const AS3 unsigned short*)(uintptr_t)a;
  r.y = *(const AS3 unsigned short*)(uintptr_t)b;
  return r;
}

__device__ __forceinline__ us2 pk_min(us2 a, us2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ us2 pk_max(us2 a, us2 b) { return __builtin_elementwise_max(a, b); }

// Batcher odd-even merge sort over packed u16 pairs (two rows at once)
template <int P>
__device__ __forceinline__ void sort_network_pk(uint32_t* a) {
#pragma unroll
  for (int p = 1; p < P; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < P; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          if (i + j + k < P && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const us2 x = as_us2(a[i + j]), y = as_us2(a[i + j + k]);
            a[i + j] = as_u32(pk_min(x, y));
            a[i + j + k] = as_u32(pk_max(x, y));
          }
        }
      }
    }
  }
}

// The KO smallest of the union of two ascending lists A (KA entries) and y
// (KY entries), ascending: the k-th is the min over the splits (k+1-j from A,
// j from y) of max(A[k-j], y[j-1]).  T: u32 (min/max) or us2 (two lists at
// once, packed halves).
template <int KA, int KY, int KO, class T>
__device__ __forceinline__ void merge_lists(const T* A, const T* y, T* L) {
#pragma unroll
  for (int k = 0; k < KO; ++k) {
    T z = k < KA ? A[k < KA ? k : 0] : y[0];
    bool have = k < KA;
#pragma unroll
    for (int j = 1; j <= KY && j <= k + 1; ++j) {
      const int i = k + 1 - j;  // elements taken from A
      if (i > KA) continue;
      const T c = i == 0 ? y[j - 1] : __builtin_elementwise_max(A[i > 0 ? i - 1 : 0], y[j - 1]);
      z = have ? __builtin_elementwise_min(z, c) : c;
      have = true;
    }
    L[k] = z;
  }
}

// The SCORE objective's screen as one integer compare (DEF kernels: objective
// 0).  A config's score numerator T = sum over f of (ff.s1 - af.s1) +
// 30 (e.s1 - af.s1) is an exact integer (|T| < 2^27), and the config can beat
// the block list's threshold key only if (double)T >= (tscore - 1e-6) nc,
// tscore the key's score: for a finite bound b that is T >= ceil(b).  The
// bound is kept in LDS next to the block lock (lock[1]) and recomputed when the
// threshold moves (the list's K-th record, under the lock: a few times per
// block), instead of decoding the key and comparing in f64 every step.  It only
// rises as the threshold falls, so a stale read is a looser screen.
__device__ __forceinline__ int32_t score_tlo(uint64_t tkey, uint32_t nc) {
  if (tkey == ~0ull) return INT32_MIN;  // (no threshold yet)
  const uint64_t ob = ~tkey;
  const uint64_t bits = (ob >> 63) ? (ob & 0x7FFFFFFFFFFFFFFFull) : ~ob;
  const double tscore = __longlong_as_double((long long)bits);
  if (!(tscore == tscore)) return INT32_MIN;  // (a NaN threshold: every config may beat it)
  const double b = (tscore - 1e-6) * (double)nc;
  if (b <= -2147483648.0) return INT32_MIN;
  if (b > 1073741824.0) return 1073741824;  // (above every |T| < 2^27)
  return (int32_t)ceil(b);
}

// The COV-af1 objective's screen bound (DEF kernels: objective 3): its key is
// the bits of V / S^2 as a double (cov_key), so a config may beat the
// threshold only if V <= key S^2; f32 with a 2^-10 margin over the screen's
// rounding, +inf with no threshold (the all-ones key), kept in LDS at lock[2]
// like score_tlo.  A NaN bound lets every config through (always safe: the
// merge is exact).
__device__ __forceinline__ float cov_tf32(uint64_t tkey) {
  if (tkey == ~0ull) return __builtin_inff();
  return (float)__longlong_as_double((long long)tkey) * (1.0f + 0x1p-10f);
}

// The 4 smallest of the union of two ascending lists A (KA real entries, the
// rest absent) and y (KY), ascending: the elementwise minimum of A and y
// reversed (absent entries are +inf) holds the 4 smallest as a bitonic
// sequence (Batcher), which one bitonic merge stage of 4 compare-exchanges
// sorts.  KA = 3, KY = 3: 2 mins + 8 ops, where the split form (merge_lists)
// takes 15.  T: u32 or us2 (two lists at once).
template <int KA, int KY, class T>
__device__ __forceinline__ void merge_top4(const T* A, const T* y, T* L) {
  static_assert(KA >= 1 && KY >= 1 && KA + KY >= 4 && KA <= 4 && KY <= 4, "4 smallest of KA + KY >= 4 entries");
  T B[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 3 - i;  // y reversed
    if (i < KA && j < KY) B[i] = __builtin_elementwise_min(A[i < KA ? i : 0], y[j < KY ? j : 0]);
    else if (i < KA) B[i] = A[i < KA ? i : 0];
    else B[i] = y[j < KY ? j : 0];
  }
  auto ce = [&](int a, int b) {
    const T lo = __builtin_elementwise_min(B[a], B[b]);
    B[b] = __builtin_elementwise_max(B[a], B[b]);
    B[a] = lo;
  };
  ce(0, 2);
  ce(1, 3);
  ce(0, 1);
  ce(2, 3);
#pragma unroll
  for (int i = 0; i < 4; ++i) L[i] = B[i];
}

// the KO smallest: merge_top4 where KO = 4 (n = 6, 7), the split form otherwise
template <int KA, int KY, int KO, class T>
__device__ __forceinline__ void merge_k(const T* A, const T* y, T* L) {
  if constexpr (KO == 4 && KA + KY >= 4) merge_top4<KA, KY>(A, y, L);
  else merge_lists<KA, KY, KO>(A, y, L);
}

// ------------------------------------------------ wave-level top-K merge --
// Called by a whole wavefront (uniform branch).  Takes the block's LDS lock,
// merges every lane record that beats its objective's K-th record (exact
// (key, rank) order), updates the thresholds, releases the lock.  The block
// lists hold exactly K records each (K <= KP).
// Each output position is a count: a list record's index plus the candidates
// below it, a candidate's lower bound in the list plus the candidates below it.
// The candidates stay in their lanes and are read with v_readlane (the loop
// over them is a chain of scalar reads, not of dependent LDS loads: in the
// fill phase, 64 candidates per objective, that latency chain held the block's
// lock for microseconds per merge and was a fixed ~1 ms per launch).
__device__ __forceinline__ void wave_topk(const TopkLds& t, int* lock, uint32_t nc, int n_obj, uint32_t K,
                                          const uint64_t (&key)[MAXOBJ], const bool (&ok)[MAXOBJ], uint64_t rank) {
  const uint32_t lane = threadIdx.x & 63;
  const int KL = (int)K;
  if (lane == 0) {
    while (atomicCAS(lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const uint32_t rlo = (uint32_t)rank, rhi = (uint32_t)(rank >> 32);
#pragma unroll
  for (int o = 0; o < MAXOBJ; ++o) {
    if (o >= n_obj) break;
    Rec* top = t.top + o * KL;
    const Rec mine = Rec{key[o], rank};
    // thr: the lesser of the list's K-th record and the seed (never above it)
    const bool p = ok[o] && rec_lt(mine, t.thr[o]);
    const uint64_t m = __ballot(p);
    if (m == 0) continue;
    // the list records this lane places (e = lane, lane + 64 < K)
    const bool h0 = (int)lane < KL, h1 = (int)lane + 64 < KL;
    const Rec x0 = h0 ? top[lane] : rec_max(), x1 = h1 ? top[lane + 64] : rec_max();
    int r0 = (int)lane, r1 = (int)lane + 64;
    int rc = p ? lower_bound_rec(top, KL, mine) : 0;
    const uint32_t klo = (uint32_t)key[o], khi = (uint32_t)(key[o] >> 32);
    for (uint64_t mm = m; mm; mm &= mm - 1) {
      const int src = __builtin_ctzll(mm);
      // (readlane returns int: widen through uint32_t, not by sign extension)
      const uint64_t ck = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(khi, src) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane(klo, src);
      const uint64_t cr = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rhi, src) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane(rlo, src);
      const Rec c = Rec{ck, cr};
      r0 += rec_lt(c, x0);
      r1 += rec_lt(c, x1);
      rc += rec_lt(c, mine);
    }
    if (h0 && r0 < KL) t.tmp[r0] = x0;
    if (h1 && r1 < KL) t.tmp[r1] = x1;
    if (p && rc < KL) t.tmp[rc] = mine;
    wave_sync();
#pragma unroll
    for (int h = 0; h < KP / 64; ++h)
      if ((int)lane + 64 * h < KL) top[lane + 64 * h] = t.tmp[lane + 64 * h];
    wave_sync();
    if (lane == 0 && rec_lt(top[K - 1], t.thr[o])) {
      t.thr[o] = top[K - 1];
      // (the DEF kernels' screens of objectives 0, SCORE, and 3, COV af1)
      if (o == 0) lock[1] = score_tlo(top[K - 1].key, nc);
      if (o == 3) lock[2] = __float_as_int(cov_tf32(top[K - 1].key));
    }
    wave_sync();
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) atomicExch(lock, 0);
}

// -------------------------------------- exact-order COV comparisons -------
// sign of V_x * S_y^2 - V_y * S_x^2 (cov_x^2 vs cov_y^2): -1 / +1, or 0 when
// inside the ambiguity band.  f32 screen first (S exact below 2^24; V carries
// one rounding, every product one more): decided outside a 2^-18 relative
// band; else f64 from the exact V (dVx(), dVy()) with the 2^-32 band the
// generic path uses.
template <class FX, class FY>
__device__ __forceinline__ int cov2_sign(float Vx, uint32_t Sx, float Vy, uint32_t Sy, const FX& dVx, const FY& dVy) {
  const float fx = (float)Sx, fy = (float)Sy;
  const float x = Vx * (fy * fy), y = Vy * (fx * fx);
  const float d = x - y, tol = 0x1p-18f * fmaxf(x, y);
  if (d < -tol) return -1;
  if (d > tol) return 1;
  const double sx = (double)Sx, sy = (double)Sy;
  const double X = dVx() * (sy * sy), Y = dVy() * (sx * sx);
  const double D = X - Y, T = 0x1p-32 * fmax(X, Y);
  return D < -T ? -1 : (D > T ? 1 : 0);
}

// The validity form (cov_f >= cov_a): the same band, decided with one
// product per side, x (1 - 2^-18) >= y and x < y (1 - 2^-18), so that both V
// zero (COV 0 >= COV 0) is decided 1 by the screen itself
template <class FX, class FY>
__device__ __forceinline__ int cov2_sign_ge(float Vx, uint32_t Sx, float Vy, uint32_t Sy, const FX& dVx, const FY& dVy) {
  const float fx = (float)Sx, fy = (float)Sy;
  const float x = Vx * (fy * fy), y = Vy * (fx * fx);
  constexpr float c = 1.0f - 0x1p-18f;
  if (x * c >= y) return 1;
  if (x < y * c) return -1;
  const double sx = (double)Sx, sy = (double)Sy;
  const double X = dVx() * (sy * sy), Y = dVy() * (sx * sx);
  const double D = X - Y, T = 0x1p-32 * fmax(X, Y);
  return D < -T ? -1 : (D > T ? 1 : 0);
}

// u64 -> f32 in three instructions (two conversions and an fma): within
// 2^-23 relative, inside the screens' error budget
__device__ __forceinline__ float u64_to_f32(uint64_t x) {
  return __builtin_fmaf((float)(uint32_t)(x >> 32), 0x1p32f, (float)(uint32_t)x);
}

// ---------------------------------------------------------- the kernel ----
// DEF: the default objective set (bote.py DEFAULT_OBJECTIVES: SCORE, MEAN af1,
// MEAN ff1, COV af1, MEAN e), compiled in; otherwise the objectives come from
// the arguments (finish_config, bote_fast.hpp).
// SI ("bench-shaped" default-objective sweeps): the servers are the planet's
// regions in order (srv[p] == p), the digest is on and ft_metric is F1F2,
// compiled in: the position -> region lookups and the flag tests vanish, and
// with them uniform masks the kernel had spilled to VGPR lanes
// XK: the extended key set (BASELINE config 5: Tempo tiny/write keys and
// every leader's FPaxos moments; include/bote_hip.h BOTE_KEYS_TEMPO_ALL_LEADERS)
// on the PERM kernels, with config 5's objective set compiled in (the
// default five, then MEAN tt1, MEAN tw2, MEAN fl1: bote.py CONFIG5_OBJECTIVES)
// The extended key set keeps NT = 3..4 tables of byte planes and sums live
// through the client loop: at 4 waves per SIMD (128 VGPRs) part of that state
// lives in scratch, and still the extra wave per SIMD hides more latency than
// the scratch traffic costs (config 5: 186 vs 198 ms at 3 waves, 168 VGPRs)
// (BOTE_GROUP_WAVES_XK, GROUP_XK_MAX_BD = 256 x that: bote_kernels.hpp)
// client-loop quads per iteration of the register-lookup (PERM) loop
constexpr uint32_t GROUP_UNROLL = 4;
// The binned client loop (BIN, below) runs before the Q phase on the XK
// kernels and after the leader choice on the others (BIN_FIRST): config 5's
// XK kernel 178.1 / 178.6 vs 182.1 / 182.6 ms with it first, the R=64 n=7
// kernel 14.07 / 14.05 vs 13.87 / 13.83 ms (r05aa).  The only live -D knob of
// this file; the decided A/Bs of rounds 4-5 (one-byte tables, late kernel
// arguments, the binned loop on every PERM kernel, the unrolls) are DESIGN.md
// history, not code.
#ifndef BOTE_BIN_FIRST
#define BOTE_BIN_FIRST 0
#endif
#ifndef BOTE_BIN_FIRST_XK
#define BOTE_BIN_FIRST_XK 1
#endif
// binned loop with client lines: quads per unrolled iteration (2 without
// lines: 4 sources per pair of quads would hold 32 VGPRs of reads at 4)
constexpr uint32_t BIN_UB = 4;
// BN: the base key set with the member-binned client loop (the extended key
// set's, below); the host picks it for bench-shaped sweeps with >= 96 clients
// (FastArgs::gbins: R=128 n=6 179.8 -> 168.2 ms; neutral at 64 clients)
template <int N, bool DEF, bool SI, bool RXC, bool XK, bool BN = false>
__global__ void __launch_bounds__(XK ? GROUP_XK_MAX_BD : GROUP_MAX_BD,
                                  XK ? BOTE_GROUP_WAVES_XK : (GCfg<N>::PERM ? BOTE_GROUP_WAVES_PERM : BOTE_GROUP_WAVES))
    sweep_group_kernel(FastArgs a) {
  const bool sid = SI || a.srv_identity;
  // S32 (the SI kernels; the host admits them only where FastArgs::s32
  // holds): every slot's sum of squares fits 32 bits, so the moments, the
  // leader columns' sums of squares and the digest folds stay 32-bit
  constexpr bool S32 = SI;
  // the position table: a launch argument, compiled in (RXC) on SI kernels
  const bool use_rx = GCfg<N>::RX && (SI ? RXC : a.grx != 0);
  using QC = QCfg<N>;
  using GC = GCfg<N>;
  constexpr int NL = QC::NL;
  constexpr int NLW = NL <= 2 ? 1 : 2;
  constexpr int F = GC::F;
  constexpr int FP = GC::FP;
  constexpr int KQ = GC::KQ;
  constexpr int PV = Pow2<N - 1>::v;                 // variable row: N-1 values, padded
  constexpr int PF = Pow2<F>::v;                     // fixed-to-fixed row: F values (self = INF), padded
  constexpr bool PERM = GC::PERM;
  constexpr bool BIN = XK || (PERM && BN);  // the member-binned client loop
  constexpr bool BIN_FIRST = BIN && (XK ? BOTE_BIN_FIRST_XK : BOTE_BIN_FIRST);  // (its loop before the Q phase)
  static_assert(!XK || (PERM && DEF), "the extended key set runs on the PERM kernels with the default objectives");
  using QT = QTab<N, XK>;
  constexpr int NT = QT::NT;  // leaderless tables (PERM: register byte planes); == NL without XK
  extern __shared__ __align__(16) unsigned char smem[];
  size_t off[16];
  group_layout(a, N, NLW, KQ, PERM, off);
  const uint32_t LB = lds_base(smem);
  const uint32_t qtab = LB + (uint32_t)off[0];
  const uint32_t cqt = LB + (uint32_t)off[1];
  const uint32_t rqt = LB + (uint32_t)(a.rq_separate ? off[2] : off[1]);
  uint32_t* srv = (uint32_t*)(smem + off[3]);
  uint2* lrec = (uint2*)(smem + off[4]);  // per position: .x column sum S1, .y f32 bits of 1 / sqrt(V)
  uint64_t* cs2 = (uint64_t*)(smem + off[5]);
  double* vcol = (double*)(smem + off[6]);
  float* vcol32 = (float*)(smem + off[7]);
  const uint64_t* binom = a.binom;
  TopkLds tk;
  tk.top = (Rec*)(smem + off[9]);
  tk.cand = (Rec*)(smem + off[10]);
  tk.tmp = (Rec*)(smem + off[11]);
  tk.thr = (Rec*)(smem + off[12]);
  const uint32_t thra = LB + (uint32_t)off[12];  // (the thresholds' LDS address)
  tk.cnt = nullptr;
  int* lock = (int*)(smem + off[13]);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, BD = blockDim.x, WPB = BD >> 6;
  const uint32_t qsh = a.gqsh;  // log2 of the qtab plane stride (bytes)

  // ---- stage: quad matrices, server list, binomials; then per-position sums
  {
    const uint32_t cw = a.R * a.cq_stride * 2;
    const uint32_t* src = (const uint32_t*)a.cqt;
    uint32_t* dst = (uint32_t*)(smem + off[1]);
    for (uint32_t i = tid; i < cw; i += BD) dst[i] = src[i];
    if (a.rq_separate) {
      const uint32_t rw = a.R * a.rq_stride * 2;
      const uint32_t* rs = (const uint32_t*)a.rqt;
      uint32_t* rd = (uint32_t*)(smem + off[2]);
      for (uint32_t i = tid; i < rw; i += BD) rd[i] = rs[i];
    }
  }
  for (uint32_t i = tid; i < a.ns; i += BD) srv[i] = a.srv[i];
  for (uint32_t i = tid; i < (uint32_t)a.n_obj * a.K; i += BD) tk.top[i] = rec_max();
  // thresholds start at the seed keys (FastArgs::tseed: a bound on each
  // objective's K-th key over the launch range, from the sample launch)
  if (tid < MAXOBJ) tk.thr[tid] = a.tseed && tid < a.n_obj ? Rec{a.tseed[tid], ~0ull} : rec_max();
  if (tid == 0) {
    lock[0] = 0;
    lock[1] = score_tlo(a.tseed && a.n_obj ? a.tseed[0] : ~0ull, a.nc);
    lock[2] = __float_as_int(cov_tf32(a.tseed && a.n_obj > 3 ? a.tseed[3] : ~0ull));
  }
  // sample launch with a slot per wave: lane o clears the wave's slot of
  // objective o (no memset before the launch); the same lane's atomicMin
  // per chunk follows it in program order
  if (a.smin && a.smin_wave && lane < a.n_obj)
    a.smin[(size_t)lane * gridDim.x * WPB + (size_t)blockIdx.x * WPB + wid] = ~0ull;
  // BIN: the member bins start at zero (each lane re-zeroes its own after use)
  if constexpr (BIN)
    for (uint32_t i = tid; i < (BD >> 6) * N * 64; i += BD) ((uint32_t*)(smem + off[14]))[i] = 0;
  ((uint64_t*)(smem + off[15]))[tid] = 0;  // this thread's digest
  __syncthreads();
  const uint32_t cstride = a.cq_stride * 8;  // bytes per CQT column
  const uint32_t rstride = a.rq_stride * 8;
  for (uint32_t i = tid; i < a.ns; i += BD) {
    const uint32_t col = cqt + srv[i] * cstride;
    uint64_t c1 = 0, c2 = 0;
    for (uint32_t c = 0; c < a.nc; ++c) {
      uint64_t v = l16(col + 2 * c) >> LAT_SHIFT;
      c1 += v;
      c2 += v * v;
    }
    cs2[i] = c2;
    const double v = (double)((uint64_t)a.nc * c2 - c1 * c1);  // exact: < 2^53
    vcol[i] = v;
    vcol32[i] = (float)v;
    // w = 1 / sqrt(V): a member's COV is sqrt(V) / S, so the leader screen
    // maximises S * w with no transcendental per config (+inf: COV 0)
    const float w = v > 0.0 ? (float)(1.0 / sqrt(v)) : __builtin_inff();
    lrec[i] = make_uint2((uint32_t)c1, __float_as_uint(w));
  }
  __syncthreads();

  const uint32_t nc = a.nc, nq = nc >> 2, rem = nc & 3;
  const uint32_t qlane = qtab + tid * 4;
  // PERM: this wave's client lines (one per distinct (p1, p2) of a step),
  // then the pairs' keys (lowtab entries)
  const uint32_t lines = qtab + wid * lines_wave_bytes(a);
  const uint32_t keys = lines + a.gslots * cstride;
  const uint32_t gl = LB + (uint32_t)off[8] + wid * gline_bytes(a, N, KQ);  // this wave's group line
  const uint32_t rxt = gl;                                                 // per-position table (RX)
  const uint32_t mfl = gl + gline_rx_bytes(a, N);                          // nearest fixed member per client
  const uint32_t upk = mfl + cstride;                                      // packed fixed-row lists
  const uint32_t fS1 = upk + FP * KQ * 4;                                  // fixed column sums
  const uint32_t fVf = fS1 + F * 4;                                        // fixed column 1 / sqrt(V) (f32)
  const double pnc1 = a.p_fmean * (double)nc, pnc2 = a.p_emean * (double)nc;
  // the wave's valid-config count (uniform: a popcount of the valid lanes per
  // step, scalar adds) and each lane's running digest in LDS (off[15]):
  // neither holds vector registers across the step loop
  uint64_t valid_cnt = 0;
  // (the slot address is rebuilt at each add from the bins' lane address,
  // binb = LB + off[14] + 256 N wid + 4 lane, live through the step anyway:
  // the slot's own address, live across the step loop, was spilled and
  // reloaded from scratch every step)
  const uint32_t dofs = uni(LB + (uint32_t)off[15] + wid * 512u - 2u * (LB + (uint32_t)off[14] + wid * (N * 256u)));
  auto digest_add = [&](uint32_t binb_, uint64_t d) {
    uint32_t ad;
    asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(ad) : "v"(binb_), "s"(dofs));
    __hip_atomic_fetch_add((AS3 uint64_t*)(uintptr_t)ad, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  };

  // Work: either this wave's equal share of [rb, re), or (nwchunks > 0)
  // chunks of equal estimated cost taken from a ticket counter until none is
  // left.  Rank shares of equal size are not equal work: a group of C(p3, 3)
  // configs costs ceil(C(p3, 3) / 64) steps plus its precompute, and the
  // regions of small groups cost up to several times the average.
  bool static_done = false;
  // The next chunk's ticket is claimed when a chunk starts (its atomic's
  // latency overlaps the chunk's work), so each wave holds one claimed ticket
  // ahead; a claimed ticket is always swept by its wave, and every wave ends
  // on a ticket past the last chunk.
  const uint32_t wsh = a.wshards ? a.wshards : 1u, wx = blockIdx.x % wsh;
  unsigned int* const tctr = a.wctr + 32 * wx;  // this block's counter shard
  uint32_t cnext = 0;
  if (a.nwchunks && lane == 0) cnext = atomicAdd(tctr, 1u);  // (vector atomic, one lane)
  for (;;) {
  uint64_t r, rend;
  uint32_t chunk = ~0u;
  if (a.nwchunks) {
    const uint32_t c = wx + wsh * uni(cnext);
    if (c >= a.nwchunks) break;
    if (lane == 0) cnext = atomicAdd(tctr, 1u);
    chunk = c;
    PSTAT(a, 13, true);  // chunks
    r = uni64(a.wchunks[c]);
    rend = a.smin ? min(r + 64ull * a.ssteps, a.re) : uni64(a.wchunks[c + 1]);  // (sample chunks: ssteps steps)
    GASSERT(a, a.rb <= r && r <= rend && rend <= a.re, 0);  // chunk inside the launch range
  } else {
    if (static_done) break;
    static_done = true;
    const uint64_t nwaves = (uint64_t)gridDim.x * WPB;
    const uint64_t gw = (uint64_t)blockIdx.x * WPB + wid;
    const uint64_t total = a.re - a.rb;
    r = uni64(a.rb + (uint64_t)(((unsigned __int128)total * gw) / nwaves));
    rend = uni64(a.rb + (uint64_t)(((unsigned __int128)total * (gw + 1)) / nwaves));
  }

  if (r < rend) {
    uint32_t hq[F];  // fixed positions p_3 .. p_{N-1} (uniform)
    uint64_t base = 0;
    if (a.wstate && chunk != ~0u) {
      // the chunk's first group, unranked on the host (bote_capi.hip
      // sweep_chunks): the colex rank of its fixed part, then the positions
      // as bytes (a device unrank is ~45 dependent binomial loads)
      const uint64_t* st = a.wstate + 4 * (size_t)chunk;
      base = uni64(st[0]);
      const uint64_t b0 = uni64(st[1]), b1 = uni64(st[2]);
#pragma unroll
      for (int k = 0; k < F; ++k) hq[k] = (uint32_t)((k < 8 ? b0 >> (8 * k) : b1 >> (8 * (k - 8))) & 0xFFu);
    } else {
      uint32_t p[N];
      colex_unrank<N>(binom, a.ns, r, p);
#pragma unroll
      for (int k = 0; k < F; ++k) {
        hq[k] = uni(p[3 + k]);
        base += binom[hq[k] * (N + 1) + (k + 4)];
      }
      base = uni64(base);
    }
    uint64_t low = r - base;
#ifdef BOTE_DEBUG
    {
      bool okq = hq[0] >= 3 && hq[F - 1] < a.ns;
      for (int k = 1; k < F; ++k) okq = okq && hq[k - 1] < hq[k];
      GASSERT(a, okq, 1);  // fixed positions: ascending, above the 3 variable ones, < ns
    }
#endif
    for (;;) {
      const uint64_t gend = base + uni64(binom[hq[0] * (N + 1) + 3]);
      PSTAT(a, 12, true);  // groups (precomputes)
      // ---------------- per-group, wave-uniform precompute -> group line
      uint32_t freg[F];
#pragma unroll
      for (int k = 0; k < F; ++k) freg[k] = uni(sid ? hq[k] : srv[hq[k]]);
      if (lane < (uint32_t)F) {
        uint32_t pos = 0;
#pragma unroll
        for (int k = 0; k < F; ++k) pos = lane == (uint32_t)k ? hq[k] : pos;
        const uint2 lr = lrec[pos];
        s32(fS1 + 4 * lane, lr.x);
        s32(fVf + 4 * lane, lr.y);
      }
      if (lane < (uint32_t)FP) {
        // rows 2*lane and 2*lane+1: sorted distances to the other fixed
        // members (the self entry is INF, so it sorts last)
        uint32_t v[2][PF];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t k = 2 * lane + h;
          uint32_t rk = 0;
#pragma unroll
          for (int kk = 0; kk < F; ++kk) rk = k == (uint32_t)kk ? freg[kk] : rk;
#pragma unroll
          for (int m = 0; m < PF; ++m) {
            uint32_t d = 0xFFFFu;
            if (m < F && k < (uint32_t)F && (uint32_t)m != k) d = l16(rqt + freg[m < F ? m : 0] * rstride + 2 * rk) >> LAT_SHIFT;
            v[h][m] = d;
          }
          sort_network<PF>(v[h]);
        }
#pragma unroll
        for (int i = 0; i < KQ; ++i) {
          const uint32_t lo = i < F - 1 ? v[0][i < PF ? i : 0] : 0xFFFFu;
          const uint32_t hi = i < F - 1 ? v[1][i < PF ? i : 0] : 0xFFFFu;
          s32(upk + (lane * KQ + i) * 4, lo | (hi << 16));
        }
      }
      // each client's nearest fixed member: latency << 4 | member index (3 + k)
      for (uint32_t c = lane; c < (nq + 1) * 4; c += 64) {
        uint32_t key = 3u;
        if (c < nc) {
          key = 0xFFFFu;
#pragma unroll
          for (int k = 0; k < F; ++k) key = min(key, l16(cqt + freg[k] * cstride + 2 * c) | (uint32_t)(3 + k));
        }
        s16(mfl + 2 * c, key);
      }
      GASSERT(a, PERM || (tid + 1) * 4 <= (1u << qsh), 6);  // qtab plane holds every thread's word
      if (use_rx) {
        GASSERT(a, hq[0] <= a.ns, 5);  // position table rows (ns x 16 B per wave)
        // positions below the smallest fixed one: sorted distances to the
        // fixed members (row part), the fixed members' distances to x
        // (column part, packed as the fixed-row pairs); absent members INF
        for (uint32_t x = lane; x < hq[0]; x += 64) {
          const uint32_t rg = sid ? x : srv[x];
          uint32_t rf[4], cf[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t fk = freg[k < F ? k : 0];
            rf[k] = k < F ? l16(rqt + fk * rstride + 2 * rg) >> LAT_SHIFT : 0xFFFFu;
            cf[k] = k < F ? l16(rqt + rg * rstride + 2 * fk) >> LAT_SHIFT : 0xFFFFu;
          }
          sort_network<4>(rf);
          s128(rxt + 16 * x, make_uint4(rf[0] | (rf[1] << 16), rf[2] | (rf[3] << 16), cf[0] | (cf[1] << 16),
                                        cf[2] | (cf[3] << 16)));
        }
        // a fixed member's row at its own position (no variable member sits
        // there): the column part only, its distances to the fixed members,
        // itself included; the colocated leader-column sums read the leader's
        // row whichever member leads
        if (lane < (uint32_t)F) {
          uint32_t rj = 0, pj = 0;
#pragma unroll
          for (int k = 0; k < F; ++k) {
            rj = lane == (uint32_t)k ? freg[k] : rj;
            pj = lane == (uint32_t)k ? hq[k] : pj;
          }
          uint32_t cf[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) cf[k] = k < F ? l16(rqt + rj * rstride + 2 * freg[k < F ? k : 0]) >> LAT_SHIFT : 0xFFFFu;
          s64(rxt + 16 * pj + 8, cf[0] | (cf[1] << 16), cf[2] | (cf[3] << 16));
        }
      }
      wave_sync();

      // ---------------- the group's configs, 64 per step
      const uint64_t cend = uni64(gend < rend ? gend : rend);
      GASSERT(a, low + (cend - r) <= a.lowtab_n, 2);  // low-table rows of the group's configs
      // the step loop counts in 32 bits (a group holds C(p3, 3) < 2^32
      // configs, and the low table's rows are indexed in 32 bits), so its
      // control stays on the scalar unit (there is no 64-bit scalar compare)
      uint32_t left = uni((uint32_t)(cend - r)), lo32 = uni((uint32_t)low);
      // a per-lane pointer into the low table (lane-varying, so it lives in
      // VGPRs: the table's base is a spilled SGPR pair the step loop would
      // otherwise reload from VGPR lanes every step); the host pads the table
      // with 64 rows, so lanes past the group's end read in bounds
      const uint32_t* ltp = a.lowtab + lo32 + lane;
      uint32_t lp3 = *ltp;  // prefetched
      while (left) {
        const uint32_t len = min(64u, left);
        bool have = lane < len;
        PSTAT(a, 0, true);  // steps
        const uint32_t cur = lp3;
        // prefetch the next step's low part (the load overlaps this step)
        ltp += len;
        if (left > len) lp3 = *ltp;
        uint64_t key[MAXOBJ];
        bool ok[MAXOBJ];
        bool vflag = false;  // this lane's config is valid (counted by a ballot where the wave has reconverged)
#pragma unroll
        for (int o = 0; o < MAXOBJ; ++o) {
          key[o] = 0;
          ok[o] = false;
        }
        const uint64_t rank = r + lane;
        // ---- PERM: client lines.  Lanes with equal (p1, p2) (consecutive in
        //      colex order; a lane starts a new pair when p0 == 0) share
        //      min(member 1, member 2, nearest fixed) per client, built once
        //      per step, so the client loop merges one lane column into it.
        //      More distinct pairs than slots: the loop merges all four.
        uint32_t ll = lines;
        bool use_lines = false;
        if constexpr (PERM) {
          const uint64_t nk = __ballot(have && ((cur & 0xFFu) == 0 || lane == 0));
          const uint32_t nsl = (uint32_t)__popcll(nk);
          use_lines = nsl <= a.gslots && !ABLATE(a, 4096);
          PSTAT(a, 1, !use_lines);  // more distinct (p1, p2) than line slots
          if (use_lines) {
            // slot = index of the lane's pair among the step's pairs; the
            // first lane of each pair publishes its key to the wave's slot table
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(nk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nk, 0));
            const bool starts = (nk >> lane) & 1;
            const uint32_t slot = below + (starts ? 1u : 0u) - 1;
            ll = lines + slot * cstride;
            GASSERT(a, !have || slot < a.gslots, 4);  // client-line slot
            if (starts) s32(keys + 4 * slot, cur);
            wave_sync();
            // then lpl lanes per line (one quad = 4 clients each), 64 / lpl
            // lines per pass
            const uint32_t nqq = nq + (rem ? 1u : 0u);
            const uint32_t lsh = nqq <= 16 ? 3u : (nqq <= 32 ? 4u : 5u), lpl = 1u << lsh;
            const uint32_t li = lane >> lsh, qx = lane & (lpl - 1);
            for (uint32_t sl = 0; sl < nsl; sl += 64u >> lsh) {
              const uint32_t sx = sl + li;
              if (sx < nsl) {
                const uint32_t k = l32(keys + 4 * sx);
                const uint32_t p1 = (k >> 8) & 0xFFu, p2 = k >> 16;
                const uint32_t b1 = cqt + (sid ? p1 : srv[p1]) * cstride;
                const uint32_t b2 = cqt + (sid ? p2 : srv[p2]) * cstride;
                const uint32_t dst = lines + sx * cstride;
                for (uint32_t x = qx; x < nqq; x += lpl) {
                  const uint2 v1 = l64(b1 + 8 * x), v2 = l64(b2 + 8 * x), vf = l64(mfl + 8 * x);
                  const us2 lo = pk_min(pk_min(as_us2(v1.x | 0x00010001u), as_us2(v2.x | 0x00020002u)), as_us2(vf.x));
                  const us2 hi = pk_min(pk_min(as_us2(v1.y | 0x00010001u), as_us2(v2.y | 0x00020002u)), as_us2(vf.y));
                  s64(dst + 8 * x, as_u32(lo), as_u32(hi));
                }
              }
            }
            wave_sync();
          }
        }
        if (have) {
          uint32_t pv[3], rv[3];
          pv[0] = cur & 0xFF;
          pv[1] = (cur >> 8) & 0xFF;
          pv[2] = cur >> 16;
          GASSERT(a, pv[0] < pv[1] && pv[1] < pv[2] && pv[2] < hq[0], 3);  // variable positions below the fixed ones
#pragma unroll
          for (int i = 0; i < 3; ++i) rv[i] = sid ? pv[i] : srv[pv[i]];
          uint32_t cv[3];  // RQT column of each variable member
#pragma unroll
          for (int i = 0; i < 3; ++i) cv[i] = __umul24(rv[i], rstride) + rqt;  // (one v_mad_u32_u24)
          // ---- BIN: the member-binned client loop, one body for both of its
          //      places (before the Q phase with BIN_FIRST: it needs only the
          //      members' columns and the client line, and its results are the
          //      lane's bins in LDS and one squared-key sum, so none of the Q
          //      phase, leader choice or every-leader state is live through it;
          //      else after the leader choice).  Per client one LDS add of
          //      (key | 1 << 24) into its nearest member's bin (this lane's
          //      word of member m at binb + 256 m): the bin holds cnt_m (bits
          //      24..31) and K_m, the sum of keys (latency << 4 | m) of the
          //      member's clients = 16 D1_m + m cnt_m; the squared keys go to a
          //      v_dot2 sum (returned).  The epilogue (below) turns the bins
          //      into every table's sums.
          const uint32_t binb = LB + (uint32_t)off[14] + wid * (N * 256) + lane * 4;
          (void)binb;
          auto binned_clients = [&](auto lines_c, uint32_t c0, uint32_t c1, uint32_t c2) -> uint64_t {
            const us2 K1 = {1, 1}, K2 = {2, 2};
            // each client's nearest member, packed (latency << 4 | member):
            // the lane's member-0 column against its client line, or against
            // the other three sources when no line was built; two quads per
            // ds_read_b128 (g16: a 16-B aligned offset)
            auto nearest = [&](uint32_t g8, uint32_t& L, uint32_t& H) {
              const uint2 wa = l64(c0 + g8);
              us2 lo, hi;
              if constexpr (decltype(lines_c)::value) {
                const uint2 wl = l64(ll + g8);
                lo = pk_min(as_us2(wa.x), as_us2(wl.x));
                hi = pk_min(as_us2(wa.y), as_us2(wl.y));
              } else {
                const uint2 wb = l64(c1 + g8), wc = l64(c2 + g8), wf = l64(mfl + g8);
                lo = pk_min(pk_min(as_us2(wa.x), as_us2(wb.x) | K1), pk_min(as_us2(wc.x) | K2, as_us2(wf.x)));
                hi = pk_min(pk_min(as_us2(wa.y), as_us2(wb.y) | K1), pk_min(as_us2(wc.y) | K2, as_us2(wf.y)));
              }
              L = as_u32(lo);
              H = as_u32(hi);
            };
            auto nearest2 = [&](uint32_t g16, uint32_t& L0, uint32_t& H0, uint32_t& L1, uint32_t& H1) {
              const uint4 wa = l128(c0 + g16);
              us2 lo0, hi0, lo1, hi1;
              if constexpr (decltype(lines_c)::value) {
                const uint4 wl = l128(ll + g16);
                lo0 = pk_min(as_us2(wa.x), as_us2(wl.x));
                hi0 = pk_min(as_us2(wa.y), as_us2(wl.y));
                lo1 = pk_min(as_us2(wa.z), as_us2(wl.z));
                hi1 = pk_min(as_us2(wa.w), as_us2(wl.w));
              } else {
                const uint4 wb = l128(c1 + g16), wc = l128(c2 + g16), wf = l128(mfl + g16);
                lo0 = pk_min(pk_min(as_us2(wa.x), as_us2(wb.x) | K1), pk_min(as_us2(wc.x) | K2, as_us2(wf.x)));
                hi0 = pk_min(pk_min(as_us2(wa.y), as_us2(wb.y) | K1), pk_min(as_us2(wc.y) | K2, as_us2(wf.y)));
                lo1 = pk_min(pk_min(as_us2(wa.z), as_us2(wb.z) | K1), pk_min(as_us2(wc.z) | K2, as_us2(wf.z)));
                hi1 = pk_min(pk_min(as_us2(wa.w), as_us2(wb.w) | K1), pk_min(as_us2(wc.w) | K2, as_us2(wf.w)));
              }
              L0 = as_u32(lo0);
              H0 = as_u32(hi0);
              L1 = as_u32(lo1);
              H1 = as_u32(hi1);
            };
            uint32_t s2l = 0;
            uint64_t L2 = 0;
            auto badd = [&](uint32_t addr, uint32_t v) {
              __hip_atomic_fetch_add((AS3 uint32_t*)(uintptr_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            };
            // bin address of a member tag t: binb + (t << 8) in one v_lshl_add
            auto baddr = [&](uint32_t t) {
              uint32_t r;
              asm("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(r) : "v"(t), "v"(binb));
              return r;
            };
            // both bin addresses of a packed pair of keys: the tags masked
            // together (t = w & 0x000F000F, one v_and, fast class), then
            // binb + 256 t.lo16 and binb + 256 t.hi16 by v_mad_u32_u16
            // (op_sel selects the half; profiles/r05e: v_mad_u32_u16 0.91,
            // v_and 1.62, v_bfe and v_lshl_add 0.95 wave-instructions per
            // CU-clock)
            const uint32_t k256 = 256u;
            auto baddr2 = [&](uint32_t w, uint32_t& lo, uint32_t& hi) {
              const uint32_t t = w & 0x000F000Fu;
              asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(lo) : "v"(t), "v"(k256), "v"(binb));
              asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(hi) : "v"(t), "v"(k256), "v"(binb));
            };
            // a client's bin value (key | 1 << 24) by v_perm, every operand in
            // VGPRs (the compiler would pass the count word as an SGPR operand:
            // config 5 182.7 / 182.9 vs 185.0 / 185.2 ms, r05t)
            const uint32_t kcnt = 0x01000000u, sel_lo = 0x070C0100u, sel_hi = 0x070C0302u;
            auto bval = [&](uint32_t w, uint32_t sel) {
              uint32_t r;
              asm("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(kcnt), "v"(w), "v"(sel));
              return r;
            };
            // (the keys of a group of quads are read before any of their bin
            // adds: the compiler cannot tell the bins from the CQT and lines, so
            // it keeps program order between LDS reads and adds)
            auto quad_bin = [&](uint32_t L, uint32_t H, uint32_t nv) {
#ifdef BOTE_DEBUG
              GASSERT(a, (L & 15u) < (uint32_t)N && ((L >> 16) & 15u) < (uint32_t)N && (H & 15u) < (uint32_t)N &&
                             ((H >> 16) & 15u) < (uint32_t)N, 8);
#endif
              if (nv < 4) {  // (the last, partial quad: uniform)
                L &= nv >= 2 ? ~0u : 0x0000FFFFu;
                H &= nv == 3 ? 0x0000FFFFu : 0u;
              }
              // squared keys (16 lat + m)^2 = 256 lat^2 + 32 lat m + m^2: L2
              // follows from their sum and the bins (epilogue)
              s2l = __builtin_amdgcn_udot2(as_us2(L), as_us2(L), s2l, false);
              s2l = __builtin_amdgcn_udot2(as_us2(H), as_us2(H), s2l, false);
              if (nv >= 4) {
                uint32_t aL0, aL1, aH0, aH1;
                baddr2(L, aL0, aL1);
                baddr2(H, aH0, aH1);
                badd(aL0, bval(L, sel_lo));
                badd(aL1, bval(L, sel_hi));
                badd(aH0, bval(H, sel_lo));
                badd(aH1, bval(H, sel_hi));
                return;
              }
              badd(baddr(L & 15u), __builtin_amdgcn_perm(0x01000000u, L, 0x070C0100u));
              if (nv >= 2) badd(baddr(__builtin_amdgcn_ubfe(L, 16, 4)), __builtin_amdgcn_perm(0x01000000u, L, 0x070C0302u));
              if (nv >= 3) badd(baddr(H & 15u), __builtin_amdgcn_perm(0x01000000u, H, 0x070C0100u));
            };
            // s2l (squared keys) is flushed to 64 bits every k_flush quads
            constexpr uint32_t UB = decltype(lines_c)::value ? BIN_UB : 2u;
            const uint32_t nql = ABLATE(a, 1) ? 0u : nq;
            const uint32_t kfl = a.k_flush, fU = kfl / UB ? kfl / UB : 1u;
            uint32_t g = 0, k = 0;
            auto ub_body = [&](uint32_t g0) {
              uint32_t Lk[UB], Hk[UB];
#pragma unroll
              for (uint32_t u = 0; u < UB; u += 2) nearest2(g0 * 8 + 8 * u, Lk[u], Hk[u], Lk[u + 1], Hk[u + 1]);
#pragma unroll
              for (uint32_t u = 0; u < UB; ++u) quad_bin(Lk[u], Hk[u], 4u);
            };
            if (kfl >= nql + UB) {
              // one 32-bit sum holds every client's squared key: no flush test
              // in the loop (a uniform branch; at R=64 the test cost two VCC
              // v_cndmask and a 64-bit add per iteration).  Two bodies per
              // trip: the second's reads take immediate offsets, so the lane
              // addresses advance once per 2 UB quads
              for (; g + 2 * UB <= nql; g += 2 * UB) {
                ub_body(g);
                ub_body(g + UB);
              }
              for (; g + UB <= nql; g += UB) ub_body(g);
            } else if (kfl >= UB) {
              for (; g + UB <= nql; g += UB) {
                uint32_t Lk[UB], Hk[UB];
#pragma unroll
                for (uint32_t u = 0; u < UB; u += 2) nearest2(g * 8 + 8 * u, Lk[u], Hk[u], Lk[u + 1], Hk[u + 1]);
#pragma unroll
                for (uint32_t u = 0; u < UB; ++u) quad_bin(Lk[u], Hk[u], 4u);
                if (++k == fU) {
                  L2 += s2l;
                  s2l = 0;
                  k = 0;
                }
              }
              L2 += s2l;
              s2l = 0;
            }
            for (; g < nql; ++g) {
              uint32_t Lk, Hk;
              nearest(g * 8, Lk, Hk);
              quad_bin(Lk, Hk, 4u);
              L2 += s2l;
              s2l = 0;
            }
            if (rem && !ABLATE(a, 1)) {
              uint32_t Lk, Hk;
              nearest(nq * 8, Lk, Hk);
              quad_bin(Lk, Hk, rem);
            }
            return L2 + s2l;
          };
          uint64_t L2first = 0;
          if constexpr (BIN && BIN_FIRST) {
            const uint32_t f0 = __umul24(rv[0], cstride) + cqt, f1 = __umul24(rv[1], cstride) + cqt,
                           f2 = __umul24(rv[2], cstride) + cqt;
            L2first = use_lines ? binned_clients(BoolC<true>{}, f0, f1, f2) : binned_clients(BoolC<false>{}, f0, f1, f2);
          }
          // member m: 0..2 variable, 3.. fixed (config order = ascending positions)
          uint32_t Q2[N], Q3[N];
          // PERM: Q2 and Q3 also as the packed pair words of the rows (index
          // as wp's: 0 members (0, 1), 1 member 2, 2 + pp fixed (3 + 2pp,
          // 4 + 2pp); a lone member's high half 0): the leader choice reads a
          // half with v_mad_u32_u16 op_sel, the leader's values come out by
          // byte selection (v_perm), so neither needs the unpacked values
          uint32_t Q2w[4] = {0u, 0u, 0u, 0u}, Q3w[4] = {0u, 0u, 0u, 0u};
          uint32_t cS1p = 0, cS1e = 0;  // colocated sums: packed (t0 | t1 << 16), third table
          uint32_t cS2[NT], cS1t[NT];  // (PERM: per table)
#pragma unroll
          for (int t = 0; t < NT; ++t) cS2[t] = cS1t[t] = 0;
          // PERM: each table's member latencies as packed pair words, index
          // 0: members (0, 1), 1: member 2, 2 + pp: fixed members (3 + 2pp, 4 + 2pp)
          uint32_t wp[NT][2 + FP];
          // sorted row (packed pair: lo = member j, hi = member j + 1)
          auto emit_pk = [&](int j, bool has_hi, const uint32_t* L) {
            const uint32_t w0 = L[QC::lq(0) - 2], w1 = L[(NL >= 2 ? QC::lq(1) : QC::lq(0)) - 2];
            if constexpr (PERM) {
              Q2[j] = L[0] & 0xFFFFu;
              Q3[j] = L[1] & 0xFFFFu;
              if (has_hi) {
                Q2[j + 1] = L[0] >> 16;
                Q3[j + 1] = L[1] >> 16;
              }
              const int pi = j == 0 ? 0 : (j == 2 ? 1 : 2 + (j - 3) / 2);
              const uint32_t hm = has_hi ? ~0u : 0xFFFFu;
#pragma unroll
              for (int t = 0; t < NT; ++t) wp[t][pi] = L[QT::q(t) - 2] & hm;
              Q2w[pi] = L[0] & hm;
              Q3w[pi] = L[1] & hm;
              (void)w0;
              (void)w1;
              return;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              if (h == 1 && !has_hi) break;
              const uint32_t sel = h ? 0x07060302u : 0x05040100u;
              const uint32_t sh = h ? 16u : 0u;
              Q2[j + h] = (L[0] >> sh) & 0xFFFFu;
              Q3[j + h] = (L[1] >> sh) & 0xFFFFu;
              const uint32_t word = NL >= 2 ? __builtin_amdgcn_perm(w1, w0, sel) : ((w0 >> sh) & 0xFFFFu);
              if (!ABLATE(a, 1024)) s32(qlane + ((uint32_t)(j + h) << qsh), word);
              cS1p += word;
              const uint32_t q0 = word & 0xFFFFu;
              cS2[0] += q0 * q0;
              if (NL >= 2) {
                const uint32_t q1 = word >> 16;
                cS2[NL >= 2 ? 1 : 0] += q1 * q1;
              }
              if (NL == 3) {
                const uint32_t q2 = (L[QC::lq(NL - 1) - 2] >> sh) & 0xFFFFu;
                s32(qlane + ((uint32_t)(N + j + h) << qsh), q2);
                cS1e += q2;
                cS2[NL - 1] += q2 * q2;
              }
            }
          };
          if (use_rx) {
            // ---- Q phase from the group's position table: each variable
            //      row = its sorted fixed part + the 2 distances to the other
            //      variable members; each fixed row = the group's sorted
            //      fixed-to-fixed list + the lane's 3 distances (packed)
            uint4 X0, X1, X2;
            if (ABLATE(a, 8192)) {  // timing only: no table reads
              X0 = make_uint4(pv[0], pv[1], pv[2], pv[0] ^ pv[1]);
              X1 = make_uint4(pv[2], pv[0], pv[1], pv[1] ^ pv[2]);
              X2 = make_uint4(pv[1], pv[2], pv[0], pv[0] ^ pv[2]);
            } else {
              X0 = l128(rxt + 16 * pv[0]);
              X1 = l128(rxt + 16 * pv[1]);
              X2 = l128(rxt + 16 * pv[2]);
            }
            {  // rows 0 and 1, packed (lo: member 0, hi: member 1)
              us2 A[4], y[2], L[KQ];
              A[0] = as_us2(__builtin_amdgcn_perm(X1.x, X0.x, 0x05040100u));
              A[1] = as_us2(__builtin_amdgcn_perm(X1.x, X0.x, 0x07060302u));
              A[2] = as_us2(__builtin_amdgcn_perm(X1.y, X0.y, 0x05040100u));
              A[3] = as_us2(__builtin_amdgcn_perm(X1.y, X0.y, 0x07060302u));
              // (stored latencies are << 4, so one shift of the packed pair is exact)
              y[0] = as_us2((l16(cv[1] + 2 * rv[0]) | (l16(cv[0] + 2 * rv[1]) << 16)) >> LAT_SHIFT);  // d(0,1) | d(1,0)
              y[1] = as_us2((l16(cv[2] + 2 * rv[0]) | (l16(cv[2] + 2 * rv[1]) << 16)) >> LAT_SHIFT);  // d(0,2) | d(1,2)
              const us2 t = pk_min(y[0], y[1]);
              y[1] = pk_max(y[0], y[1]);
              y[0] = t;
              if (ABLATE(a, 32)) {
#pragma unroll
                for (int k = 0; k < KQ; ++k) L[k] = pk_min(A[k], y[k & 1]);
              } else {
                merge_k<F < 4 ? F : 4, 2, KQ>(A, y, L);
              }
              uint32_t W[KQ];
#pragma unroll
              for (int k = 0; k < KQ; ++k) W[k] = as_u32(L[k]);
              emit_pk(0, true, W);
            }
            {  // row 2
              uint32_t A[4], y[2], L[KQ];
              A[0] = X2.x & 0xFFFFu;
              A[1] = X2.x >> 16;
              A[2] = X2.y & 0xFFFFu;
              A[3] = X2.y >> 16;
              const uint32_t d20 = l16(cv[0] + 2 * rv[2]) >> LAT_SHIFT, d21 = l16(cv[1] + 2 * rv[2]) >> LAT_SHIFT;
              y[0] = min(d20, d21);
              y[1] = max(d20, d21);
              merge_k<F < 4 ? F : 4, 2, KQ>(A, y, L);
              emit_pk(2, false, L);
            }
#pragma unroll
            for (int pp = 0; pp < FP; ++pp) {
              us2 A[KQ];  // the group's sorted fixed-row lists (uniform)
#pragma unroll
              for (int i = 0; i < KQ; ++i) A[i] = as_us2(l32(upk + (pp * KQ + i) * 4));
              const bool has_hi = 2 * pp + 1 < F;
              us2 y[3];  // the 3 lane distances (d(f, m) | d(f', m)), sorted
              y[0] = as_us2(pp == 0 ? X0.z : X0.w);
              y[1] = as_us2(pp == 0 ? X1.z : X1.w);
              y[2] = as_us2(pp == 0 ? X2.z : X2.w);
              {
                us2 t = pk_min(y[0], y[1]);
                y[1] = pk_max(y[0], y[1]);
                y[0] = t;
                t = pk_min(y[1], y[2]);
                y[2] = pk_max(y[1], y[2]);
                y[1] = t;
                t = pk_min(y[0], y[1]);
                y[1] = pk_max(y[0], y[1]);
                y[0] = t;
              }
              us2 L[KQ];
              if (ABLATE(a, 64)) {
#pragma unroll
                for (int k = 0; k < KQ; ++k) L[k] = pk_min(A[k], y[k < 3 ? k : 2]);
              } else {
                // (the group's fixed-row lists hold F - 1 real distances, the
                // self entry and padding sort last as +inf)
                merge_k<(F - 1 < KQ ? F - 1 : KQ), 3, KQ>(A, y, L);
              }
              uint32_t W[KQ];
#pragma unroll
              for (int k = 0; k < KQ; ++k) W[k] = as_u32(L[k]);
              emit_pk(3 + 2 * pp, has_hi, W);
            }
          } else {
            // ---- Q phase, variable rows 0 and 1 (packed), row 2 (lo half)
            {
              uint32_t v[PV];
              // (stored latencies are << 4, so one shift of the packed pair is exact)
              v[0] = (l16(cv[1] + 2 * rv[0]) | (l16(cv[0] + 2 * rv[1]) << 16)) >> LAT_SHIFT;  // d(0,1) | d(1,0)
              v[1] = (l16(cv[2] + 2 * rv[0]) | (l16(cv[2] + 2 * rv[1]) << 16)) >> LAT_SHIFT;  // d(0,2) | d(1,2)
  #pragma unroll
              for (int k = 0; k < F; ++k) {
                const uint32_t fc = rqt + freg[k] * rstride;
                v[2 + k] = (l16(fc + 2 * rv[0]) | (l16(fc + 2 * rv[1]) << 16)) >> LAT_SHIFT;
              }
  #pragma unroll
              for (int k = N - 1; k < PV; ++k) v[k] = 0xFFFFFFFFu;
              if (!ABLATE(a, 32)) sort_network_pk<PV>(v);
              emit_pk(0, true, v);
            }
            {
              uint32_t v[PV];
              v[0] = l16(cv[0] + 2 * rv[2]) >> LAT_SHIFT;
              v[1] = l16(cv[1] + 2 * rv[2]) >> LAT_SHIFT;
  #pragma unroll
              for (int k = 0; k < F; ++k) v[2 + k] = l16(rqt + freg[k] * rstride + 2 * rv[2]) >> LAT_SHIFT;
  #pragma unroll
              for (int k = N - 1; k < PV; ++k) v[k] = 0xFFFFu;
              if (!ABLATE(a, 32)) sort_network<PV>(v);
              emit_pk(2, false, v);
            }
            // ---- fixed rows (pairs): insert the 3 lane distances into the
            //      group's packed sorted lists
  #pragma unroll
            for (int pp = 0; pp < FP; ++pp) {
              us2 A[KQ];  // the group's sorted fixed-row lists (uniform)
  #pragma unroll
              for (int i = 0; i < KQ; ++i) A[i] = as_us2(l32(upk + (pp * KQ + i) * 4));
              const bool has_hi = 2 * pp + 1 < F;
              us2 y[3];  // the 3 lane distances, then sorted (3 compare-exchanges)
  #pragma unroll
              for (int m = 0; m < 3; ++m) {
                const uint32_t lo = l16(cv[m] + 2 * freg[2 * pp]);
                const uint32_t hi = has_hi ? l16(cv[m] + 2 * freg[has_hi ? 2 * pp + 1 : 2 * pp]) : 0xFFF0u;
                y[m] = as_us2((lo | (hi << 16)) >> LAT_SHIFT);
                if (!has_hi) y[m] = as_us2(as_u32(y[m]) | 0xFFFF0000u);
              }
              {
                us2 t = pk_min(y[0], y[1]);
                y[1] = pk_max(y[0], y[1]);
                y[0] = t;
                t = pk_min(y[1], y[2]);
                y[2] = pk_max(y[1], y[2]);
                y[1] = t;
                t = pk_min(y[0], y[1]);
                y[1] = pk_max(y[0], y[1]);
                y[0] = t;
              }
              // merge: the k-th smallest of A u y is the min over the splits
              // (k+1-j from A, j from y) of max(A[k-j], y[j-1])
              uint32_t L[KQ];
  #pragma unroll
              for (int k = 0; k < KQ; ++k) {
                us2 z = A[k];
                if (ABLATE(a, 64)) {
                  L[k] = as_u32(pk_min(z, y[k < 3 ? k : 2]));
                  continue;
                }
  #pragma unroll
                for (int j = 1; j <= 3 && j <= k + 1; ++j) {
                  const int i = k + 1 - j;  // elements taken from A
                  z = pk_min(z, i == 0 ? y[j - 1] : pk_max(A[i > 0 ? i - 1 : 0], y[j - 1]));
                }
                L[k] = as_u32(z);
              }
              emit_pk(3 + 2 * pp, has_hi, L);
            }
          }
          // ---- PERM: byte planes (member m's latency: low byte in byte m of
          //      QL, high byte in byte m of QH; members 0..3 in .x, 4..6 in
          //      .y) and the colocated sums over the members
          uint2 QL[NT], QH[NT];
          // BIN kernels with an odd number of fixed members (n = 4, 6): the
          // two lone members, 2 and N - 1, share one table word (q_2 | q_{N-1}
          // << 16), so the colocated sums and the bin epilogue's per-table
          // dot products run over one word fewer (config 5, n = 6: 3 words)
          constexpr bool PAIR2 = BIN && (F % 2 == 1);
          constexpr int NWB = PAIR2 ? 1 + FP : 2 + FP;
          if constexpr (PAIR2) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wp[t][1] |= wp[t][1 + FP] << 16;
          }
          if constexpr (PERM) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const uint32_t w01 = wp[t][0], w2 = wp[t][1], w34 = wp[t][2], w56 = FP >= 2 ? wp[t][FP >= 2 ? 3 : 2] : 0u;
              if constexpr (!BIN) {  // (BIN bins the clients by member instead)
                QL[t].x = __builtin_amdgcn_perm(w2, w01, 0x0C040200u) | (w34 << 24);
                QH[t].x = __builtin_amdgcn_perm(w34, __builtin_amdgcn_perm(w2, w01, 0x0C050301u), 0x05020100u);
                QL[t].y = __builtin_amdgcn_perm(w56, w34, 0x0C060402u);
                QH[t].y = __builtin_amdgcn_perm(w56, w34, 0x0C070503u);
              }
              uint32_t ps = 0, sq = 0;
#pragma unroll
              for (int i = 0; i < NWB; ++i) {
                ps += wp[t][i];
                sq = __builtin_amdgcn_udot2(as_us2(wp[t][i]), as_us2(wp[t][i]), sq, false);
              }
              cS2[t] = sq;
              cS1t[t] = (ps & 0xFFFFu) + (ps >> 16);
            }
          }
          // ---- FPaxos leader (f = 1, q = 2, min COV, first in config order)
          auto pos_of = [&](int l) { return l < 3 ? pv[l] : hq[l - 3]; };
          auto reg_of = [&](int l) { return l < 3 ? rv[l] : freg[l - 3]; };
          uint2 vrec[3];  // the variable members' (S1, f32 1 / sqrt(V)): one 8-byte LDS read each
#pragma unroll
          for (int i = 0; i < 3; ++i) vrec[i] = lrec[pv[i]];
          auto s1_of = [&](int l) { return l < 3 ? vrec[l].x : l32(fS1 + 4 * (l - 3)); };
          auto wf_of = [&](int l) { return l < 3 ? __uint_as_float(vrec[l].y) : lf32(fVf + 4 * (l - 3)); };
          auto vf_of = [&](int l) { return (float)vcol[pos_of(l)]; };  // (exact re-scan only)
          // 1 / COV proxy t = S / sqrt(V) = S * w per member in f32 (S exact
          // below 2^24, w and the product one rounding each): within 2^-23
          // of exact, so comparisons outside a 2^-18 band are decided; any
          // closer call re-runs the scan exactly (cov2_sign) or defers.
          // Decided without a sequential scan: m = max t (a tree), the
          // leader is the first member at m, and the decision is ambiguous
          // when m is finite and another member lies within the 2^-18 band
          // below m (exact zeros, V = 0, t = inf, tie exactly and keep the
          // first, as the reference's first-minimum does).
          uint32_t bi = 0;
          // PERM (n <= 7): the leader's byte code, member l -> l + (l >= 3),
          // so that codes 0..2 name the bytes of the step's packed variable
          // positions (cur) and 4..7 those of the packed fixed ones, and a
          // code's low 2 bits index its member within the Q2w / Q3w byte pool
          uint32_t lcode = 0;
          auto code_of = [](int l) { return (uint32_t)(l + (l >= 3 ? 1 : 0)); };
          // S = s1 + nc Q2 for member l from its packed word (op_sel: the half)
          auto s_of = [&](int l) {
            if constexpr (PERM) {
              const int pi = l < 2 ? 0 : (l == 2 ? 1 : 2 + (l - 3) / 2);
              const bool hi = l < 2 ? l == 1 : (l > 2 && (l - 3) % 2 == 1);
              uint32_t r;
              if (hi) asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(Q2w[pi]), "s"(nc), "v"(s1_of(l)));
              else asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(Q2w[pi]), "s"(nc), "v"(s1_of(l)));
              return r;
            } else {
              return s1_of(l) + __umul24(nc, Q2[l]);
            }
          };
          bool amb = false;
          if (!ABLATE(a, 128)) {
            // t >= 0 and never NaN here (S >= nc * Q2 > 0: server-server
            // latencies are > 0 on the fast path, so Q2 > 0).  Non-negative
            // floats order as their bit patterns, so each t's low IB mantissa
            // bits carry IM - l instead (a change below 2^-19 relative, inside
            // the band below): the integer max is the largest t with the
            // FIRST member on exact ties, and no compare/select chain is needed.
            constexpr uint32_t IM = N <= 8 ? 7u : 15u;
            uint32_t u[N];
#pragma unroll
            for (int l = 0; l < N; ++l) {
              const float t = (float)s_of(l) * wf_of(l);
              u[l] = (__float_as_uint(t) & ~IM) | (IM - (PERM ? code_of(l) : (uint32_t)l));
            }
            // the largest and second largest (with multiplicity) t: a
            // running max and median-of-three, 2 ops per member
            uint32_t mu = u[0], m2u = 0;
#pragma unroll
            for (int l = 1; l < N; ++l) {
              m2u = max(min(mu, m2u), min(max(mu, m2u), u[l]));  // (v_med3_u32)
              mu = max(mu, u[l]);
            }
            bi = (mu & IM) ^ IM;  // the first member at the maximum
            if constexpr (PERM) {
              lcode = bi;
              bi = lcode - (lcode >> 2);  // (codes 4..7: members 3..6)
            }
            const float m = __uint_as_float(mu & ~IM), m2 = __uint_as_float(m2u & ~IM);
            amb = m < __builtin_inff() && m2 >= m * (1.0f - 0x1p-18f);
          }
          PSTAT(a, 2, amb);  // leader within the f32 band: exact re-scan
          if (amb) {  // exact re-scan in the generic path's arithmetic
            amb = false;
            bi = 0;
            lcode = 0;
            uint32_t bpos = pv[0];
            uint32_t bS = s1_of(0) + nc * Q2[0];
            float bV = vf_of(0);
#pragma unroll
            for (int l = 1; l < N; ++l) {
              const uint32_t S = s1_of(l) + nc * Q2[l];
              const float V = vf_of(l);
              if (V == 0.0f && bV == 0.0f) continue;  // both COV exactly 0: keep the first
              const uint32_t pl = pos_of(l);
              const int c = cov2_sign(V, S, bV, bS, [&] { return vcol[pl]; }, [&] { return vcol[bpos]; });
              if (c == 0) amb = true;
              if (c < 0) {
                bi = l;
                lcode = code_of(l);
                bS = S;
                bV = V;
                bpos = pl;
              }
            }
          }
          GASSERT(a, bi < (uint32_t)N, 7);  // leader member
          PSTAT(a, 3, amb);  // leader deferred
          if (amb) {
            if (!a.smin) defer_rank(a, rank);
            have = false;
            if constexpr (BIN && BIN_FIRST) {  // the epilogue will not run: re-zero the bins here
#pragma unroll
              for (int m = 0; m < N; ++m) s32(binb + 256u * m, 0u);
            }
          }
          if (have) {
            uint32_t lpos = pv[0], lq2 = Q2[0], lq3 = Q3[0], lreg = rv[0];
            if constexpr (PERM && SI) {
              // the leader's values by byte selection on its code: Q2 / Q3
              // from the pool of members 0..2 (Q2w[0..1]) or 3..6 (Q2w[2..3]),
              // 2 bytes at 2 (code & 3); its position from the step's packed
              // variable positions (cur: p0 | p1 << 8 | p2 << 16) or the
              // group's fixed ones (hqw); 11 ops where the compare/select
              // chain over the members took 28
              uint32_t hqw = 0;
#pragma unroll
              for (int k = 0; k < F; ++k) hqw |= hq[k] << (8 * k);
              const uint32_t sel = 0x0C0C0100u + (lcode & 3u) * 0x0202u;
              const bool pb = lcode >= 4u;
              lq2 = pb ? __builtin_amdgcn_perm(Q2w[3], Q2w[2], sel) : __builtin_amdgcn_perm(Q2w[1], Q2w[0], sel);
              lq3 = pb ? __builtin_amdgcn_perm(Q3w[3], Q3w[2], sel) : __builtin_amdgcn_perm(Q3w[1], Q3w[0], sel);
              lpos = __builtin_amdgcn_perm(hqw, cur, 0x0C0C0C00u | lcode);
            } else {
#pragma unroll
              for (int l = 1; l < N; ++l)
                if (bi == (uint32_t)l) {
                  lpos = pos_of(l);
                  lq2 = Q2[l];
                  lq3 = Q3[l];
                  if constexpr (!SI) lreg = reg_of(l);
                }
            }
            if constexpr (SI) lreg = lpos;  // (servers in region order: position = region)
            Mom mom[NSLOT];
            // XK: the extended slots and every leader's FPaxos moments are
            // folded into the digest (a linear fold: any order) as they are
            // produced, so none stays live to the end of the config;
            // objectives 5..7 keep one sum each (tt1, tw2, fl1)
            uint32_t hx = 0;
            uint32_t x_tt1 = 0, x_tw2 = 0, x_fl1 = 0;
            auto xslot = [&](uint32_t sl, uint64_t s1, uint64_t s2) { hx = digest_fold(hx, sl, s1, s2); };
            (void)xslot;
            // ---- XK, before the client loop (so that none of it stays live
            //      through it; with BIN_FIRST the loop has run already): FPaxos all leaders (Bote::all_leaders_stats, lib.rs:129-150)
            //      over the Input clients at q = f + 1, members in config
            //      order, from the column sums (closed form, as ff1/ff2); the
            //      digest consumes every one, and slots fl1/fl2 take the best
            //      leader by Stats::Mean (lib.rs:99-121: the first minimum)
            if constexpr (XK) {
              // 32-bit arithmetic: the host runs XK here only when every sum
              // of squares fits (nc * (2 * max latency)^2 < 2^32), so
              // S2 = c2 + q (c1 + S1) with 24-bit multiplies (c1, S1 < 2^24)
              uint32_t b1 = ~0u, b2 = ~0u, b1s = 0, b2s = 0;
#pragma unroll
              for (int f = 0; f < 2; ++f) {
#pragma unroll
                for (int l = 0; l < N; ++l) {
                  const uint32_t c1 = s1_of(l), c2 = (uint32_t)cs2[pos_of(l)];
                  const uint32_t q = f == 0 ? Q2[l] : Q3[l];
                  const uint32_t m1 = __umul24(nc, q) + c1;  // (nc, q, c1 + m1 < 2^24)
                  const uint32_t m2 = __umul24(q, c1 + m1) + c2;
                  hx = digest_fold_leader(hx, f, l, m1, m2);
                  if (f == 0 && m1 < b1) {
                    b1 = m1;
                    b1s = m2;
                  }
                  if (f == 1 && m1 < b2) {
                    b2 = m1;
                    b2s = m2;
                  }
                }
              }
              xslot(18, b1, b1s);  // fl1
              xslot(19, b2, b2s);  // fl2
              x_fl1 = (uint32_t)b1;
              // Colocated Tempo: the members' own quorum latencies (slots 14..17)
              constexpr int t2 = QT::idx(2), t3 = QT::idx(3), t4 = QT::idx(4);
              xslot(14, cS1t[t2], cS2[t2]);  // ttC1
              xslot(15, cS1t[t4], cS2[t4]);  // ttC2
              xslot(16, cS1t[t2], cS2[t2]);  // twC1
              xslot(17, cS1t[t3], cS2[t3]);  // twC2
            }
            // ---- Input leaderless: 3 lane columns + the wave's nearest-fixed line
            {
              const us2 J1 = {1, 1}, J2 = {2, 2};
              // Sums use full-rate 32-bit adds on packed u16 pairs (no half
              // overflows: lat + q < 2^15, and p1 is flushed every g_flush
              // quads), squares the 2-wide dot product (s2, flushed to 64 bits)
              uint32_t S1[NT], s2[NT], p1[NT];
              uint64_t S2[NT];
#pragma unroll
              for (int t = 0; t < NT; ++t) {
                S1[t] = 0;
                S2[t] = 0;
                s2[t] = 0;
                p1[t] = 0;
              }
              const uint32_t c0 = __umul24(rv[0], cstride) + cqt, c1 = __umul24(rv[1], cstride) + cqt,
                             c2 = __umul24(rv[2], cstride) + cqt;
              // (m << qsh) + qlane in one instruction (the compiler would
              // otherwise re-associate it into shift, and, add)
              auto qaddr = [&](uint32_t m) {
                uint32_t r;
                asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(qsh), "v"(qlane));
                return r;
              };
              // each client's nearest member, packed (latency << 4 | member):
              // the lane's member-0 column against its client line, or
              // against the other three sources when no line was built
              auto nearest = [&](auto lines_c, uint32_t g8, us2& lo, us2& hi) {
                const uint2 wa = l64(c0 + g8);
                if constexpr (decltype(lines_c)::value) {
                  const uint2 wl = l64(ll + g8);
                  lo = pk_min(as_us2(wa.x), as_us2(wl.x));
                  hi = pk_min(as_us2(wa.y), as_us2(wl.y));
                } else {
                  const uint2 wb = l64(c1 + g8), wc = l64(c2 + g8), wf = l64(mfl + g8);
                  lo = pk_min(pk_min(as_us2(wa.x), as_us2(wb.x) | J1), pk_min(as_us2(wc.x) | J2, as_us2(wf.x)));
                  hi = pk_min(pk_min(as_us2(wa.y), as_us2(wb.y) | J1), pk_min(as_us2(wc.y) | J2, as_us2(wf.y)));
                }
              };
              // two quads at once (g16: a 16-B aligned offset): one ds_read_b128
              // per source (4 LDS cycles for 16 B per lane, where the pair of
              // 8-B reads the compiler would merge into a ds_read2_b64 takes 8;
              // the column stride is an odd number of 16-B units: quad_stride)
              auto nearest2 = [&](auto lines_c, uint32_t g16, us2& lo0, us2& hi0, us2& lo1, us2& hi1) {
                const uint4 wa = l128(c0 + g16);
                if constexpr (decltype(lines_c)::value) {
                  const uint4 wl = l128(ll + g16);
                  lo0 = pk_min(as_us2(wa.x), as_us2(wl.x));
                  hi0 = pk_min(as_us2(wa.y), as_us2(wl.y));
                  lo1 = pk_min(as_us2(wa.z), as_us2(wl.z));
                  hi1 = pk_min(as_us2(wa.w), as_us2(wl.w));
                } else {
                  const uint4 wb = l128(c1 + g16), wc = l128(c2 + g16), wf = l128(mfl + g16);
                  lo0 = pk_min(pk_min(as_us2(wa.x), as_us2(wb.x) | J1), pk_min(as_us2(wc.x) | J2, as_us2(wf.x)));
                  hi0 = pk_min(pk_min(as_us2(wa.y), as_us2(wb.y) | J1), pk_min(as_us2(wc.y) | J2, as_us2(wf.y)));
                  lo1 = pk_min(pk_min(as_us2(wa.z), as_us2(wb.z) | J1), pk_min(as_us2(wc.z) | J2, as_us2(wf.z)));
                  hi1 = pk_min(pk_min(as_us2(wa.w), as_us2(wb.w) | J1), pk_min(as_us2(wc.w) | J2, as_us2(wf.w)));
                }
              };
              auto quad_at = [&](us2 lo, us2 hi, uint32_t mlo, uint32_t mhi) {
                const uint32_t L = as_u32(lo), H = as_u32(hi);
#ifdef BOTE_DEBUG
                // every client's nearest-member tag names a member (low 4 bits)
                GASSERT(a, (L & 15u) < (uint32_t)N && ((L >> 16) & 15u) < (uint32_t)N && (H & 15u) < (uint32_t)N &&
                               ((H >> 16) & 15u) < (uint32_t)N, 8);
#endif
                const us2 dlo = lo >> (us2)4, dhi = hi >> (us2)4;
                auto acc1 = [&](int t, us2 q01, us2 q23) {
                  // packed adds as one 32-bit add: no carry crosses the halves
                  const uint32_t a01 = (as_u32(dlo) + as_u32(q01)) & mlo;
                  const uint32_t a23 = (as_u32(dhi) + as_u32(q23)) & mhi;
                  p1[t] += a01 + a23;
                  s2[t] = __builtin_amdgcn_udot2(as_us2(a01), as_us2(a01), s2[t], false);
                  s2[t] = __builtin_amdgcn_udot2(as_us2(a23), as_us2(a23), s2[t], false);
                };
                if constexpr (PERM) {
                  // the 4 clients' member tags as byte selectors, then per
                  // table the low and high bytes of their members' latencies
                  // (v_perm over the byte planes), interleaved into u16 pairs
                  const uint32_t sel = __builtin_amdgcn_perm(H, L, 0x06040200u) & 0x0F0F0F0Fu;
#pragma unroll
                  for (int t = 0; t < NT; ++t) {
                    const uint32_t bl = __builtin_amdgcn_perm(QL[t].y, QL[t].x, sel);
                    const uint32_t bh = __builtin_amdgcn_perm(QH[t].y, QH[t].x, sel);
                    acc1(t, as_us2(__builtin_amdgcn_perm(bh, bl, 0x05010400u)),
                         as_us2(__builtin_amdgcn_perm(bh, bl, 0x07030602u)));
                  }
                } else {
                  // qtab address of each client's nearest member: one bitfield
                  // extract + one v_lshl_add per client; the two tables are the
                  // halves of the member's word, read straight into packed pairs
                  const uint32_t a0 = qaddr(L & 15u), a1 = qaddr(__builtin_amdgcn_ubfe(L, 16, 4));
                  const uint32_t a2 = qaddr(H & 15u), a3 = qaddr(__builtin_amdgcn_ubfe(H, 16, 4));
                  // (16-bit loads into packed halves would need d16 loads, which
                  //  gfx950 with sramecc does not preserve; read words and perm)
                  const uint32_t w0 = l32(a0), w1 = l32(a1), w2 = l32(a2), w3 = l32(a3);
                  acc1(0, as_us2(__builtin_amdgcn_perm(w1, w0, 0x05040100u)), as_us2(__builtin_amdgcn_perm(w3, w2, 0x05040100u)));
                  if (NL >= 2)
                    acc1(NL >= 2 ? 1 : 0, as_us2(__builtin_amdgcn_perm(w1, w0, 0x07060302u)),
                         as_us2(__builtin_amdgcn_perm(w3, w2, 0x07060302u)));
                  if (NL == 3) {
                    const uint32_t P2 = (uint32_t)N << qsh;
                    const uint32_t x0 = l32(a0 + P2), x1 = l32(a1 + P2), x2 = l32(a2 + P2), x3 = l32(a3 + P2);
                    acc1(NL - 1, as_us2(__builtin_amdgcn_perm(x1, x0, 0x05040100u)),
                         as_us2(__builtin_amdgcn_perm(x3, x2, 0x05040100u)));
                  }
                }
              };
              auto quad = [&](auto lines_c, uint32_t g8, uint32_t mlo, uint32_t mhi) {
                us2 lo, hi;
                nearest(lines_c, g8, lo, hi);
                quad_at(lo, hi, mlo, mhi);
              };
              auto quad2 = [&](auto lines_c, uint32_t g16) {
                us2 lo0, hi0, lo1, hi1;
                nearest2(lines_c, g16, lo0, hi0, lo1, hi1);
                quad_at(lo0, hi0, ~0u, ~0u);
                quad_at(lo1, hi1, ~0u, ~0u);
              };
              auto flush = [&]() {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                  S2[t] = S32 ? (uint64_t)((uint32_t)S2[t] + s2[t]) : S2[t] + s2[t];
                  s2[t] = 0;
                  S1[t] += (p1[t] & 0xFFFFu) + (p1[t] >> 16);
                  p1[t] = 0;
                }
              };
              const uint32_t nql = ABLATE(a, 1) ? 0u : nq;
              // 4 quads per iteration (constant offsets fold into the ds_read
              // offset fields); s2 is flushed to 64 bits every s2_flush quads
              // (XK: 2 quads per iteration; its 4 tables' temporaries of 4
              // unrolled quads spill)
              constexpr uint32_t U = XK ? 2u : GROUP_UNROLL;
              static_assert(U % 2 == 0, "quads are read in 16-B pairs");
              auto clients = [&](auto lines_c) {
                const uint32_t fU = a.g_flush / U ? a.g_flush / U : 1u;
                uint32_t g = 0, k = 0;
                if (a.g_flush >= U) {
                  for (; g + U <= nql; g += U) {
#pragma unroll
                    for (uint32_t u = 0; u < U; u += 2) quad2(lines_c, g * 8 + 8 * u);  // (g, U even: 16-B aligned)
                    if (++k == fU) {
                      flush();
                      k = 0;
                    }
                  }
                  flush();
                }
                for (uint32_t g0 = g; g0 < nql; g0 += a.g_flush) {
                  const uint32_t ge = min(nql, g0 + a.g_flush);
                  for (g = g0; g < ge; ++g) quad(lines_c, g * 8, ~0u, ~0u);
                  flush();
                }
                if (rem && !ABLATE(a, 1)) {
                  quad(lines_c, nq * 8, rem >= 2 ? ~0u : 0x0000FFFFu, rem == 3 ? 0x0000FFFFu : 0u);
                  flush();
                }
              };
              if constexpr (BIN) {
                // ---- BIN: the clients binned by nearest member (binned_clients,
                //      above), so the loop does not depend on the number of
                //      tables (4 with the extended keys).  Per table t, exactly,
                //        S1_t = L1 + sum_m cnt_m q_t[m],
                //        S2_t = L2 + 2 sum_m D1_m q_t[m] + sum_m cnt_m q_t[m]^2
                //      (L1 = sum of latencies = sum_m D1_m, L2 = sum of squares).
                //      The host runs this only where the fields cannot overflow
                //      (nc < 256, nc (16 max + 15) < 2^24; bote_capi.hip).
                uint64_t L2;
                if constexpr (BIN_FIRST) L2 = L2first;  // (the loop ran before the Q phase)
                else if (use_lines) L2 = binned_clients(BoolC<true>{}, c0, c1, c2);
                else L2 = binned_clients(BoolC<false>{}, c0, c1, c2);
                // the bins (re-zeroed for the next config of this lane), in
                // packed member pairs laid out as the tables' words wp[t][i]
                // (members (0, 1), 2, (3, 4), (5, 6) at n = 7; (0, 1), (2, 5),
                // (3, 4) at n = 6, PAIR2; a lone member's high half is
                // don't-care: its table word's high half is 0), so
                // each table's sums are one v_dot2 per word.  The host admits
                // the bins only where nc max < 2^16 (bote_capi.hip), so every
                // count, every D1_m and every cnt_m q product fits a u16.
                constexpr int NW = NWB;
                // the members of word i (low, high; -1: none), as in wp[t][i]
                auto wlo = [](int i) { return i == 0 ? 0 : (i == 1 ? 2 : 3 + 2 * (i - 2)); };
                auto whi = [](int i) {
                  return i == 0 ? 1 : (i == 1 ? (PAIR2 ? N - 1 : -1) : (4 + 2 * (i - 2) < N ? 4 + 2 * (i - 2) : -1));
                };
                uint32_t wv[N], hv[N];  // bin words; (K_m - m cnt_m) >> 4 = D1_m | cnt_m << 20
#pragma unroll
                for (int m = 0; m < N; ++m) {
                  wv[m] = l32(binb + 256u * m);
                  s32(binb + 256u * m, 0u);
                  hv[m] = (m ? wv[m] - (uint32_t)m * (wv[m] >> 24) : wv[m]) >> 4;
                }
                uint32_t cW[NW], dW[NW];  // (cnt_m | cnt_m' << 16), (D1_m | D1_m' << 16)
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                  const int ml = wlo(i), mh = whi(i);
                  if (mh >= 0) {
                    cW[i] = __builtin_amdgcn_perm(wv[mh], wv[ml], 0x0C070C03u);
                    dW[i] = __builtin_amdgcn_perm(hv[mh], hv[ml], 0x05040100u);
                  } else {
                    cW[i] = wv[ml] >> 24;
                    dW[i] = hv[ml];
                  }
                }
                // L1 = sum_m D1_m; corr = 32 sum_m m D1_m + sum_m m^2 cnt_m
                // (per word constant pairs; a lone member's high weight 0)
                uint32_t L1 = 0, corr = 0;
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                  const int ml = wlo(i), mh = whi(i);
                  const uint32_t one = mh >= 0 ? 0x00010001u : 1u;
                  const uint32_t k32 = (uint32_t)(32 * ml) | (mh >= 0 ? (uint32_t)(32 * mh) << 16 : 0u);
                  const uint32_t kmm = (uint32_t)(ml * ml) | (mh >= 0 ? (uint32_t)(mh * mh) << 16 : 0u);
                  L1 = __builtin_amdgcn_udot2(as_us2(dW[i]), as_us2(one), L1, false);
                  corr = __builtin_amdgcn_udot2(as_us2(dW[i]), as_us2(k32), corr, false);
                  corr = __builtin_amdgcn_udot2(as_us2(cW[i]), as_us2(kmm), corr, false);
                }
                L2 = (L2 - corr) >> 8;  // exact: the sum of squared keys is 256 L2 + corr
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                  // S1 = L1 + sum cnt q;  S2 = L2 + 2 sum D1 q + sum (cnt q) q
                  uint32_t s1 = L1, x = 0, qq = 0;
#pragma unroll
                  for (int i = 0; i < NW; ++i) {
                    const us2 q = as_us2(wp[t][i]);
                    s1 = __builtin_amdgcn_udot2(as_us2(cW[i]), q, s1, false);
                    x = __builtin_amdgcn_udot2(as_us2(dW[i]), q, x, false);
                    const us2 cq = as_us2(cW[i]) * q;  // (v_pk_mul_lo_u16: cnt q < 2^16)
                    qq = __builtin_amdgcn_udot2(cq, q, qq, false);
                  }
                  S1[t] = s1;
                  S2[t] = L2 + ((uint64_t)x << 1) + qq;
                  if constexpr (S32) S2[t] = (uint32_t)S2[t];  // (< 2^32: FastArgs::s32)
                }
              } else {
                if (PERM && use_lines) clients(BoolC<PERM>{});
                else clients(BoolC<false>{});
              }
              if (ABLATE(a, 1)) {  // timing only: non-degenerate dummy sums
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                  S1[t] = 1000u + rv[0] + t;
                  S2[t] = (uint64_t)S1[t] * S1[t] + 12345u;
                }
              }
              mom[SLOT_AF1] = Mom{S1[QC::idx_a1], S2[QC::idx_a1], nc};
              mom[SLOT_AF2] = Mom{S1[QC::idx_a2], S2[QC::idx_a2], nc};
              mom[SLOT_E] = Mom{S1[QC::idx_e], S2[QC::idx_e], nc};
              if constexpr (XK) {
                // Tempo tiny (2f) and write (f + 1) quorums, Input: slots 10..13
                constexpr int t2 = QT::idx(2), t3 = QT::idx(3), t4 = QT::idx(4);
                xslot(10, S1[t2], S2[t2]);  // tt1
                xslot(11, S1[t4], S2[t4]);  // tt2
                xslot(12, S1[t2], S2[t2]);  // tw1
                xslot(13, S1[t3], S2[t3]);  // tw2
                x_tt1 = S1[t2];
                x_tw2 = S1[t3];
              }
            }
            // ---- Input FPaxos from the leader column's sums
            const uint32_t lc1 = lrec[lpos].x;
            if constexpr (S32) {
              // sum (L + q) and sum (L + q)^2 = c2 + q (c1 + S1), in 32 bits,
              // with 24-bit multiplies (FastArgs::s32: c1 + S1 <= 3 nc max < 2^24)
              const uint32_t lc2 = (uint32_t)cs2[lpos];
              const uint32_t m2 = __umul24(nc, lq2) + lc1, m3 = __umul24(nc, lq3) + lc1;
              mom[SLOT_FF1] = Mom{m2, __umul24(lq2, lc1 + m2) + lc2, nc};
              mom[SLOT_FF2] = Mom{m3, __umul24(lq3, lc1 + m3) + lc2, nc};
            } else {
              const uint64_t lc2 = cs2[lpos];
              mom[SLOT_FF1] = leader_mom(lc1, lc2, nc, lq2);
              mom[SLOT_FF2] = leader_mom(lc1, lc2, nc, lq3);
            }
            // ---- Colocated: FPaxos reads the leader's column of the config
            //      submatrix; leaderless values are the members' own quorums
            {
              const uint32_t lcol = __umul24(lreg, rstride) + rqt;
              // sum_k (v_k + q) and sum_k (v_k + q)^2 from sum v and sum v^2
              uint32_t sv = 0, sv2 = 0;
              int k0 = 0;
              if (use_rx) {
                // the fixed members' part from the column words of the
                // leader's position-table row (packed u16 pairs: v_dot2; the
                // pad halves past F are INF and masked off), then the three
                // variable members' distances
                const uint2 cw = l64(rxt + 16 * lpos + 8);
                const uint32_t w0 = F >= 2 ? cw.x : (cw.x & 0xFFFFu), w1 = F >= 4 ? cw.y : (cw.y & 0xFFFFu);
                sv = __builtin_amdgcn_udot2(as_us2(w0), as_us2(0x00010001u), 0u, false);
                sv2 = __builtin_amdgcn_udot2(as_us2(w0), as_us2(w0), 0u, false);
                if constexpr (F >= 3) {
                  sv = __builtin_amdgcn_udot2(as_us2(w1), as_us2(0x00010001u), sv, false);
                  sv2 = __builtin_amdgcn_udot2(as_us2(w1), as_us2(w1), sv2, false);
                }
                k0 = 3;
              }
#pragma unroll
              for (int k = 0; k < N; ++k) {
                if (ABLATE(a, 512)) break;
                if (k >= 3 && k0 == 3) break;
                const uint32_t v = l16(lcol + 2 * reg_of(k)) >> LAT_SHIFT;
                sv += v;
                sv2 += v * v;
              }
              const uint32_t f1 = sv + N * lq2, f2 = sv + N * lq3;
              const uint32_t f1s = sv2 + 2 * lq2 * sv + N * lq2 * lq2, f2s = sv2 + 2 * lq3 * sv + N * lq3 * lq3;
              mom[5 + SLOT_FF1] = Mom{f1, f1s, (uint32_t)N};
              mom[5 + SLOT_FF2] = Mom{f2, f2s, (uint32_t)N};
              uint32_t cl1[NT > 3 ? NT : 3];
              if constexpr (PERM) {
#pragma unroll
                for (int t = 0; t < NT; ++t) cl1[t] = cS1t[t];
              } else {
                cl1[0] = cS1p & 0xFFFFu;
                cl1[1] = cS1p >> 16;
                cl1[2] = cS1e;
              }
              mom[5 + SLOT_AF1] = Mom{cl1[QC::idx_a1], cS2[QC::idx_a1], (uint32_t)N};
              mom[5 + SLOT_AF2] = Mom{cl1[QC::idx_a2], cS2[QC::idx_a2], (uint32_t)N};
              mom[5 + SLOT_E] = Mom{cl1[QC::idx_e], cS2[QC::idx_e], (uint32_t)N};
            }
            // the leader column's V: f32 for the screens (0 exactly when V is),
            // the exact f64 read only inside a screen's ambiguity band
            const float vlead32 = vcol32[lpos];
            // af1's exact V (leaderless sums S1 < 2^21, so one 32x32 square),
            // shared by the validity test and the COV-af1 objective screen
            auto mom_v32 = [](const Mom& m) {
              const uint32_t s1 = (uint32_t)m.s1;
              return (uint64_t)m.cnt * m.s2 - (uint64_t)s1 * s1;
            };
            // V and its f32 value; on the S32 kernels every V = cnt s2 - s1^2
            // fits 32 bits (the host admits them only with FastArgs::v32), so
            // 32-bit products give it exactly (mod 2^32)
            auto vmom = [&](const Mom& m, uint64_t& V, float& vf) {
              if constexpr (S32) {
                const uint32_t v = m.cnt * (uint32_t)m.s2 - (uint32_t)m.s1 * (uint32_t)m.s1;
                V = v;
                vf = (float)v;
              } else {
                V = mom_v32(m);
                vf = u64_to_f32(V);
              }
            };
            uint64_t Va1;
            float va1;
            vmom(mom[SLOT_AF1], Va1, va1);
            if constexpr (DEF) {
              // ---- compute_score validity (search.rs:421-472), exact.  The
              //      integer mean tests of every f first; the COV tests only
              //      for configs that pass them, and a config is deferred
              //      only when its validity hinges on an ambiguous COV call.
              bool valid = false;
              const int fcap = min(N / 2, SI ? 2 : a.ft_metric);
              bool defer = false;
              if (!ABLATE(a, 256)) {  // (the default objectives imply want_score)
                valid = true;
#pragma unroll
                for (int f = 1; f <= 2; ++f) {
                  if (f > fcap) break;
                  const Mom& ma = mom[f == 1 ? SLOT_AF1 : SLOT_AF2];
                  const Mom& mf = mom[f == 1 ? SLOT_FF1 : SLOT_FF2];
                  // fmi >= p1: decided on the integer difference outside
                  // [m1_lo, m1_hi], by the reference's f64 arithmetic inside
                  const int32_t D = (int32_t)((uint32_t)mf.s1 - (uint32_t)ma.s1);
                  const int32_t m1lo = a.m1_lo, m1hi = a.m1_hi;
                  bool mok = D > m1hi;
                  PSTAT(a, 4 + f - 1, D >= m1lo && D <= m1hi);  // f64 mean test (f = 1, 2)
                  if (D >= m1lo && D <= m1hi) mok = (mom_mean(mf) - mom_mean(ma)) >= a.p_fmean;
                  valid = valid && mok;
                  if (N == 11 || N == 13) {
                    const int32_t De = (int32_t)((uint32_t)mom[SLOT_E].s1 - (uint32_t)ma.s1);
                    bool eok = De > a.m2_hi;
                    if (De >= a.m2_lo && De <= a.m2_hi) eok = (mom_mean(mom[SLOT_E]) - mom_mean(ma)) >= a.p_emean;
                    valid = valid && eok;
                  }
                }
                PSTAT(a, 6, valid);  // COV validity tests
                if (valid) {
                  // cov_f >= cov_a (min_fairness_fpaxos_improv == 0 on this path):
                  // cross-multiplied f32 screen, then f64 (cov2_sign)
                  bool lt = false, amb_c = false;
#pragma unroll
                  for (int f = 1; f <= 2; ++f) {
                    if (f > fcap) break;
                    const Mom& ma = mom[f == 1 ? SLOT_AF1 : SLOT_AF2];
                    const Mom& mf = mom[f == 1 ? SLOT_FF1 : SLOT_FF2];
                    uint64_t Va = Va1;
                    float vaf = va1;
                    if (f != 1) vmom(ma, Va, vaf);
                    const int c = cov2_sign_ge(vlead32, (uint32_t)mf.s1, vaf, (uint32_t)ma.s1, [&] { return vcol[lpos]; },
                                            [&] { return (double)Va; });
                    lt = lt || c < 0;
                    amb_c = amb_c || c == 0;
                  }
                  valid = !lt && !amb_c;
                  defer = !lt && amb_c;
                }
              }
              PSTAT(a, 8, defer);  // validity deferred
              if (defer) {
                if (!a.smin) defer_rank(a, rank);
              } else {
                vflag = valid;
                if ((SI || a.want_digest) && !ABLATE(a, 16)) {
                  uint32_t h = hx;  // (0 without XK)
#pragma unroll
                  for (int sl = 0; sl < NSLOT; ++sl) h = digest_fold(h, sl, mom[sl].s1, mom[sl].s2);
                  digest_add(binb, digest_final(rank, bi, h));
                }
                // ---- default objectives: 0 SCORE, 1 MEAN af1, 2 MEAN ff1, 3 COV af1, 4 MEAN e
                if (ABLATE(a, 2048)) valid = false;
                ok[1] = ok[2] = ok[4] = true;
                key[1] = mom[SLOT_AF1].s1;
                key[2] = mom[SLOT_FF1].s1;
                key[4] = mom[SLOT_E].s1;
                if constexpr (XK) {  // 5 MEAN tt1, 6 MEAN tw2, 7 MEAN fl1
                  ok[5] = ok[6] = ok[7] = true;
                  key[5] = x_tt1;
                  key[6] = x_tw2;
                  key[7] = x_fl1;
                }
                if (valid) {
                  // (32-bit: every S1 here is below 2^21, so |T| < 2^27)
                  int32_t T = 0;
#pragma unroll
                  for (int f = 1; f <= 2; ++f) {
                    if (f > fcap) break;
                    const int32_t a1 = (int32_t)(uint32_t)mom[f == 1 ? SLOT_AF1 : SLOT_AF2].s1;
                    T += (int32_t)(uint32_t)mom[f == 1 ? SLOT_FF1 : SLOT_FF2].s1 - a1 +
                         30 * ((int32_t)(uint32_t)mom[SLOT_E].s1 - a1);
                  }
                  const bool maybe = T >= *(volatile int*)(lock + 1);  // (score_tlo)
                  PSTAT(a, 9, maybe);  // f64 score
                  if (maybe) {
                    double score = 0.0;
                    const double me = mom_mean(mom[SLOT_E]);
#pragma unroll
                    for (int f = 1; f <= 2; ++f) {
                      if (f > fcap) break;
                      const double mA = mom_mean(mom[f == 1 ? SLOT_AF1 : SLOT_AF2]);
                      const double fmi = mom_mean(mom[f == 1 ? SLOT_FF1 : SLOT_FF2]) - mA;
                      const double emi = me - mA;
                      double t = 30.0 * emi;
                      t = fmi + t;
                      score = score + t;
                    }
                    ok[0] = true;
                    key[0] = ~orderable_f64(score);
                  }
                }
                {
                  const Mom& m = mom[SLOT_AF1];
                  // f32 screen with a 2^-10 margin (conservative: offers a
                  // superset): V / S^2 <= the threshold key's V / S^2,
                  // cross-multiplied, the threshold's f32 bound from LDS
                  // (cov_tf32; +inf, or a NaN key: every config passes)
                  const float S = (float)(uint32_t)m.s1;
                  const bool maybe = !(va1 > __int_as_float(*(volatile int*)(lock + 2)) * (S * S));
                  PSTAT(a, 10, maybe);  // COV af1 key (f64)
                  if (maybe) {
                    ok[3] = true;
                    key[3] = cov_key(m);
                  }
                }
              }
            } else {
              uint64_t vc = 0, dg = 0;  // (this config's: finish_config adds to them)
              if (!finish_config<N>(a, mom, vcol[lpos], bi, rank, tk.thr, pnc1, pnc2, vc, dg, key, ok) && !a.smin)
                defer_rank(a, rank);
              vflag = vc != 0;
              if (dg) digest_add(binb, dg);
            }
          }
        }
        valid_cnt += (uint64_t)__popcll(__ballot(vflag));  // (every lane active here: a uniform count)
        // ---- top-K: lock-free screen, exact merge under the block lock
        if (a.smin) {
          // sample launch: per objective the least key of this chunk's configs
          const int nobj = XK ? 8 : (DEF ? 5 : a.n_obj);
#pragma unroll
          for (int o = 0; o < MAXOBJ; ++o) {
            if (o >= nobj) break;
            uint64_t v = ok[o] ? key[o] : ~0ull;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
              const uint64_t w = ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), d) << 32) |
                                 (uint32_t)__shfl_xor((int)(uint32_t)v, d);
              v = w < v ? w : v;
            }
            uint32_t ch = uni(chunk);
            // (an opaque copy: the compiler hoisted these 8 slot addresses out
            // of the step loop into the chunk head, where the register-bound
            // XK kernel spilled them -- 4 KB of scratch writes per chunk of the
            // sweep launch, which never takes this branch: most of config 5's
            // 7.5e8 B of WRITE_SIZE per launch, r06d)
            asm volatile("" : "+s"(ch));
            const size_t slot = a.smin_wave ? (size_t)o * gridDim.x * WPB + (size_t)blockIdx.x * WPB + wid
                                            : (size_t)o * a.nwchunks + ch;
            if (lane == (a.smin_wave ? (uint32_t)o : 0u) && v != ~0ull)
              atomicMin((unsigned long long*)&a.smin[slot], v);
          }
        } else if (!ABLATE(a, 4)) {
          const int nobj = XK ? 8 : (DEF ? 5 : a.n_obj);
          // (the thresholds read first, from one LDS address with immediate
          // offsets: read under the short-circuit test, each cost a spilled
          // SGPR reload and an address move)
          uint64_t th[MAXOBJ];
#pragma unroll
          for (int o = 0; o < MAXOBJ; ++o)
            if (o < nobj) {
              const uint2 t = l64(thra + 16u * o);
              th[o] = ((uint64_t)t.y << 32) | t.x;
            }
          bool pass = false;
#pragma unroll
          for (int o = 0; o < MAXOBJ; ++o)
            if (o < nobj) pass = pass || (ok[o] && key[o] <= th[o]);
          PSTAT(a, 11, pass);  // block top-K merge
          if (__ballot(pass)) wave_topk(tk, lock, a.nc, nobj, a.K, key, ok, rank);
        }
        r += len;
        left -= len;
      }
      // (a sample chunk stops at its first group's end: any subset of the
      // range bounds its K-th key, and a sample across many small groups,
      // as at rank 0, cost one precompute each: the launch's slowest wave)
      if (r >= rend || a.smin) break;
      // ---------------- next group: colex successor of the fixed positions
      // (a combination of {3 .. ns-1}; the smallest fixed position is >= 3)
      {
        int js = F;
#pragma unroll
        for (int k = F - 1; k >= 0; --k) {
          const uint32_t nxt = (k == F - 1) ? a.ns : hq[k + 1];
          if (hq[k] + 1 < nxt) js = k;
        }
        base = 0;
#pragma unroll
        for (int k = 0; k < F; ++k) {
          hq[k] = uni(k < js ? (uint32_t)(3 + k) : (k == js ? hq[k] + 1 : hq[k]));
          base += binom[hq[k] * (N + 1) + (k + 4)];
        }
        base = uni64(base);
        low = 0;
      }
      wave_sync();  // the group line is rewritten next
    }
  }
  wave_sync();  // (the next chunk rewrites the group line)
  }
  if (a.smin) return;  // (the sample launch: no counters, no lists; no barrier follows)
  if (valid_cnt && lane == 0) atomicAdd(&a.out_counters[0], (unsigned long long)valid_cnt);  // (uniform)
  const uint64_t digest = *(const AS3 uint64_t*)(uintptr_t)(LB + (uint32_t)off[15] + tid * 8);
  if (digest) atomicAdd(&a.out_counters[1], (unsigned long long)digest);
  __syncthreads();
  Rec* dst = a.out_top + (size_t)blockIdx.x * a.n_obj * KP;
  if (a.kbound) {
    // the one-launch merge follows: publish this list's K-th key (a bound on
    // the union's K-th key), then write only the records within the least
    // bound seen so far and a terminator (tk.thr is free now: its key holds
    // the bound).  The terminator/padding is (~0, ~0): a real record may
    // have key ~0 (a NaN COV key, cov_key) but its rank is < C(R, n) < 2^64
    // - 1, so the two never match, and a ~0 key is written only when no
    // bound is known (b == ~0)
    if (tid < a.n_obj) {
      const Rec kth = tk.top[tid * a.K + a.K - 1];
      uint64_t b = ~0ull;
      if (!(kth.key == ~0ull && kth.rank == ~0ull)) {
        b = atomicMin(&a.kbound[tid], (unsigned long long)kth.key);  // (vector atomic)
        b = b < kth.key ? b : kth.key;
      } else {
        b = __hip_atomic_load(&a.kbound[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      tk.thr[tid].key = b;
    }
    __syncthreads();
    for (uint32_t i = tid; i < (uint32_t)a.n_obj * a.K; i += BD) {
      const uint32_t o = i / a.K, e = i % a.K;
      const uint64_t b = tk.thr[o].key;
      const Rec r = tk.top[i];
      const bool in = !(r.key == ~0ull && r.rank == ~0ull) && r.key <= b;
      bool prev = true;
      if (e) {
        const Rec q = tk.top[i - 1];
        prev = !(q.key == ~0ull && q.rank == ~0ull) && q.key <= b;
      }
      if (in) dst[o * KP + e] = r;
      else if (prev) dst[o * KP + e] = rec_max();  // the terminator
    }
    return;
  }
  for (uint32_t i = tid; i < (uint32_t)a.n_obj * KP; i += BD) {
    const uint32_t o = i / KP, e = i % KP;
    dst[i] = e < a.K ? tk.top[o * a.K + e] : rec_max();
  }
}

// ------------------------------------------------------------- launcher ---
template <int N, bool DEF, bool SI, bool RXC, bool XK, bool BN = false>
static hipError_t launch_group_n(const FastArgs& a, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0,
                                 hipEvent_t e1) {
  auto k = sweep_group_kernel<N, DEF, SI, RXC, XK, BN>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (e != hipSuccess) return e;
  // (timed launches carry their events in the dispatch: no marker packets
  // before and after the kernel, which cost ~10 us of idle GPU each)
  if (e0) hipExtLaunchKernelGGL(k, dim3(grid), dim3(a.gbd), (uint32_t)shm, st, e0, e1, 0u, a);
  else hipLaunchKernelGGL(k, dim3(grid), dim3(a.gbd), shm, st, a);
  return hipGetLastError();
}

// The instantiation launch_group runs for these arguments (its occupancy
// decides the persistent grid, so it must be the kernel that runs).
// (S32 kernels also take every V in 32 bits: FastArgs::v32)
static bool group_si(const FastArgs& a) { return a.srv_identity && a.want_digest && a.ft_metric == 2 && a.s32 && a.v32; }

// the extended key set: PERM kernels (n = 4..7) with the default objectives
bool group_supports_keys(uint32_t n, uint32_t bd) { return n >= 4 && n <= 7 && group_uses_lines(n) && bd <= GROUP_XK_MAX_BD; }

template <int N, bool XK>
static const void* group_fn_n(const FastArgs& a, bool def) {
  if constexpr (XK) {
    return group_si(a) ? (a.grx ? (const void*)sweep_group_kernel<N, true, true, true, true>
                                : (const void*)sweep_group_kernel<N, true, true, false, true>)
                       : (const void*)sweep_group_kernel<N, true, false, false, true>;
  } else {
    if (def && group_si(a) && a.gbins)
      return a.grx ? (const void*)sweep_group_kernel<N, true, true, true, false, true>
                   : (const void*)sweep_group_kernel<N, true, true, false, false, true>;
    return def ? (group_si(a) ? (a.grx ? (const void*)sweep_group_kernel<N, true, true, true, false>
                                       : (const void*)sweep_group_kernel<N, true, true, false, false>)
                              : (const void*)sweep_group_kernel<N, true, false, false, false>)
               : (const void*)sweep_group_kernel<N, false, false, false, false>;
  }
}

template <int N, bool XK>
static hipError_t launch_group_x(const FastArgs& a, bool def, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0,
                                 hipEvent_t e1) {
  if constexpr (XK) {
    return group_si(a) ? (a.grx ? launch_group_n<N, true, true, true, true>(a, grid, shm, st, e0, e1)
                                : launch_group_n<N, true, true, false, true>(a, grid, shm, st, e0, e1))
                       : launch_group_n<N, true, false, false, true>(a, grid, shm, st, e0, e1);
  } else {
    if (def && group_si(a) && a.gbins)
      return a.grx ? launch_group_n<N, true, true, true, false, true>(a, grid, shm, st, e0, e1)
                   : launch_group_n<N, true, true, false, false, true>(a, grid, shm, st, e0, e1);
    return def ? (group_si(a) ? (a.grx ? launch_group_n<N, true, true, true, false>(a, grid, shm, st, e0, e1)
                                       : launch_group_n<N, true, true, false, false>(a, grid, shm, st, e0, e1))
                              : launch_group_n<N, true, false, false, false>(a, grid, shm, st, e0, e1))
               : launch_group_n<N, false, false, false, false>(a, grid, shm, st, e0, e1);
  }
}

static const void* group_fn(const FastArgs& a, uint32_t n, bool def) {
  switch (n) {
#define FN_CASE(NN) case NN: return a.keys ? group_fn_n<NN, true>(a, def) : group_fn_n<NN, false>(a, def);
#define FN_CASE0(NN) case NN: return a.keys ? nullptr : group_fn_n<NN, false>(a, def);
#ifdef BOTE_ISA_N7
    FN_CASE(7)
#elif defined(BOTE_ISA_N6)
    FN_CASE(6)
#elif defined(BOTE_ISA_N5)
    FN_CASE(5)
#else
    FN_CASE(4) FN_CASE(5) FN_CASE(6) FN_CASE(7) FN_CASE0(8) FN_CASE0(9) FN_CASE0(10) FN_CASE0(11) FN_CASE0(12)
    FN_CASE0(13) FN_CASE0(14) FN_CASE0(15) FN_CASE0(16)
#endif
#undef FN_CASE
#undef FN_CASE0
    default: return nullptr;
  }
}

int group_occupancy(const FastArgs& a, uint32_t n, size_t shm, bool def) {
  int nb = 0;
  const void* k = group_fn(a, n, def);
  if (!k) return 0;
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, (int)a.gbd, shm) != hipSuccess) return 0;
  return nb > 0 ? nb : 0;
}

hipError_t launch_group(const FastArgs& a, uint32_t n, bool def, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0,
                        hipEvent_t e1) {
  switch (n) {
#define GS_CASE(NN) \
  case NN: return a.keys ? launch_group_x<NN, true>(a, def, grid, shm, st, e0, e1) : launch_group_x<NN, false>(a, def, grid, shm, st, e0, e1);
#define GS_CASE0(NN) \
  case NN: return a.keys ? hipErrorInvalidValue : launch_group_x<NN, false>(a, def, grid, shm, st, e0, e1);
#ifdef BOTE_ISA_N7  // (analysis builds only: the n = 7 kernels, for assembly listings)
    GS_CASE(7)
#elif defined(BOTE_ISA_N6)  // (the n = 6 kernels: BASELINE config 5)
    GS_CASE(6)
#elif defined(BOTE_ISA_N5)
    GS_CASE(5)
#else
    GS_CASE(4) GS_CASE(5) GS_CASE(6) GS_CASE(7) GS_CASE0(8) GS_CASE0(9) GS_CASE0(10) GS_CASE0(11) GS_CASE0(12)
    GS_CASE0(13) GS_CASE0(14) GS_CASE0(15) GS_CASE0(16)
#endif
#undef GS_CASE
#undef GS_CASE0
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bote
