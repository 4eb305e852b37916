// bote_sweep.hip — the fast-path sweep kernel (gfx950): exhaustive search over
// colex ranks with a block top-K, for planets that meet the fast-path
// preconditions checked on the host (bote_capi.hip, fast_eligible):
//   * every latency <= 4095 (packed u16 keys: latency << 4 | member)
//   * the server set is "simple": self latency 0, latency between two servers
//     > 0 (a colocated client's nearest server is itself)
//   * servers in name order, >= 2 clients, min_fairness_fpaxos_improv == 0
// Anything else runs the generic kernel (bote_kernels.hip), which is also the
// exact path for the rare configs this kernel defers (COV near-ties).
//
// Data layout in LDS (DESIGN.md "Data layout"):
//   CQT[t][g]  uint2 = 4 x u16 (latency << 4) from clients 4g..4g+3 to region
//              t; column stride (nq + 1) * 8 bytes, an odd number of 8-byte
//              slots, so distinct columns spread over the ds_read_b64 banks.
//   RQT        the same layout with ALL regions as the rows (== CQT when the
//              client list is 0..R-1): L[a][b] = RQT[b][a >> 2].u16[a & 3].
//   qtab       per lane and member: packed leaderless quorum latencies,
//              plane-major [member][lane] (conflict-free).
//
// Per config (one lane; reference functions in bote_kernels.hip's header):
// quorum latencies by sorting each member's off-diagonal distances; FPaxos
// leader by exact-COV comparison (variance is shift invariant, so leader l's
// V = nc*sum(L^2) - (sum L)^2 of its column, precomputed per position); the
// Input leaderless keys by the packed client-quad loop; compute_score validity
// by integer / f64-margin decisions; digest; block top-K.
#include "bote_fast.hpp"


namespace bote {


constexpr uint32_t QSH = 10;  // log2(FAST_BD * 4): byte stride between qtab member planes
static_assert((1u << QSH) == FAST_BD * 4, "qtab plane stride");

struct FastSmem {
  unsigned char* base;  // dynamic LDS base; byte offsets below are relative to it
  uint32_t cqt, rqt, qtab;
  uint32_t* srv;
  uint32_t* cs1;
  uint64_t* cs2;
  double* vcol;
  uint64_t* binom;
  TopkLds tk;
};

__host__ __device__ inline size_t fast_layout(const FastArgs& a, int N, int NLW, size_t* off) {
  size_t o = 0;
  off[0] = o; o += (size_t)N * FAST_BD * NLW * 4;  // qtab first: offsets stay small
  off[1] = o; o += (size_t)a.R * a.cq_stride * 8;
  off[2] = o; o += a.rq_separate ? (size_t)a.R * a.rq_stride * 8 : 0;
  off[3] = o; o += (size_t)a.ns * 4;  // srv
  off[4] = o; o += (size_t)a.ns * 4;  // cs1
  o = (o + 15) & ~(size_t)15;
  off[5] = o; o += (size_t)a.ns * 8;                   // cs2
  off[6] = o; o += (size_t)a.ns * 8;                   // vcol
  off[7] = o; o += (size_t)(a.ns + 1) * (N + 1) * 8;  // binom
  o = (o + 15) & ~(size_t)15;
  off[8] = o; o += (size_t)a.n_obj * KP * 16;  // top
  off[9] = o; o += (size_t)FAST_BD * 16;      // cand
  off[10] = o; o += (size_t)KP * 16;          // tmp
  off[11] = o; o += (size_t)MAXOBJ * 16;      // thr
  off[12] = o; o += 48;                       // cnt[1 + MAXOBJ]
  return o;
}

size_t fast_smem_bytes(const FastArgs& a, uint32_t n) {
  size_t off[13];
  int nl = 0;
  switch (n) {
#define NL_CASE(NN) case NN: nl = QCfg<NN>::NL; break;
    NL_CASE(2) NL_CASE(3) NL_CASE(4) NL_CASE(5) NL_CASE(6) NL_CASE(7) NL_CASE(8) NL_CASE(9)
    NL_CASE(10) NL_CASE(11) NL_CASE(12) NL_CASE(13) NL_CASE(14) NL_CASE(15) NL_CASE(16)
#undef NL_CASE
    default: return 0;
  }
  return fast_layout(a, (int)n, nl <= 2 ? 1 : 2, off);
}

template <int N>
__device__ __forceinline__ uint32_t sel_u(const uint32_t (&arr)[N], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) r |= arr[j] & (0u - (uint32_t)(i == (uint32_t)j));
  return r;
}


// ------------------------------------------------------------ hot loop ----
// Input leaderless keys over client quads.  Per quad and member: one
// ds_read_b64 (4 clients), a packed OR of the member index and a packed min
// (v_pk_min_u16: ties go to the lower member = the lower name); per client:
// one qtab read for the nearest member's quorum latencies; packed adds and
// v_dot2_u32_u16 accumulate the sum and the sum of squares.  Squares are
// accumulated in 32 bits and flushed to 64 bits every `flushQ` quads.
template <int N, int NL>
__device__ __forceinline__ void client_quads(const unsigned char* B, uint32_t cqt, uint32_t nq, uint32_t rem,
                                             uint32_t flushQ, const uint32_t (&colT)[N], uint32_t qlane,
                                             uint32_t (&S1)[NL], uint64_t (&S2)[NL]) {
  const us2 ones = {1, 1};
  constexpr int NQ = NL == 3 ? 8 : 4;  // qtab words per quad
  uint32_t s2[NL];
#pragma unroll
  for (int t = 0; t < NL; ++t) {
    S1[t] = 0;
    S2[t] = 0;
    s2[t] = 0;
  }
  uint32_t col[N];
#pragma unroll
  for (int j = 0; j < N; ++j) col[j] = cqt + colT[j];

  // stage 1: the quad's N member columns
  auto load = [&](uint32_t g8, uint2 (&w)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) w[j] = ld64(B, col[j] + g8);
  };
  // stage 2: nearest member per client (packed min of latency<<4 | member)
  auto nearest = [&](const uint2 (&w)[N], us2& lo, us2& hi) {
    lo = as_us2(w[0].x);
    hi = as_us2(w[0].y);
#pragma unroll
    for (int j = 1; j < N; ++j) {
      const us2 J = {(unsigned short)j, (unsigned short)j};
      lo = __builtin_elementwise_min(lo, as_us2(w[j].x) | J);
      hi = __builtin_elementwise_min(hi, as_us2(w[j].y) | J);
    }
  };
  // stage 3a: the nearest members' quorum latencies (qtab sits at LDS offset
  // 0, so qlane < 2^QSH and the member plane offset can be OR-ed in)
  auto qread = [&](us2 lo, us2 hi, uint32_t (&q)[NQ]) {
    constexpr uint32_t QM = 15u << QSH;
    const uint32_t L = as_u32(lo), H = as_u32(hi);
    q[0] = ld32(B, ((L << QSH) & QM) | qlane);
    q[1] = ld32(B, ((L >> (16 - QSH)) & QM) | qlane);
    q[2] = ld32(B, ((H << QSH) & QM) | qlane);
    q[3] = ld32(B, ((H >> (16 - QSH)) & QM) | qlane);
    if (NL == 3) {
      const uint32_t P2 = (uint32_t)N << QSH;  // second plane follows the first
      q[NQ - 4] = ld32(B, qlane + P2 + ((L & 15u) << QSH));
      q[NQ - 3] = ld32(B, qlane + P2 + (((L >> 16) & 15u) << QSH));
      q[NQ - 2] = ld32(B, qlane + P2 + ((H & 15u) << QSH));
      q[NQ - 1] = ld32(B, qlane + P2 + (((H >> 16) & 15u) << QSH));
    }
  };
  // stage 3b: client latency = distance + quorum latency; S1 and S2 by dot2
  auto acc1 = [&](int t, us2 dlo, us2 dhi, uint32_t ql01, uint32_t ql23, uint32_t mlo, uint32_t mhi) {
    us2 a01 = dlo + as_us2(ql01), a23 = dhi + as_us2(ql23);
    a01 = as_us2(as_u32(a01) & mlo);
    a23 = as_us2(as_u32(a23) & mhi);
    S1[t] = __builtin_amdgcn_udot2(a01, ones, S1[t], false);
    S1[t] = __builtin_amdgcn_udot2(a23, ones, S1[t], false);
    s2[t] = __builtin_amdgcn_udot2(a01, a01, s2[t], false);
    s2[t] = __builtin_amdgcn_udot2(a23, a23, s2[t], false);
  };
  auto accum = [&](us2 lo, us2 hi, const uint32_t (&q)[NQ], uint32_t mlo, uint32_t mhi) {
    const us2 dlo = lo >> (us2)4, dhi = hi >> (us2)4;
    acc1(0, dlo, dhi, __builtin_amdgcn_perm(q[1], q[0], 0x05040100u), __builtin_amdgcn_perm(q[3], q[2], 0x05040100u),
         mlo, mhi);
    if (NL >= 2)
      acc1(NL >= 2 ? 1 : 0, dlo, dhi, __builtin_amdgcn_perm(q[1], q[0], 0x07060302u),
           __builtin_amdgcn_perm(q[3], q[2], 0x07060302u), mlo, mhi);
    if (NL == 3)
      acc1(NL - 1, dlo, dhi, __builtin_amdgcn_perm(q[NQ - 3], q[NQ - 4], 0x05040100u),
           __builtin_amdgcn_perm(q[NQ - 1], q[NQ - 2], 0x05040100u), mlo, mhi);
  };
  auto quad = [&](uint32_t g8, uint32_t mlo, uint32_t mhi) {
    uint2 w[N];
    uint32_t q[NQ];
    us2 lo, hi;
    load(g8, w);
    nearest(w, lo, hi);
    qread(lo, hi, q);
    accum(lo, hi, q, mlo, mhi);
  };
  auto flush = [&]() {
#pragma unroll
    for (int t = 0; t < NL; ++t) {
      S2[t] += s2[t];
      s2[t] = 0;
    }
  };

  uint32_t g = 0;
  if (N <= 8 && flushQ >= 2) {
    // Software-pipelined pairs: the next pair's 2N column reads (merged
    // into ds_read2_b64) are in flight while this pair's qtab reads and
    // sums run; the scheduling barriers keep the compiler from serialising
    // the reads behind their first use, which it otherwise does to save
    // registers under the 128-VGPR cap.
    const uint32_t np = nq >> 1;
    const uint32_t fp = flushQ >> 1;
    if (np) {
      uint2 wa[N], wb[N];
      load(0, wa);
      load(8, wb);
      uint32_t k = 0;
      for (uint32_t p = 0; p < np; ++p) {
        us2 loA, hiA, loB, hiB;
        nearest(wa, loA, hiA);
        nearest(wb, loB, hiB);
        uint32_t qA[NQ], qB[NQ];
        qread(loA, hiA, qA);
        qread(loB, hiB, qB);
        const uint32_t gn = min(p + 1, np - 1) * 16;
        load(gn, wa);
        load(gn + 8, wb);
        __builtin_amdgcn_sched_barrier(0);
        accum(loA, hiA, qA, ~0u, ~0u);
        accum(loB, hiB, qB, ~0u, ~0u);
        if (++k == fp) {
          flush();
          k = 0;
        }
      }
      flush();
      g = np << 1;
    }
  }
  for (uint32_t g0 = g; g0 < nq; g0 += flushQ) {
    const uint32_t ge = min(nq, g0 + flushQ);
    for (g = g0; g < ge; ++g) quad(g * 8, ~0u, ~0u);
    flush();
  }
  if (rem) {
    const uint32_t mlo = rem >= 2 ? ~0u : 0x0000FFFFu, mhi = rem == 3 ? 0x0000FFFFu : 0u;
    quad(nq * 8, mlo, mhi);
    flush();
  }
}

// ---------------------------------------------------------- the kernel ----
template <int N>
__global__ void __launch_bounds__(FAST_BD, 4) sweep_fast_kernel(FastArgs a) {
  using QC = QCfg<N>;
  constexpr int NL = QC::NL;
  constexpr int NLW = NL <= 2 ? 1 : 2;
  constexpr int P = Pow2<N - 1>::v;  // off-diagonal row values, padded
  extern __shared__ __align__(16) unsigned char smem[];
  size_t off[13];
  fast_layout(a, N, NLW, off);
  FastSmem s;
  s.base = smem;
  s.qtab = (uint32_t)off[0];
  s.cqt = (uint32_t)off[1];
  s.rqt = a.rq_separate ? (uint32_t)off[2] : (uint32_t)off[1];
  s.srv = (uint32_t*)(smem + off[3]);
  s.cs1 = (uint32_t*)(smem + off[4]);
  s.cs2 = (uint64_t*)(smem + off[5]);
  s.vcol = (double*)(smem + off[6]);
  s.binom = (uint64_t*)(smem + off[7]);
  s.tk.top = (Rec*)(smem + off[8]);
  s.tk.cand = (Rec*)(smem + off[9]);
  s.tk.tmp = (Rec*)(smem + off[10]);
  s.tk.thr = (Rec*)(smem + off[11]);
  s.tk.cnt = (int*)(smem + off[12]);
  const uint32_t tid = threadIdx.x;
  const unsigned char* B = smem;

  // ---- stage: quad matrices, server list, binomials; then per-position sums
  {
    const uint32_t cw = a.R * a.cq_stride * 2;  // 32-bit words
    const uint32_t* src = (const uint32_t*)a.cqt;
    uint32_t* dst = (uint32_t*)(smem + s.cqt);
    for (uint32_t i = tid; i < cw; i += FAST_BD) dst[i] = src[i];
    if (a.rq_separate) {
      const uint32_t rw = a.R * a.rq_stride * 2;
      const uint32_t* rs = (const uint32_t*)a.rqt;
      uint32_t* rd = (uint32_t*)(smem + s.rqt);
      for (uint32_t i = tid; i < rw; i += FAST_BD) rd[i] = rs[i];
    }
  }
  for (uint32_t i = tid; i < a.ns; i += FAST_BD) s.srv[i] = a.srv[i];
  for (uint32_t i = tid; i < (a.ns + 1) * (N + 1); i += FAST_BD) s.binom[i] = a.binom[i];
  topk_init(s.tk, a.n_obj);
  __syncthreads();
  const uint32_t cstride = a.cq_stride * 8;  // bytes per CQT column
  const uint32_t rstride = a.rq_stride * 8;
  for (uint32_t i = tid; i < a.ns; i += FAST_BD) {
    const uint32_t col = s.cqt + s.srv[i] * cstride;
    uint64_t c1 = 0, c2 = 0;
    for (uint32_t c = 0; c < a.nc; ++c) {
      uint64_t v = ld16(B, col + (c >> 2) * 8 + (c & 3) * 2) >> LAT_SHIFT;
      c1 += v;
      c2 += v * v;
    }
    s.cs1[i] = (uint32_t)c1;
    s.cs2[i] = c2;
    s.vcol[i] = (double)((uint64_t)a.nc * c2 - c1 * c1);  // exact: < 2^53
  }
  __syncthreads();

  const uint32_t nc = a.nc, nq = nc >> 2, rem = nc & 3;
  const uint32_t qlane = s.qtab + tid * 4;
  const uint64_t total = a.re - a.rb;
  const uint64_t runlen = a.runlen;
  const uint64_t njobs = (total + runlen - 1) / runlen;
  const uint64_t G = (uint64_t)gridDim.x * FAST_BD;
  const uint64_t outer = (njobs + G - 1) / G;
  const double pnc1 = a.p_fmean * (double)nc, pnc2 = a.p_emean * (double)nc;
  uint64_t valid_cnt = 0, digest = 0;

  for (uint64_t it = 0; it < outer; ++it) {
    const uint64_t job = it * G + (uint64_t)blockIdx.x * FAST_BD + tid;
    const bool jobok = job < njobs;
    uint64_t rank = a.rb + job * runlen;
    uint32_t p[N];
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = j;
    if (jobok) colex_unrank<N>(s.binom, a.ns, rank, p);
    for (uint64_t tt = 0; tt < runlen; ++tt) {
      bool have = jobok && rank < a.re;
      uint64_t key[MAXOBJ];
      bool ok[MAXOBJ];
#pragma unroll
      for (int o = 0; o < MAXOBJ; ++o) {
        key[o] = 0;
        ok[o] = false;
      }
      if (have) {
        // ---- members (positions ascending == names ascending)
        uint32_t colT[N], colR[N], rowq[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const uint32_t r = a.srv_identity ? p[j] : s.srv[p[j]];
          colT[j] = r * cstride;
          colR[j] = s.rqt + r * rstride;
          rowq[j] = (r >> 2) * 8 + (r & 3) * 2;
        }
        // ---- Q phase: sorted off-diagonal distances of each member's row
        uint32_t Q2[N], Q3[N];
        uint32_t cS1[NL], cS2[NL];
#pragma unroll
        for (int t = 0; t < NL; ++t) cS1[t] = cS2[t] = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          uint32_t v[P];
          int t = 0;
          if (ABLATE(a, 2)) {
#pragma unroll
            for (int k = 0; k < N; ++k)
              if (k != j) v[t++] = colR[k] + rowq[j] + k;
          } else {
#pragma unroll
            for (int k = 0; k < N; ++k)
              if (k != j) v[t++] = ld16(B, colR[k] + rowq[j]) >> LAT_SHIFT;
          }
#pragma unroll
          for (int k = N - 1; k < P; ++k) v[k] = 0xFFFFFFFFu;
          sort_network<P>(v);
          // the row's q-th smallest (self = 0 first) is the (q-1)-th off-diagonal
          Q2[j] = v[0];
          Q3[j] = QC::maxf >= 2 ? v[QC::maxf >= 2 ? 1 : 0] : 0u;
          uint32_t ql[NL];
#pragma unroll
          for (int t2 = 0; t2 < NL; ++t2) {
            ql[t2] = v[QC::lq(t2) - 2];
            cS1[t2] += ql[t2];
            cS2[t2] += ql[t2] * ql[t2];
          }
          *(uint32_t*)(smem + qlane + ((uint32_t)j << QSH)) = ql[0] | (NL >= 2 ? ql[NL >= 2 ? 1 : 0] << 16 : 0u);
          if (NL == 3) *(uint32_t*)(smem + qlane + ((uint32_t)(N + j) << QSH)) = ql[NL - 1];
          // one member row at a time: keeps the row's reads and sort network
          // from being interleaved with the next rows (register pressure)
          __builtin_amdgcn_sched_barrier(0);
        }
        // ---- FPaxos leader (f = 1, q = 2, min COV, first in config order)
        uint32_t bi = 0;
        bool amb = false;
        // the leader's position, quorum latencies and column, carried along
        uint32_t lp = p[0], lq2 = Q2[0], lq3 = Q3[0], lcol = colR[0];
        {
          uint32_t c1 = s.cs1[p[0]];
          double bS = (double)(c1 + nc * Q2[0]);
          bS = bS * bS;
          double bV = s.vcol[p[0]];
#pragma unroll
          for (int l = 1; l < N; ++l) {
            const double V = s.vcol[p[l]];
            double S = (double)(s.cs1[p[l]] + nc * Q2[l]);
            S = S * S;
            const double x = V * bS, y = bV * S;  // cov_l^2 < cov_best^2  <=>  x < y
            const bool zero = (V == 0.0) && (bV == 0.0);
            const double d = x - y, tol = 0x1p-32 * fmax(x, y);
            if (!zero && fabs(d) <= tol) amb = true;
            if (!zero && d < -tol) {
              bi = l;
              bS = S;
              bV = V;
              lp = p[l];
              lq2 = Q2[l];
              lq3 = Q3[l];
              lcol = colR[l];
            }
          }
        }
        if (amb) {  // defer to the exact generic kernel (see bote_sweep_launch)
          defer_rank(a, rank);
          have = false;
        }
        if (have) {
          Mom mom[NSLOT];
          // Input leaderless: the hot loop (first, so little is live across it)
          {
            uint32_t S1[NL];
            uint64_t S2[NL];
            client_quads<N, NL>(B, s.cqt, ABLATE(a, 1) ? 0u : nq, ABLATE(a, 1) ? 0u : rem, a.s2_flush, colT,
                                qlane, S1, S2);
            if (ABLATE(a, 1)) {  // timing only: non-degenerate dummy sums (nothing defers)
#pragma unroll
              for (int t = 0; t < NL; ++t) {
                S1[t] = 1000u + colT[0] + t;
                S2[t] = (uint64_t)S1[t] * S1[t] + 12345u;
              }
            }
            mom[SLOT_AF1] = Mom{S1[QC::idx_a1], S2[QC::idx_a1], nc};
            mom[SLOT_AF2] = Mom{S1[QC::idx_a2], S2[QC::idx_a2], nc};
            mom[SLOT_E] = Mom{S1[QC::idx_e], S2[QC::idx_e], nc};
          }
          // Input FPaxos: moments from the leader column's sums
          mom[SLOT_FF1] = leader_mom(s.cs1[lp], s.cs2[lp], nc, lq2);
          mom[SLOT_FF2] = leader_mom(s.cs1[lp], s.cs2[lp], nc, lq3);
          // Colocated: leaderless values are the members' own quorum latencies;
          // FPaxos reads the leader's column of the config submatrix.
          {
            uint32_t f1 = 0, f1s = 0, f2 = 0, f2s = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) {
              const uint32_t v = ld16(B, lcol + rowq[k]) >> LAT_SHIFT;
              const uint32_t x1 = v + lq2, x2 = v + lq3;
              f1 += x1;
              f1s += x1 * x1;
              f2 += x2;
              f2s += x2 * x2;
            }
            mom[5 + SLOT_FF1] = Mom{f1, f1s, (uint32_t)N};
            mom[5 + SLOT_FF2] = Mom{f2, f2s, (uint32_t)N};
            mom[5 + SLOT_AF1] = Mom{cS1[QC::idx_a1], cS2[QC::idx_a1], (uint32_t)N};
            mom[5 + SLOT_AF2] = Mom{cS1[QC::idx_a2], cS2[QC::idx_a2], (uint32_t)N};
            mom[5 + SLOT_E] = Mom{cS1[QC::idx_e], cS2[QC::idx_e], (uint32_t)N};
          }
          if (!finish_config<N>(a, mom, s.vcol[lp], bi, rank, s.tk.thr, pnc1, pnc2, valid_cnt, digest, key, ok)) {
            defer_rank(a, rank);
            have = false;
          }
        }
      }
      if (!ABLATE(a, 4)) topk_step(s.tk, a.n_obj, a.K, key, ok, rank);
      if (jobok && rank < a.re) colex_next<N>(a.ns, p);
      ++rank;
    }
  }
  if (valid_cnt) atomicAdd(&a.out_counters[0], (unsigned long long)valid_cnt);
  if (digest) atomicAdd(&a.out_counters[1], (unsigned long long)digest);
  __syncthreads();
  Rec* dst = a.out_top + (size_t)blockIdx.x * a.n_obj * KP;
  for (uint32_t i = tid; i < (uint32_t)a.n_obj * KP; i += FAST_BD) dst[i] = s.tk.top[i];
}

// ------------------------------------------------------------- launcher ---
template <int N>
static hipError_t launch_fast_n(const FastArgs& a, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0,
                                hipEvent_t e1) {
  auto k = sweep_fast_kernel<N>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (e != hipSuccess) return e;
  if (e0) hipExtLaunchKernelGGL(k, dim3(grid), dim3(FAST_BD), (uint32_t)shm, st, e0, e1, 0u, a);
  else hipLaunchKernelGGL(k, dim3(grid), dim3(FAST_BD), shm, st, a);
  return hipGetLastError();
}

int fast_occupancy(uint32_t n, size_t shm) {
  int nb = 0;
  const void* k = nullptr;
  switch (n) {
#define OCC_CASE(NN) case NN: k = (const void*)sweep_fast_kernel<NN>; break;
    OCC_CASE(2) OCC_CASE(3) OCC_CASE(4) OCC_CASE(5) OCC_CASE(6) OCC_CASE(7) OCC_CASE(8) OCC_CASE(9)
    OCC_CASE(10) OCC_CASE(11) OCC_CASE(12) OCC_CASE(13) OCC_CASE(14) OCC_CASE(15) OCC_CASE(16)
#undef OCC_CASE
    default: return 0;
  }
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess) return 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, (int)FAST_BD, shm) != hipSuccess) return 1;
  return nb > 0 ? nb : 1;
}

hipError_t launch_fast(const FastArgs& a, uint32_t n, uint32_t grid, size_t shm, hipStream_t st, hipEvent_t e0,
                       hipEvent_t e1) {
  switch (n) {
#define FS_CASE(NN) case NN: return launch_fast_n<NN>(a, grid, shm, st, e0, e1);
    FS_CASE(2) FS_CASE(3) FS_CASE(4) FS_CASE(5) FS_CASE(6) FS_CASE(7) FS_CASE(8) FS_CASE(9)
    FS_CASE(10) FS_CASE(11) FS_CASE(12) FS_CASE(13) FS_CASE(14) FS_CASE(15) FS_CASE(16)
#undef FS_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bote
