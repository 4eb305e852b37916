// bote_kernels.hip — gfx950 kernels for fantoch_bote's configuration search.
//
// Work mapping (DESIGN.md "Kernels"): one LANE evaluates one configuration at a
// time; a wavefront holds 64 neighbouring configurations (colex-consecutive
// ranks), so every per-client step is wave-uniform in the client and
// lane-varying only in the config's members.  The R x R latency matrix (stored
// latency << 4) and the client row offsets live in LDS; per-lane quorum tables
// live in an LDS plane indexed [member][lane] (bank-conflict free).
//
// Reference map:
//   eval_config            Search::compute_stats   fantoch_bote/src/search.rs:262-319
//     Q phase              Bote::quorum_latency    fantoch_bote/src/lib.rs:155-163,169-185
//     leader selection     Bote::best_leader (COV) fantoch_bote/src/lib.rs:99-150
//     client loop          Bote::leaderless        fantoch_bote/src/lib.rs:38-59
//     FPaxos moments       Bote::leader            fantoch_bote/src/lib.rs:67-89
//     score / validity     Search::compute_score   fantoch_bote/src/search.rs:421-472
//   rank enumeration       Search::compute_configs fantoch_bote/src/search.rs:234-260
//                          (permutator combination -> colex ranks)
//   k_single_*             Bote::{leaderless, leader, all_leaders_stats, best_leader}
#include <atomic>
#include "bote_kernels.hpp"

namespace bote {

// ------------------------------------------------------------ LDS carving --
struct Smem {
  uint32_t* mat;     // R*R   latency << 4, row = from
  uint32_t* clioff;  // nc    client row offsets (cli[c] * R)
  uint32_t* srv;     // ns    server region ids
  uint64_t* cs;      // 2*ns  per position: sum_c L[c][srv[p]], sum_c L^2
  uint64_t* binom;   // (ns+1)*(N+1)
  uint32_t* qtab;    // N * BD * NLW
  TopkLds tk;        // top MAXOBJ*KP, cand BD, tmp KP, thr MAXOBJ, cnt
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// One layout function used by host (sizing) and device (carving).
__host__ __device__ inline size_t smem_layout(const EvalArgs& a, int N, int NLW, uint32_t BD, bool topk,
                                              size_t* off) {
  size_t o = 0;
  off[0] = o; o += (size_t)a.R * a.R * 4;
  off[1] = o; o += (size_t)a.nc * 4;
  off[2] = o; o += (size_t)a.ns * 4;
  o = align_up(o, 16);
  off[3] = o; o += (size_t)a.ns * 16;
  off[4] = o; o += a.cfgs ? 0 : (size_t)(a.ns + 1) * (N + 1) * 8;
  o = align_up(o, 16);
  off[5] = o; o += (size_t)N * BD * NLW * 4;
  o = align_up(o, 16);
  off[6] = o; o += topk ? (size_t)MAXOBJ * KP * 16 : 0;
  off[7] = o; o += topk ? (size_t)BD * 16 : 0;
  off[8] = o; o += topk ? (size_t)KP * 16 : 0;
  off[9] = o; o += topk ? (size_t)MAXOBJ * 16 : 0;
  off[10] = o; o += 48;
  return o;
}

template <int N>
__device__ inline Smem carve(const EvalArgs& a, unsigned char* base, int NLW) {
  size_t off[11];
  smem_layout(a, N, NLW, blockDim.x, a.out_top != nullptr, off);
  Smem s;
  s.mat = (uint32_t*)(base + off[0]);
  s.clioff = (uint32_t*)(base + off[1]);
  s.srv = (uint32_t*)(base + off[2]);
  s.cs = (uint64_t*)(base + off[3]);
  s.binom = (uint64_t*)(base + off[4]);
  s.qtab = (uint32_t*)(base + off[5]);
  s.tk.top = (Rec*)(base + off[6]);
  s.tk.cand = (Rec*)(base + off[7]);
  s.tk.tmp = (Rec*)(base + off[8]);
  s.tk.thr = (Rec*)(base + off[9]);
  s.tk.cnt = (int*)(base + off[10]);
  return s;
}

// arr[i] for a lane-varying i without an indexed private array: an OR of
// masked registers (a plain select chain is turned into a scratch lookup).
template <int N>
__device__ __forceinline__ uint32_t sel(const uint32_t (&arr)[N], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) r |= arr[j] & (0u - (uint32_t)(i == (uint32_t)j));
  return r;
}

// --------------------------------------------------------- config result --
// X: the extended key set (slots 10..19 and every leader's FPaxos moments,
// al[f - 1][config-order leader], Input clients)
template <int N, bool X>
struct CfgOut {
  static constexpr int NS = X ? NSLOT_X : NSLOT;
  Mom mom[NS];
  Mom al[X ? 2 : 1][X ? N : 1];
  uint32_t lead_orig;
  double score;
  bool valid;
};

// Slot presence for a config of size N (af2/ff2 need max_f >= 2).
template <int N>
__device__ __forceinline__ bool slot_has(int s) {
  return slot_exists<N>(s);
}

// ------------------------------------------------------------- eval one ---
// Evaluate the configuration whose members are positions p[0..N) of the
// server list (given order = config order).  `oi` is the output row (FULL).
template <int N, bool FULL, bool X>
__device__ __forceinline__ void eval_config(const EvalArgs& a, const Smem& s, const uint32_t (&p)[N], bool sorted_in, uint64_t oi,
                            CfgOut<N, X>& out) {
  using QC = QCfg<N>;
  using QT = QTab<N, X>;
  constexpr int NL = QT::NT;  // leaderless tables: compute_stats' q's, then the extended ones
  constexpr int NLW = (NL + 1) / 2;
  constexpr int P = Pow2<N>::v;
  const uint32_t BD = blockDim.x, tid = threadIdx.x;
  const uint32_t R = a.R, nc = a.nc;

  // --- members, sorted by region id (== name order) for the closest-server
  //     tie-break; `orig` keeps the config order for the leader tie-break.
  uint32_t mk[P];
#pragma unroll
  for (int j = 0; j < N; ++j) mk[j] = (s.srv[p[j]] << 12) | (p[j] << 4) | (uint32_t)j;
#pragma unroll
  for (int j = N; j < P; ++j) mk[j] = 0xFFFFFFFFu;
  if (!sorted_in) sort_network<P>(mk);
  uint32_t mreg[N], mpos[N], morig[N], moff[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    mreg[j] = mk[j] >> 12;
    mpos[j] = (mk[j] >> 4) & 0xFF;
    morig[j] = mk[j] & 15;
    moff[j] = mreg[j] * R;
  }

  // --- Q phase: per member j, the sorted distances to the config (row j of
  //     the config submatrix, self included); colocated closest server.
  uint32_t Qf1[N], Qf2[N], Ql[NL][N], cdk[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    uint32_t v[P];
    uint32_t key = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      uint32_t w = s.mat[moff[j] + mreg[k]];
      v[k] = w >> LAT_SHIFT;
      key = min(key, w | (uint32_t)k);
    }
#pragma unroll
    for (int k = N; k < P; ++k) v[k] = 0xFFFFFFFFu;
    sort_network<P>(v);
    Qf1[j] = v[QC::qf1 - 1];
    Qf2[j] = QC::maxf >= 2 ? v[(QC::maxf >= 2 ? QC::qf2 : 1) - 1] : 0;
#pragma unroll
    for (int t = 0; t < NL; ++t) Ql[t][j] = v[QT::q(t) - 1];
    cdk[j] = key;
    // the lane's quorum tables, two u16 per word: word w of member j at
    // qtab[(j * NLW + w) * BD + tid] (bank-conflict free)
#pragma unroll
    for (int w = 0; w < NLW; ++w)
      s.qtab[(j * NLW + w) * BD + tid] = Ql[2 * w][j] | (2 * w + 1 < NL ? (Ql[2 * w + 1 < NL ? 2 * w + 1 : 0][j] << 16) : 0u);
  }

  // --- FPaxos leader: min COV over the Input clients at f = 1 (q = 2),
  //     first in config order on ties.  Exact moments from the per-position
  //     column sums: sum_c (L[c][l] + Q)^k expands in sum_c L and sum_c L^2.
  Mom lm[N];
#pragma unroll
  for (int l = 0; l < N; ++l) {
    uint64_t c1 = s.cs[2 * mpos[l]], c2 = s.cs[2 * mpos[l] + 1], q = Qf1[l];
    lm[l] = Mom{c1 + (uint64_t)nc * q, c2 + 2ull * q * c1 + (uint64_t)nc * q * q, nc};
  }
  Mom bm = lm[0];
  uint32_t bo = morig[0], bi = 0;
  bool amb = false;
#pragma unroll
  for (int l = 1; l < N; ++l) {
    int c = cov_cmp(lm[l], bm);
    if (c == CMP_AMBIG) {
      amb = true;
    } else if (c == CMP_LT || (c == CMP_EQ && morig[l] < bo)) {
      bm = lm[l];
      bo = morig[l];
      bi = l;
    }
  }
  if (amb) {
    // Near-tie: replay the reference's f64 arithmetic for every leader.
    double cv[N];
#pragma unroll
    for (int l = 0; l < N; ++l) {
      const uint32_t col = mreg[l], q = Qf1[l];
      auto gen = [&](uint32_t c) { return (s.mat[s.clioff[c] + col] >> LAT_SHIFT) + q; };
      cv[l] = ref_cov(gen, nc, lm[l].s1);
    }
    double bc = cv[0];
    bo = morig[0];
    bi = 0;
#pragma unroll
    for (int l = 1; l < N; ++l) {
      int c = f64_cmp(cv[l], bc);
      if (c < 0 || (c == 0 && morig[l] < bo)) {
        bc = cv[l];
        bo = morig[l];
        bi = l;
      }
    }
  }
  const uint32_t lreg = sel(mreg, bi), lpos = sel(mpos, bi);
  const uint32_t lq1 = sel(Qf1, bi), lq2 = sel(Qf2, bi);
  out.lead_orig = bo;

  const uint32_t stride = 5 * nc + 5 * N;
  const bool wv = FULL && a.out_vals != nullptr;  // write per-client values
  uint32_t* ov = wv ? a.out_vals + oi * stride : nullptr;

  // --- Input FPaxos (search.rs:291-302): moments from column sums.
  {
    uint64_t c1 = s.cs[2 * lpos], c2 = s.cs[2 * lpos + 1];
    uint64_t q = lq1;
    out.mom[SLOT_FF1] = Mom{c1 + (uint64_t)nc * q, c2 + 2ull * q * c1 + (uint64_t)nc * q * q, nc};
    q = lq2;
    out.mom[SLOT_FF2] = Mom{c1 + (uint64_t)nc * q, c2 + 2ull * q * c1 + (uint64_t)nc * q * q, nc};
  }

  // --- Colocated keys: clients are the config members (config order).
  {
    uint64_t f1 = 0, f1s = 0, f2 = 0, f2s = 0;
    uint64_t l1[NL], l2[NL];
#pragma unroll
    for (int t = 0; t < NL; ++t) l1[t] = l2[t] = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      uint32_t v = s.mat[moff[k] + lreg] >> LAT_SHIFT;  // ping_latency(client k, leader)
      uint32_t x1 = v + lq1, x2 = v + lq2;
      f1 += x1; f1s += (uint64_t)x1 * x1;
      f2 += x2; f2s += (uint64_t)x2 * x2;
      uint32_t d = cdk[k] >> LAT_SHIFT, js = cdk[k] & 15;
      uint32_t A[NL];
#pragma unroll
      for (int t = 0; t < NL; ++t) {
        A[t] = d + sel(Ql[t], js);
        l1[t] += A[t];
        l2[t] += (uint64_t)A[t] * A[t];
      }
      if (wv) {
        uint32_t* oc = ov + 5 * nc;
        uint32_t o = morig[k];
        oc[SLOT_AF1 * N + o] = A[QC::idx_a1];
        oc[SLOT_FF1 * N + o] = x1;
        oc[SLOT_AF2 * N + o] = QC::maxf >= 2 ? A[QC::idx_a2] : 0xFFFFFFFFu;
        oc[SLOT_FF2 * N + o] = QC::maxf >= 2 ? x2 : 0xFFFFFFFFu;
        oc[SLOT_E * N + o] = A[QC::idx_e];
      }
    }
    out.mom[5 + SLOT_FF1] = Mom{f1, f1s, (uint32_t)N};
    out.mom[5 + SLOT_FF2] = Mom{f2, f2s, (uint32_t)N};
    out.mom[5 + SLOT_AF1] = Mom{l1[QC::idx_a1], l2[QC::idx_a1], (uint32_t)N};
    out.mom[5 + SLOT_AF2] = Mom{l1[QC::idx_a2], l2[QC::idx_a2], (uint32_t)N};
    out.mom[5 + SLOT_E] = Mom{l1[QC::idx_e], l2[QC::idx_e], (uint32_t)N};
    if constexpr (X) {
      constexpr int t2 = QT::idx(2), t3 = QT::idx(3) < 0 ? 0 : QT::idx(3), t4 = QT::idx(4) < 0 ? 0 : QT::idx(4);
      out.mom[4 + SLOT_TT1] = Mom{l1[t2], l2[t2], (uint32_t)N};
      out.mom[4 + SLOT_TW1] = Mom{l1[t2], l2[t2], (uint32_t)N};
      out.mom[4 + SLOT_TT2] = Mom{l1[t4], l2[t4], (uint32_t)N};
      out.mom[4 + SLOT_TW2] = Mom{l1[t3], l2[t3], (uint32_t)N};
    }
  }

  // --- Input leaderless: the hot loop.  Per client (wave-uniform): the
  //     nearest member by packed (latency << 4 | member) min, then the
  //     member's quorum latencies from the lane's LDS table.
  {
    uint32_t S1[NL];
    uint64_t S2[NL];
#pragma unroll
    for (int t = 0; t < NL; ++t) { S1[t] = 0; S2[t] = 0; }
    for (uint32_t c = 0; c < nc; ++c) {
      const uint32_t off = s.clioff[c];
      uint32_t m = 0xFFFFFFFFu;
#pragma unroll
      for (int k = 0; k < N; ++k) m = min(m, s.mat[off + mreg[k]] | (uint32_t)k);
      const uint32_t js = m & 15, d = m >> LAT_SHIFT;
      uint32_t A[NL];
#pragma unroll
      for (int w = 0; w < NLW; ++w) {
        const uint32_t wd = s.qtab[(js * NLW + w) * BD + tid];
        A[2 * w] = d + (wd & 0xFFFF);
        if (2 * w + 1 < NL) A[2 * w + 1 < NL ? 2 * w + 1 : 0] = d + (wd >> 16);
      }
#pragma unroll
      for (int t = 0; t < NL; ++t) {
        S1[t] += A[t];
        S2[t] += (uint64_t)A[t] * A[t];
      }
      if (wv) {
        uint32_t v = s.mat[off + lreg] >> LAT_SHIFT;
        ov[SLOT_AF1 * nc + c] = A[QC::idx_a1];
        ov[SLOT_FF1 * nc + c] = v + lq1;
        ov[SLOT_AF2 * nc + c] = QC::maxf >= 2 ? A[QC::idx_a2] : 0xFFFFFFFFu;
        ov[SLOT_FF2 * nc + c] = QC::maxf >= 2 ? v + lq2 : 0xFFFFFFFFu;
        ov[SLOT_E * nc + c] = A[QC::idx_e];
      }
    }
    out.mom[SLOT_AF1] = Mom{S1[QC::idx_a1], S2[QC::idx_a1], nc};
    out.mom[SLOT_AF2] = Mom{S1[QC::idx_a2], S2[QC::idx_a2], nc};
    out.mom[SLOT_E] = Mom{S1[QC::idx_e], S2[QC::idx_e], nc};
    if constexpr (X) {
      // Tempo tiny (2f) and write (f + 1) quorums, Input
      constexpr int t2 = QT::idx(2), t3 = QT::idx(3) < 0 ? 0 : QT::idx(3), t4 = QT::idx(4) < 0 ? 0 : QT::idx(4);
      out.mom[SLOT_TT1] = Mom{S1[t2], S2[t2], nc};
      out.mom[SLOT_TW1] = Mom{S1[t2], S2[t2], nc};
      out.mom[SLOT_TT2] = Mom{S1[t4], S2[t4], nc};
      out.mom[SLOT_TW2] = Mom{S1[t3], S2[t3], nc};
    }
  }
  if constexpr (X) {
    // FPaxos all leaders (Bote::all_leaders_stats, lib.rs:129-150), Input
    // clients, q = f + 1, leaders in config order, and the best leader by
    // Stats::Mean (lib.rs:99-121: the first minimum, exact sums)
#pragma unroll
    for (int o = 0; o < N; ++o) {
      uint32_t l = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) l = morig[k] == (uint32_t)o ? (uint32_t)k : l;
      const uint32_t pl = sel(mpos, l);
      const uint64_t c1 = s.cs[2 * pl], c2 = s.cs[2 * pl + 1];
      const uint64_t q1 = sel(Qf1, l), q2 = sel(Qf2, l);
      out.al[0][o] = Mom{c1 + (uint64_t)nc * q1, c2 + 2ull * q1 * c1 + (uint64_t)nc * q1 * q1, nc};
      out.al[1][o] = Mom{c1 + (uint64_t)nc * q2, c2 + 2ull * q2 * c1 + (uint64_t)nc * q2 * q2, nc};
    }
    Mom b1 = out.al[0][0], b2 = out.al[1][0];
#pragma unroll
    for (int o = 1; o < N; ++o) {
      if (out.al[0][o].s1 < b1.s1) b1 = out.al[0][o];
      if (out.al[1][o].s1 < b2.s1) b2 = out.al[1][o];
    }
    out.mom[SLOT_FL1] = b1;
    out.mom[SLOT_FL2] = b2;
  }

  // --- Search::compute_score (search.rs:421-472), bit-exact.
  out.valid = false;
  out.score = 0.0;
  if (a.want_score) {
    const int fmax = min(N / 2, a.ft_metric);
    bool valid = true;
    double score = 0.0;
#pragma unroll
    for (int f = 1; f <= 2; ++f) {
      if (f > fmax) break;
      const int sa = f == 1 ? SLOT_AF1 : SLOT_AF2, sf = f == 1 ? SLOT_FF1 : SLOT_FF2;
      const Mom& ma = out.mom[sa];
      const Mom& mf = out.mom[sf];
      double fmi = mom_mean(mf) - mom_mean(ma);
      bool fair;
      if (cov_nan(mf) || cov_nan(ma)) {
        fair = false;  // NaN - x >= p is false
      } else {
        int c = CMP_AMBIG;
        if (a.p_fair == 0.0) {
          c = cov_cmp(mf, ma);
          fair = c != CMP_LT;
        } else {
          double d = mom_cov(mf) - mom_cov(ma);
          double tol = 1e-9 * (1.0 + fabs(mom_cov(mf)) + fabs(mom_cov(ma)));
          if (fabs(d - a.p_fair) > tol) c = CMP_EQ;
          fair = d >= a.p_fair;
        }
        if (c == CMP_AMBIG) {
          // replay the reference's f64 covs of ff_f and af_f (Input)
          const uint32_t qfl = f == 1 ? lq1 : lq2;
          auto genf = [&](uint32_t cc) { return (s.mat[s.clioff[cc] + lreg] >> LAT_SHIFT) + qfl; };
          const int ti = f == 1 ? QC::idx_a1 : QC::idx_a2;
          auto gena = [&](uint32_t cc) {
            const uint32_t off = s.clioff[cc];
            uint32_t m = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < N; ++k) m = min(m, s.mat[off + mreg[k]] | (uint32_t)k);
            uint32_t js = m & 15;
            uint32_t q = 0;
#pragma unroll
            for (int t = 0; t < NL; ++t)
              if (t == ti) q = sel(Ql[t], js);
            return (m >> LAT_SHIFT) + q;
          };
          double cf = ref_cov(genf, nc, mf.s1), ca = ref_cov(gena, nc, ma.s1);
          fair = (cf - ca) >= a.p_fair;
        }
      }
      valid = valid && fmi >= a.p_fmean && fair;
      double emi = mom_mean(out.mom[SLOT_E]) - mom_mean(ma);
      if (N == 11 || N == 13) valid = valid && emi >= a.p_emean;
      double t = 30.0 * emi;
      t = fmi + t;
      score = score + t;
    }
    out.valid = valid;
    out.score = score;
  }
}

// ------------------------------------------------------------ the kernel --
template <int N, bool FULL, bool X>
__global__ void __launch_bounds__(256) eval_kernel(EvalArgs a) {
  constexpr int NLW = (QTab<N, X>::NT + 1) / 2;
  constexpr int NS = CfgOut<N, X>::NS;
  extern __shared__ __align__(16) unsigned char smem[];
  if (a.run_if_over && *a.run_if_over <= a.over_cap) return;  // block-uniform, before any barrier
  const Smem s = carve<N>(a, smem, NLW);
  const uint32_t BD = blockDim.x, tid = threadIdx.x;
  const bool topk = !FULL && a.out_top != nullptr;
  if (a.rank_list && *a.rank_count == 0) {
    // the deferred-config fix-up with nothing deferred (the common case):
    // empty lists for the merge, nothing staged (block-uniform)
    if (topk) {
      Rec* dst = a.out_top + (size_t)blockIdx.x * a.n_obj * KP;
      for (uint32_t i = tid; i < (uint32_t)a.n_obj * KP; i += BD) dst[i] = rec_max();
    }
    return;
  }

  // stage the planet, client offsets, server list, column sums, binomials
  for (uint32_t i = tid; i < a.R * a.R; i += BD) s.mat[i] = a.mat[i];
  for (uint32_t i = tid; i < a.nc; i += BD) s.clioff[i] = a.cli[i] * a.R;
  for (uint32_t i = tid; i < a.ns; i += BD) s.srv[i] = a.srv[i];
  if (!a.cfgs)
    for (uint32_t i = tid; i < (a.ns + 1) * (N + 1); i += BD) s.binom[i] = a.binom[i];
  if (topk) topk_init(s.tk, a.n_obj);
  __syncthreads();
  for (uint32_t i = tid; i < a.ns; i += BD) {
    uint64_t c1 = 0, c2 = 0;
    const uint32_t col = s.srv[i];
    for (uint32_t c = 0; c < a.nc; ++c) {
      uint64_t v = s.mat[s.clioff[c] + col] >> LAT_SHIFT;
      c1 += v;
      c2 += v * v;
    }
    s.cs[2 * i] = c1;
    s.cs[2 * i + 1] = c2;
  }
  __syncthreads();

  uint64_t total = a.re - a.rb;
  if (a.rank_list) {  // deferred configs: the count is known only on the device
    const uint64_t c = *a.rank_count;
    total = c < total ? c : total;
  }
  const uint64_t runlen = a.rank_list ? 1 : a.runlen;
  const uint64_t njobs = (total + runlen - 1) / runlen;
  const uint64_t G = (uint64_t)gridDim.x * BD;
  const uint64_t outer = (njobs + G - 1) / G;
  const bool sorted_in = !a.cfgs && a.srv_sorted;
  uint64_t valid_cnt = 0, digest = 0;

  for (uint64_t it = 0; it < outer; ++it) {
    const uint64_t job = it * G + (uint64_t)blockIdx.x * BD + tid;
    const bool jobok = job < njobs;
    uint64_t rank = a.rb + job * runlen;  // rank or config index
    uint32_t p[N];
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = j;
    uint64_t rend = a.re;
    if (jobok) {
      if (a.cfgs) {
#pragma unroll
        for (int j = 0; j < N; ++j) p[j] = a.cfgs[rank * N + j];
      } else {
        if (a.rank_list) {
          rank = a.rank_list[job];
          rend = rank + 1;
        }
        colex_unrank<N>(s.binom, a.ns, rank, p);
      }
    }
    for (uint64_t t = 0; t < runlen; ++t) {
      const bool have = jobok && rank < rend;
      CfgOut<N, X> r;
      if (have) {
        eval_config<N, FULL, X>(a, s, p, sorted_in, rank - a.rb, r);
        if (r.valid) ++valid_cnt;
        if (a.want_digest) {
          uint32_t h = 0;
#pragma unroll
          for (int sl = 0; sl < NSLOT; ++sl)
            if (slot_has<N>(sl)) h = digest_fold(h, sl, r.mom[sl].s1, r.mom[sl].s2);
          if constexpr (X) {  // the extended key set: every leader, then slots 10..19
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              if (f >= QCfg<N>::maxf) break;
#pragma unroll
              for (int l = 0; l < N; ++l) h = digest_fold_leader(h, f, l, r.al[f][l].s1, r.al[f][l].s2);
            }
#pragma unroll
            for (int sl = 10; sl < 20; ++sl)
              if (slot_has<N>(sl)) h = digest_fold(h, sl, r.mom[sl].s1, r.mom[sl].s2);
          }
          digest += digest_final(rank, r.lead_orig, h);
        }
        if (FULL) {
          const uint64_t oi = rank - a.rb;
          if (a.out_leader) a.out_leader[oi] = r.lead_orig;
#pragma unroll
          for (int sl = 0; sl < NS; ++sl) {
            const bool h = slot_has<N>(sl);
            if (a.out_s1) a.out_s1[oi * NS + sl] = h ? r.mom[sl].s1 : ~0ull;
            if (a.out_s2) a.out_s2[oi * NS + sl] = h ? r.mom[sl].s2 : ~0ull;
            if (a.out_mean) a.out_mean[oi * NS + sl] = h ? mom_mean(r.mom[sl]) : __longlong_as_double(0x7FF8000000000000ll);
            if (a.out_cov) a.out_cov[oi * NS + sl] = h ? mom_cov(r.mom[sl]) : __longlong_as_double(0x7FF8000000000000ll);
          }
          if constexpr (X) {
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
              for (int l = 0; l < N; ++l) {
                const bool h = f < QCfg<N>::maxf;
                if (a.out_al_s1) a.out_al_s1[(oi * 2 + f) * N + l] = h ? r.al[f][l].s1 : ~0ull;
                if (a.out_al_s2) a.out_al_s2[(oi * 2 + f) * N + l] = h ? r.al[f][l].s2 : ~0ull;
              }
          }
          if (a.out_score) a.out_score[oi] = r.score;
          if (a.out_valid) a.out_valid[oi] = r.valid ? 1 : 0;
        }
      }
      if (topk) {
        uint64_t key[MAXOBJ];
        bool ok[MAXOBJ];
#pragma unroll
        for (int o = 0; o < MAXOBJ; ++o) {
          ok[o] = false;
          key[o] = 0;
          if (o < a.n_obj && have) {
            const uint32_t kind = a.obj_kind[o], sl = a.obj_slot[o];
            ok[o] = true;
            if (kind == OBJ_SCORE) {
              ok[o] = r.valid;
              key[o] = ~orderable_f64(r.score);
            } else {
              // `sl` is uniform: one scalar branch per slot keeps r.mom in
              // registers (a select chain here gets turned into scratch).
#pragma unroll
              for (int q = 0; q < NS; ++q)
                if ((uint32_t)q == sl) key[o] = kind == OBJ_MEAN ? r.mom[q].s1 : cov_key(r.mom[q]);
            }
          }
        }
        topk_step(s.tk, a.n_obj, a.K, key, ok, rank);
      }
      if (have && !a.cfgs) colex_next<N>(a.ns, p);
      ++rank;
    }
  }

  if (a.out_counters) {
    if (valid_cnt) atomicAdd(&a.out_counters[0], (unsigned long long)valid_cnt);
    if (digest) atomicAdd(&a.out_counters[1], (unsigned long long)digest);
  }
  if (topk) {
    __syncthreads();
    Rec* dst = a.out_top + (size_t)blockIdx.x * a.n_obj * KP;
    for (uint32_t i = tid; i < (uint32_t)a.n_obj * KP; i += BD) dst[i] = s.tk.top[i];
  }
}

// ----------------------------------------------------- top-K list merge --
// (one thread per record of the G_MERGE_LISTS x KP inputs: each launch of
// the merge chain is latency-bound, 23 us per level at 256 threads)
constexpr int MERGE_BD = G_MERGE_LISTS * KP;
// lists: n_lists lists, list i of objective o at src[i * list_stride + o * KP]
// out:   one list per group of G_MERGE_LISTS lists, at dst[g * out_stride + o * KP]
// Every input list is sorted (block top-K lists, padded with rec_max), so each
// record's output slot is its rank in the union: its index in its own list
// plus, per other list, how many records precede it there (ties go to the
// lower list index).  One pass of binary searches in LDS, no sort; a block
// that finds an unsorted input falls back to the full bitonic sort.
__global__ void __launch_bounds__(1024) merge_kernel(const Rec* src, uint32_t n_lists, uint64_t list_stride, Rec* dst,
                                                     uint64_t out_stride, const Rec* alt, uint32_t alt_lists,
                                                     const unsigned long long* sel, uint64_t cap) {
  if (sel && *sel > cap) {  // device-side choice of the input (fast sweep overflow fallback)
    src = alt;
    n_lists = alt_lists;
  }
  __shared__ Rec buf[G_MERGE_LISTS * KP];
  __shared__ int unsorted;
  const uint32_t g = blockIdx.x, o = blockIdx.y;
  if (threadIdx.x == 0) unsorted = 0;
  for (uint32_t i = threadIdx.x; i < G_MERGE_LISTS * KP; i += blockDim.x) {
    uint32_t l = g * G_MERGE_LISTS + i / KP;
    buf[i] = l < n_lists ? src[l * list_stride + o * KP + i % KP] : rec_max();
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < G_MERGE_LISTS * KP; i += blockDim.x)
    if (i % KP && rec_lt(buf[i], buf[i - 1])) unsorted = 1;
  __syncthreads();
  Rec* out = dst + g * out_stride + o * KP;
  if (unsorted) {  // block-uniform
    block_bitonic(buf, G_MERGE_LISTS * KP);
    for (uint32_t i = threadIdx.x; i < KP; i += blockDim.x) out[i] = buf[i];
    return;
  }
  for (uint32_t i = threadIdx.x; i < G_MERGE_LISTS * KP; i += blockDim.x) {
    const uint32_t l = i / KP;
    const Rec x = buf[i];
    uint32_t pos = i % KP;
    for (uint32_t m = 0; m < (uint32_t)G_MERGE_LISTS && pos < (uint32_t)KP; ++m) {
      if (m == l) continue;
      pos += m < l ? upper_bound_rec(buf + m * KP, KP, x) : lower_bound_rec(buf + m * KP, KP, x);
    }
    if (pos < (uint32_t)KP) out[pos] = x;
  }
}

// ------------------------------------------------- single-config kernels --
// Shared by Bote::{leaderless, leader, all_leaders_stats, best_leader}.
// Server membership is a set (the reference filters with `contains`).


// q-th closest (1-based) from row `from` over the member set: counting
// selection, O(R) per call over the set members in (latency, id) order.
__device__ inline uint32_t quorum_lat(const uint32_t* smat, const uint8_t* member, uint32_t R, uint32_t from, uint32_t q,
                                      int* err) {
  // the q-th smallest of { L[from][t] : member[t] } (ties irrelevant for the value)
  for (uint32_t t = 0; t < R; ++t) {
    if (!member[t]) continue;
    uint32_t v = smat[from * R + t] >> LAT_SHIFT;
    uint32_t lt = 0, le = 0;
    for (uint32_t u = 0; u < R; ++u) {
      if (!member[u]) continue;
      uint32_t w = smat[from * R + u] >> LAT_SHIFT;
      lt += w < v;
      le += w <= v;
    }
    if (lt < q && q <= le) return v;
  }
  if (err) *err = 1;
  return 0;
}

__device__ inline uint32_t closest_member(const uint32_t* smat, const uint8_t* member, uint32_t R, uint32_t from) {
  // packed (latency << 8 | id) min: the (latency, name) order with id == name rank
  uint32_t key = 0xFFFFFFFFu;
  for (uint32_t t = 0; t < R; ++t)
    if (member[t]) key = min(key, ((smat[from * R + t] >> LAT_SHIFT) << 8) | t);
  return key;
}

// mode 0: quorum latencies of `froms`; 1: leaderless; 2: leader; 3: all leaders
__global__ void __launch_bounds__(256) single_kernel(SingleArgs a, int mode) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* smat = (uint32_t*)smem;
  uint8_t* member = (uint8_t*)(smat + a.R * a.R);
  uint32_t* qlat = (uint32_t*)(smem + align_up(a.R * a.R * 4 + a.R, 16));
  for (uint32_t i = threadIdx.x; i < a.R * a.R; i += blockDim.x) smat[i] = a.mat[i];
  for (uint32_t i = threadIdx.x; i < a.R; i += blockDim.x) member[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < a.ns; i += blockDim.x) member[a.servers[i]] = 1;
  __syncthreads();
  // quorum latency of every region (only member rows are used)
  for (uint32_t r = threadIdx.x; r < a.R; r += blockDim.x) qlat[r] = quorum_lat(smat, member, a.R, r, a.q, a.err);
  __syncthreads();
  if (mode == 0) {
    for (uint32_t i = threadIdx.x; i < a.nf; i += blockDim.x) a.out[i] = qlat[a.froms[i]];
  } else if (mode == 1) {
    for (uint32_t i = threadIdx.x; i < a.nc; i += blockDim.x) {
      uint32_t c = a.clients[i];
      uint32_t key = closest_member(smat, member, a.R, c);
      a.out[i] = (uint64_t)(key >> 8) + qlat[key & 0xFF];
    }
  } else if (mode == 2) {
    for (uint32_t i = threadIdx.x; i < a.nc; i += blockDim.x) {
      uint32_t c = a.clients[i];
      a.out[i] = (uint64_t)(smat[c * a.R + a.leader] >> LAT_SHIFT) + qlat[a.leader];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < a.ns * a.nc; i += blockDim.x) {
      uint32_t l = a.servers[i / a.nc], c = a.clients[i % a.nc];
      a.out[i] = (uint64_t)(smat[c * a.R + l] >> LAT_SHIFT) + qlat[l];
    }
  }
}

// Bote::best_leader: one thread per leader computes the reference's f64 stat
// (ordered sums), then thread 0 takes the first minimum under F64's order.
__global__ void __launch_bounds__(256) best_leader_kernel(SingleArgs a, const uint64_t* vals, double* stat) {
  for (uint32_t l = threadIdx.x; l < a.ns; l += blockDim.x) {
    const uint64_t* v = vals + (size_t)l * a.nc;
    uint64_t s1 = 0;
    for (uint32_t c = 0; c < a.nc; ++c) s1 += v[c];
    auto gen = [&](uint32_t c) { return (uint32_t)v[c]; };
    double x;
    if (a.stat == 0) x = (double)s1 / (double)a.nc;
    else if (a.stat == 1) x = ref_cov(gen, a.nc, s1);
    else x = ref_mdtm(gen, a.nc, s1);
    stat[l] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (uint32_t l = 1; l < a.ns; ++l)
      if (f64_cmp(stat[l], stat[b]) < 0) b = l;
    *a.out_pos = b;
  }
}

// ------------------------------------------------------------- launchers --
template <int N, bool FULL, bool X>
static hipError_t launch_eval_n(const EvalArgs& a, uint32_t grid, uint32_t bd, size_t shm, hipStream_t st) {
  auto k = eval_kernel<N, FULL, X>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(bd), shm, st, a);
  return hipGetLastError();
}

size_t eval_smem_bytes(const EvalArgs& a, uint32_t n, uint32_t bd, bool topk) {
  size_t off[11];
  int nl = 0;
  const bool x = a.keys != 0;
  switch (n) {
#define NL_CASE(NN) case NN: nl = x ? QTab<NN, true>::NT : QTab<NN, false>::NT; break;
    NL_CASE(2) NL_CASE(3) NL_CASE(4) NL_CASE(5) NL_CASE(6) NL_CASE(7) NL_CASE(8) NL_CASE(9)
    NL_CASE(10) NL_CASE(11) NL_CASE(12) NL_CASE(13) NL_CASE(14) NL_CASE(15) NL_CASE(16)
#undef NL_CASE
    default: return 0;
  }
  return smem_layout(a, (int)n, (nl + 1) / 2, bd, topk, off);
}

int eval_occupancy(uint32_t n, bool full, uint32_t bd, size_t shm, bool x) {
  int nb = 0;
  const void* k = nullptr;
  switch (n) {
#define OCC_CASE(NN)                                                                                       \
  case NN:                                                                                                 \
    k = x ? (full ? (const void*)eval_kernel<NN, true, true> : (const void*)eval_kernel<NN, false, true>)  \
          : (full ? (const void*)eval_kernel<NN, true, false> : (const void*)eval_kernel<NN, false, false>); \
    break;
    OCC_CASE(2) OCC_CASE(3) OCC_CASE(4) OCC_CASE(5) OCC_CASE(6) OCC_CASE(7) OCC_CASE(8) OCC_CASE(9)
    OCC_CASE(10) OCC_CASE(11) OCC_CASE(12) OCC_CASE(13) OCC_CASE(14) OCC_CASE(15) OCC_CASE(16)
#undef OCC_CASE
    default: return 0;
  }
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess) return 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, (int)bd, shm) != hipSuccess) return 1;
  return nb > 0 ? nb : 1;
}

hipError_t launch_eval(const EvalArgs& a, uint32_t n, bool full, uint32_t grid, uint32_t bd, size_t shm,
                       hipStream_t st) {
  switch (n) {
#define EV_CASE(NN)                                                                                 \
  case NN:                                                                                          \
    return a.keys ? (full ? launch_eval_n<NN, true, true>(a, grid, bd, shm, st)                     \
                          : launch_eval_n<NN, false, true>(a, grid, bd, shm, st))                   \
                  : (full ? launch_eval_n<NN, true, false>(a, grid, bd, shm, st)                    \
                          : launch_eval_n<NN, false, false>(a, grid, bd, shm, st));
    EV_CASE(2) EV_CASE(3) EV_CASE(4) EV_CASE(5) EV_CASE(6) EV_CASE(7) EV_CASE(8) EV_CASE(9)
    EV_CASE(10) EV_CASE(11) EV_CASE(12) EV_CASE(13) EV_CASE(14) EV_CASE(15) EV_CASE(16)
#undef EV_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_merge(const Rec* src, uint32_t n_lists, uint64_t list_stride, Rec* dst, uint64_t out_stride,
                        uint32_t n_obj, hipStream_t st) {
  uint32_t groups = (n_lists + G_MERGE_LISTS - 1) / G_MERGE_LISTS;
  hipLaunchKernelGGL(merge_kernel, dim3(groups, n_obj), dim3(MERGE_BD), 0, st, src, n_lists, list_stride, dst, out_stride,
                     (const Rec*)nullptr, 0u, (const unsigned long long*)nullptr, (uint64_t)0);
  return hipGetLastError();
}

hipError_t launch_merge_sel(const Rec* src, uint32_t n_lists, const Rec* alt, uint32_t alt_lists, uint64_t list_stride,
                            const unsigned long long* sel, uint64_t cap, Rec* dst, uint64_t out_stride, uint32_t n_obj,
                            hipStream_t st) {
  // groups cover the larger input; the surplus groups emit all-padding lists
  const uint32_t m = n_lists > alt_lists ? n_lists : alt_lists;
  uint32_t groups = (m + G_MERGE_LISTS - 1) / G_MERGE_LISTS;
  hipLaunchKernelGGL(merge_kernel, dim3(groups, n_obj), dim3(MERGE_BD), 0, st, src, n_lists, list_stride, dst, out_stride,
                     alt, alt_lists, sel, cap);
  return hipGetLastError();
}

// ------------------------------------------------- one-launch list merge --
// One workgroup per objective merges a sweep's per-block top-K lists (sorted,
// padded with rec_max) into the K least of their union.  The group kernel's
// dump (bote_group.hip, FastArgs::kbound) writes each list only up to the
// least K-th key of any block, which still leaves most of every list: the
// blocks take statistically similar chunks, so the least of 512 per-block
// K-th order statistics leaves ~70 of each block's 100 records below it
// (round 4: ~36 k records per objective, 1.07 ms per step).  So the merge
// first tightens the bound from the lists' heads:
//   t = a key with at least K head records at or below it,
// where the head records (the first WIDE_HEAD of each list) are distinct
// configs, so the union's K-th key is <= t.  With 512 lists and K = 100 the
// K-th least head lies at about the 20th percentile of the block minima, and
// the union holds ~K + K/8 records at or below it.  t is found by a radix
// select with 10-bit digits over (key - least head) that stops as soon as the
// chosen digit's bin holds at most WIDE_SLACK heads beyond the K-th (one or
// two passes for mean keys), and t is that bin's upper edge.  Each list's
// prefix at or below min(t, kbound) is counted, the counts are scanned, and
// when the gathered records fit one pass (<= WIDE_RANK_MAX) each record's
// output slot is its rank among them (a count over LDS; the (key, rank) order
// is total, so ranks are distinct); larger fills (the overflow fallback's full
// lists, heavy ties at t) take the windowed bitonic path: passes of <=
// WIDE_SORT - K records sorted with the running K least.  The result is the K
// least of the union whatever the fill (tests/test_merge_model.py restates the
// procedure and bounds the gathered count).
constexpr int WIDE_BD = 1024, WIDE_SORT = 4096, WIDE_LISTS_PER_THREAD = 4, WIDE_HEAD = 2;
constexpr int WIDE_BINS = 1024, WIDE_WAVES = WIDE_BD / 64, WIDE_SLACK = 32, WIDE_RANK_MAX = 1024;
// A record with key == ~0 (a NaN COV key) has a real rank < C(R, n) < 2^64 - 1,
// so only padding matches both fields.
__device__ __forceinline__ bool is_rec_max(const Rec& r) { return r.key == ~0ull && r.rank == ~0ull; }
static_assert(WIDE_MERGE_LISTS == (uint32_t)(WIDE_BD * WIDE_LISTS_PER_THREAD), "one thread per WIDE_LISTS_PER_THREAD lists");
static_assert(WIDE_BINS == WIDE_BD, "the digit histogram shares the scan array");
constexpr int WIDE_FEW = 64;  // a bin this small is finished by one wave (wide_select)
// LDS: the head records of every list (thread-minor; the windowed path's
// sort buffer reuses them), the one-pass gather, the scan / digit histogram,
// control words, per-wave reductions and a small bin's values: 149 KB
constexpr size_t WIDE_HEADS_BYTES = (size_t)WIDE_LISTS_PER_THREAD * WIDE_HEAD * WIDE_BD * 16;
static_assert(WIDE_HEADS_BYTES >= (size_t)WIDE_SORT * 16, "the windowed sort buffer fits the head records");
size_t merge_wide_smem() {
  return WIDE_HEADS_BYTES + (size_t)WIDE_RANK_MAX * 16 + (WIDE_BD + 8) * sizeof(uint32_t) +
         4 * WIDE_WAVES * sizeof(uint64_t) + 2 * WIDE_FEW * sizeof(uint64_t);
}

// inclusive prefix sum over the wavefront
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(v, d);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}

// Block-wide selection for merge_wide_kernel: among the values the threads
// visit (each(f) calls f(v) for each of this thread's values), a value x with
// at least `need` values <= x, by an MSB-first radix select with 10-bit digits
// over (v - least value) that stops as soon as the chosen digit's bin holds at
// most WIDE_SLACK values beyond the need-th, or at the exact value.  `left` is
// then the need-th value's position among the values of the final bin and
// `inbin` their number (exact: x is the need-th value itself).  none: fewer
// than `need` values.  Every thread of the block calls it (it has barriers).
struct WideSel {
  uint64_t x;
  uint32_t left, inbin;
  bool exact, none;
  bool has_aux;  // a small final bin was ranked by (value, aux): aux is the selected item's
  uint64_t aux;
};
template <class Each>
__device__ WideSel wide_select(Each each, uint64_t need, uint32_t* hist, uint32_t* ctl, uint64_t* red, bool slack) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t* few = red + 4 * WIDE_WAVES;  // the values of a small final bin
  uint64_t* fewa = few + WIDE_FEW;       // and their aux words (ranks: the items are then distinct)
  uint64_t mn = ~0ull, mx = 0, nv = 0;
  each([&](uint64_t v, uint64_t) {
    mn = min(mn, v);
    mx = max(mx, v);
    ++nv;
  });
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, (uint64_t)__shfl_xor((long long)mn, d));
    mx = max(mx, (uint64_t)__shfl_xor((long long)mx, d));
    nv += (uint64_t)__shfl_xor((long long)nv, d);
  }
  if (lane == 0) {
    red[wv] = mn;
    red[WIDE_WAVES + wv] = mx;
    red[2 * WIDE_WAVES + wv] = nv;
  }
  __syncthreads();
  mn = ~0ull;
  mx = 0;
  nv = 0;
#pragma unroll
  for (int w = 0; w < WIDE_WAVES; ++w) {
    mn = min(mn, red[w]);
    mx = max(mx, red[WIDE_WAVES + w]);
    nv += red[2 * WIDE_WAVES + w];
  }
  WideSel r{~0ull, 0, 0, false, true, false, 0};
  if (nv >= need && need > 0) {  // (block-uniform)
    r.none = false;
    if (mx == mn) {
      r = WideSel{mn, (uint32_t)need, (uint32_t)nv, true, false, false, 0};
    } else {
      uint32_t s_hi = 64 - (uint32_t)__clzll(mx - mn);  // every (v - mn) < 2^s_hi
      uint64_t prefix = 0;
      for (;;) {
        const uint32_t s_lo = s_hi > 10 ? s_hi - 10 : 0, w = s_hi - s_lo;
        hist[tid] = 0;
        __syncthreads();
        // (shared-count audit, round 6: the adds follow the zeroing barrier;
        // wave 0 reads the bins only after the barrier below; every thread
        // reads the pick (ctl[2..4]) after the next one, and the histogram is
        // zeroed again only after the loop's closing barrier, so no thread can
        // add into a pass while another still reads the last)
        each([&](uint64_t v, uint64_t) {
          v -= mn;
          if (s_hi >= 64 || (v >> s_hi) == prefix) atomicAdd(&hist[(uint32_t)(v >> s_lo) & ((1u << w) - 1)], 1u);
        });
        __syncthreads();
        if (wv == 0) {  // one wave: the bin holding the need-th value, 16 bins per lane
          uint32_t cb[WIDE_BINS / 64], sl = 0;
#pragma unroll
          for (int q = 0; q < WIDE_BINS / 64; ++q) {
            cb[q] = hist[lane * (WIDE_BINS / 64) + q];
            sl += cb[q];
          }
          uint32_t before = wave_incl_scan(sl) - sl;
#pragma unroll
          for (int q = 0; q < WIDE_BINS / 64; ++q) {
            if (before < need && need <= before + cb[q]) {  // exactly one lane, one bin
              ctl[2] = lane * (WIDE_BINS / 64) + q;
              ctl[3] = (uint32_t)(need - before);
              ctl[4] = cb[q];
            }
            before += cb[q];
          }
          if (lane == 0) ctl[5] = 0;  // (slots of a small bin's values)
        }
        __syncthreads();
        const uint32_t d = ctl[2], left = ctl[3], inbin = ctl[4];
        prefix = (prefix << w) | d;
        need = left;
        s_hi = s_lo;
        if (s_hi == 0 || (slack && inbin - left <= (uint32_t)WIDE_SLACK)) {  // (block-uniform)
          r.left = left;
          r.inbin = inbin;
          r.exact = s_hi == 0;
          break;
        }
        if (inbin <= (uint32_t)WIDE_FEW) {  // (block-uniform) the bin's values to one wave: exact
          each([&](uint64_t v, uint64_t aux) {
            v -= mn;
            if ((v >> s_hi) == prefix) {
              // (audit: ctl[5] was zeroed by wave 0 before the pick barrier;
              // the adds precede the barrier below, after which only wave 0
              // reads the slots, and every path out of here passes a barrier
              // before ctl is written again)
              const uint32_t k = atomicAdd(&ctl[5], 1u);
              few[k] = v;
              fewa[k] = aux;
            }
          });
          __syncthreads();
          if (wv == 0) {
            // the left-th least item in (value, aux) order: fewer than `left`
            // items below it and at least `left` at or below it (equal items:
            // every lane holding one agrees); with distinct aux words (ranks)
            // it is one item, so the caller has its aux without a second select
            const uint64_t x = lane < inbin ? few[lane] : ~0ull, xa = lane < inbin ? fewa[lane] : ~0ull;
            uint32_t lt = 0, le = 0, vlt = 0, vle = 0;
            for (uint32_t j = 0; j < inbin; j += 4) {  // (4 reads in flight; inbin <= 64 = the buffer)
#pragma unroll
              for (uint32_t u = 0; u < 4; ++u) {
                const uint64_t y = few[j + u], ya = fewa[j + u];
                const bool in = j + u < inbin;
                lt += (uint32_t)(in && (y < x || (y == x && ya < xa)));
                le += (uint32_t)(in && (y < x || (y == x && ya <= xa)));
                vlt += (uint32_t)(in && y < x);
                vle += (uint32_t)(in && y <= x);
              }
            }
            if (lane < inbin && lt < left && left <= le) {
              red[0] = x;
              red[1] = xa;
              ctl[3] = left - vlt;  // (its position among the values equal to it)
              ctl[4] = vle - vlt;
            }
          }
          __syncthreads();
          r.x = mn + red[0];
          r.aux = red[1];
          r.has_aux = true;
          r.left = ctl[3];
          r.inbin = ctl[4];
          r.exact = true;
          __syncthreads();
          return r;
        }
        __syncthreads();  // (the histogram and ctl are rewritten by the next pass)
      }
      const uint64_t x = (prefix << s_hi) | ((1ull << s_hi) - 1);  // (s_hi < 64 after a pass)
      r.x = x > ~0ull - mn ? ~0ull : mn + x;
    }
  }
  __syncthreads();  // (red, hist and ctl are reused by the caller)
  return r;
}

__global__ void __launch_bounds__(WIDE_BD) merge_wide_kernel(const Rec* src, uint32_t n_lists, uint64_t list_stride,
                                                             Rec* dst, const Rec* alt, uint32_t alt_lists,
                                                             const unsigned long long* sel, uint64_t cap,
                                                             const unsigned long long* kbound, uint32_t K,
                                                             const unsigned long long* csrc,
                                                             const unsigned long long* calt, uint64_t* cdst) {
#ifdef BOTE_MERGE_PRINTF
  const uint64_t T0 = wall_clock64();
  uint64_t TT[4] = {0, 0, 0, 0};
  int tn = 0;
#define WIDE_T(name) TT[tn++ & 3] = wall_clock64() - T0;
#else
#define WIDE_T(name)
#endif
  const bool use_alt = sel && *sel > cap;
  if (use_alt) {  // device-side choice of the input (fast sweep overflow fallback)
    src = alt;
    n_lists = alt_lists;
  }
  // the result's counters (valid, digest) from the same choice (what
  // pick_counters_kernel does for the merge tree; one launch fewer)
  if (cdst && blockIdx.x == 0 && threadIdx.x < 2) cdst[threadIdx.x] = (use_alt ? calt : csrc)[threadIdx.x];
  extern __shared__ __align__(16) unsigned char wsm[];
  Rec* hr = (Rec*)wsm;                              // head records (then the windowed path's buffer)
  Rec* buf = hr;                                    // the windowed path's sort buffer
  Rec* gbuf = (Rec*)(wsm + WIDE_HEADS_BYTES);       // the one-pass gather
  uint32_t* scan = (uint32_t*)(wsm + WIDE_HEADS_BYTES + (size_t)WIDE_RANK_MAX * 16);  // also the digit histogram
  uint32_t* ctl = scan + WIDE_BD;  // [0] next window start, [1] records this pass; [2..4] the digit pick
  uint64_t* red = (uint64_t*)(ctl + 8);  // per wave: least and greatest value, count
  const uint32_t o = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t KK = K < (uint32_t)KP ? K : (uint32_t)KP;
  Rec* out = dst + o * KP;
  if (KK == 0) {
    for (uint32_t i = tid; i < (uint32_t)KP; i += WIDE_BD) out[i] = rec_max();
    return;
  }
  constexpr int LT = WIDE_LISTS_PER_THREAD, H = WIDE_HEAD;
  auto list = [&](int j) { return src + (size_t)(tid * LT + j) * list_stride + o * KP; };
  auto live = [&](int j) { return tid * LT + (uint32_t)j < n_lists; };
  // records above the bound on the K-th key (the least K-th key of the
  // group blocks' full lists) cannot be among the K least of the union
  const uint64_t b0 = kbound && !use_alt ? kbound[o] : ~0ull;
  // the first WIDE_HEAD records of all of a thread's lists load together
  // (one round trip to memory: the lists were written by blocks on every
  // XCD) into LDS, thread-minor (in registers they spilled at 1,024
  // threads); everything up to the gather then reads LDS
  auto hrec = [&](int j, int c) -> Rec& { return hr[(c * LT + j) * WIDE_BD + tid]; };
  auto hk = [&](int j, int c) -> uint64_t { return hrec(j, c).key; };
  {
    Rec t[LT][H];
#pragma unroll
    for (int j = 0; j < LT; ++j)
#pragma unroll
      for (int c = 0; c < H; ++c) t[j][c] = live(j) && (uint32_t)c < KK ? list(j)[c] : Rec{~0ull, ~0ull};
#pragma unroll
    for (int j = 0; j < LT; ++j)
#pragma unroll
      for (int c = 0; c < H; ++c) hrec(j, c) = t[j][c];
  }
  WIDE_T("heads")
  // the bound record (bk, br): the union's K least are at or below it
  uint64_t bk = ~0ull, br = ~0ull;
  {
    // the heads' kept prefix per list (a list's records end at its
    // terminator: what follows it in memory is stale; a key of all ones, a
    // NaN COV, also ends it here: fewer heads only loosen the bound)
    uint32_t hn[LT];
#pragma unroll
    for (int j = 0; j < LT; ++j) {
      uint32_t c = 0;
#pragma unroll
      for (int i = 0; i < H; ++i) c += (uint32_t)(c == (uint32_t)i && hk(j, i) != ~0ull && hk(j, i) <= b0);
      hn[j] = c;
    }
    auto each_head = [&](auto f) {
#pragma unroll
      for (int j = 0; j < LT; ++j)
#pragma unroll
        for (int c = 0; c < H; ++c)
          if ((uint32_t)c < hn[j]) f(hk(j, c), hrec(j, c).rank);
    };
    // (to the exact key: a bin's worth of heads above the K-th could stand
    // for many more tied records beyond the heads)
    const WideSel ks = wide_select(each_head, KK, scan, ctl, red, false);
    WIDE_T("keysel")
    if (!ks.none) {
      bk = ks.x;
      if (ks.has_aux && ks.inbin > 1) {
        br = ks.aux;  // (a small final bin ranked by (key, rank): the K-th head record itself)
      } else if (ks.inbin > 1) {
        // heads tie at the K-th key (FPaxos means: round 5 measured 1,186
        // records at one key on a 1/8 shard): the left-th least rank among
        // them makes (bk, br) the K-th least head record itself
        auto each_tie = [&](auto f) {
#pragma unroll
          for (int j = 0; j < LT; ++j)
#pragma unroll
            for (int c = 0; c < H; ++c)
              if ((uint32_t)c < hn[j] && hk(j, c) == bk) f(hrec(j, c).rank, 0ull);
        };
        const WideSel rs = wide_select(each_tie, ks.left, scan, ctl, red, true);
        if (!rs.none) br = rs.x;
      }
    }
  }
  const uint64_t kb = min(b0, bk);
  // a record is gathered when it is a real record at or below both bounds
  auto keep = [&](const Rec& r) {
    return !is_rec_max(r) && r.key <= kb && (r.key < bk || r.rank <= br);
  };
  // per list: the filled prefix length at or below the bound (keys from the
  // registers; a rank is read only where it decides)
  uint32_t cnt[LT], off[LT], mine = 0;
#pragma unroll
  for (int j = 0; j < LT; ++j) {
    uint32_t c = 0;
    bool go = live(j);
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if (go && (uint32_t)i < KK) {
        const uint64_t k = hk(j, i);
        bool in = k <= kb;
        if (in && (k == ~0ull || (k == bk && br != ~0ull))) in = keep(hrec(j, i));
        c += in ? 1u : 0u;
        go = in;
      } else {
        go = false;
      }
    }
    if (go) {  // a long list (rare): walk the rest
      const Rec* L = list(j);
      while (c < KK && keep(L[c])) ++c;
    }
    cnt[j] = c;
    off[j] = mine;
    mine += c;
  }
  // exclusive scan of the threads' totals (list order = thread order): per
  // wave by shuffles, then the waves' totals
  const uint32_t incl = wave_incl_scan(mine);
  if (lane == 63) scan[wv] = incl;
  __syncthreads();
  uint32_t base = incl - mine, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < (uint32_t)WIDE_WAVES; ++w) {
    const uint32_t x = scan[w];
    base += w < wv ? x : 0u;
    total += x;
  }
#pragma unroll
  for (int j = 0; j < LT; ++j) off[j] += base;
  WIDE_T("scan")
  if (total <= (uint32_t)WIDE_RANK_MAX) {  // (block-uniform) one pass: slot = rank among the gathered
#pragma unroll
    for (int j = 0; j < LT; ++j) {
#pragma unroll
      for (int c = 0; c < H; ++c)
        if ((uint32_t)c < cnt[j]) gbuf[off[j] + c] = hrec(j, c);
      if (cnt[j] > (uint32_t)H) {  // (rare: beyond the heads)
        const Rec* L = list(j);
        for (uint32_t c = H; c < cnt[j]; ++c) gbuf[off[j] + c] = L[c];
      }
    }
    // (padded with rec_max to a multiple of 8: the count loop below keeps 8
    // independent LDS reads in flight; padding is never below a record)
    const uint32_t tot8 = (total + 7) & ~7u;
    if (tid >= total && tid < tot8) gbuf[tid] = rec_max();
    __syncthreads();
    for (uint32_t i = tid; i < total; i += WIDE_BD) {
      const Rec x = gbuf[i];
      uint32_t r = 0;
      for (uint32_t m = 0; m < tot8; m += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) r += (uint32_t)rec_lt(gbuf[m + u], x);
      }
      if (r < KK) out[r] = x;
    }
    for (uint32_t i = min(total, KK) + tid; i < (uint32_t)KP; i += WIDE_BD) out[i] = rec_max();
    WIDE_T("done")
#ifdef BOTE_MERGE_PRINTF
    if (tid == 0)
      printf("merge o=%u lists=%u total=%u bk=%llx br=%llx ticks heads %llu keysel %llu scan %llu done %llu\n", o,
             n_lists, total, (unsigned long long)bk, (unsigned long long)br, (unsigned long long)TT[0],
             (unsigned long long)TT[1], (unsigned long long)TT[2], (unsigned long long)TT[3]);
#endif
    return;
  }
  // running K least: buf[0 .. have) (buf overwrites the head records: the
  // windowed passes gather from memory)
  uint32_t have = 0;
  const uint32_t room = WIDE_SORT - KK;  // records gathered per pass
  uint32_t w0 = 0;  // window start (in the concatenated order)
  while (w0 < total) {
    __syncthreads();
    if (tid == 0) {
      ctl[0] = total;  // the next window starts at the first list that does not fit
      ctl[1] = 0;
    }
    __syncthreads();
    // lists inside [w0, w0 + room) are copied after the running list
#pragma unroll
    for (int j = 0; j < LT; ++j) {
      if (cnt[j] == 0 || off[j] < w0) continue;
      if (off[j] + cnt[j] - w0 <= room) {
        Rec* d = buf + KK + off[j] - w0;
        const Rec* L = list(j);
        for (uint32_t c = 0; c < cnt[j]; ++c) d[c] = L[c];
        atomicMax(&ctl[1], off[j] + cnt[j] - w0);
      } else {
        // (audit: thread 0 resets ctl[0..1] between the two barriers at the
        // window's start; the atomics follow them, every thread reads
        // got / next after the barrier below, and the next window's reset
        // waits for the barrier that opens it)
        atomicMin(&ctl[0], off[j]);
      }
    }
    __syncthreads();
    const uint32_t got = ctl[1], next = ctl[0];
    // compact: running records at [0, have), the pass's at [KK, KK + got)
    uint32_t n = KK + got, P = 2;
    while (P < n) P <<= 1;
    for (uint32_t i = tid; i < P; i += WIDE_BD)
      if ((i >= have && i < KK) || i >= n) buf[i] = rec_max();
    __syncthreads();
    block_bitonic(buf, (int)P);
    have = min(KK, n);
    w0 = next;
  }
  __syncthreads();
  for (uint32_t i = tid; i < (uint32_t)KP; i += WIDE_BD) out[i] = i < have && i < KK ? buf[i] : rec_max();
}
#undef WIDE_T

hipError_t launch_merge_wide(const Rec* src, uint32_t n_lists, const Rec* alt, uint32_t alt_lists, uint64_t list_stride,
                             const unsigned long long* sel, uint64_t cap, const unsigned long long* kbound, Rec* dst,
                             uint32_t n_obj, uint32_t K, const unsigned long long* csrc, const unsigned long long* calt,
                             uint64_t* cdst, hipStream_t st) {
  if (n_lists > (uint32_t)(WIDE_BD * WIDE_LISTS_PER_THREAD) || alt_lists > (uint32_t)(WIDE_BD * WIDE_LISTS_PER_THREAD))
    return hipErrorInvalidValue;
  const size_t shm = merge_wide_smem();
  // (the LDS limit above 64 KB, once per device)
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = 1ull << (dev & 63);
  if (!(done.load(std::memory_order_relaxed) & bit)) {
    e = hipFuncSetAttribute((const void*)merge_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    done.fetch_or(bit, std::memory_order_relaxed);
  }
  hipLaunchKernelGGL(merge_wide_kernel, dim3(n_obj), dim3(WIDE_BD), shm, st, src, n_lists, list_stride, dst, alt,
                     alt_lists, sel, cap, kbound, K, csrc, calt, cdst);
  return hipGetLastError();
}

__global__ void pick_counters_kernel(const unsigned long long* src, const unsigned long long* alt,
                                     const unsigned long long* sel, uint64_t cap, uint64_t* dst) {
  if (threadIdx.x < 2) dst[threadIdx.x] = (*sel > cap ? alt : src)[threadIdx.x];
}

// the per-launch control words of a fast-path sweep zeroed in one launch
// (valid/digest counters, the deferred-queue count, the work-ticket counter,
// the overflow fallback's counters) instead of four memsets
__global__ void zero_ctl_kernel(unsigned long long* counters, unsigned long long* qcount, unsigned int* wctr,
                                unsigned long long* counters_alt, unsigned long long* kbound) {
  const uint32_t t = threadIdx.x;
  if (t < 2) counters[t] = 0;
  if (t == 2) *qcount = 0;
  if (t >= 4 && t < 6) counters_alt[t - 4] = 0;
  if (t >= 8 && t < 24 && wctr) wctr[32 * (t - 8)] = 0;  // the 8 ticket-counter shards, main and sample launch
  if (t >= 32 && t < 32 + MAXOBJ && kbound) kbound[t - 32] = ~0ull;  // the lists' K-th key bound (no bound)
}

hipError_t launch_zero_ctl(unsigned long long* counters, unsigned long long* qcount, unsigned int* wctr,
                           unsigned long long* counters_alt, unsigned long long* kbound, hipStream_t st) {
  hipLaunchKernelGGL(zero_ctl_kernel, dim3(1), dim3(64), 0, st, counters, qcount, wctr, counters_alt, kbound);
  return hipGetLastError();
}

// The top-K seed: per objective (one block each) the K-th least of the
// sample launch's per-chunk minima, by an exact MSB-first radix select (8-bit
// digits: a 256-bin LDS histogram of the keys that share the prefix so far,
// then the digit holding the K-th); all-ones (no bound) when fewer than K
// samples have the objective.  The bytes above the highest one in which the
// keys differ (found first from their AND and OR) are taken as known: mean
// keys (S1 < 2^21) skip 5 of the 8 passes, whose histograms would all hit one
// bin.  (A bitonic sort of 4096 keys took 56 us: 78 barrier-separated stages.)
__global__ void __launch_bounds__(1024) seed_kernel(const uint64_t* smin, uint32_t nsamp, uint32_t K, uint64_t* tseed) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t sel[3];  // prefix, remaining rank, keys in the chosen bin
  __shared__ uint64_t red[2][16];
  __shared__ uint64_t few[64];  // a small final bin's keys
  __shared__ uint32_t nfew;
  const uint32_t o = blockIdx.x, tid = threadIdx.x, BD = blockDim.x;
  if (nsamp < K || K == 0) {
    if (tid == 0) tseed[o] = ~0ull;
    return;
  }
  const uint64_t* x = smin + (size_t)o * nsamp;
  // up to RP keys per thread stay in registers across the passes (32,768 keys
  // re-read from memory every pass took 72 us); larger samples re-read
  constexpr int RP = 32;
  const bool inreg = nsamp <= (uint32_t)RP * BD;
  uint64_t xr[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) {
    const uint32_t k = tid + (uint32_t)i * BD;
    xr[i] = inreg && k < nsamp ? x[k] : ~0ull;
  }
  // the AND and OR of all keys: the bits above their highest difference are common
  uint64_t va = ~0ull, vo = 0;
  if (inreg) {
#pragma unroll
    for (int i = 0; i < RP; ++i)
      if (tid + (uint32_t)i * BD < nsamp) {
        va &= xr[i];
        vo |= xr[i];
      }
  } else {
    for (uint32_t k = tid; k < nsamp; k += BD) {
      va &= x[k];
      vo |= x[k];
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    va &= (uint64_t)__shfl_xor((long long)va, d);
    vo |= (uint64_t)__shfl_xor((long long)vo, d);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = va;
    red[1][tid >> 6] = vo;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t a = ~0ull, b = 0;
    for (uint32_t w = 0; w < (BD >> 6); ++w) {
      a &= red[0][w];
      b |= red[1][w];
    }
    const uint64_t diff = a ^ b;  // bits in which some keys differ
    const int top = diff ? 63 - __clzll(diff) : -1;  // highest such bit
    const int pass0 = top < 0 ? -1 : top / 8;        // first byte to select on
    // the known high bytes; the rank within them is K
    sel[0] = pass0 < 0 ? a : (pass0 == 7 ? 0 : a >> (8 * (pass0 + 1)));
    sel[1] = K;
    red[0][0] = (uint64_t)(int64_t)pass0;
  }
  __syncthreads();
  const int pass0 = (int)(int64_t)red[0][0];
  for (int pass = pass0; pass >= 0; --pass) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    const uint64_t prefix = sel[0];
    const int sh = 8 * pass;
    // (audit: the bins are zeroed before the barrier above; wave 0 reads
    // them after the barrier below and publishes sel[] before the next one;
    // every thread reads sel[] after it, and the next pass zeroes the bins
    // only after that barrier, so no add lands in a pass still being read)
    auto count = [&](uint64_t v) {
      if (pass == 7 || (v >> (sh + 8)) == prefix) atomicAdd(&hist[(v >> sh) & 0xFFu], 1u);
    };
    if (inreg) {
#pragma unroll
      for (int i = 0; i < RP; ++i)
        if (tid + (uint32_t)i * BD < nsamp) count(xr[i]);
    } else {
      for (uint32_t k = tid; k < nsamp; k += BD) count(x[k]);
    }
    __syncthreads();
    if (tid < 64) {  // one wave: inclusive scan of the 256 bins, 4 per lane
      uint32_t c[4], s = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) c[b] = hist[4 * tid + b];
#pragma unroll
      for (int b = 0; b < 4; ++b) s += c[b];
      uint32_t incl = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if ((int)tid >= d) incl += y;
      }
      const uint64_t need = sel[1];
      uint32_t before = incl - s;  // keys in the bins of the lanes below
      int digit = -1;
      uint64_t left = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (digit < 0 && before < need && need <= before + c[b]) {
          digit = 4 * (int)tid + b;
          left = need - before;
        }
        before += c[b];
      }
      if (digit >= 0) {  // exactly one lane holds the K-th key's digit
        sel[0] = (sel[0] << 8) | (uint64_t)digit;
        sel[1] = left;
        sel[2] = hist[digit];
      }
      if (tid == 0) nfew = 0;
    }
    __syncthreads();
    if (pass > 0 && sel[2] <= 64) {  // (block-uniform) a small bin: one wave ranks its keys
      const uint64_t pfx = sel[0];
      const int shb = 8 * pass;
      // (audit: nfew is zeroed by thread 0 before the pick barrier; the
      // adds follow it and wave 0 reads nfew after the barrier below, then
      // the block returns: nfew is never added to again in this launch)
      auto push = [&](uint64_t v) {
        if ((v >> shb) == pfx) few[atomicAdd(&nfew, 1u)] = v;
      };
      if (inreg) {
#pragma unroll
        for (int i = 0; i < RP; ++i)
          if (tid + (uint32_t)i * BD < nsamp) push(xr[i]);
      } else {
        for (uint32_t k = tid; k < nsamp; k += BD) push(x[k]);
      }
      __syncthreads();
      if (tid < 64) {  // the sel[1]-th least of the bin's keys
        const uint32_t nb = nfew, need = (uint32_t)sel[1];
        const uint64_t v = tid < nb ? few[tid] : ~0ull;
        uint32_t lt = 0, le = 0;
        for (uint32_t j = 0; j < nb; j += 4) {  // (4 reads in flight; nb <= 64 = the buffer)
#pragma unroll
          for (uint32_t u = 0; u < 4; ++u) {
            const uint64_t y = few[j + u];
            lt += (uint32_t)(j + u < nb && y < v);
            le += (uint32_t)(j + u < nb && y <= v);
          }
        }
        if (tid < nb && lt < need && need <= le) tseed[o] = v;  // (every lane holding it writes the same)
      }
      return;
    }
  }
  if (tid == 0) tseed[o] = sel[0];
}

hipError_t launch_seed(const uint64_t* smin, uint32_t nsamp, uint32_t n_obj, uint32_t K, uint64_t* tseed,
                       hipStream_t st) {
  hipLaunchKernelGGL(seed_kernel, dim3(n_obj), dim3(1024), 0, st, smin, nsamp, K, tseed);
  return hipGetLastError();
}

hipError_t launch_pick_counters(const unsigned long long* src, const unsigned long long* alt,
                                const unsigned long long* sel, uint64_t cap, uint64_t* dst, hipStream_t st) {
  hipLaunchKernelGGL(pick_counters_kernel, dim3(1), dim3(64), 0, st, src, alt, sel, cap, dst);
  return hipGetLastError();
}

__global__ void sum_counters_kernel(const uint64_t* src, uint32_t n, uint64_t stride, uint64_t off, uint64_t* dst) {
  if (threadIdx.x < 2) {
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; ++i) s += src[i * stride + off + threadIdx.x];
    dst[threadIdx.x] = s;
  }
}

hipError_t launch_sum_counters(const uint64_t* src, uint32_t n, uint64_t stride, uint64_t off, uint64_t* dst,
                               hipStream_t st) {
  hipLaunchKernelGGL(sum_counters_kernel, dim3(1), dim3(64), 0, st, src, n, stride, off, dst);
  return hipGetLastError();
}

hipError_t launch_single(const SingleArgs& a, int mode, hipStream_t st) {
  size_t shm = align_up((size_t)a.R * a.R * 4 + a.R, 16) + (size_t)a.R * 4;
  hipError_t e = hipFuncSetAttribute((const void*)single_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(single_kernel, dim3(1), dim3(256), shm, st, a, mode);
  return hipGetLastError();
}

hipError_t launch_best_leader(const SingleArgs& a, const uint64_t* vals, double* stat, hipStream_t st) {
  hipLaunchKernelGGL(best_leader_kernel, dim3(1), dim3(256), 0, st, a, vals, stat);
  return hipGetLastError();
}

}  // namespace bote
