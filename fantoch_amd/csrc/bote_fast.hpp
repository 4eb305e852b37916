// bote_fast.hpp — device pieces shared by the two fast-path sweep kernels
// (bote_sweep.hip: every member lane-varying; bote_group.hip: wave-uniform
// fixed members).  Both produce the same per-config results as the exact
// generic kernel (bote_kernels.hip) or defer the config to it.
#pragma once
#include "bote_kernels.hpp"

namespace bote {

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }
__device__ __forceinline__ uint32_t as_u32(us2 x) { return __builtin_bit_cast(uint32_t, x); }

__device__ __forceinline__ uint32_t ld16(const unsigned char* b, uint32_t off) { return *(const uint16_t*)(b + off); }
__device__ __forceinline__ uint32_t ld32(const unsigned char* b, uint32_t off) { return *(const uint32_t*)(b + off); }
__device__ __forceinline__ uint2 ld64(const unsigned char* b, uint32_t off) { return *(const uint2*)(b + off); }

// Deferred configs (COV near-ties) go to the exact generic kernel.
__device__ __forceinline__ void defer_rank(const FastArgs& a, uint64_t rank) {
  unsigned long long q = atomicAdd(a.queue_count, 1ull);
  if (q < a.queue_cap) a.queue[q] = rank;
}

// FPaxos Input moments from the leader column's sums (Bote::leader,
// fantoch_bote/src/lib.rs:67-89): sum_c (L + q) and sum_c (L + q)^2.
__device__ __forceinline__ Mom leader_mom(uint64_t c1, uint64_t c2, uint32_t nc, uint64_t q) {
  return Mom{c1 + (uint64_t)nc * q, c2 + 2ull * q * c1 + (uint64_t)nc * q * q, nc};
}

// compute_score validity (search.rs:421-472), digest and objective keys of one
// evaluated configuration.  `vcol_lead` is V of the leader's column (variance
// is shift invariant, so it is also V of ff1 and ff2).  `thr` holds the
// block's current K-th record per objective (only .key is read).  Returns
// false when a COV decision is within the ambiguity band: the caller defers
// the config and offers nothing to the top-K.
template <int N>
__device__ __forceinline__ bool finish_config(const FastArgs& a, const Mom (&mom)[NSLOT], double vcol_lead,
                                              uint32_t lead_member, uint64_t rank, const Rec* thr, double pnc1,
                                              double pnc2, uint64_t& valid_cnt, uint64_t& digest,
                                              uint64_t (&key)[MAXOBJ], bool (&ok)[MAXOBJ]) {
  using QC = QCfg<N>;
  const uint32_t nc = a.nc;
  bool amb = false;
  bool valid = false;
  const int fcap = min(N / 2, a.ft_metric);
  if (a.want_score && !ABLATE(a, 8)) {
    valid = true;
#pragma unroll
    for (int f = 1; f <= 2; ++f) {
      if (f > fcap) break;
      const Mom& ma = mom[f == 1 ? SLOT_AF1 : SLOT_AF2];
      const Mom& mf = mom[f == 1 ? SLOT_FF1 : SLOT_FF2];
      // fmi >= p1: exact in integers unless the sums meet exactly
      const double D = (double)(int64_t)(mf.s1 - ma.s1);
      bool mok;
      if (a.p_int && D != pnc1) mok = D > pnc1;
      else mok = (mom_mean(mf) - mom_mean(ma)) >= a.p_fmean;
      valid = valid && mok;
      if (valid) {
        // cov_f >= cov_a  <=>  V_f * S1_a^2 >= V_a * S1_f^2
        const double Vf = vcol_lead;
        const double Va = (double)mom_v(ma);
        const double sa = (double)ma.s1 * (double)ma.s1, sf = (double)mf.s1 * (double)mf.s1;
        const double x = Vf * sa, y = Va * sf;
        if (!(Vf == 0.0 && Va == 0.0)) {
          const double d = x - y, tol = 0x1p-32 * fmax(x, y);
          if (fabs(d) <= tol) amb = true;
          valid = valid && d > 0.0;
        }
      }
      if (N == 11 || N == 13) {
        const double De = (double)(int64_t)(mom[SLOT_E].s1 - ma.s1);
        bool eok;
        if (a.p_int && De != pnc2) eok = De > pnc2;
        else eok = (mom_mean(mom[SLOT_E]) - mom_mean(ma)) >= a.p_emean;
        valid = valid && eok;
      }
    }
  }
  if (amb) return false;
  if (valid) ++valid_cnt;
  if (a.want_digest && !ABLATE(a, 16)) {
    uint32_t h = 0;
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl)
      if (QC::maxf >= 2 || (sl % 5 != SLOT_AF2 && sl % 5 != SLOT_FF2)) h = digest_fold(h, sl, mom[sl].s1, mom[sl].s2);
    digest += digest_final(rank, lead_member, h);
  }
  // ---- objective keys
#pragma unroll
  for (int o = 0; o < MAXOBJ; ++o) {
    if (o >= a.n_obj) break;
    const uint32_t kind = a.obj_kind[o], sl = a.obj_slot[o];
    if (kind == OBJ_SCORE) {
      if (!valid) continue;
      // score * nc = sum_f (S1_ff - S1_af) + 30 (S1_e - S1_af) exactly; the
      // f64 score (search.rs:445-468) is within 1e-9 of it, so it is
      // computed only when it may beat the objective's threshold.
      const uint64_t tkey = thr[o].key;
      bool maybe = tkey == ~0ull;
      if (!maybe) {
        const uint64_t ob = ~tkey;  // orderable bits of the threshold score
        const uint64_t bits = (ob >> 63) ? (ob & 0x7FFFFFFFFFFFFFFFull) : ~ob;
        const double tscore = __longlong_as_double((long long)bits);
        int64_t T = 0;
#pragma unroll
        for (int f = 1; f <= 2; ++f) {
          if (f > fcap) break;
          const int64_t a1 = (int64_t)mom[f == 1 ? SLOT_AF1 : SLOT_AF2].s1;
          T += (int64_t)mom[f == 1 ? SLOT_FF1 : SLOT_FF2].s1 - a1 + 30 * ((int64_t)mom[SLOT_E].s1 - a1);
        }
        maybe = !(tscore == tscore) || (double)T >= (tscore - 1e-6) * (double)nc;
      }
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
        ok[o] = true;
        key[o] = ~orderable_f64(score);
      }
      continue;
    }
#pragma unroll
    for (int q = 0; q < NSLOT; ++q) {
      if ((uint32_t)q != sl) continue;
      const Mom& m = mom[q];
      if (kind == OBJ_MEAN) {
        ok[o] = true;
        key[o] = m.s1;
      } else {
        // COV key fl(V / S1^2): divide only when it may beat the threshold
        const uint64_t tk = thr[o].key;
        const double V = (double)mom_v(m), S = (double)m.s1 * (double)m.s1;
        const bool maybe = tk == ~0ull || V <= __longlong_as_double((long long)tk) * S * (1.0 + 0x1p-40);
        if (maybe) {
          ok[o] = true;
          key[o] = cov_key(m);
        }
      }
    }
  }
  return true;
}

}  // namespace bote
