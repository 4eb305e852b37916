// bote_quorums.hip — Bote::leaderless (fantoch_bote/src/lib.rs:38-59) for a
// batch of configurations and several quorum sizes per launch (gfx950).
//
// This carries the protocols whose quorums the reference's compute_stats
// (search.rs:262-319) does not key: Tempo's fast quorum (non-tiny n/2+f, tiny
// 2f) and its write quorum f+1 (fantoch/src/config.rs:317-329), or any other
// leaderless quorum size.  Per configuration and quorum size q it produces the
// per-client latencies of `leaderless(config, clients, q)` (Input placement)
// and `leaderless(config, config, q)` (Colocated, config order) and their exact
// sums and sums of squares.
//
// One lane = one configuration.  Members are sorted by region id (== name
// order), so the packed (latency << 4 | member) minimum is the reference's
// (latency, name) nearest-server order (planet/mod.rs:122-140, lib.rs:169-185);
// the q-th entry of a member's sorted config row is quorum_latency
// (lib.rs:155-163).  Integer work only (VALU + LDS); no MFMA.
#include "bote_kernels.hpp"

namespace bote {

// OR-of-masked-registers select for a lane-varying index (no scratch array)
template <int P>
__device__ __forceinline__ uint32_t pick(const uint32_t (&v)[P], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) r |= v[j] & (0u - (uint32_t)(i == (uint32_t)j));
  return r;
}

template <int N>
__global__ void __launch_bounds__(256) leaderless_q_kernel(LqArgs a) {
  constexpr int P = Pow2<N>::v;
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* mat = (uint32_t*)smem;                    // R*R, latency << 4
  uint32_t* clioff = mat + a.R * a.R;                 // nc
  uint32_t* srv = clioff + a.nc;                      // ns
  uint64_t* binom = (uint64_t*)(((uintptr_t)(srv + a.ns) + 15) & ~(uintptr_t)15);  // (ns+1)(N+1)
  const uint32_t tid = threadIdx.x, BD = blockDim.x;
  for (uint32_t i = tid; i < a.R * a.R; i += BD) mat[i] = a.mat[i];
  for (uint32_t i = tid; i < a.nc; i += BD) clioff[i] = a.cli[i] * a.R;
  for (uint32_t i = tid; i < a.ns; i += BD) srv[i] = a.srv[i];
  if (!a.cfgs)
    for (uint32_t i = tid; i < (a.ns + 1) * (N + 1); i += BD) binom[i] = a.binom[i];
  __syncthreads();

  const uint32_t nc = a.nc, R = a.R;
  for (uint64_t job = (uint64_t)blockIdx.x * BD + tid; job < a.ncfg; job += (uint64_t)gridDim.x * BD) {
    uint32_t p[N];
    if (a.cfgs) {
#pragma unroll
      for (int j = 0; j < N; ++j) p[j] = a.cfgs[job * N + j];
    } else {
      colex_unrank<N>(binom, a.ns, a.rank_begin + job, p);
    }
    // members in name order; morig = position in config order
    uint32_t mk[P];
#pragma unroll
    for (int j = 0; j < N; ++j) mk[j] = (srv[p[j]] << 12) | ((uint32_t)j << 4);
#pragma unroll
    for (int j = N; j < P; ++j) mk[j] = 0xFFFFFFFFu;
    sort_network<P>(mk);
    uint32_t mreg[N], morig[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      mreg[j] = mk[j] >> 12;
      morig[j] = (mk[j] >> 4) & 0xFF;
    }
    const uint32_t vstride = nc + N;
    for (uint32_t qi = 0; qi < a.nq; ++qi) {
      const uint32_t q = a.qs[qi];
      // quorum_latency(member j, config, q): the q-th of row j, self (0) first
      uint32_t Q[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        uint32_t v[P];
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = mat[mreg[j] * R + mreg[k]] >> LAT_SHIFT;
#pragma unroll
        for (int k = N; k < P; ++k) v[k] = 0xFFFFFFFFu;
        sort_network<P>(v);
        Q[j] = pick<P>(v, q - 1);
      }
      uint32_t* ov = a.out_vals ? a.out_vals + (job * a.nq + qi) * vstride : nullptr;
      uint64_t s1[2] = {0, 0}, s2[2] = {0, 0};
      // Input clients, then Colocated (the members, config order)
      for (uint32_t c = 0; c < nc + N; ++c) {
        uint32_t off, slot;
        if (c < nc) {
          off = clioff[c];
          slot = c;
        } else {
          const uint32_t j = c - nc;  // config-order member j
          uint32_t reg = 0;
#pragma unroll
          for (int k = 0; k < N; ++k) reg = morig[k] == j ? mreg[k] : reg;
          off = reg * R;
          slot = c;
        }
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < N; ++k) m = min(m, mat[off + mreg[k]] | (uint32_t)k);
        const uint32_t v = (m >> LAT_SHIFT) + pick<N>(Q, m & 15);
        const int pl = c < nc ? 0 : 1;
        s1[pl] += v;
        s2[pl] += (uint64_t)v * v;
        if (ov) ov[slot] = v;
      }
      if (a.out_sum) {
        a.out_sum[(job * a.nq + qi) * 2] = s1[0];
        a.out_sum[(job * a.nq + qi) * 2 + 1] = s1[1];
      }
      if (a.out_sumsq) {
        a.out_sumsq[(job * a.nq + qi) * 2] = s2[0];
        a.out_sumsq[(job * a.nq + qi) * 2 + 1] = s2[1];
      }
    }
  }
}

size_t lq_smem_bytes(const LqArgs& a, uint32_t n) {
  size_t o = (size_t)a.R * a.R * 4 + (size_t)a.nc * 4 + (size_t)a.ns * 4;
  o = (o + 15) & ~(size_t)15;
  return o + (a.cfgs ? 0 : (size_t)(a.ns + 1) * (n + 1) * 8);
}

template <int N>
static hipError_t launch_lq_n(const LqArgs& a, uint32_t grid, size_t shm, hipStream_t st) {
  auto k = leaderless_q_kernel<N>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), shm, st, a);
  return hipGetLastError();
}

hipError_t launch_leaderless_q(const LqArgs& a, uint32_t n, uint32_t grid, size_t shm, hipStream_t st) {
  switch (n) {
#define LQ_CASE(NN) case NN: return launch_lq_n<NN>(a, grid, shm, st);
    LQ_CASE(1) LQ_CASE(2) LQ_CASE(3) LQ_CASE(4) LQ_CASE(5) LQ_CASE(6) LQ_CASE(7) LQ_CASE(8) LQ_CASE(9)
    LQ_CASE(10) LQ_CASE(11) LQ_CASE(12) LQ_CASE(13) LQ_CASE(14) LQ_CASE(15) LQ_CASE(16)
#undef LQ_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bote
