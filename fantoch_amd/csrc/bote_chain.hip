// bote_chain.hip — Search::sorted_evolving_configs on the device (gfx950).
//
// Reference: fantoch_bote/src/search.rs:97-178 (chains n = 3 -> 5 -> ... -> 13),
// super_configs :378-401 (BTreeSet::is_superset), min_mean_decrease :403-419,
// and the final BTreeMap<F64, Vec<_>> order: score descending, chains of equal
// score in enumeration order.
//
// Levels l = 0..5 hold the ranked (valid) configs of n = 3 + 2l in the order
// the host enumerated them, as position bitmasks of the server list.  A chain
// prefix ending at config M of level l extends by every config of level l+1
// that contains M: those are M plus two positions, so instead of scanning the
// whole next level each prefix enumerates its C(ns - n, 2) supersets and
// finds them by binary search in the level's mask-sorted index (integer
// bitmask work: VALU + LDS-free global reads, no MFMA).  Extensions are
// written in enumeration order (count pass, exclusive scan, emit pass, then a
// per-prefix insertion sort of its segment), so chain index order is the
// reference's nested-loop order; the final ordering is a stable radix sort on
// ~orderable(score), which keeps equal scores in that order.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "bote_kernels.hpp"

namespace bote {

struct LevelDev {
  const uint64_t* mask;     // [cnt] masks in enumeration order
  const double* score;      // [cnt]
  const double* mean;       // [cnt][2] Atlas Input mean f=1, f=2
  const uint64_t* smask;    // [cnt] masks sorted ascending
  const uint32_t* sidx;     // [cnt] enumeration index of smask[i]
  uint32_t cnt;
  uint32_t n;
};

__device__ __forceinline__ int64_t find_mask(const LevelDev& L, uint64_t m) {
  uint32_t lo = 0, hi = L.cnt;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint64_t v = L.smask[mid];
    if (v < m) lo = mid + 1;
    else hi = mid;
  }
  return (lo < L.cnt && L.smask[lo] == m) ? (int64_t)L.sidx[lo] : -1;
}

// search.rs:403-419: compare only for the f values of n - 2
__device__ __forceinline__ bool mean_decrease_ok(const LevelDev& prev, uint32_t pi, const LevelDev& cur, uint32_t ci,
                                                 uint32_t n, int ft_metric, double min_dec) {
  const uint32_t m = n - 2;
  const uint32_t fmax = min(m / 2, (uint32_t)ft_metric);
  for (uint32_t f = 1; f <= fmax; ++f) {
    const double d = prev.mean[2 * pi + f - 1] - cur.mean[2 * ci + f - 1];
    if (!(d >= min_dec)) return false;
  }
  return true;
}

// One thread per prefix: enumerate the supersets of its last config in the
// next level.  EMIT = false: count them; EMIT = true: write (parent, index,
// partial score) at the prefix's offset, then sort the segment by index.
template <bool EMIT>
__global__ void __launch_bounds__(256) chain_join_kernel(LevelDev prev, LevelDev cur, const uint32_t* plast,
                                                         const double* pscore, uint64_t nprefix, uint32_t ns,
                                                         int ft_metric, double min_dec, uint32_t* count,
                                                         const uint64_t* offset, uint32_t* out_parent,
                                                         uint32_t* out_last, double* out_score) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nprefix) return;
  const uint32_t last = plast[k];
  const uint64_t M = prev.mask[last];
  uint32_t c = 0;
  const uint64_t base = EMIT ? offset[k] : 0;
  for (uint32_t a = 0; a < ns; ++a) {
    if (M >> a & 1) continue;
    for (uint32_t b = a + 1; b < ns; ++b) {
      if (M >> b & 1) continue;
      const int64_t j = find_mask(cur, M | (1ull << a) | (1ull << b));
      if (j < 0 || !mean_decrease_ok(prev, last, cur, (uint32_t)j, cur.n, ft_metric, min_dec)) continue;
      if (EMIT) {
        out_parent[base + c] = (uint32_t)k;
        out_last[base + c] = (uint32_t)j;
      }
      ++c;
    }
  }
  if (!EMIT) {
    count[k] = c;
    return;
  }
  // enumeration order inside the segment (the reference iterates the next
  // level's ranked list in order): insertion sort by index
  for (uint32_t i = 1; i < c; ++i) {
    const uint32_t x = out_last[base + i];
    uint32_t j = i;
    while (j > 0 && out_last[base + j - 1] > x) {
      out_last[base + j] = out_last[base + j - 1];
      --j;
    }
    out_last[base + j] = x;
  }
  // partial score, summed in the reference's order: s3 + s5 + ... (search.rs:146-151)
  for (uint32_t i = 0; i < c; ++i) out_score[base + i] = pscore[k] + cur.score[out_last[base + i]];
}

__global__ void chain_seed_kernel(LevelDev L, uint32_t* last, double* score) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L.cnt) return;
  last[i] = i;
  score[i] = L.score[i];
}

__global__ void chain_keys_kernel(const double* score, uint64_t n, uint64_t* key, uint32_t* val) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double s = score[i] + 0.0;  // F64 equality: -0.0 == 0.0 (-0.0 + 0.0 = +0.0)
  key[i] = ~orderable_f64(s);  // ascending key = descending score; NaN (greatest) first
  val[i] = (uint32_t)i;
}

// Walk the parent pointers of the first `nout` sorted chains.
__global__ void chain_gather_kernel(const uint32_t* order, uint64_t nout, const uint32_t* const* parent,
                                    const uint32_t* const* last, const double* score, uint32_t* out_idx,
                                    double* out_score) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nout) return;
  uint32_t c = order[i];
  out_score[i] = score[c];
  for (int l = 5; l >= 0; --l) {
    out_idx[i * 6 + l] = last[l][c];
    if (l > 0) c = parent[l][c];
  }
}

// ------------------------------------------------------------------ host --

hipError_t chain_search(const ChainHostLevel* lv, uint32_t ns, int ft_metric, double min_dec, uint64_t max_out,
                        uint32_t* out_idx, double* out_score, uint64_t* out_total, hipStream_t st, int* too_many) {
  *too_many = 0;
  *out_total = 0;
  std::vector<void*> owned;
  auto dalloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
    owned.push_back(p);
    return p;
  };
  auto cleanup = [&](hipError_t e) {
    (void)hipStreamSynchronize(st);
    for (void* p : owned) (void)hipFree(p);
    return e;
  };
#define CH_TRY(x)                      \
  do {                                 \
    hipError_t _e = (x);               \
    if (_e != hipSuccess) return cleanup(_e); \
  } while (0)
  LevelDev L[6];
  for (int l = 0; l < 6; ++l) {
    const uint32_t c = lv[l].cnt;
    L[l].cnt = c;
    L[l].n = lv[l].n;
    // host-side mask sort for the lookup index
    std::vector<std::pair<uint64_t, uint32_t>> srt(c);
    for (uint32_t i = 0; i < c; ++i) srt[i] = {lv[l].mask[i], i};
    std::sort(srt.begin(), srt.end());
    std::vector<uint64_t> sm(c);
    std::vector<uint32_t> si(c);
    for (uint32_t i = 0; i < c; ++i) {
      sm[i] = srt[i].first;
      si[i] = srt[i].second;
    }
    uint64_t* dm = (uint64_t*)dalloc(c * 8);
    double* ds = (double*)dalloc(c * 8);
    double* dmean = (double*)dalloc(c * 16);
    uint64_t* dsm = (uint64_t*)dalloc(c * 8);
    uint32_t* dsi = (uint32_t*)dalloc(c * 4);
    if (!dm || !ds || !dmean || !dsm || !dsi) return cleanup(hipErrorOutOfMemory);
    if (c) {
      CH_TRY(hipMemcpyAsync(dm, lv[l].mask, c * 8, hipMemcpyHostToDevice, st));
      CH_TRY(hipMemcpyAsync(ds, lv[l].score, c * 8, hipMemcpyHostToDevice, st));
      CH_TRY(hipMemcpyAsync(dmean, lv[l].mean, c * 16, hipMemcpyHostToDevice, st));
      CH_TRY(hipMemcpyAsync(dsm, sm.data(), c * 8, hipMemcpyHostToDevice, st));
      CH_TRY(hipMemcpyAsync(dsi, si.data(), c * 4, hipMemcpyHostToDevice, st));
      CH_TRY(hipStreamSynchronize(st));  // the host vectors die at the end of this iteration
    }
    L[l].mask = dm;
    L[l].score = ds;
    L[l].mean = dmean;
    L[l].smask = dsm;
    L[l].sidx = dsi;
  }
  // level 0: every ranked n = 3 config starts a chain
  uint32_t* parent[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  uint32_t* last[6];
  double* score[6];
  uint64_t np = L[0].cnt;
  last[0] = (uint32_t*)dalloc(np * 4);
  score[0] = (double*)dalloc(np * 8);
  if (!last[0] || !score[0]) return cleanup(hipErrorOutOfMemory);
  if (np) hipLaunchKernelGGL(chain_seed_kernel, dim3((np + 255) / 256), dim3(256), 0, st, L[0], last[0], score[0]);
  CH_TRY(hipGetLastError());
  for (int l = 1; l < 6; ++l) {
    uint32_t* cnt = (uint32_t*)dalloc(np * 4 + 4);
    uint64_t* off = (uint64_t*)dalloc(np * 8 + 8);
    if (!cnt || !off) return cleanup(hipErrorOutOfMemory);
    uint64_t total = 0;
    if (np) {
      hipLaunchKernelGGL(chain_join_kernel<false>, dim3((np + 255) / 256), dim3(256), 0, st, L[l - 1], L[l], last[l - 1],
                         score[l - 1], np, ns, ft_metric, min_dec, cnt, (const uint64_t*)nullptr, (uint32_t*)nullptr,
                         (uint32_t*)nullptr, (double*)nullptr);
      CH_TRY(hipGetLastError());
      // exclusive scan of the counts (64-bit offsets)
      size_t tmp_bytes = 0;
      CH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, np + 1, st));
      void* tmp = dalloc(tmp_bytes);
      if (!tmp) return cleanup(hipErrorOutOfMemory);
      CH_TRY(hipMemsetAsync(cnt + np, 0, 4, st));
      CH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, np + 1, st));
      CH_TRY(hipMemcpyAsync(&total, off + np, 8, hipMemcpyDeviceToHost, st));
      CH_TRY(hipStreamSynchronize(st));
    }
    if (total > 0x7FFFFFFFull) {  // u32 parent pointers, int radix-sort sizes
      *too_many = 1;
      return cleanup(hipSuccess);
    }
    parent[l] = (uint32_t*)dalloc(total * 4);
    last[l] = (uint32_t*)dalloc(total * 4);
    score[l] = (double*)dalloc(total * 8);
    if (!parent[l] || !last[l] || !score[l]) return cleanup(hipErrorOutOfMemory);
    if (total) {
      hipLaunchKernelGGL(chain_join_kernel<true>, dim3((np + 255) / 256), dim3(256), 0, st, L[l - 1], L[l], last[l - 1],
                         score[l - 1], np, ns, ft_metric, min_dec, cnt, off, parent[l], last[l], score[l]);
      CH_TRY(hipGetLastError());
    }
    np = total;
  }
  *out_total = np;
  const uint64_t nout = std::min<uint64_t>(np, max_out);
  if (nout) {
    uint64_t* key = (uint64_t*)dalloc(np * 8);
    uint64_t* key2 = (uint64_t*)dalloc(np * 8);
    uint32_t* val = (uint32_t*)dalloc(np * 4);
    uint32_t* val2 = (uint32_t*)dalloc(np * 4);
    uint32_t* didx = (uint32_t*)dalloc(nout * 24);
    double* dsc = (double*)dalloc(nout * 8);
    const uint32_t** dpar = (const uint32_t**)dalloc(6 * sizeof(void*));
    const uint32_t** dlast = (const uint32_t**)dalloc(6 * sizeof(void*));
    if (!key || !key2 || !val || !val2 || !didx || !dsc || !dpar || !dlast) return cleanup(hipErrorOutOfMemory);
    hipLaunchKernelGGL(chain_keys_kernel, dim3((np + 255) / 256), dim3(256), 0, st, score[5], np, key, val);
    CH_TRY(hipGetLastError());
    size_t tmp_bytes = 0;
    CH_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, key, key2, val, val2, (int)np, 0, 64, st));
    void* tmp = dalloc(tmp_bytes);
    if (!tmp) return cleanup(hipErrorOutOfMemory);
    CH_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key, key2, val, val2, (int)np, 0, 64, st));
    CH_TRY(hipMemcpyAsync(dpar, parent, 6 * sizeof(void*), hipMemcpyHostToDevice, st));
    CH_TRY(hipMemcpyAsync(dlast, last, 6 * sizeof(void*), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(chain_gather_kernel, dim3((nout + 255) / 256), dim3(256), 0, st, val2, nout, dpar, dlast,
                       score[5], didx, dsc);
    CH_TRY(hipGetLastError());
    CH_TRY(hipMemcpyAsync(out_idx, didx, nout * 24, hipMemcpyDeviceToHost, st));
    CH_TRY(hipMemcpyAsync(out_score, dsc, nout * 8, hipMemcpyDeviceToHost, st));
  }
  return cleanup(hipSuccess);
#undef CH_TRY
}

}  // namespace bote
