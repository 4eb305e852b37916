// bote_kernels.hpp — launch interface between the C ABI (bote_capi.hip) and
// the gfx950 kernels (bote_kernels.hip).
#pragma once
#include "bote_device.hpp"

namespace bote {

constexpr int NSLOT = 10;
constexpr int G_MERGE_LISTS = 8;  // lists merged per workgroup
enum { SLOT_AF1 = 0, SLOT_FF1 = 1, SLOT_AF2 = 2, SLOT_FF2 = 3, SLOT_E = 4 };
enum { OBJ_SCORE = 0, OBJ_MEAN = 1, OBJ_COV = 2 };

struct EvalArgs {
  // planet (device): latency << 4, row = from
  const uint32_t* mat;
  uint32_t R;
  // server list (region ids; positions index it) and client list
  const uint32_t* srv;
  uint32_t ns;
  const uint32_t* cli;
  uint32_t nc;
  int srv_sorted;  // srv ascending => colex positions are already in name order
  // work: explicit configs (positions, n per config) or colex ranks
  const uint32_t* cfgs;
  uint64_t rb, re;  // [rb, re) ranks, or config indices when cfgs != null
  uint32_t runlen;  // consecutive ranks per lane job
  const uint64_t* binom;  // (ns+1) x (n+1)
  // ranking params (compute_score)
  int want_score;
  double p_fmean, p_emean, p_fair;
  int ft_metric;
  // FULL outputs
  uint32_t* out_vals;
  uint32_t* out_leader;
  uint64_t* out_s1;
  uint64_t* out_s2;
  double* out_mean;
  double* out_cov;
  double* out_score;
  uint8_t* out_valid;
  // TOP-K outputs
  int n_obj;
  uint32_t obj_kind[MAXOBJ];
  uint32_t obj_slot[MAXOBJ];
  uint32_t K;
  Rec* out_top;                      // [grid][n_obj][KP]
  unsigned long long* out_counters;  // [0] valid count, [1] digest
  int want_digest;
};

struct SingleArgs {
  const uint32_t* mat;  // latency << 4
  uint32_t R;
  const uint32_t* servers;
  uint32_t ns;
  const uint32_t* clients;
  uint32_t nc;
  const uint32_t* froms;
  uint32_t nf;
  uint32_t q;
  uint32_t leader;
  int stat;
  uint64_t* out;
  uint32_t* out_pos;
  int* err;
};

size_t eval_smem_bytes(const EvalArgs& a, uint32_t n, uint32_t bd, bool topk);
int eval_occupancy(uint32_t n, bool full, uint32_t bd, size_t shm);
hipError_t launch_eval(const EvalArgs& a, uint32_t n, bool full, uint32_t grid, uint32_t bd, size_t shm,
                       hipStream_t st);
hipError_t launch_merge(const Rec* src, uint32_t n_lists, uint64_t list_stride, Rec* dst, uint64_t out_stride,
                        uint32_t n_obj, hipStream_t st);

hipError_t launch_sum_counters(const uint64_t* src, uint32_t n, uint64_t stride, uint64_t off, uint64_t* dst,
                               hipStream_t st);
hipError_t launch_single(const SingleArgs& a, int mode, hipStream_t st);
hipError_t launch_best_leader(const SingleArgs& a, const uint64_t* vals, double* stat, hipStream_t st);

}  // namespace bote
