// bote_host.hpp — host-only pieces of libbote_hip.so (plain C++, no HIP): the
// combinatorics of colex ranks, the group walk behind the cost-balanced work
// chunks and shard splits, the client-quad layouts, the fast-path eligibility
// test and the result-block unpacking.  Compiled by g++ into the library and,
// separately, under ASan/UBSan by tests/test_sanitize.py (tests/native/
// host_check.cpp), so the driver's host code runs under the sanitizers the
// oracle does.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace bote {
namespace host {

// C(m, k) as u64 (0 when k > m or on overflow).
uint64_t binom_u64(uint32_t m, uint32_t k);
// (ns + 1) x (n + 1) table, row m, column k: C(m, k).
std::vector<uint64_t> binom_table(uint32_t ns, uint32_t n);
// rank -> n ascending positions < ns (colex: rank = sum_j C(p_j, j + 1)).
// False when rank >= C(ns, n).
bool colex_unrank(uint64_t rank, uint32_t n, uint32_t ns, uint32_t* out);
uint64_t colex_rank(const uint32_t* pos, uint32_t n);

// ------------------------------------------------------------ group walk --
// Colex ranks of n-subsets sharing their n - 3 largest members form one
// contiguous "group" of C(p3, 3) ranks (bote_group.hip).  The group kernel
// runs a group in ceil(len / 64) wavefront steps plus a per-group precompute
// (group_cost: fitted), so the cost of a rank range is a sum
// over the groups it touches.  A GroupWalk holds the groups of one rank range
// [rb, re), clipped to it, in rank order.
struct GroupWalk {
  uint32_t ns = 0, n = 0, nc = 0;
  uint64_t rb = 0, re = 0;
  double group_cost = 0;
  std::vector<uint64_t> start;  // clipped group start ranks, ascending
  std::vector<uint64_t> len;    // clipped lengths (> 0)
  bool covers(uint64_t b, uint64_t e) const { return rb <= b && e <= re; }
};
// One group's precompute in wavefront steps for nc clients.
double group_cost(uint32_t nc);
// Walk the groups of [rb, re).  Null when n < 4, the range is empty or it
// touches more than max_groups groups (callers then split ranks evenly).
std::shared_ptr<GroupWalk> walk_groups(uint32_t ns, uint32_t n, uint32_t nc, uint64_t rb, uint64_t re,
                                       uint64_t max_groups = 40000000);
// nchunks + 1 ascending boundaries from b to e cutting [b, e) (inside the
// walk's range) into parts of equal estimated cost; empty if the walk does not
// cover [b, e).
std::vector<uint64_t> cut_chunks(const GroupWalk& w, uint64_t b, uint64_t e, uint32_t nchunks);
// The work-chunk table of a launch (guided): chunks of the base size
// (total / nchunks) for most of the range, then `levels` rounds of
// `tail_waves` chunks each of 1/2, 1/4, ... of it, so that the waves that
// take the last chunks finish close together.  cut_chunks when the launch
// is small (nchunks < 16 tail_waves) or tail_waves == 0.
std::vector<uint64_t> cut_chunks_guided(const GroupWalk& w, uint64_t b, uint64_t e, uint32_t nchunks,
                                        uint32_t tail_waves, uint32_t levels);
// Work chunks per wavefront for a launch of `ranks` configs on `nwaves`
// waves with nc clients: every chunk re-runs its first group's precompute
// (group_cost steps) and the launch ends about one chunk after the mean, so C
// chunks per wave cost C * g + T / C steps for T steps per wave: C = sqrt(T /
// g), between 4 and cap.  (32 per wave on a 1/64 shard of R=64 n=7 spent
// about half of its time in chunk-start precomputes.)
uint32_t chunks_per_wave(uint64_t ranks, uint32_t nwaves, uint32_t nc, uint32_t cap);
// Expected lane utilisation of the group kernel over the whole rank space.
double group_utilisation(uint32_t ns, uint32_t n);
// Group-kernel geometry choice between two workgroup sizes, each with the
// workgroups per CU (occ) and client lines per wave (gslots) it fits: true
// when (bd, occ, gslots) should replace the best so far (best_occ == 0: none).
bool pick_group_geometry(uint32_t bd, int occ, uint32_t gslots, uint32_t best_bd, int best_occ,
                         uint32_t best_gslots);

// ------------------------------------------------------------ layouts ----
// Column-major packed-u16 quad layout of `rows` (client ids) against every
// region t of an R x R matrix (row = from): entry [t][c] = lat[rows[c]][t] <<
// shift, column stride `stride` quads (quad_stride: at least one pad quad).
std::vector<uint16_t> quad_layout(const uint16_t* lat, uint32_t R, const uint32_t* rows, uint32_t nrows,
                                  uint32_t shift, uint32_t& quads, uint32_t& stride);
// Column stride in quads (8 B) for `quads` data quads: at least quads + 1,
// and an odd number of 16-B units, so that a column starts 16-B aligned
// (ds_read_b128 of two quads) and 16 lanes at consecutive columns hit 16
// distinct 4-bank groups (conflict-free 16-B reads, MI355X_MICROARCH.md LDS).
uint32_t quad_stride(uint32_t quads);
// Packed (p0 | p1 << 8 | p2 << 16) 3-subsets of [0, m) in colex order.
std::vector<uint32_t> low_table(uint32_t m);
// The fast path's preconditions (bote_sweep.hip header): every latency <=
// 4095, servers ascending, self latency 0 and server-server latency > 0 among
// the servers, >= 2 clients, and no fairness threshold.
bool fast_eligible(const uint16_t* lat, uint32_t R, const uint32_t* servers, uint32_t ns, uint32_t nc,
                   bool fairness_threshold);

// -------------------------------------------------------- result blocks --
// A result block is [n_obj x kp records {key, rank} (16 B), ascending, padded
// with all-ones records][valid u64][digest u64].  Copies the first K records
// of each objective to out (n_obj x K, padding past the filled ones).
struct TopkRecord {
  uint64_t key, rank;
};
void unpack_result(const uint8_t* blk, uint32_t n_obj, uint32_t K, uint32_t kp, TopkRecord* out, uint32_t* out_count,
                   uint64_t* out_valid, uint64_t* out_digest);

}  // namespace host
}  // namespace bote
