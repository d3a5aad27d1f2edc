// Layout of one rank's IPC-shared xGMI region, shared by the one-shot all-reduce kernel
// (xgmi_allreduce.hip, the two-launch path) and the one-launch exchange inside grad_reduce
// (kernels/reduce_sgd.hip).
//
//   [flag table: XG_MAX_RANKS x max_blocks words]  step flags of xgmi_allreduce_kernel,
//                                                  row = writer rank, column = its workgroup
//   [slot 0 | slot 1]                              fp32 gradient slots of the two-launch path,
//                                                  alternated by step parity
//   [granule slot 0 | granule slot 1]              one 8-byte granule per arena element for the
//                                                  one-launch exchange: {fp32 value, step tag},
//                                                  written by ONE 64-bit store, so a reader that
//                                                  sees the tag also sees the value (no flag, no
//                                                  ordering between two stores to rely on)
//
// A flag word is written only by its writer rank (remote store over xGMI) and polled only by
// the region's owner (local load); a granule is written only by the region's owner and read
// by the peers (remote loads).
#pragma once

namespace dnn {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_CHUNK = 1024;       // elements per xgmi_allreduce workgroup
constexpr int XP_MAX_BLOCKS = 128;   // grad_reduce blocks that take part in the exchange (counters)

inline long long xg_round_up(long long x, long long m) { return (x + m - 1) / m * m; }
inline int xgmi_max_blocks(long long capacity) { return (int)((capacity + XG_CHUNK - 1) / XG_CHUNK); }
inline long long xgmi_flag_bytes(long long capacity) {
  return xg_round_up((long long)XG_MAX_RANKS * xgmi_max_blocks(capacity) * 4, 4096);
}
inline long long xgmi_slot_bytes(long long capacity) {
  return xg_round_up((long long)xgmi_max_blocks(capacity) * XG_CHUNK * 4, 4096);
}
// granule slots of the one-launch exchange
inline long long xgmi_gslot_off(long long capacity) {
  return xgmi_flag_bytes(capacity) + 2 * xgmi_slot_bytes(capacity);
}
inline long long xgmi_gslot_bytes(long long capacity) { return xg_round_up(capacity * 8, 4096); }
inline long long xgmi_region_bytes(long long capacity) {
  return xgmi_gslot_off(capacity) + 2 * xgmi_gslot_bytes(capacity);
}

}  // namespace dnn
