// Layout of one rank's IPC-shared xGMI region, shared by the one-shot all-reduce kernel
// (xgmi_allreduce.hip) and the one-launch exchange inside grad_reduce (kernels/reduce_sgd.hip).
//
//   [flag table A: XG_MAX_RANKS x max_blocks words]  step flags of xgmi_allreduce_kernel,
//                                                    row = writer rank, column = its workgroup
//   [flag table B: XG_MAX_RANKS x XP_MAX_BLOCKS words] step flags of the grad_reduce exchange,
//                                                    row = writer rank, column = reduce block
//   [slot 0 | slot 1]                                gradient slots, alternated by step parity
//
// A flag word is written only by its writer rank (remote store over xGMI) and polled only by
// the region's owner (local load).  Element e of a step's gradient lives at slot[par][e].
#pragma once

namespace dnn {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_CHUNK = 1024;       // elements per xgmi_allreduce workgroup
constexpr int XP_MAX_BLOCKS = 128;   // grad_reduce blocks that take part in the exchange

inline long long xg_round_up(long long x, long long m) { return (x + m - 1) / m * m; }
inline int xgmi_max_blocks(long long capacity) { return (int)((capacity + XG_CHUNK - 1) / XG_CHUNK); }
// byte offset of flag table B
inline long long xgmi_xp_flag_off(long long capacity) {
  return xg_round_up((long long)XG_MAX_RANKS * xgmi_max_blocks(capacity) * 4, 256);
}
inline long long xgmi_flag_bytes(long long capacity) {
  return xg_round_up(xgmi_xp_flag_off(capacity) + (long long)XG_MAX_RANKS * XP_MAX_BLOCKS * 4, 4096);
}
inline long long xgmi_slot_bytes(long long capacity) {
  return xg_round_up((long long)xgmi_max_blocks(capacity) * XG_CHUNK * 4, 4096);
}
inline long long xgmi_region_bytes(long long capacity) {
  return xgmi_flag_bytes(capacity) + 2 * xgmi_slot_bytes(capacity);
}

}  // namespace dnn
