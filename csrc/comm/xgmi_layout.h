// Layout of one rank's IPC-shared xGMI region, shared by the one-launch exchange inside
// grad_reduce (kernels/reduce_sgd.hip) and the one-shot all-reduce kernel
// (xgmi_allreduce.hip: the two-launch fallback and the layer engine's all-reduce).
//
//   [slot 0 | slot 1]        granules of xgmi_allreduce_kernel (step = its per-workgroup counters)
//   [slot 0 | slot 1]        granules of the grad_reduce exchange (step = its per-block counters)
//   [ag: parity]             all-gather slot of the two-hop form: the owner of an element stores
//                            the rank-order sum {sum, step} here, the other ranks read it
//
// A granule is one 8-byte word per element: {fp32 value, step}, written by ONE 64-bit store
// of the region's owner and read by the peers (remote loads); slots alternate by step parity.
// A reader that sees the tag also sees the value - no flag, and no ordering between two stores
// to rely on.  The two paths count steps independently, so each has its own slots (a tag of
// one could otherwise match a stale granule of the other).
#pragma once

namespace dnn {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_CHUNK = 1024;       // elements per xgmi_allreduce workgroup
constexpr int XP_MAX_BLOCKS = 128;   // grad_reduce blocks that take part in the exchange (counters)
constexpr int XP_WAIT_RING = 1024;   // per-step exchange-wait records (launchers.h ReduceArgs::xp_wait)

inline long long xg_round_up(long long x, long long m) { return (x + m - 1) / m * m; }
inline int xgmi_max_blocks(long long capacity) { return (int)((capacity + XG_CHUNK - 1) / XG_CHUNK); }
inline long long xgmi_gslot_bytes(long long capacity) { return xg_round_up(capacity * 8, 4096); }
inline long long xgmi_xp_off(long long capacity) { return 2 * xgmi_gslot_bytes(capacity); }  // exchange slots
inline long long xgmi_ag_off(long long capacity) { return 4 * xgmi_gslot_bytes(capacity); }
inline long long xgmi_region_bytes(long long capacity) { return 6 * xgmi_gslot_bytes(capacity); }

}  // namespace dnn
