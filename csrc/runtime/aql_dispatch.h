// Direct AQL dispatch: a user-mode HSA queue of this process's own, for launches whose cost is
// the runtime's launch + completion path rather than the kernel (the persistent training window).
//
// The bench's 20-step window is ONE persistent kernel of ~310 us, yet it paid ~26 us more than
// its steps: a graph of one trivial kernel costs the same ~25 us from replay to the synchronize's
// return (profiles/r6/window/hostprobe.json).  Here the host writes the kernel dispatch packet
// itself into a queue it created (hsa_queue_create on the HIP device's agent), rings the doorbell
// and spins on the packet's completion signal: no stream, marker or interrupt in the path.
//
// The kernel object is the one the HIP runtime loaded for the device (found through the AMD
// loader extension by the kernel's name), so both paths run the very same code.  Kernel
// arguments are the kernel's explicit parameter block (the caller's struct, checked against the
// symbol's kernarg segment size).  A dispatch is synchronous: run() returns once the packet's
// completion signal reached 0, so the HIP stream work before it must be finished (the caller
// checks) and HIP work after it is ordered by program order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace dnn {

struct AqlKernel {
  uint64_t object = 0;         // kernel descriptor address (HSA kernel object)
  uint32_t group_static = 0;   // static LDS bytes
  uint32_t private_bytes = 0;  // scratch per work-item
  uint32_t kernarg_bytes = 0;  // explicit (+ hidden) kernarg segment size
  std::string name;
};

class AqlQueue;

// The queue of HIP device `hip_device` (created on first use; nullptr + *why if this process
// cannot have one: no HSA agent with the device's PCI address, queue creation refused, ...).
AqlQueue* aql_queue(int hip_device, std::string* why = nullptr);

// The HSA kernel object of a kernel the HIP runtime loads for the queue's device: host_fn is the
// kernel's host stub (hipFuncGetAttributes on it makes HIP load the code object first), name_part
// a substring that must match exactly one kernel symbol of the device's executables.
AqlKernel aql_kernel(AqlQueue* q, const void* host_fn, const char* name_part);

// Dispatch (1-D grid of grid_x workgroups of block_x work-items, dyn_lds bytes of dynamic LDS)
// and wait for completion (spin, bounded by timeout_s: an overrun throws and leaves the queue
// unusable).  args / bytes: the explicit parameter block - host memory (copied into the queue's
// kernarg buffer), or with args_on_device a 16-B aligned device-memory copy the packet points at
// (HIP's own placement: a kernel that re-reads its arguments pays host-link latency otherwise).
void aql_run(AqlQueue* q, const AqlKernel& k, const void* args, size_t bytes, unsigned grid_x, unsigned block_x,
             unsigned dyn_lds, double timeout_s, bool args_on_device = false);
// aql_run's halves: dispatch (returns after the doorbell) and wait (no-op if nothing is in flight)
void aql_dispatch(AqlQueue* q, const AqlKernel& k, const void* args, size_t bytes, unsigned grid_x,
                  unsigned block_x, unsigned dyn_lds, double timeout_s, bool args_on_device = false);
void aql_wait(AqlQueue* q);

// Prepared launches (the AQL counterpart of a captured graph): the kernel object of host_fn
// (aql_kernel on the current HIP device's queue, cached per device and name), its explicit
// parameter block copied once into device memory (checked against the symbol's kernarg size) and
// the launch shape.  Returns a handle for aql_prepared_run.  Throws if the device has no queue.
int aql_prepare(const void* host_fn, const char* name_part, const void* args, size_t bytes, unsigned grid_x,
                unsigned block_x, unsigned dyn_lds, double timeout_s, hipStream_t stream);
// Run a prepared launch: after the stream's earlier work (one query; a synchronize if it is busy),
// dispatch and wait for completion.  Refuses a stream that is being captured.
void aql_prepared_run(int handle);
// The same in two halves, so host work can overlap the kernel: launch returns after the doorbell,
// wait spins until it completed (one dispatch in flight per queue: a second launch before the
// wait throws).  Nothing but wait orders later HIP work after the kernel.
void aql_prepared_launch(int handle);
void aql_prepared_wait(int handle);

// Host-clock microseconds of the last aql_run: doorbell -> completion seen, and the whole call.
double aql_last_us(AqlQueue* q, bool whole = false);

}  // namespace dnn
