// pybind11 bindings of the gfx950 kernels.  Device pointers and HIP streams cross
// the boundary as integers (tensor.data_ptr(), torch.cuda.Stream.cuda_stream), so the
// extension does not depend on libtorch's C++ ABI and launches onto whatever stream
// python (or a hipGraph capture) is using.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <tuple>
#include <vector>
#include <string>

#include "comm/xgmi_layout.h"
#include "kernels/launchers.h"
#include "runtime/aql_dispatch.h"



namespace dnn {
int rccl_open(const std::string& path);
std::string rccl_unique_id();
uintptr_t rccl_init(const std::string& id_bytes, int nranks, int rank, int device, int blocking, double timeout_s);
void rccl_allreduce(uintptr_t comm, uintptr_t buf, size_t count, int dtype, int op, uintptr_t stream);
void rccl_broadcast(uintptr_t comm, uintptr_t buf, size_t count, int root, uintptr_t stream);
int rccl_async_error(uintptr_t comm);
void rccl_abort(uintptr_t comm);
void rccl_destroy(uintptr_t comm);
// one-shot xGMI all-reduce (comm/xgmi_allreduce.hip)
std::tuple<uintptr_t, std::string, std::string> xgmi_alloc(long long capacity);
uintptr_t uncached_alloc(long long bytes);
void uncached_free(uintptr_t p);
std::tuple<long long, long long, long long> uncached_pool_stats();
void lds_poison(unsigned pattern, hipStream_t stream);
void lds_squat(int bytes, double spin_us, int blocks, uintptr_t bad, hipStream_t stream);
bool aql_selftest(std::string* why);
uintptr_t xgmi_open(const std::string& handle);
void xgmi_close(uintptr_t p);
std::string xgmi_device_id();
void xgmi_free(uintptr_t p);
std::pair<uintptr_t, uintptr_t> xgmi_abort_word();
void xgmi_set_abort(uintptr_t host_word, unsigned v);
void xgmi_free_abort_word(uintptr_t host_word);
void launch_xgmi_allreduce(const std::vector<uintptr_t>& regions, int rank, long long capacity, int n,
                           const float* grad, float* out, float* master, float* mom, bf16* shadow, float lr,
                           float momentum, float scale, int mode, unsigned* ctr, const unsigned* abort_w,
                           double timeout_s, hipStream_t stream, int form, unsigned long long* wait);
}  // namespace dnn

namespace py = pybind11;
using u = uintptr_t;

template <typename T>
static T* P(u x) { return reinterpret_cast<T*>(x); }
static hipStream_t S(u x) { return reinterpret_cast<hipStream_t>(x); }
// pipelined step: grad_reduce(defer=2) stores the previous step's reduction for the next
// fused_train_pipe launch
static dnn::ReduceArgs g_pending_pipe{};
static bool g_pending_pipe_set = false;

PYBIND11_MODULE(_dnn_hip, m) {
  m.doc() = "MI355X (gfx950) HIP kernels for the data-parallel CIFAR-10 CNN engine";
  m.def("layout", []() {
    py::dict d;
    d["conv1.weight"] = dnn::OFF_C1W; d["conv1.bias"] = dnn::OFF_C1B;
    d["conv2.weight"] = dnn::OFF_C2W; d["conv2.bias"] = dnn::OFF_C2B;
    d["fc1.weight"] = dnn::OFF_F1W; d["fc1.bias"] = dnn::OFF_F1B;
    d["fc2.weight"] = dnn::OFF_F2W; d["fc2.bias"] = dnn::OFF_F2B;
    d["fc3.weight"] = dnn::OFF_F3W; d["fc3.bias"] = dnn::OFF_F3B;
    d["arena"] = dnn::ARENA; d["slab"] = dnn::SLAB; d["shadow_total"] = dnn::SH_TOTAL;
    d["sh_w1f"] = dnn::SH_W1F; d["sh_w2f"] = dnn::SH_W2F; d["sh_wf"] = dnn::SH_WF;
    d["sh_w2t"] = dnn::SH_W2T; d["sh_w3t"] = dnn::SH_W3T;
    return d;
  });
  m.def("fused_train",
        [](u images, u labels, u order, int order_len, int batch, u state, u master, u shadow, u a0, u h1, u h2,
           u z1, u z2, u z3, u slab, u loss, u correct, u stream, u stamps, u next_ids, u stage, u codes) {
          dnn::launch_fused_train(P<const uint8_t>(images), P<const int32_t>(labels), P<const int32_t>(order),
                                  order_len, batch, P<int32_t>(state), P<const float>(master),
                                  P<const bf16>(shadow), P<float>(a0), P<float>(h1), P<float>(h2), P<float>(z1),
                                  P<float>(z2), P<float>(z3), P<float>(slab), P<float>(loss), P<int32_t>(correct),
                                  P<long long>(stamps), P<const int32_t>(next_ids), P<unsigned char>(stage),
                                  S(stream), P<uint8_t>(codes));
        },
        py::arg("images"), py::arg("labels"), py::arg("order"), py::arg("order_len"), py::arg("batch"),
        py::arg("state"), py::arg("master"), py::arg("shadow"), py::arg("a0"), py::arg("h1"), py::arg("h2"),
        py::arg("z1"), py::arg("z2"), py::arg("z3"), py::arg("slab"), py::arg("loss"), py::arg("correct"),
        py::arg("stream"), py::arg("stamps") = 0, py::arg("next_ids") = 0, py::arg("stage") = 0,
        py::arg("codes") = 0);
  m.def("fused_train_f32", [](u images, u labels, u order, int order_len, int batch, u state, u master, u a0, u h1,
                              u h2, u z1, u z2, u z3, u slab, u loss, u correct, u stream, u stamps) {
    dnn::launch_fused_train_f32(P<const uint8_t>(images), P<const int32_t>(labels), P<const int32_t>(order), order_len,
                                batch, P<const int32_t>(state), P<const float>(master), P<float>(a0), P<float>(h1),
                                P<float>(h2), P<float>(z1), P<float>(z2), P<float>(z3), P<float>(slab), P<float>(loss),
                                P<int32_t>(correct), S(stream), P<long long>(stamps));
  }, py::arg("images"), py::arg("labels"), py::arg("order"), py::arg("order_len"), py::arg("batch"), py::arg("state"),
     py::arg("master"), py::arg("a0"), py::arg("h1"), py::arg("h2"), py::arg("z1"), py::arg("z2"), py::arg("z3"),
     py::arg("slab"), py::arg("loss"), py::arg("correct"), py::arg("stream"), py::arg("stamps") = 0);
  m.def("fused_eval_f32", [](u images, u labels, int n, int base, int count, u master, u loss, u correct, u stream) {
    dnn::launch_fused_eval_f32(P<const uint8_t>(images), P<const int32_t>(labels), n, base, count,
                               P<const float>(master), P<float>(loss), P<int32_t>(correct), S(stream));
  });
  m.def("fused_eval", [](u images, u labels, u order, int n, int base, int count, u master, u shadow, u loss,
                         u correct, u stream) {
    dnn::launch_fused_eval(P<const uint8_t>(images), P<const int32_t>(labels), P<const int32_t>(order), n, base,
                           count, P<const float>(master), P<const bf16>(shadow), P<float>(loss), P<int32_t>(correct),
                           S(stream));
  });
  m.def("grad_reduce", [](u a0, u h1, u h2, u z1, u z2, u z3, u slab, u loss, u correct, int batch, u master,
                          u grad, u mom, u shadow, u state, u stats, float lr, float momentum, float grad_scale,
                          int fuse_sgd, int lo, int hi, int bookkeeping, u order, int order_len, u batch_ids,
                          u stream, u stamps, const std::vector<u>& xp_regions, int xp_rank, long long xp_capacity, u xp_ctr,
                          u xp_err, u xp_abort, double xp_timeout_s, float xp_scale, u next_ids, int xp_mode,
                          u xp_wait, int defer, u bk_bv_in,
                          u bk_bv_out, int bk_adv, int bk_stats) {
    dnn::ReduceArgs a{P<const float>(a0), P<const float>(h1), P<const float>(h2), P<const float>(z1),
                      P<const float>(z2), P<const float>(z3), P<const float>(slab), P<const float>(loss),
                      P<const int32_t>(correct), batch, P<float>(master), P<float>(grad), P<float>(mom),
                      P<bf16>(shadow), P<int32_t>(state), P<double>(stats), P<const int32_t>(order), order_len,
                      P<int32_t>(batch_ids), lr, momentum, grad_scale, fuse_sgd, lo, hi, bookkeeping,
                      P<long long>(stamps)};
    a.next_ids = P<int32_t>(next_ids);
    a.bk_bv_in = P<const int32_t>(bk_bv_in);
    a.bk_bv_out = P<int32_t>(bk_bv_out);
    if (bk_adv < 0 || bk_adv > 1) throw std::runtime_error("grad_reduce: bk_adv is 0 or 1");
    a.bk_adv = bk_adv;
    a.bk_stats = bk_stats;
    if (!xp_regions.empty()) {
      if ((int)xp_regions.size() > dnn::XG_MAX_RANKS || xp_rank < 0 || xp_rank >= (int)xp_regions.size())
        throw std::runtime_error("grad_reduce exchange: 1..8 ranks, rank in range");
      // the exchange takes the whole arena (every block's elements have one step counter)
      if (!(lo == 0 && hi >= dnn::ARENA) || xp_capacity < dnn::ARENA || !xp_ctr || !xp_err || !xp_abort)
        throw std::runtime_error("grad_reduce exchange: the whole arena, region capacity >= arena, counters set");
      for (size_t r = 0; r < xp_regions.size(); ++r) a.xp_region[r] = P<unsigned char>(xp_regions[r]);
      a.xp_rank = xp_rank;
      a.xp_nranks = (int)xp_regions.size();
      a.xp_ctr = P<unsigned>(xp_ctr);
      a.xp_err = P<unsigned>(xp_err);
      a.xp_abort = P<const unsigned>(xp_abort);
      a.xp_timeout_ticks = (long long)(xp_timeout_s * 1.0e8);
      a.xp_scale = xp_scale;
      a.xp_gslot_off = dnn::xgmi_xp_off(xp_capacity);
      a.xp_gslot_bytes = dnn::xgmi_gslot_bytes(xp_capacity);
      if (xp_mode < 0 || xp_mode > 6 || (xp_mode & 1))
        throw std::runtime_error("grad_reduce exchange: xp_mode 0 (pull) or 2 (two-hop pull), + 4 for bf16 granules");
      a.xp_mode = xp_mode;
      a.xp_ag_off = dnn::xgmi_ag_off(xp_capacity);
      a.xp_wait = P<unsigned long long>(xp_wait);
    }
    if (defer == 2) {  // (pipelined step) kept for the next fused_train_pipe launch
      g_pending_pipe = a;
      g_pending_pipe_set = true;
      return;
    }
    if (defer) throw std::runtime_error("grad_reduce: defer is 0 or 2 (the pipelined / persistent launch)");
    dnn::launch_grad_reduce(a, S(stream));
  }, py::arg("a0"), py::arg("h1"), py::arg("h2"), py::arg("z1"), py::arg("z2"), py::arg("z3"), py::arg("slab"),
     py::arg("loss"), py::arg("correct"), py::arg("batch"), py::arg("master"), py::arg("grad"), py::arg("mom"),
     py::arg("shadow"), py::arg("state"), py::arg("stats"), py::arg("lr"), py::arg("momentum"),
     py::arg("grad_scale"), py::arg("fuse_sgd"), py::arg("lo"), py::arg("hi"), py::arg("bookkeeping"),
     py::arg("order"), py::arg("order_len"), py::arg("batch_ids"), py::arg("stream"), py::arg("stamps") = 0,
     py::arg("xp_regions") = std::vector<u>{}, py::arg("xp_rank") = 0, py::arg("xp_capacity") = 0,
     py::arg("xp_ctr") = 0, py::arg("xp_err") = 0, py::arg("xp_abort") = 0, py::arg("xp_timeout_s") = 60.0,
     py::arg("xp_scale") = 1.0f, py::arg("next_ids") = 0, py::arg("xp_mode") = 0, py::arg("xp_wait") = 0,
     py::arg("defer") = 0, py::arg("bk_bv_in") = 0, py::arg("bk_bv_out") = 0, py::arg("bk_adv") = 1,
     py::arg("bk_stats") = 1);
  // the pipelined step's merged launch (lenet_fused.hip PIPE): the reduction of the previous
  // step (the last grad_reduce(defer=2) call) + this step's samples
  m.def("fused_train_pipe", [](u images, u labels, int order_len, int batch, u master, u shadow, u a0, u h1, u h2,
                               u z1, u z2, u z3, u slab, u loss, u correct, u next_ids, u stage, u ctr, int par,
                               int wait, int nred, u bvalid, u err, double timeout_s, u stream, u stamps,
                               int flags, u flg) {
    if (!g_pending_pipe_set) throw std::runtime_error("fused_train_pipe needs a grad_reduce(defer=2) call first");
    g_pending_pipe_set = false;
    dnn::PipeCtl pc;
    pc.ctr = P<unsigned>(ctr);
    pc.par = par;
    pc.wait = wait;
    pc.nred = nred;
    pc.bvalid = P<const int32_t>(bvalid);
    pc.err = P<unsigned>(err);
    pc.timeout_ticks = (long long)(timeout_s * 1.0e8);
    pc.flags = flags;
    pc.flg = P<unsigned>(flg);
    dnn::launch_fused_train_pipe(P<const uint8_t>(images), P<const int32_t>(labels), order_len, batch,
                                 P<const float>(master), P<const bf16>(shadow), P<float>(a0), P<float>(h1),
                                 P<float>(h2), P<float>(z1), P<float>(z2), P<float>(z3), P<float>(slab),
                                 P<float>(loss), P<int32_t>(correct), P<long long>(stamps), P<const int32_t>(next_ids),
                                 P<unsigned char>(stage), g_pending_pipe, pc, S(stream));
  }, py::arg("images"), py::arg("labels"), py::arg("order_len"), py::arg("batch"), py::arg("master"),
     py::arg("shadow"), py::arg("a0"), py::arg("h1"), py::arg("h2"), py::arg("z1"), py::arg("z2"), py::arg("z3"),
     py::arg("slab"), py::arg("loss"), py::arg("correct"), py::arg("next_ids"), py::arg("stage"), py::arg("ctr"),
     py::arg("par"), py::arg("wait"), py::arg("nred"), py::arg("bvalid"), py::arg("err"), py::arg("timeout_s"),
     py::arg("stream"), py::arg("stamps") = 0, py::arg("flags") = 0, py::arg("flg") = 0);
  // the persistent launch (lenet_fused.hip PERS): nsteps steps in ONE launch; the reduction is the
  // last grad_reduce(defer=2) call's (rows of parity 0, parity 1 right after them)
  m.def("fused_train_persist", [](u images, u labels, int order_len, int batch, u master, u shadow, u a0, u h1, u h2,
                                  u z1, u z2, u z3, u slab, u loss, u correct, u stage, u ctl, int nsteps, u bv0,
                                  u bv1, u nid0, u nid1, u err, double timeout_s, u stream, u stamps, int flags,
                                  bool direct) {
    if (!g_pending_pipe_set) throw std::runtime_error("fused_train_persist needs a grad_reduce(defer=2) call first");
    g_pending_pipe_set = false;
    dnn::PipeCtl pc;
    pc.ctr = P<unsigned>(ctl);
    pc.nsteps = nsteps;
    pc.bv_slot[0] = P<int32_t>(bv0);
    pc.bv_slot[1] = P<int32_t>(bv1);
    pc.nid_slot[0] = P<int32_t>(nid0);
    pc.nid_slot[1] = P<int32_t>(nid1);
    pc.err = P<unsigned>(err);
    pc.timeout_ticks = (long long)(timeout_s * 1.0e8);
    pc.flags = flags;
    return dnn::launch_fused_train_persist(P<const uint8_t>(images), P<const int32_t>(labels), order_len, batch,
                                    P<const float>(master), P<const bf16>(shadow), P<float>(a0), P<float>(h1),
                                    P<float>(h2), P<float>(z1), P<float>(z2), P<float>(z3), P<float>(slab),
                                    P<float>(loss), P<int32_t>(correct), P<long long>(stamps), P<unsigned char>(stage),
                                    g_pending_pipe, pc, S(stream), direct);
  }, py::arg("images"), py::arg("labels"), py::arg("order_len"), py::arg("batch"), py::arg("master"),
     py::arg("shadow"), py::arg("a0"), py::arg("h1"), py::arg("h2"), py::arg("z1"), py::arg("z2"), py::arg("z3"),
     py::arg("slab"), py::arg("loss"), py::arg("correct"), py::arg("stage"), py::arg("ctl"), py::arg("nsteps"),
     py::arg("bv0"), py::arg("bv1"), py::arg("nid0"), py::arg("nid1"), py::arg("err"), py::arg("timeout_s"),
     py::arg("stream"), py::arg("stamps") = 0, py::arg("flags") = 0, py::arg("direct") = false);
  // the fp32 kernel's persistent launch (lenet_f32.hip PERS): the reduction is the last
  // grad_reduce(defer=2) call's
  m.def("fused_train_persist_f32", [](u images, u labels, int order_len, int batch, u master, u a0, u h1, u h2, u z1,
                                      u z2, u z3, u slab, u loss, u correct, u ctl, int nsteps, u bv0, u bv1, u nid0,
                                      u nid1, u err, double timeout_s, u stream, int flags, u stamps, bool direct) {
    if (!g_pending_pipe_set) throw std::runtime_error("fused_train_persist_f32 needs a grad_reduce(defer=2) call first");
    g_pending_pipe_set = false;
    dnn::PipeCtl pc;
    pc.ctr = P<unsigned>(ctl);
    pc.nsteps = nsteps;
    pc.bv_slot[0] = P<int32_t>(bv0);
    pc.bv_slot[1] = P<int32_t>(bv1);
    pc.nid_slot[0] = P<int32_t>(nid0);
    pc.nid_slot[1] = P<int32_t>(nid1);
    pc.err = P<unsigned>(err);
    pc.timeout_ticks = (long long)(timeout_s * 1.0e8);
    pc.flags = flags;
    return dnn::launch_fused_train_persist_f32(P<const uint8_t>(images), P<const int32_t>(labels), order_len, batch,
                                               P<const float>(master), P<float>(a0), P<float>(h1), P<float>(h2),
                                               P<float>(z1), P<float>(z2), P<float>(z3), P<float>(slab),
                                               P<float>(loss), P<int32_t>(correct), g_pending_pipe, pc, S(stream),
                                               P<long long>(stamps), direct);
  }, py::arg("images"), py::arg("labels"), py::arg("order_len"), py::arg("batch"), py::arg("master"), py::arg("a0"),
     py::arg("h1"), py::arg("h2"), py::arg("z1"), py::arg("z2"), py::arg("z3"), py::arg("slab"), py::arg("loss"),
     py::arg("correct"), py::arg("ctl"), py::arg("nsteps"), py::arg("bv0"), py::arg("bv1"), py::arg("nid0"),
     py::arg("nid1"), py::arg("err"), py::arg("timeout_s"), py::arg("stream"), py::arg("flags") = 0,
     py::arg("stamps") = 0, py::arg("direct") = false);
  m.def("persist_max_batch_f32", []() { return dnn::persist_max_batch_f32(); });
  m.def("persist_resident_workgroups_f32", []() { return dnn::persist_resident_workgroups_f32(); });
  m.def("persist_wg_f32", []() { return dnn::persist_wg_f32(); });
  m.def("persist_conv_wg_f32", []() { return dnn::persist_conv_wg_f32(); });
  m.def("persist_ctl_bytes_f32", [](int batch) { return dnn::persist_ctl_bytes_f32(batch); });
  m.def("persist_max_batch", []() { return dnn::persist_max_batch(); });
  m.def("persist_resident_workgroups", []() { return dnn::persist_resident_workgroups(); });
  m.def("persist_ctl_bytes", [](int batch) { return dnn::persist_ctl_bytes(batch); });
  // direct AQL dispatch (runtime/aql_dispatch.h): "" when this process has a queue on the device,
  // else why not; the host-clock cost of the last direct dispatch (doorbell -> completion, whole call)
  m.def("aql_status", [](int device) {
    std::string why;
    return dnn::aql_queue(device, &why) != nullptr ? std::string() : why;
  });
  // the direct dispatch path end to end on a trivial kernel (csrc/kernels/diag.hip): "" or why not
  m.def("aql_selftest", []() {
    std::string why;
    return dnn::aql_selftest(&why) ? std::string() : why;
  });
  m.def("persist_direct_run", [](int handle) { dnn::aql_prepared_run(handle); }, py::arg("handle"),
        py::call_guard<py::gil_scoped_release>());
  m.def("persist_direct_launch", [](int handle) { dnn::aql_prepared_launch(handle); }, py::arg("handle"));
  m.def("persist_direct_wait", [](int handle) { dnn::aql_prepared_wait(handle); }, py::arg("handle"),
        py::call_guard<py::gil_scoped_release>());
  m.def("aql_last_us", [](int device, bool whole) { return dnn::aql_last_us(dnn::aql_queue(device), whole); },
        py::arg("device"), py::arg("whole") = false);
  m.def("pipe_reduce_blocks", []() { return dnn::pipe_reduce_blocks(); });
  m.def("pipe_groups", []() { return dnn::pipe_groups(); });
  m.def("init", []() { dnn::init_kernels(); });
  // ---- Linear layers on MFMA (kernels/linear.hip) ----
  m.def("linear_fwd", [](u x, u w, u b, u y, int B, int K, int N, int relu, u stream) {
    dnn::launch_linear_fwd(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), B, K, N, relu,
                           S(stream));
  });
  m.def("linear_splitk_splits", [](int B, int K, int N) { return dnn::linear_splitk_splits(B, K, N); });
  m.def("linear_fwd_splitk", [](u x, u w, u b, u y, u part, int splits, int B, int K, int N, int relu, u stream) {
    dnn::launch_linear_fwd_splitk(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), P<float>(part),
                                  splits, B, K, N, relu, S(stream));
  });
  m.def("linear_dgrad", [](u dy, u y, u w, u dx, int B, int K, int N, u stream) {
    dnn::launch_linear_dgrad(P<const float>(dy), P<const float>(y), P<const float>(w), P<float>(dx), B, K, N,
                             S(stream));
  });
  m.def("linear_wgrad", [](u dy, u y, u x, u dw, u db, int B, int K, int N, u stream) {
    dnn::launch_linear_wgrad(P<const float>(dy), P<const float>(y), P<const float>(x), P<float>(dw), P<float>(db), B,
                             K, N, S(stream));
  });
  m.def("linear_fwd_xent", [](u x, u w, u b, u y, u labels, u state, u loss, u correct, u dlogits, int B, int K,
                              int N, u stream) {
    dnn::launch_linear_fwd_xent(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y),
                                P<const int32_t>(labels), P<const int32_t>(state), P<float>(loss), P<int32_t>(correct),
                                P<float>(dlogits), B, K, N, S(stream));
  });
  m.def("linear_bwd", [](u dy, u y, u w, u x, u dx, u dw, u db, int B, int K, int N, u stream) {
    dnn::launch_linear_bwd(P<const float>(dy), P<const float>(y), P<const float>(w), P<const float>(x), P<float>(dx),
                           P<float>(dw), P<float>(db), B, K, N, S(stream));
  });
  // ---- generic layer kernels (kernels/layers.hip), used by runtime/layer_engine.py ----
  m.def("ingest", [](u images, u labels, u ids, int batch, int per_img, u out, u lab_out, u stream) {
    dnn::launch_ingest(P<const uint8_t>(images), P<const int32_t>(labels), P<const int32_t>(ids), batch, per_img,
                       P<float>(out), P<int32_t>(lab_out), S(stream));
  });
  m.def("relu_pool_fwd", [](u x, int BC, int H, int W, u y, u code, u stream) {
    dnn::launch_relu_pool_fwd(P<const float>(x), BC, H, W, P<float>(y), P<uint8_t>(code), S(stream));
  });
  m.def("relu_pool_bwd", [](u dy, u code, int BC, int H, int W, u dx, u stream) {
    dnn::launch_relu_pool_bwd(P<const float>(dy), P<const uint8_t>(code), BC, H, W, P<float>(dx), S(stream));
  });
  m.def("relu_fwd", [](u x, long n, u y, u stream) { dnn::launch_relu_fwd(P<const float>(x), n, P<float>(y), S(stream)); });
  m.def("relu_bwd", [](u dy, u y, long n, u dx, u stream) {
    dnn::launch_relu_bwd(P<const float>(dy), P<const float>(y), n, P<float>(dx), S(stream));
  });
  m.def("chan_parts", [](int B, int L) { return dnn::chan_parts(B, L); });
  m.def("bn_fwd_train", [](u x, int B, int C, int L, u state, u gamma, u beta, float eps, float mom, u rmean,
                           u rvar, u y, u smean, u sinvstd, u part, u stream) {
    dnn::launch_bn_fwd_train(P<const float>(x), B, C, L, P<const int32_t>(state), P<const float>(gamma),
                             P<const float>(beta), eps, mom, P<float>(rmean), P<float>(rvar), P<float>(y),
                             P<float>(smean), P<float>(sinvstd), P<double>(part), S(stream));
  });
  m.def("bn_fwd_eval", [](u x, int B, int C, int L, u gamma, u beta, float eps, u rmean, u rvar, u y, u stream) {
    dnn::launch_bn_fwd_eval(P<const float>(x), B, C, L, P<const float>(gamma), P<const float>(beta), eps,
                            P<const float>(rmean), P<const float>(rvar), P<float>(y), S(stream));
  });
  m.def("bn_bwd", [](u dy, u x, int B, int C, int L, u state, u gamma, u smean, u sinvstd, u dx, u dgamma,
                     u dbeta, u part, u stream) {
    dnn::launch_bn_bwd(P<const float>(dy), P<const float>(x), B, C, L, P<const int32_t>(state), P<const float>(gamma),
                       P<const float>(smean), P<const float>(sinvstd), P<float>(dx), P<float>(dgamma),
                       P<float>(dbeta), P<double>(part), S(stream));
  });
  // ext_parts > 0: part holds that many statistics partials per channel already (conv epilogue)
  m.def(
      "bn_act_fwd_train",
      [](u x, int B, int C, int H, int W, u state, u gamma, u beta, float eps, float mom, u rmean, u rvar, u y, u code,
         u smean, u sinvstd, u part, int act, u stream, int ext_parts) {
        dnn::launch_bn_act_fwd_train(P<const float>(x), B, C, H, W, P<const int32_t>(state), P<const float>(gamma),
                                     P<const float>(beta), eps, mom, P<float>(rmean), P<float>(rvar), P<float>(y),
                                     P<uint8_t>(code), P<float>(smean), P<float>(sinvstd), P<double>(part), act,
                                     S(stream), ext_parts);
      },
      py::arg("x"), py::arg("B"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("state"), py::arg("gamma"),
      py::arg("beta"), py::arg("eps"), py::arg("mom"), py::arg("rmean"), py::arg("rvar"), py::arg("y"),
      py::arg("code"), py::arg("smean"), py::arg("sinvstd"), py::arg("part"), py::arg("act"), py::arg("stream"),
      py::arg("ext_parts") = 0);
  m.def(
      "bn_act_bwd",
      [](u dy, u x, int B, int C, int H, int W, u state, u gamma, u beta, u smean, u sinvstd, u code, u dx, u dgamma,
         u dbeta, u part, int act, u stream, int ext_parts) {
        dnn::launch_bn_act_bwd(P<const float>(dy), P<const float>(x), B, C, H, W, P<const int32_t>(state),
                               P<const float>(gamma), P<const float>(beta), P<const float>(smean),
                               P<const float>(sinvstd), P<const uint8_t>(code), P<float>(dx), P<float>(dgamma),
                               P<float>(dbeta), P<double>(part), act, S(stream), ext_parts);
      },
      py::arg("dy"), py::arg("x"), py::arg("B"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("state"),
      py::arg("gamma"), py::arg("beta"), py::arg("smean"), py::arg("sinvstd"), py::arg("code"), py::arg("dx"),
      py::arg("dgamma"), py::arg("dbeta"), py::arg("part"), py::arg("act"), py::arg("stream"),
      py::arg("ext_parts") = 0);
  m.def("chan_sum", [](u a, int B, int C, int L, u out, u part, u stream) {
    dnn::launch_chan_sum(P<const float>(a), B, C, L, P<float>(out), P<double>(part), S(stream));
  });
  m.def("xent", [](u logits, u labels, int B, int NC, u state, u loss, u correct, u dlogits, u stream) {
    dnn::launch_xent(P<const float>(logits), P<const int32_t>(labels), B, NC, P<const int32_t>(state), P<float>(loss),
                     P<int32_t>(correct), P<float>(dlogits), S(stream));
  });
  auto book_args = [](u loss, u correct, int batch, u state, u stats, u order, int order_len, u batch_ids) {
    dnn::ReduceArgs a{};
    a.loss = P<const float>(loss);
    a.correct = P<const int32_t>(correct);
    a.batch = batch;
    a.state = P<int32_t>(state);
    a.stats = P<double>(stats);
    a.order = P<const int32_t>(order);
    a.order_len = order_len;
    a.batch_ids = P<int32_t>(batch_ids);
    return a;
  };
  m.def("layer_bookkeeping", [book_args](u loss, u correct, int batch, u state, u stats, u order, int order_len,
                                         u batch_ids, u stream) {
    dnn::launch_layer_bookkeeping(book_args(loss, correct, batch, state, stats, order, order_len, batch_ids),
                                  S(stream));
  });
  // SGD + packed conv-weight images + bookkeeping (loss == 0: no bookkeeping) in one launch;
  // slices: (part, S, M, Kd, dw arena offset, db arena offset) of deferred conv wgrad slice sums
  m.def("sgd_tail", [book_args](u p, u g, u mom, long n, float lr, float momentum, float grad_scale,
                                std::vector<std::tuple<u, u, int, int, int, int, int, int, int, int, int>> jobs,
                                u arena, std::vector<std::tuple<u, int, int, int, long, long>> slices, u loss,
                                u correct, int batch, u state, u stats, u order, int order_len, u batch_ids,
                                u stream) {
    std::vector<dnn::ConvPackJob> js;
    for (const auto& t : jobs)
      js.push_back(dnn::ConvPackJob{P<const float>(std::get<0>(t)), P<void>(std::get<1>(t)), std::get<2>(t),
                                    std::get<3>(t), std::get<4>(t), std::get<5>(t), std::get<6>(t), std::get<7>(t),
                                    std::get<8>(t), std::get<9>(t), std::get<10>(t)});
    const dnn::ReduceArgs a = book_args(loss, correct, batch, state, stats, order, order_len, batch_ids);
    std::vector<dnn::SliceJob> sl;
    for (const auto& t : slices)
      sl.push_back(dnn::SliceJob{P<const float>(std::get<0>(t)), std::get<1>(t), std::get<2>(t), std::get<3>(t),
                                 std::get<4>(t), std::get<5>(t)});
    dnn::launch_sgd_tail(P<float>(p), P<float>(g), P<float>(mom), n, lr, momentum, grad_scale, js.data(),
                         (int)js.size(), P<const float>(arena), sl.data(), (int)sl.size(), loss != 0 ? &a : nullptr,
                         S(stream));
  });
  m.def("conv_fwd", [](u x, u w, u bias, u y, u ws, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops,
                       int flip, u stream) {
    dnn::launch_conv_fwd(P<const float>(x), P<const float>(w), P<const float>(bias), P<float>(y), P<void>(ws), B, C, H,
                         W, M, K, pad, bf16_ops, flip, S(stream));
  });
  m.def("conv_fwd_workspace", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int flip) {
    return (long)dnn::conv_fwd_workspace(B, C, H, W, M, K, pad, bf16_ops, flip);
  });
  m.def("conv_fwd_fast", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
    return dnn::conv_fwd_fast(B, C, H, W, M, K, pad, bf16_ops);
  });
  // jobs: [(w, dst, B, C, H, W, M, K, pad, bf16_ops, flip), ...]
  m.def("conv_pack_all", [](std::vector<std::tuple<u, u, int, int, int, int, int, int, int, int, int>> jobs, u stream) {
    std::vector<dnn::ConvPackJob> js;
    for (const auto& t : jobs)
      js.push_back(dnn::ConvPackJob{P<const float>(std::get<0>(t)), P<void>(std::get<1>(t)), std::get<2>(t),
                                    std::get<3>(t), std::get<4>(t), std::get<5>(t), std::get<6>(t), std::get<7>(t),
                                    std::get<8>(t), std::get<9>(t), std::get<10>(t)});
    dnn::launch_conv_pack_all(js.data(), (int)js.size(), S(stream));
  });
  m.def("conv_fwd_packed", [](u x, u wp, u bias, u y, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops,
                              u stream) {
    dnn::launch_conv_fwd_packed(P<const float>(x), P<const void>(wp), P<const float>(bias), P<float>(y), B, C, H, W, M,
                                K, pad, bf16_ops, S(stream));
  });
  m.def("conv_fwd_ingest_ok", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, int epi) {
    return dnn::conv_fwd_ingest_ok(B, C, H, W, M, K, pad, bf16_ops, epi);
  });
  // first conv of a training step reading the u8 images of the batch ids (ingest folded in)
  m.def("conv_fwd_packed_ingest", [](u images, u ids, u labels, u x_out, u lab_out, u wp, u bias, u y, u code, u stats,
                                     u state, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops,
                                     u stream) {
    dnn::launch_conv_fwd_packed_ingest(P<const uint8_t>(images), P<const int32_t>(ids), P<const int32_t>(labels),
                                       P<float>(x_out), P<int32_t>(lab_out), P<const void>(wp), P<const float>(bias),
                                       P<float>(y), P<uint8_t>(code), P<double>(stats), P<const int32_t>(state), B, C,
                                       H, W, M, K, pad, bf16_ops, S(stream));
  });
  m.def("conv_fwd_unpool_ok", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
    return dnn::conv_fwd_unpool_ok(B, C, H, W, M, K, pad, bf16_ops);
  });
  // data gradient of a pooled conv straight from the pooled gradient + argmax codes
  m.def("conv_fwd_packed_unpool", [](u x, u code, u wp, u y, int B, int C, int H, int W, int M, int K, int pad,
                                     int bf16_ops, u stream) {
    dnn::launch_conv_fwd_packed_unpool(P<const float>(x), P<const uint8_t>(code), P<const void>(wp), P<float>(y), B, C,
                                       H, W, M, K, pad, bf16_ops, S(stream));
  });
  m.def("conv_fwd_pool_ok", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
    return dnn::conv_fwd_pool_ok(B, C, H, W, M, K, pad, bf16_ops);
  });
  m.def("conv_fwd_packed_pool", [](u x, u wp, u bias, u y, u code, int B, int C, int H, int W, int M, int K, int pad,
                                   int bf16_ops, u stream) {
    dnn::launch_conv_fwd_packed_pool(P<const float>(x), P<const void>(wp), P<const float>(bias), P<float>(y),
                                     P<uint8_t>(code), B, C, H, W, M, K, pad, bf16_ops, S(stream));
  });
  m.def("conv_fwd_stat_parts", [](int B, int C, int H, int W, int M, int K, int pad, int bf16_ops) {
    return dnn::conv_fwd_stat_parts(B, C, H, W, M, K, pad, bf16_ops);
  });
  m.def("conv_fwd_packed_stats", [](u x, u wp, u bias, u y, u stats, u state, int B, int C, int H, int W, int M, int K,
                                    int pad, int bf16_ops, u stream) {
    dnn::launch_conv_fwd_packed_stats(P<const float>(x), P<const void>(wp), P<const float>(bias), P<float>(y),
                                      P<double>(stats), P<const int32_t>(state), B, C, H, W, M, K, pad, bf16_ops,
                                      S(stream));
  });
  m.def("conv_fwd_packed_bnbwd", [](u x, u wp, u y, u stats, u state, u bn_z, u bn_mean, u bn_invstd, u bn_gamma,
                                    u bn_beta, u bn_code, int zH, int zW, int B, int C, int H, int W, int M, int K,
                                    int pad, int bf16_ops, u stream) {
    dnn::launch_conv_fwd_packed_bnbwd(P<const float>(x), P<const void>(wp), P<float>(y), P<double>(stats),
                                      P<const int32_t>(state), P<const float>(bn_z), P<const float>(bn_mean),
                                      P<const float>(bn_invstd), P<const float>(bn_gamma), P<const float>(bn_beta),
                                      P<const uint8_t>(bn_code), zH, zW, B, C, H, W, M, K, pad, bf16_ops, S(stream));
  });
  m.def("conv_wgrad_slices", [](int B, int C, int H, int W, int M, int K, int pad) {
    int s = 1, cps = 1;
    dnn::conv_wgrad_split(B, C, H, W, M, K, pad, &s, &cps);
    return s;
  });
  m.def(
      "conv_wgrad",
      [](u x, u dy, u part, u dw, u db, int B, int C, int H, int W, int M, int K, int pad, int bf16_ops, u stream,
         u pool_code) {
        dnn::launch_conv_wgrad(P<const float>(x), P<const float>(dy), P<float>(part), P<float>(dw), P<float>(db), B, C,
                               H, W, M, K, pad, bf16_ops, S(stream), P<const uint8_t>(pool_code));
      },
      py::arg("x"), py::arg("dy"), py::arg("part"), py::arg("dw"), py::arg("db"), py::arg("B"), py::arg("C"),
      py::arg("H"), py::arg("W"), py::arg("M"), py::arg("K"), py::arg("pad"), py::arg("bf16_ops"), py::arg("stream"),
      py::arg("pool_code") = 0);
  m.def("flip_weights", [](u w, int O, int C, int K, u wf, u stream) {
    dnn::launch_flip_weights(P<const float>(w), O, C, K, P<float>(wf), S(stream));
  });
  m.def("sgd_flat", [](u p, u g, u mom, long n, float lr, float momentum, float grad_scale, u stream) {
    dnn::launch_sgd_flat(P<float>(p), P<const float>(g), P<float>(mom), n, lr, momentum, grad_scale, S(stream));
  });
  // native RCCL communicator (comm/rccl_comm.cpp)
  m.def("rccl_open", &dnn::rccl_open, py::arg("path"));
  m.def("rccl_unique_id", []() { return py::bytes(dnn::rccl_unique_id()); });
  m.def(
      "rccl_init",
      [](py::bytes id, int nranks, int rank, int device, int blocking, double timeout_s) {
        const std::string idb(id);      // (converted under the GIL)
        py::gil_scoped_release nogil;   // waits until every rank joined (non-blocking: <= timeout_s)
        return dnn::rccl_init(idb, nranks, rank, device, blocking, timeout_s);
      },
      py::arg("id"), py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("blocking") = 0,
      py::arg("timeout_s") = 120.0);
  m.def("rccl_allreduce", &dnn::rccl_allreduce, py::arg("comm"), py::arg("buf"), py::arg("count"),
        py::arg("dtype"), py::arg("op"), py::arg("stream"));
  m.def("rccl_broadcast", &dnn::rccl_broadcast);
  m.def("rccl_async_error", &dnn::rccl_async_error);
  m.def("rccl_abort", [](uintptr_t c) { py::gil_scoped_release nogil; dnn::rccl_abort(c); });
  m.def("rccl_destroy", [](uintptr_t c) { py::gil_scoped_release nogil; dnn::rccl_destroy(c); });
  // one-shot xGMI all-reduce (+ fused SGD) over IPC-mapped peer regions
  m.def("xgmi_alloc", [](long long capacity) {
    auto [p, h, kind] = dnn::xgmi_alloc(capacity);
    return py::make_tuple(p, py::bytes(h), kind);
  });
  m.def("xgmi_open", [](py::bytes h) { return dnn::xgmi_open(std::string(h)); });
  m.def("xgmi_close", &dnn::xgmi_close);
  m.def("xgmi_device_id", &dnn::xgmi_device_id);
  m.def("xgmi_free", &dnn::xgmi_free);
  m.def("uncached_alloc", &dnn::uncached_alloc);
  m.def("uncached_free", &dnn::uncached_free);
  // A stream with a hardware queue of its own: HIP multiplexes ordinary streams onto a few
  // hardware queues (GPU_MAX_HW_QUEUES), in order, so two streams of one process can land on
  // the same queue and run one after the other.  Kernels that wait for each other (the
  // in-process exchange harness: two ranks' grids polling each other's granules) must not: a
  // CU-masked stream (all CUs) gets a dedicated queue.  Never destroyed (parallel/inproc.py).
  m.def("stream_create_own_queue", []() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev))
      throw std::runtime_error("stream_create_own_queue: device query failed");
    std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
    return reinterpret_cast<u>(s);
  });
  m.def("uncached_pool_stats", &dnn::uncached_pool_stats);
  m.def("lds_poison", [](unsigned pattern, u stream) { dnn::lds_poison(pattern, S(stream)); }, py::arg("pattern"),
        py::arg("stream"));
  m.def("lds_squat", [](int bytes, double spin_us, int blocks, u bad, u stream) {
    dnn::lds_squat(bytes, spin_us, blocks, bad, S(stream));
  }, py::arg("bytes"), py::arg("spin_us"), py::arg("blocks"), py::arg("bad"), py::arg("stream"));
  m.def("xgmi_abort_word", &dnn::xgmi_abort_word);
  m.def("xgmi_set_abort", &dnn::xgmi_set_abort);
  m.def("xgmi_free_abort_word", &dnn::xgmi_free_abort_word);
  m.def("xgmi_max_blocks", &dnn::xgmi_max_blocks);
  m.def("xgmi_region_bytes", &dnn::xgmi_region_bytes);
  m.def("xgmi_gslot_bytes", &dnn::xgmi_gslot_bytes);
  m.def("xgmi_xp_max_blocks", []() { return dnn::XP_MAX_BLOCKS; });
  m.def("xgmi_wait_ring", []() { return py::make_tuple(dnn::XP_WAIT_RING, dnn::XP_MAX_BLOCKS, 4); });
  m.def("grad_reduce_blocks", []() { return dnn::grad_reduce_blocks(); });
  m.def("xgmi_allreduce", [](std::vector<u> regions, int rank, long long capacity, int n, u grad, u out, u master,
                             u mom, u shadow, float lr, float momentum, float scale, int mode, u ctr, u abort_w,
                             double timeout_s, u stream, int form, u wait) {
    dnn::launch_xgmi_allreduce(regions, rank, capacity, n, P<const float>(grad), P<float>(out), P<float>(master),
                               P<float>(mom), P<bf16>(shadow), lr, momentum, scale, mode, P<unsigned>(ctr),
                               P<const unsigned>(abort_w), timeout_s, S(stream), form,
                               P<unsigned long long>(wait));
  }, py::arg("regions"), py::arg("rank"), py::arg("capacity"), py::arg("n"), py::arg("grad"), py::arg("out"),
     py::arg("master"), py::arg("mom"), py::arg("shadow"), py::arg("lr"), py::arg("momentum"), py::arg("scale"),
     py::arg("mode"), py::arg("ctr"), py::arg("abort_w"), py::arg("timeout_s"), py::arg("stream"), py::arg("form") = 0,
     py::arg("wait") = 0);
  m.def("epoch_begin", [](u staged, u order, int n, u state, u batch_ids, int batch, u stream, u images, u labels,
                          u next_ids, u stage) {
    dnn::launch_epoch_begin(P<const int32_t>(staged), P<int32_t>(order), n, P<int32_t>(state), P<int32_t>(batch_ids),
                            batch, P<const uint8_t>(images), P<const int32_t>(labels), P<int32_t>(next_ids),
                            P<unsigned char>(stage), S(stream));
  }, py::arg("staged"), py::arg("order"), py::arg("n"), py::arg("state"), py::arg("batch_ids"), py::arg("batch"),
     py::arg("stream"), py::arg("images") = 0, py::arg("labels") = 0, py::arg("next_ids") = 0, py::arg("stage") = 0);
  m.def("sgd_apply", [](u master, u grad, u mom, u shadow, int n, float lr, float momentum, float grad_scale,
                        int pack_only, u stream) {
    dnn::launch_sgd_apply(P<float>(master), P<const float>(grad), P<float>(mom), P<bf16>(shadow), n, lr, momentum,
                          grad_scale, pack_only, S(stream));
  });
}
