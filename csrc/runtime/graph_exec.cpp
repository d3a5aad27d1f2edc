// hipGraph helpers the Python engines need beyond torch.cuda.CUDAGraph.
//
// graph_upload: hipGraphUpload of an instantiated step-chunk graph.  The first replay of a
// freshly instantiated graph otherwise pays the upload of its launch packets / kernel
// arguments inside that replay; the engines upload every chunk graph right after capture
// (prepare_graphs), so a short timed run does not carry that one-time cost.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace dnn {

void graph_upload(uintptr_t exec, uintptr_t stream) {
  hipError_t e = hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) throw std::runtime_error(std::string("hipGraphUpload: ") + hipGetErrorString(e));
}

}  // namespace dnn
