// Host side of the one-shot IPC all-gather (kernels in csrc/kernels/comm.hip): allocation, handle
// export/import, epoch bookkeeping, copy-out into a torch tensor, timeout reporting.
// Exposed to Python as attackfl_amd._C.IpcContext (wrapped by attackfl_amd/parallel/ipc.py).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <string>
#include <vector>

#include "kernels.h"

namespace {

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

#define IPC_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));            \
  } while (0)

class IpcContext {
 public:
  IpcContext(int rank, int world, int64_t cap) : rank_(rank), world_(world), cap_(cap) {
    TORCH_CHECK(world >= 1 && world <= AFL_IPC_MAX_PEERS, "IPC all-gather supports 1..16 ranks");
    TORCH_CHECK(rank >= 0 && rank < world, "bad rank");
    float* base = nullptr;
    IPC_OK((hipError_t)afl_ipc_alloc(world, cap, &base));
    local_ = base;
    IPC_OK(hipMalloc((void**)&status_, sizeof(int)));
    IPC_OK(hipMemset(status_, 0, sizeof(int)));
    for (int i = 0; i < AFL_IPC_MAX_PEERS; ++i) peers_.base[i] = nullptr;
    peers_.world = world;
    peers_.base[rank] = local_;
  }
  ~IpcContext() { close(); }

  // 64-byte IPC handle of the local receive buffer
  py::bytes handle() const {
    hipIpcMemHandle_t h;
    IPC_OK(hipIpcGetMemHandle(&h, local_));
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == world_, "need one handle per rank");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "bad handle size");
      hipIpcMemHandle_t h;
      memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      IPC_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_.base[r] = (float*)p;
      opened_.push_back(p);
    }
    ready_ = true;
  }

  // out[r * n : (r+1) * n] = rank r's `src` (n floats); blocks the host until done, raises on timeout
  torch::Tensor all_gather(torch::Tensor src, int64_t max_polls) {
    TORCH_CHECK(ready_, "IPC context not opened");
    TORCH_CHECK(src.is_cuda() && src.is_contiguous() && src.scalar_type() == torch::kFloat32, "src: fp32 device");
    const long n = src.numel();
    TORCH_CHECK(n <= cap_, "block larger than the IPC buffer");
    ++epoch_;
    hipStream_t s = cur();
    IPC_OK((hipError_t)afl_ipc_all_gather(src.data_ptr<float>(), n, peers_, rank_, cap_, epoch_, status_, max_polls,
                                          s));
    auto out = torch::empty({(long)world_ * n}, src.options());
    const float* region = local_ + (long)(epoch_ & 1u) * world_ * cap_;
    IPC_OK(hipMemcpy2DAsync(out.data_ptr<float>(), n * sizeof(float), region, cap_ * sizeof(float),
                            n * sizeof(float), world_, hipMemcpyDeviceToDevice, s));
    int st = 0;
    IPC_OK(hipMemcpyAsync(&st, status_, sizeof(int), hipMemcpyDeviceToHost, s));
    IPC_OK(hipStreamSynchronize(s));
    TORCH_CHECK(st == 0, "IPC all-gather timed out waiting for a peer (epoch ", epoch_, ")");
    return out;
  }

  void close() {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    if (local_) (void)hipFree(local_);
    if (status_) (void)hipFree(status_);
    local_ = nullptr;
    status_ = nullptr;
    ready_ = false;
  }

  int64_t capacity() const { return cap_; }

 private:
  int rank_, world_;
  long cap_;
  float* local_ = nullptr;
  int* status_ = nullptr;
  uint32_t epoch_ = 0;
  bool ready_ = false;
  AflIpcPeers peers_{};
  std::vector<void*> opened_;
};

}  // namespace

void afl_register_ipc(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<IpcContext>(m, "IpcContext")
      .def(py::init<int, int, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("cap"))
      .def("handle", &IpcContext::handle)
      .def("open", &IpcContext::open)
      .def("all_gather", &IpcContext::all_gather, py::arg("src"), py::arg("max_polls") = 20000000)
      .def("close", &IpcContext::close)
      .def("capacity", &IpcContext::capacity);
}
