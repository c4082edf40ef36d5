// Host side of the one-shot IPC all-gather (kernels in csrc/kernels/comm.hip): allocation, handle
// export/import, epoch bookkeeping, timeout reporting.  Exposed to Python as attackfl_amd._C.IpcContext
// (wrapped by attackfl_amd/parallel/ipc.py).
//
// all_gather() only enqueues (push + signal/wait on the current stream) and returns a VIEW of this
// epoch's receive region: no host synchronisation and no copy-out.  The view stays valid until the
// call after next reuses its parity; the caller consumes it on the same stream before then.  A
// deadline miss inside the wait kernel shows up in status() (pinned host word) once the stream has
// passed the wait.
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
  IpcContext(int rank, int world, int64_t cap) : rank_(rank), world_(world), cap_((cap + 3) / 4 * 4) {
    TORCH_CHECK(world >= 1 && world <= AFL_IPC_MAX_PEERS, "IPC all-gather supports 1..16 ranks");
    TORCH_CHECK(rank >= 0 && rank < world, "bad rank");
    TORCH_CHECK(cap >= 1, "bad capacity");
    IPC_OK(hipGetDevice(&device_));
    float* base = nullptr;
    IPC_OK((hipError_t)afl_ipc_alloc(world, cap_, &base));
    local_ = base;
    IPC_OK(hipHostMalloc((void**)&status_, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
    *status_ = 0;
    for (int i = 0; i < AFL_IPC_MAX_PEERS; ++i) peers_.base[i] = nullptr;
    peers_.world = world;
    peers_.base[rank] = local_;
  }
  ~IpcContext() { close(); }

  // 64-byte IPC handle of the local receive buffer
  py::bytes handle() const {
    TORCH_CHECK(local_ != nullptr, "IPC context closed");
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

  // enqueue: rank r's `src` (n floats) -> row r of the returned [world, n] view (row stride = capacity)
  torch::Tensor all_gather(torch::Tensor src, double timeout_s) {
    TORCH_CHECK(ready_, "IPC context not opened");
    TORCH_CHECK(src.is_cuda() && src.is_contiguous() && src.scalar_type() == torch::kFloat32, "src: fp32 device");
    TORCH_CHECK(src.get_device() == device_, "src is on another device than the IPC buffers");
    const long n = src.numel();
    TORCH_CHECK(n <= cap_, "block larger than the IPC buffer");
    ++epoch_;
    const uint64_t ticks = (uint64_t)(timeout_s > 0 ? timeout_s * 1e8 : 6e9);  // s_memrealtime: 100 MHz
    IPC_OK((hipError_t)afl_ipc_all_gather(src.data_ptr<float>(), n, peers_, rank_, cap_, epoch_, status_, ticks,
                                          cur()));
    float* region = local_ + (long)(epoch_ & 1u) * world_ * cap_;
    return torch::from_blob(region, {(long)world_, n}, {cap_, 1L},
                            torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device_));
  }

  // bitmask of senders some wait timed out on (valid for every gather the host has synchronised past)
  int status() const { return status_ ? __atomic_load_n(status_, __ATOMIC_ACQUIRE) : 0; }

  void close() {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    if (local_) (void)hipFree(local_);
    if (status_) (void)hipHostFree(status_);
    local_ = nullptr;
    status_ = nullptr;
    ready_ = false;
  }

  int64_t capacity() const { return cap_; }
  int64_t epoch() const { return epoch_; }

 private:
  int rank_, world_;
  long cap_;
  int device_ = 0;
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
      .def("all_gather", &IpcContext::all_gather, py::arg("src"), py::arg("timeout_s") = 60.0)
      .def("status", &IpcContext::status)
      .def("close", &IpcContext::close)
      .def("capacity", &IpcContext::capacity)
      .def("epoch", &IpcContext::epoch);
}
