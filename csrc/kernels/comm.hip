// One-shot intra-node all-gather over xGMI peer mappings (the small-message path of the FL round
// exchange; replaces the reference's RabbitMQ UPDATE/START hops, server.py:187-275,
// src/RpcClient.py:108-114).  Every rank maps every peer's receive buffer (IPC handles), writes its
// own block straight into all of them (one hop per peer, all links at once — a ring all-gather
// needs world-1 dependent hops), then raises a per-sender epoch flag in each peer and waits for the
// flags of every sender in its own buffer.  Buffers are double-buffered by epoch parity: a rank can
// only start writing epoch e+2 after every peer has signalled epoch e+1, i.e. after every peer's
// stream has passed all work it enqueued before that gather (which is where epoch e is consumed).
//
// Everything is stream-ordered: two launches, no host synchronisation.  A wait that exceeds its
// deadline (s_memrealtime, 100 MHz) stops spinning and sets a status word in pinned host memory,
// which the host reads at its next natural synchronisation point — a missing peer becomes an error,
// never a hung GPU.
//
// Memory: receive buffers + flags are allocated uncached (hipDeviceMallocUncached), so peer stores
// land in HBM and neither the flag spin nor the consumer kernels can read stale L2 lines.
#include "common.h"
#include "kernels.h"

namespace {

// flag (uint32) of `sender` for `parity` in the receive buffer at `base`: one 128-byte line each
__device__ __forceinline__ uint32_t* ipc_flag(float* base, int world, long cap, int parity, int sender) {
  return (uint32_t*)(base + 2L * world * cap) + (long)(parity * world + sender) * AFL_IPC_FLAG_STRIDE;
}

// data push: block [n] floats -> slot `rank` of buffer `parity` of every peer (blockIdx.y = peer)
__global__ void __launch_bounds__(256) k_ipc_push(const float* __restrict__ src, long n, AflIpcPeers peers, int rank,
                                                  long cap, int parity) {
  const int peer = blockIdx.y;
  float* dst = peers.base[peer] + ((long)parity * peers.world + rank) * cap;
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
    const long n4 = n >> 2;
    for (long i = t0; i < n4; i += stride) ((float4*)dst)[i] = ((const float4*)src)[i];
    for (long i = (n4 << 2) + t0; i < n; i += stride) dst[i] = src[i];
  } else {
    for (long i = t0; i < n; i += stride) dst[i] = src[i];
  }
}

// lane r < world: raise this rank's flag in peer r (release, system scope: the push kernel's remote
// stores completed at the kernel boundary and are ordered before the flag), then wait for sender r's
// flag in the local buffer.
__global__ void __launch_bounds__(64) k_ipc_signal_wait(AflIpcPeers peers, int rank, long cap, int parity,
                                                        uint32_t epoch, int* status, uint64_t deadline_ticks) {
  const int r = threadIdx.x;
  const int world = peers.world;
  if (r >= world) return;
  __threadfence_system();
  __hip_atomic_store(ipc_flag(peers.base[r], world, cap, parity, rank), epoch, __ATOMIC_RELEASE,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t* mine = ipc_flag(peers.base[rank], world, cap, parity, r);
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
    if (__builtin_amdgcn_s_memrealtime() - t_start > deadline_ticks) {
      __hip_atomic_fetch_or(status, 1 << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // bit = missing sender
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

}  // namespace

long afl_ipc_buffer_bytes(int world, long cap) {
  return (2L * world * cap) * 4 + 2L * world * AFL_IPC_FLAG_STRIDE * 4 + 256;
}

int afl_ipc_alloc(int world, long cap, float** base) {
  const size_t bytes = (size_t)afl_ipc_buffer_bytes(world, cap);
  hipError_t e = hipExtMallocWithFlags((void**)base, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*base, 0, bytes);
}

int afl_ipc_all_gather(const float* src, long n, const AflIpcPeers& peers, int rank, long cap, uint32_t epoch,
                       int* status, uint64_t deadline_ticks, hipStream_t s) {
  if (n > cap || peers.world < 1 || peers.world > AFL_IPC_MAX_PEERS || rank < 0 || rank >= peers.world)
    return (int)hipErrorInvalidValue;
  for (int r = 0; r < peers.world; ++r)
    if (peers.base[r] == nullptr) return (int)hipErrorInvalidValue;
  const int parity = (int)(epoch & 1u);
  const long n4 = (n + 3) / 4;
  const unsigned gx = (unsigned)std::max(1L, std::min(64L, (n4 + 255) / 256));
  hipLaunchKernelGGL(k_ipc_push, dim3(gx, peers.world), dim3(256), 0, s, src, n, peers, rank, cap, parity);
  hipLaunchKernelGGL(k_ipc_signal_wait, dim3(1), dim3(64), 0, s, peers, rank, cap, parity, epoch, status,
                     deadline_ticks);
  return (int)hipGetLastError();
}
