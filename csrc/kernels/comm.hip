// One-shot intra-node all-gather over xGMI peer mappings (the small-message path of the FL round
// exchange; replaces the reference's RabbitMQ UPDATE/START hops, server.py:187-275,
// src/RpcClient.py:108-114).  Every rank maps every peer's receive buffer (IPC handles), writes its
// own block straight into all of them (one hop per peer, all links at once — a ring all-gather
// needs world-1 dependent hops), then raises a per-sender epoch flag in each peer; the receiver
// waits for all flags.  Buffers are double-buffered by epoch parity, so a fast rank cannot
// overwrite data a slow peer has not copied out yet.
//
// Memory: receive buffers + flags are allocated uncached (hipDeviceMallocUncached), so peer
// stores land in HBM and the flag spin reads them without stale L2 lines.  The spin has an
// iteration cap: a missing peer turns into an error code, never a hung GPU.
#include "common.h"
#include "kernels.h"

namespace {

// data push: block [n] floats -> slot `rank` of buffer `parity` of every peer
__global__ void __launch_bounds__(256) k_ipc_push(const float* __restrict__ src, long n, AflIpcPeers peers, int rank,
                                                  long cap, int parity) {
  const int peer = blockIdx.y;
  float* dst = peers.base[peer] + (long)parity * peers.world * cap + (long)rank * cap;
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 + 3 < n && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    *(float4*)(dst + i4) = *(const float4*)(src + i4);
  } else {
    for (long i = i4; i < min(n, i4 + 4); ++i) dst[i] = src[i];
  }
}

// flag raise: flags live after the two data buffers: [world] uint32 per parity
__global__ void k_ipc_signal(AflIpcPeers peers, int rank, long cap, int parity, uint32_t epoch) {
  const int peer = threadIdx.x;
  if (peer >= peers.world) return;
  uint32_t* fl = (uint32_t*)(peers.base[peer] + 2L * peers.world * cap) + parity * peers.world + rank;
  __threadfence_system();
  __hip_atomic_store(fl, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_ipc_wait(const float* local_base, int world, long cap, int parity, uint32_t epoch, int* status,
                           long max_polls) {
  const int r = threadIdx.x;
  if (r >= world) return;
  const uint32_t* fl = (const uint32_t*)(local_base + 2L * world * cap) + parity * world + r;
  long polls = 0;
  while (__hip_atomic_load(fl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
    if (++polls > max_polls) {
      atomicExch(status, 1);  // timed out: report instead of hanging
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

}  // namespace

long afl_ipc_buffer_bytes(int world, long cap) { return (2L * world * cap + 2L * world + 64) * 4; }

int afl_ipc_alloc(int world, long cap, float** base) {
  const size_t bytes = (size_t)afl_ipc_buffer_bytes(world, cap);
  hipError_t e = hipExtMallocWithFlags((void**)base, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*base, 0, bytes);
}

int afl_ipc_all_gather(const float* src, long n, const AflIpcPeers& peers, int rank, long cap, uint32_t epoch,
                       int* status, long max_polls, hipStream_t s) {
  if (n > cap || peers.world > AFL_IPC_MAX_PEERS) return (int)hipErrorInvalidValue;
  const int parity = (int)(epoch & 1u);
  const dim3 grid((unsigned)((n + 1023) / 1024), peers.world);
  hipLaunchKernelGGL(k_ipc_push, grid, dim3(256), 0, s, src, n, peers, rank, cap, parity);
  hipLaunchKernelGGL(k_ipc_signal, dim3(1), dim3(64), 0, s, peers, rank, cap, parity, epoch);
  hipLaunchKernelGGL(k_ipc_wait, dim3(1), dim3(64), 0, s, (const float*)peers.base[rank], peers.world, cap, parity,
                     epoch, status, max_polls);
  return (int)hipGetLastError();
}
