// CRC-32 (IEEE 802.3 polynomial, reflected — the value zlib.crc32 / zip records carry) of a device
// buffer, for the checkpoint writer (attackfl_amd/utils/ckpt.py).  The writer emits the reference's
// torch.save zip layout itself (server.py:549-553 writes one .pth per successful round): per round only
// the storage bytes and their CRC change, and the CRC of a 19.5 MB hypernetwork arena costs ~23 ms on
// one host core (zlib) — longer than a round.  Here it is two launches on the checkpoint stream:
//
//   k_crc_chunks   one thread per 256-byte chunk: slice-by-4 table CRC (tables in LDS) -> crc[chunk]
//   k_crc_combine  one workgroup: thread t folds a contiguous run of chunk CRCs, thread 0 folds the runs
//
// Folding uses CRC linearity: crc(A || B) = (x^(8|B|) mod P) (*) crc(A)  ^  crc(B), where (*) is the
// carry-less product modulo P in the reflected representation; the x^(8|B|) constants are computed on
// the host (crc32_consts in bindings.cpp) for the three run lengths that occur.
#include "common.h"
#include "kernels.h"

namespace {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kChunk = 256;  // bytes per thread

// a (*) b mod P, reflected (bit 31 = x^0); `a` must be nonzero (it is always an x^n constant here)
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

__global__ void __launch_bounds__(256) k_crc_chunks(const uint32_t* __restrict__ data, long nbytes,
                                                    uint32_t* __restrict__ crcs) {
  __shared__ uint32_t T[4][256];
  const int t = threadIdx.x;
  uint32_t c = (uint32_t)t;
  for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
  T[0][t] = c;
  __syncthreads();
  T[1][t] = (T[0][t] >> 8) ^ T[0][T[0][t] & 255];
  __syncthreads();
  T[2][t] = (T[1][t] >> 8) ^ T[0][T[1][t] & 255];
  __syncthreads();
  T[3][t] = (T[2][t] >> 8) ^ T[0][T[2][t] & 255];
  __syncthreads();
  const long chunk = (long)blockIdx.x * blockDim.x + t;
  const long b0 = chunk * kChunk;
  if (b0 >= nbytes) return;
  const long len = nbytes - b0 < kChunk ? nbytes - b0 : kChunk;  // multiple of 4
  const uint32_t* w = data + b0 / 4;
  uint32_t crc = 0xFFFFFFFFu;
  if (len == kChunk) {
#pragma unroll 4
    for (int q = 0; q < kChunk / 16; ++q) {
      const uint4 v = ((const uint4*)w)[q];
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        crc ^= vv[j];
        crc = T[3][crc & 255] ^ T[2][(crc >> 8) & 255] ^ T[1][(crc >> 16) & 255] ^ T[0][crc >> 24];
      }
    }
  } else {
    for (long j = 0; j < len / 4; ++j) {
      crc ^= w[j];
      crc = T[3][crc & 255] ^ T[2][(crc >> 8) & 255] ^ T[1][(crc >> 16) & 255] ^ T[0][crc >> 24];
    }
  }
  crcs[chunk] = ~crc;
}

__global__ void __launch_bounds__(256) k_crc_combine(const uint32_t* __restrict__ crcs, long nchunks, long per,
                                                     uint32_t x_chunk, uint32_t x_last, uint32_t x_part,
                                                     uint32_t x_part_last, uint32_t* __restrict__ out) {
  __shared__ uint32_t part[256];
  const int t = threadIdx.x;
  const long first = (long)t * per;
  const long nparts = (nchunks + per - 1) / per;
  if (first < nchunks) {
    const long end = first + per < nchunks ? first + per : nchunks;
    uint32_t acc = crcs[first];
    for (long j = first + 1; j < end; ++j) acc = multmodp(j == nchunks - 1 ? x_last : x_chunk, acc) ^ crcs[j];
    part[t] = acc;
  }
  __syncthreads();
  if (t == 0) {
    uint32_t tot = part[0];
    for (long p = 1; p < nparts; ++p) tot = multmodp(p == nparts - 1 ? x_part_last : x_part, tot) ^ part[p];
    out[0] = tot;
  }
}

}  // namespace

int afl_crc32_partials(long nbytes) { return (int)((nbytes + kChunk - 1) / kChunk); }

int afl_crc32(const void* data, long nbytes, uint32_t* chunk_crcs, uint32_t* out, uint32_t x_chunk, uint32_t x_last,
              uint32_t x_part, uint32_t x_part_last, hipStream_t s) {
  if (nbytes <= 0 || (nbytes & 3) || (((uintptr_t)data) & 15)) return (int)hipErrorInvalidValue;
  const long nchunks = afl_crc32_partials(nbytes);
  const long per = (nchunks + 255) / 256;
  hipLaunchKernelGGL(k_crc_chunks, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s, (const uint32_t*)data,
                     nbytes, chunk_crcs);
  hipLaunchKernelGGL(k_crc_combine, dim3(1), dim3(256), 0, s, chunk_crcs, nchunks, per, x_chunk, x_last, x_part,
                     x_part_last, out);
  return (int)hipGetLastError();
}
