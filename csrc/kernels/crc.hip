// CRC-32 (IEEE 802.3 polynomial, reflected — the value zlib.crc32 / zip records carry) of a device
// buffer, for the checkpoint writer (attackfl_amd/utils/ckpt.py).  The writer emits the reference's
// torch.save zip layout itself (server.py:549-553 writes one .pth per successful round): per round only
// the storage bytes and their CRC change, and the CRC of a 19.5 MB hypernetwork arena costs ~23 ms on
// one host core (zlib) — longer than a round.  Here it is ONE launch on the checkpoint stream, fully
// parallel (no sequential fold):
//
//   CRC linearity over GF(2): with R(M) the CRC register after M from a zero register (no final xor),
//   R(C_0 || ... || C_{n-1}) = XOR_i  R(C_i) (*) x^(8 * (bytes after C_i))  mod P,
//   and zlib's crc32(M) = ~(R(M) ^ (0xFFFFFFFF (*) x^(8 |M|))).
//   Thread i: slice-by-4 table CRC of its 256-byte chunk (tables in LDS) -> R(C_i); its shift constant
//   x^(8 * (L - end_i)) from the host's table of x^(2^k) (<= 40 products); the product is XORed
//   into the result with a wave xor-reduction and one atomic xor per workgroup (xor is exact and
//   order-free: the result is deterministic).  The result word is pre-set to ~(0xFFFFFFFF (*) x^(8L))
//   by the host, so it ends as the final CRC.
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

struct CrcPow {
  uint32_t x2k[48];  // x^(2^k) mod P, k = 0..47
};

__global__ void __launch_bounds__(256) k_crc32(const uint32_t* __restrict__ data, long nbytes, CrcPow pw,
                                               uint32_t* __restrict__ out) {
  __shared__ uint32_t T[4][256];
  __shared__ uint32_t red[4];
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
  uint32_t term = 0;
  if (b0 < nbytes) {
    const long len = nbytes - b0 < kChunk ? nbytes - b0 : kChunk;  // multiple of 4
    const uint32_t* w = data + b0 / 4;
    uint32_t crc = 0;  // zero register: R(C_i)
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
    // shift by the bytes behind this chunk: x^(8 * after) = prod over set bits k of 8*after of x^(2^k)
    uint64_t e = (uint64_t)(nbytes - b0 - len) * 8u;
    term = crc;
    for (int k = 0; e; ++k, e >>= 1)
      if (e & 1) term = multmodp(pw.x2k[k], term);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) term ^= __shfl_xor(term, o, 64);
  if ((t & 63) == 0) red[t >> 6] = term;
  __syncthreads();
  if (t == 0) atomicXor(out, (red[0] ^ red[1]) ^ (red[2] ^ red[3]));
}

}  // namespace

int afl_crc32(const void* data, long nbytes, const uint32_t* x2k, uint32_t* out, hipStream_t s) {
  if (nbytes <= 0 || (nbytes & 3) || (((uintptr_t)data) & 15)) return (int)hipErrorInvalidValue;
  const long nchunks = (nbytes + kChunk - 1) / kChunk;
  CrcPow pw;
  for (int k = 0; k < 48; ++k) pw.x2k[k] = x2k[k];
  hipLaunchKernelGGL(k_crc32, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s, (const uint32_t*)data,
                     nbytes, pw, out);
  return (int)hipGetLastError();
}
