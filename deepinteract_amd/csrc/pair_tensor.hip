// L1 x L2 outer-concat interaction tensor (construct_interact_tensor, pad=False,
// deepinteract_utils.py:158-172):
//     T[c, i, j] = h1[i, c]          for c <  H
//     T[c, i, j] = h2[j, c - H]      for c >= H          (NCHW, [2H, L1, L2] per complex)
// The reference materialises it with two repeat_interleave tensors plus a cat (3x the output
// bytes); here every output byte is written exactly once: a pure HBM store stream (512 MB per
// 2x1000-residue complex in bf16), with non-temporal 16-B stores (write-once data, kept out of
// the caches the concurrently running GeoT kernels use).
//
// Persistent grid: a few blocks per CU walk work items (complex, channel, 64K-element chunk);
// no LDS, so the kernel co-resides with the GeoT kernels on the other stream (which hold the
// LDS) instead of starving them of CU slots. Chain-2 planes read the transposed features hT
// [H, Nt] (written by the final node layer), so each 16-B store is fed by one 16-B load.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "common.h"
#include "../../include/deepinteract_amd.h"

namespace di {

constexpr int PAIR_THREADS = 256;
constexpr int PAIR_CHUNK = 65536;  // elements per work item
constexpr int PAIR_MAX_BLOCKS = 256;  // one 4-wave block per CU: leaves the GeoT kernels their issue slots
constexpr int PAIR_UNROLL = 4;

template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  using V = floatx4;
  static constexpr int N = 4;
};
typedef unsigned int uintx4 __attribute__((ext_vector_type(4)));
template <>
struct Vec16<u16> {
  using V = uintx4;
  static constexpr int N = 8;
};

// Row index of flat plane position q (q < 2^24, exact in fp32): the fp32 quotient is off by at
// most one and is corrected with two selects, instead of a 64-bit integer division per store.
__device__ __forceinline__ void plane_rc(uint32_t q, uint32_t l2, float inv_l2, uint32_t& i, uint32_t& j) {
  int32_t ii = (int32_t)((float)q * inv_l2);
  int32_t jj = (int32_t)q - ii * (int32_t)l2;
  if (jj < 0) { --ii; jj += (int32_t)l2; }
  if (jj >= (int32_t)l2) { ++ii; jj -= (int32_t)l2; }
  i = (uint32_t)ii;
  j = (uint32_t)jj;
}

template <typename T, bool ALIGNED>
__global__ __launch_bounds__(PAIR_THREADS) void k_pair_tensor(const di_pair_desc* __restrict__ descs, int hidden,
                                                            const T* __restrict__ h, const T* __restrict__ hT,
                                                            int nrows, int chunks, int items,
                                                            T* __restrict__ out) {
  using V = typename Vec16<T>::V;
  constexpr int VEC = Vec16<T>::N;
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int chunk = item % chunks;
    const int rest = item / chunks;
    const int c = rest % (2 * hidden);
    const int cpx = rest / (2 * hidden);
    const di_pair_desc d = descs[cpx];
    const uint32_t l2 = (uint32_t)d.l2;
    const uint32_t plane = (uint32_t)d.l1 * l2;
    const uint32_t q_begin = (uint32_t)chunk * PAIR_CHUNK;
    if (q_begin >= plane) continue;  // uniform per block
    const uint32_t q_end = q_begin + PAIR_CHUNK < plane ? q_begin + PAIR_CHUNK : plane;
    const float inv_l2 = 1.0f / (float)l2;
    T* o = out + d.out_off + (int64_t)c * plane;
    const bool second = c >= hidden;
    const T* h1c = h + d.h1_row * hidden + c;                                      // column c of chain 1
    const T* h2t = hT ? hT + (int64_t)(c - hidden) * nrows + d.h2_row : nullptr;  // row c-H of hT
    const T* h2c = h + d.h2_row * hidden + (c - hidden);                           // strided fallback
    if (ALIGNED) {
      // PAIR_UNROLL independent 16-B vectors per thread per trip: the hT loads (L2 hits) of a
      // trip are all in flight before its stores
      constexpr uint32_t STEP = PAIR_THREADS * VEC;
      for (uint32_t q0 = q_begin + threadIdx.x * VEC; q0 < q_end; q0 += PAIR_UNROLL * STEP) {
        V vals[PAIR_UNROLL];
#pragma unroll
        for (int u = 0; u < PAIR_UNROLL; ++u) {
          const uint32_t q = q0 + u * STEP;
          if (q < q_end) {
            uint32_t i, j;
            plane_rc(q, l2, inv_l2, i, j);
            if (second) {
              vals[u] = *reinterpret_cast<const V*>(h2t + j);  // j % VEC == 0, L2 % VEC == 0: no row wrap
            } else {
              const T v0 = h1c[i * hidden];
              T tmp[VEC];
#pragma unroll
              for (int t = 0; t < VEC; ++t) tmp[t] = v0;
              vals[u] = *reinterpret_cast<const V*>(tmp);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < PAIR_UNROLL; ++u) {
          const uint32_t q = q0 + u * STEP;
          if (q < q_end) __builtin_nontemporal_store(vals[u], reinterpret_cast<V*>(o + q));
        }
      }
    } else {
      for (uint32_t q = q_begin + threadIdx.x; q < q_end; q += PAIR_THREADS) {
        uint32_t i, j;
        plane_rc(q, l2, inv_l2, i, j);
        o[q] = second ? (h2t ? h2t[j] : h2c[j * hidden]) : h1c[i * hidden];
      }
    }
  }
}

}  // namespace di

using namespace di;

extern "C" int di_pair_tensor(di_dtype dt, const di_pair_desc* descs, int32_t num_complexes, int32_t max_l1,
                              int32_t max_l2, int32_t hidden, int32_t aligned16, const void* h, const void* hT,
                              int32_t num_rows, void* out, void* stream) {
  if (!descs || !h || !out || num_complexes <= 0 || max_l1 <= 0 || max_l2 <= 0 || hidden <= 0) return DI_EINVAL;
  if (aligned16 && !hT) return DI_EINVAL;
  const int64_t plane = (int64_t)max_l1 * max_l2;
  const int chunks = (int)((plane + PAIR_CHUNK - 1) / PAIR_CHUNK);
  if (plane >= (1 << 24)) return DI_ERANGE;  // flat plane offsets are exact in fp32 / uint32
  const int64_t items64 = (int64_t)num_complexes * 2 * hidden * chunks;
  if (items64 > INT32_MAX) return DI_ERANGE;
  const int items = (int)items64;
  static const int max_blocks = [] {
    const char* e = getenv("DI_PAIR_BLOCKS");  // tuning knob: resident blocks of the persistent grid
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : PAIR_MAX_BLOCKS;
  }();
  const unsigned grid = (unsigned)(items < max_blocks ? items : max_blocks);
  hipStream_t s = (hipStream_t)stream;
  // aligned16: every channel plane (L1*L2), out_off, L2 and h2_row is a multiple of 16 bytes of
  // elements: 16-B vector loads and non-temporal 16-B stores.
  if (dt == DI_BF16) {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<u16, true>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out);
    else
      hipLaunchKernelGGL((k_pair_tensor<u16, false>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out);
  } else {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<float, true>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out);
    else
      hipLaunchKernelGGL((k_pair_tensor<float, false>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
