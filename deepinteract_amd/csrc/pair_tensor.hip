// L1 x L2 outer-concat interaction tensor (construct_interact_tensor, pad=False,
// deepinteract_utils.py:158-172):
//     T[c, i, j] = h1[i, c]          for c <  H
//     T[c, i, j] = h2[j, c - H]      for c >= H          (NCHW, [2H, L1, L2] per complex)
// The reference materialises it with two repeat_interleave tensors plus a cat (3x the output
// bytes); here every output byte is written exactly once and nothing else is written or
// re-read: the kernel is a pure HBM store stream (512 MB per 2x1000-residue complex in bf16).
//
// Grid: x = 64K-element chunk of a [L1*L2] channel plane, y = channel (2H), z = complex.
// Channel planes of chain 2 are served from a copy of column h2[:, c-H] staged in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"
#include "../../include/deepinteract_amd.h"

namespace di {

constexpr int PAIR_THREADS = 256;
constexpr int PAIR_CHUNK = 65536;   // elements per block
constexpr int PAIR_MAX_L = 8192;    // longest chain the LDS column buffer holds

template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  using V = floatx4;
  static constexpr int N = 4;
};
template <>
struct Vec16<u16> {
  using V = uint4;
  static constexpr int N = 8;
};

template <typename T, bool ALIGNED>
__global__ __launch_bounds__(PAIR_THREADS) void k_pair_tensor(const di_pair_desc* __restrict__ descs, int hidden,
                                                            const T* __restrict__ h, T* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) T col[PAIR_MAX_L];
  constexpr int VEC = Vec16<T>::N;
  const di_pair_desc d = descs[blockIdx.z];
  const int c = blockIdx.y;
  const int64_t plane = (int64_t)d.l1 * d.l2;
  const int64_t q_begin = (int64_t)blockIdx.x * PAIR_CHUNK;
  if (q_begin >= plane) return;  // uniform per block
  const int64_t q_end = q_begin + PAIR_CHUNK < plane ? q_begin + PAIR_CHUNK : plane;
  T* o = out + d.out_off + (int64_t)c * plane;
  const bool second = c >= hidden;
  if (second) {
    for (int j = threadIdx.x; j < d.l2; j += PAIR_THREADS) col[j] = h[(d.h2_row + j) * hidden + (c - hidden)];
    __syncthreads();
  }
  const T* h1c = h + d.h1_row * hidden + c;
  for (int64_t q = q_begin + (int64_t)threadIdx.x * VEC; q < q_end; q += (int64_t)PAIR_THREADS * VEC) {
    T vals[VEC];
    if (ALIGNED && d.l2 >= VEC) {
      const int i = (int)(q / d.l2);
      const int j = (int)(q - (int64_t)i * d.l2);
      if (second) {
#pragma unroll
        for (int t = 0; t < VEC; ++t) {
          const int jj = j + t < d.l2 ? j + t : j + t - d.l2;
          vals[t] = col[jj];
        }
      } else {
        const T v0 = h1c[(int64_t)i * hidden];
        const T v1 = i + 1 < d.l1 ? h1c[(int64_t)(i + 1) * hidden] : v0;
#pragma unroll
        for (int t = 0; t < VEC; ++t) vals[t] = j + t < d.l2 ? v0 : v1;
      }
      *reinterpret_cast<typename Vec16<T>::V*>(o + q) = *reinterpret_cast<const typename Vec16<T>::V*>(vals);
    } else {
#pragma unroll
      for (int t = 0; t < VEC; ++t) {
        const int64_t qq = q + t;
        if (qq < q_end) {
          const int i = (int)(qq / d.l2);
          const int j = (int)(qq - (int64_t)i * d.l2);
          o[qq] = second ? col[j] : h1c[(int64_t)i * hidden];
        }
      }
    }
  }
}

}  // namespace di

using namespace di;

extern "C" int di_pair_tensor(di_dtype dt, const di_pair_desc* descs, int32_t num_complexes, int32_t max_l1,
                              int32_t max_l2, int32_t hidden, int32_t aligned16, const void* h, void* out,
                              void* stream) {
  if (!descs || !h || !out || num_complexes <= 0 || max_l1 <= 0 || max_l2 <= 0 || hidden <= 0) return DI_EINVAL;
  if (max_l2 > PAIR_MAX_L || num_complexes > 65535) return DI_EINVAL;
  const int64_t plane = (int64_t)max_l1 * max_l2;
  dim3 grid((unsigned)((plane + PAIR_CHUNK - 1) / PAIR_CHUNK), (unsigned)(2 * hidden), (unsigned)num_complexes);
  hipStream_t s = (hipStream_t)stream;
  // aligned16: the caller guarantees every channel plane (L1*L2) and every out_off is a multiple
  // of 16 bytes, which enables the 16-B vector store path.
  if (dt == DI_BF16) {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<u16, true>), grid, dim3(PAIR_THREADS), 0, s, descs, hidden, (const u16*)h, (u16*)out);
    else
      hipLaunchKernelGGL((k_pair_tensor<u16, false>), grid, dim3(PAIR_THREADS), 0, s, descs, hidden, (const u16*)h, (u16*)out);
  } else {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<float, true>), grid, dim3(PAIR_THREADS), 0, s, descs, hidden, (const float*)h, (float*)out);
    else
      hipLaunchKernelGGL((k_pair_tensor<float, false>), grid, dim3(PAIR_THREADS), 0, s, descs, hidden, (const float*)h, (float*)out);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
