// Contact-head body ops: the dilated-ResNet head stays on PyTorch-ROCm for its
// convolutions (MIOpen / hipBLASLt), but its HBM-bound normalisation passes are fused here.
//
//  * di_inorm_elu: y = ELU(InstanceNorm2d(x)) for one [C, HW] image (batch 1, NCHW), the
//    `x = conv(ELU(inorm(x)))` pattern of every inorm ResNet block (ResNet.forward,
//    deepinteract_modules.py:1075-1095; InstanceNorm2d(eps=1e-6, affine=True) :1016-1030, ELU :1080)
//    and of the head prologue (:1231-1232). Torch runs it as 2 norm kernels + 1 ELU kernel
//    (stats read, normalise read + write, ELU read + write): 5 plane passes. Here: 3.
//      k_inorm_stats  grid (split, C): each block reduces a contiguous slice of one channel
//                     plane with 16-B loads into fp64 (sum, sum of squares) partials.
//      k_inorm_apply  grid (split, C): every block folds its channel's partials (biased variance,
//                     as InstanceNorm) into mean and scale = gamma / sqrt(var + eps), then streams
//                     y = ELU((x - mean) * scale + beta) (ELU(z) = z > 0 ? z : expm1(z)).
//  * di_se_scale_add: y = (x + b[c]) * s[c] + res — the block's last conv bias, SEBlock's channel
//    gate (:954-970) and the residual add (:1095): 3 plane passes instead of 7.
//  * di_channel_mean: SEBlock's x.mean(dim=(2, 3)) (+ the deferred conv bias), one read pass.
// The convs before an InstanceNorm run without their bias (a per-channel constant cancels in
// the normalisation exactly), so the head does no separate bias-add passes.
// fp32 accumulation everywhere, fp64 for the statistics; bf16 storage rounds once (RNE).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "common.h"
#include "deepinteract_amd.h"

namespace di {

constexpr int HO_THREADS = 256;
constexpr int HO_MAX_SPLIT = 64;

typedef unsigned int u32x4h __attribute__((ext_vector_type(4)));

// 8 elements per 16-B vector for bf16, 4 for fp32; scalar access by element index for the
// unaligned head / tail of a channel plane (planes start at c * hw, any hw)
template <typename T>
struct Vec;
template <>
struct Vec<u16> {
  static constexpr int N = 8;
  __device__ static void load(const u16* p, float* v) {
    const u32x4h u = __builtin_nontemporal_load(reinterpret_cast<const u32x4h*>(p));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __builtin_bit_cast(float, u[q] << 16);
      v[2 * q + 1] = __builtin_bit_cast(float, u[q] & 0xffff0000u);
    }
  }
  __device__ static void store(u16* p, const float* v) {
    u32x4h u;
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = pack_bf16x2(v[2 * q], v[2 * q + 1]);
    *reinterpret_cast<u32x4h*>(p) = u;
  }
  __device__ static float ld1(const u16* p) { return __builtin_bit_cast(float, (uint32_t)*p << 16); }
  __device__ static void st1(u16* p, float v) { *p = (u16)(pack_bf16x2(v, 0.f) & 0xffffu); }
  __device__ static float round(float v) { return __builtin_bit_cast(float, (pack_bf16x2(v, 0.f) & 0xffffu) << 16); }
};
template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float* v) {
    const floatx4 a = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = a[q];
  }
  __device__ static void store(float* p, const float* v) {
    *reinterpret_cast<floatx4*>(p) = (floatx4){v[0], v[1], v[2], v[3]};
  }
  __device__ static float ld1(const float* p) { return *p; }
  __device__ static void st1(float* p, float v) { *p = v; }
  __device__ static float round(float v) { return v; }
};

// The plane of channel c is elements [c*hw, (c+1)*hw) of a 16-B aligned buffer. Its whole 16-B
// vectors [v0, v1) are split over the `split` blocks of the channel; the scalar head
// [c*hw, v0*N) and tail [v1*N, (c+1)*hw) go to the last block.
struct Plane {
  int64_t lo, hi;      // this block's 16-B vectors
  int64_t h0, nh, t0;  // scalar head [h0, h0 + nh), scalar tail [t0, t0 + nt)
  int64_t ns;          // nh + nt
  __device__ Plane(int64_t hw, int n, int c, int split, int b) {
    const int64_t e0 = (int64_t)c * hw, e1 = e0 + hw;
    int64_t v0 = (e0 + n - 1) / n, v1 = e1 / n;
    if (v1 <= v0) {  // no whole vector inside the plane: all scalar
      v0 = v1 = 0;
      h0 = e0, nh = hw, t0 = e1, ns = hw;
    } else {
      h0 = e0, nh = v0 * n - e0, t0 = v1 * n, ns = nh + (e1 - t0);
    }
    const int64_t per = (v1 - v0 + split - 1) / split;
    lo = v0 + per * b;
    hi = lo + per < v1 ? lo + per : v1;
    if (lo > hi) lo = hi;
  }
  __device__ int64_t nscalar(int) const { return ns; }
  __device__ int64_t scalar_at(int64_t i, int) const { return i < nh ? h0 + i : t0 + (i - nh); }
};

template <typename T>
__global__ __launch_bounds__(HO_THREADS) void k_inorm_stats(const T* __restrict__ x, int64_t hw,
                                                            double* __restrict__ part) {
  using V = Vec<T>;
  const int c = blockIdx.y, split = gridDim.x;
  const Plane P(hw, V::N, c, split, blockIdx.x);
  double s = 0.0, ss = 0.0;
  for (int64_t i = P.lo + threadIdx.x; i < P.hi; i += HO_THREADS) {
    float v[V::N];
    V::load(x + i * V::N, v);
    float fs = 0.f, fss = 0.f;  // 4-8 terms in fp32, then fp64
#pragma unroll
    for (int q = 0; q < V::N; ++q) {
      fs += v[q];
      fss = fmaf(v[q], v[q], fss);
    }
    s += fs;
    ss += fss;
  }
  if (blockIdx.x == split - 1) {
    const int64_t ns = P.nscalar(V::N);
    for (int64_t i = threadIdx.x; i < ns; i += HO_THREADS) {
      const float v = V::ld1(x + P.scalar_at(i, V::N));
      s += v;
      ss += (double)v * v;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    ss += __shfl_xor(ss, off);
  }
  __shared__ double red[2][HO_THREADS / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = s;
    red[1][wave] = ss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < HO_THREADS / 64; ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    part[((int64_t)c * split + blockIdx.x) * 2 + 0] = a;
    part[((int64_t)c * split + blockIdx.x) * 2 + 1] = b;
  }
}

__device__ __forceinline__ float elu1(float z) { return z > 0.f ? z : expm1f(z); }

template <typename T>
__global__ __launch_bounds__(HO_THREADS) void k_inorm_apply(const T* __restrict__ x, int64_t hw,
                                                            const double* __restrict__ part,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            T* __restrict__ y) {
  using V = Vec<T>;
  const int c = blockIdx.y, split = gridDim.x;
  __shared__ float sc[2];  // mean, gamma * rstd
  if (threadIdx.x < 64) {
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < split; i += 64) {
      a += part[((int64_t)c * split + i) * 2 + 0];
      b += part[((int64_t)c * split + i) * 2 + 1];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a += __shfl_xor(a, off);
      b += __shfl_xor(b, off);
    }
    if (threadIdx.x == 0) {
      const double mean = a / (double)hw;
      double var = b / (double)hw - mean * mean;  // biased, as InstanceNorm2d
      var = var > 0.0 ? var : 0.0;
      sc[0] = (float)mean;
      sc[1] = (float)((double)gamma[c] / sqrt(var + (double)eps));
    }
  }
  __syncthreads();
  // (x - mean) * (gamma * rstd) + beta: centring first keeps outputs near zero accurate when a
  // channel's mean is large against its spread (the order torch's normalisation uses)
  const float mean = sc[0], scale = sc[1], shift = beta[c];
  const Plane P(hw, V::N, c, split, blockIdx.x);
  for (int64_t i = P.lo + threadIdx.x; i < P.hi; i += HO_THREADS) {
    float v[V::N];
    V::load(x + i * V::N, v);
#pragma unroll
    for (int q = 0; q < V::N; ++q) v[q] = elu1(fmaf(v[q] - mean, scale, shift));
    V::store(y + i * V::N, v);
  }
  if (blockIdx.x == split - 1) {
    const int64_t ns = P.nscalar(V::N);
    for (int64_t i = threadIdx.x; i < ns; i += HO_THREADS) {
      const int64_t e = P.scalar_at(i, V::N);
      V::st1(y + e, elu1(fmaf(V::ld1(x + e) - mean, scale, shift)));
    }
  }
}

template <typename T>
__global__ __launch_bounds__(HO_THREADS) void k_se_scale_add(const T* __restrict__ x, const float* __restrict__ s,
                                                             const float* __restrict__ bias,
                                                             const T* __restrict__ res, int64_t hw,
                                                             T* __restrict__ y) {
#pragma clang fp contract(off)  // + bias, * s and + res round separately, as torch's kernels do
  using V = Vec<T>;
  const int c = blockIdx.y, split = gridDim.x;
  const float g = s[c], bc = bias ? bias[c] : 0.f;
  const Plane P(hw, V::N, c, split, blockIdx.x);
  for (int64_t i = P.lo + threadIdx.x; i < P.hi; i += HO_THREADS) {
    float a[V::N], r[V::N];
    V::load(x + i * V::N, a);
    V::load(res + i * V::N, r);
    // torch rounds x * s to the storage type before the residual add; so does this
#pragma unroll
    for (int q = 0; q < V::N; ++q) a[q] = V::round(V::round(a[q] + bc) * g) + r[q];
    V::store(y + i * V::N, a);
  }
  if (blockIdx.x == split - 1) {
    const int64_t ns = P.nscalar(V::N);
    for (int64_t i = threadIdx.x; i < ns; i += HO_THREADS) {
      const int64_t e = P.scalar_at(i, V::N);
      V::st1(y + e, V::round(V::round(V::ld1(x + e) + bc) * g) + V::ld1(res + e));
    }
  }
}

// mean[c] = sum of the channel's partials / hw (+ bias[c]): SEBlock's x.mean(dim=(2, 3)) of a
// conv output whose bias is applied later (di_se_scale_add)
__global__ void k_channel_mean(const double* __restrict__ part, int split, int channels, int64_t hw,
                               const float* __restrict__ bias, float* __restrict__ mean) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= channels) return;
  double a = 0.0;
  for (int i = 0; i < split; ++i) a += part[((int64_t)c * split + i) * 2];
  mean[c] = (float)(a / (double)hw + (bias ? (double)bias[c] : 0.0));
}

// blocks per channel: fill the chip (>= ~2048 blocks) without slices under 2 vectors per thread
static int ho_split(int channels, int64_t hw, int vec) {
  int split = (2048 + channels - 1) / channels;
  split = split < 1 ? 1 : (split > HO_MAX_SPLIT ? HO_MAX_SPLIT : split);
  const int64_t nvec = hw / vec;
  while (split > 1 && nvec / split < 2 * HO_THREADS) split >>= 1;  // >= 2 vectors per thread
  return split;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace di

using namespace di;

extern "C" int64_t di_inorm_work_bytes(int32_t channels, int64_t hw) {
  (void)hw;
  return (int64_t)channels * HO_MAX_SPLIT * 2 * (int64_t)sizeof(double);
}

extern "C" int di_inorm_elu(di_dtype dt, const void* x, int32_t channels, int64_t hw, const float* gamma,
                            const float* beta, float eps, void* work, void* y, void* stream) {
  if (!x || !gamma || !beta || !work || !y || channels <= 0 || channels > 65535 || hw <= 0) return DI_EINVAL;
  if ((dt != DI_F32 && dt != DI_BF16) || !aligned16(x) || !aligned16(y)) return DI_EINVAL;
  const int vec = dt == DI_BF16 ? 8 : 4;
  const int split = ho_split(channels, hw, vec);
  const dim3 grid(split, channels);
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(work);
  if (dt == DI_BF16) {
    hipLaunchKernelGGL(k_inorm_stats<u16>, grid, dim3(HO_THREADS), 0, s, (const u16*)x, hw, part);
    hipLaunchKernelGGL(k_inorm_apply<u16>, grid, dim3(HO_THREADS), 0, s, (const u16*)x, hw, part, gamma, beta,
                       eps, (u16*)y);
  } else {
    hipLaunchKernelGGL(k_inorm_stats<float>, grid, dim3(HO_THREADS), 0, s, (const float*)x, hw, part);
    hipLaunchKernelGGL(k_inorm_apply<float>, grid, dim3(HO_THREADS), 0, s, (const float*)x, hw, part, gamma,
                       beta, eps, (float*)y);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_channel_mean(di_dtype dt, const void* x, int32_t channels, int64_t hw, const float* bias,
                               void* work, float* mean, void* stream) {
  if (!x || !work || !mean || channels <= 0 || channels > 65535 || hw <= 0) return DI_EINVAL;
  if ((dt != DI_F32 && dt != DI_BF16) || !aligned16(x)) return DI_EINVAL;
  const int split = ho_split(channels, hw, dt == DI_BF16 ? 8 : 4);
  const dim3 grid(split, channels);
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(work);
  if (dt == DI_BF16)
    hipLaunchKernelGGL(k_inorm_stats<u16>, grid, dim3(HO_THREADS), 0, s, (const u16*)x, hw, part);
  else
    hipLaunchKernelGGL(k_inorm_stats<float>, grid, dim3(HO_THREADS), 0, s, (const float*)x, hw, part);
  hipLaunchKernelGGL(k_channel_mean, dim3((channels + 63) / 64), dim3(64), 0, s, part, split, channels, hw, bias, mean);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_se_scale_add(di_dtype dt, const void* x, const float* scale, const float* bias, const void* res,
                               int32_t channels, int64_t hw, void* y, void* stream) {
  if (!x || !scale || !res || !y || channels <= 0 || channels > 65535 || hw <= 0) return DI_EINVAL;
  if ((dt != DI_F32 && dt != DI_BF16) || !aligned16(x) || !aligned16(res) || !aligned16(y)) return DI_EINVAL;
  const int vec = dt == DI_BF16 ? 8 : 4;
  const dim3 grid(ho_split(channels, hw, vec), channels);
  hipStream_t s = (hipStream_t)stream;
  if (dt == DI_BF16)
    hipLaunchKernelGGL(k_se_scale_add<u16>, grid, dim3(HO_THREADS), 0, s, (const u16*)x, scale, bias,
                       (const u16*)res, hw, (u16*)y);
  else
    hipLaunchKernelGGL(k_se_scale_add<float>, grid, dim3(HO_THREADS), 0, s, (const float*)x, scale, bias,
                       (const float*)res, hw, (float*)y);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
