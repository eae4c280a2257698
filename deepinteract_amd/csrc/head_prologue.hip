// Fused head prologue: the first line of the contact head,
//     x = ELU(InstanceNorm2d(conv2d_1(T)))          ResNet2DInputWithOptAttention.forward,
//                                                   deepinteract_modules.py:1181-1184, 1228-1232
// computed WITHOUT materialising the [2H, L1, L2] pair tensor T (construct_interact_tensor,
// deepinteract_utils.py:158-172). conv2d_1 is 1x1, so on the outer concat it separates:
//     conv(T)[c, i, j] = A[c, i] + B[c, j],   A = W[:, :H] . h1[i],   B = W[:, H:] . h2[j] + b
// and the InstanceNorm statistics of a separable sum over the full L1 x L2 grid are analytic:
//     mean_c = mean_i A + mean_j B,    var_c = var_i A + var_j B      (biased, as InstanceNorm)
// so with s = gamma / sqrt(var_c + eps):
//     x[c, i, j] = ELU(a'[c, i] + b'[c, j]),  a' = s (A - mean A) + beta,  b' = s (B - mean B).
// Two kernels:
//  * k_prologue_tables: one block per (complex, group of PRO_CG channels). Rows of h are read
//    once per group with 16-B loads (one row per lane), the PRO_CG weight rows sit in LDS as
//    [2H][PRO_CG] (one broadcast ds_read_b128 per k), fp32 accumulation in k order; two-pass
//    mean / variance; the folded tables a', b' (and, for bf16, e^a', e^b') go to an fp32
//    workspace of di_head_prologue_work_bytes().
//  * k_prologue_rows: the [C, L1, L2] output as a pure store stream (the k_pair_rows structure:
//    a wave owns 64 rows, the b' segment lives in registers, a'[c, i] comes by readlane). bf16
//    uses e^(a+b) = e^a e^b: per element one add, one fma and one v_med3
//    (ELU(x) = med3(x, e^x - 1, 0), since e^x - 1 >= x) — no transcendental in the stream. A
//    channel whose tables leave the range where the product is exact in fp32 (|a'|, |b'| > 60)
//    is flagged and takes the exact exp path. fp32 output keeps expm1f (the parity mode).
// HBM: C * L1 * L2 * s bytes written, against 2H * L1 * L2 * s (pair tensor) + the
// conv / norm / ELU passes of the unfused path.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "common.h"
#include "../../include/deepinteract_amd.h"

namespace di {

constexpr int PRO_THREADS = 256;
// table-kernel launch shape, measured (profiles/r1_v8_prologue_tables_variants.json): 512 threads x
// 4 channels 47.7 us vs 256x4 57.6, 1024x4 48.4, 512x2 62.8 (bf16, 8 complexes)
constexpr int PRO_TTHREADS = 512;  // threads per table block (rows in flight)
constexpr int PRO_CG = 4;          // channels per table block (<= 4: one floatx4 of weights per k)
static_assert(PRO_CG >= 1 && PRO_CG <= 4, "PRO_CG");
constexpr int PRO_SEG = 128;       // 16-B chunks per row segment of the store stream (2 per lane)
constexpr float PRO_EXP_SAFE = 60.f;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// workspace layout, per (complex, channel): [a' (max_l1) | b' (max_l2) | e^a' (max_l1) |
// e^b' (max_l2)] fp32, then one int32 flag per (complex, channel): 1 = exact-exp path.
__host__ __device__ inline int64_t pro_table_stride(int max_l1, int max_l2) { return 2 * ((int64_t)max_l1 + max_l2); }

__device__ __forceinline__ void load8(const u16* p, float* v) {
  const u32x4 u = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __builtin_bit_cast(float, u[q] << 16);
    v[2 * q + 1] = __builtin_bit_cast(float, u[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float* v) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p);
  const floatx4 b = *reinterpret_cast<const floatx4*>(p + 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = a[q];
    v[4 + q] = b[q];
  }
}

// sum over the block of PRO_CG per-thread values (in place)
__device__ __forceinline__ void block_sum4(float* v, float* red) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q) red[w * PRO_CG + q] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i * PRO_CG + q];
    v[q] = t;
  }
}

// dot products of rows [h_row, h_row + n) of h with the PRO_CG weight rows wl[k][q]:
// out[q * stride + i] = sum_k w[q][k] h[i][k] (+ bias[q]); returns the per-thread sums.
template <typename T>
__device__ __forceinline__ void pro_dots(const T* __restrict__ h, int64_t h_row, int n, int hidden,
                                         const floatx4* wl, const float* bias, float* out, int64_t stride,
                                         float* sum) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const T* r = h + (h_row + i) * hidden;
    float acc[PRO_CG];
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q) acc[q] = 0.f;
    for (int k = 0; k < hidden; k += 8) {
      float x[8];
      load8(r + k, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const floatx4 wv = wl[k + e];
#pragma unroll
        for (int q = 0; q < PRO_CG; ++q) acc[q] = fmaf(wv[q], x[e], acc[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q) {
      const float a = acc[q] + bias[q];
      out[q * stride + i] = a;
      sum[q] += a;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(PRO_TTHREADS) void k_prologue_tables(const di_pair_desc* __restrict__ descs, int hidden,
                                                                 int channels, int max_l1, int max_l2, float eps,
                                                                 const T* __restrict__ h, const float* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 float* __restrict__ work) {
  __shared__ floatx4 wl[512];  // [2H][PRO_CG], hidden <= 256
  __shared__ float red[(PRO_TTHREADS / 64) * PRO_CG];
  const int groups = (channels + PRO_CG - 1) / PRO_CG;
  const int c0 = (blockIdx.x % groups) * PRO_CG, cpx = blockIdx.x / groups;
  const int nc = channels - c0 < PRO_CG ? channels - c0 : PRO_CG;
  const di_pair_desc d = descs[cpx];
  for (int k = threadIdx.x; k < 2 * hidden; k += blockDim.x) {
    floatx4 v;
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q) v[q] = q < nc ? w[(int64_t)(c0 + q) * 2 * hidden + k] : 0.f;
    wl[k] = v;
  }
  __syncthreads();
  const int64_t stride = pro_table_stride(max_l1, max_l2);
  float* ta = work + ((int64_t)cpx * channels + c0) * stride;  // channel q: ta + q * stride
  float* tb = ta + max_l1;
  float zero[PRO_CG], bq[PRO_CG];
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) {
    zero[q] = 0.f;
    bq[q] = q < nc ? bias[c0 + q] : 0.f;
  }
  float sa[PRO_CG], sb[PRO_CG];
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) sa[q] = sb[q] = 0.f;
  if (nc == PRO_CG) {
    pro_dots(h, d.h1_row, d.l1, hidden, wl, zero, ta, stride, sa);
    pro_dots(h, d.h2_row, d.l2, hidden, wl + hidden, bq, tb, stride, sb);
  } else {  // ragged last group (channels % PRO_CG != 0): one channel at a time
    for (int q = 0; q < nc; ++q) {
      for (int i = threadIdx.x; i < d.l1 + d.l2; i += blockDim.x) {
        const bool first = i < d.l1;
        const T* r = h + (first ? d.h1_row + i : d.h2_row + (i - d.l1)) * hidden;
        const floatx4* wk = first ? wl : wl + hidden;
        float acc = 0.f;
        for (int k = 0; k < hidden; k += 8) {
          float x[8];
          load8(r + k, x);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc = fmaf(wk[k + e][q], x[e], acc);
        }
        if (first) {
          ta[q * stride + i] = acc;
          sa[q] += acc;
        } else {
          acc += bq[q];
          tb[q * stride + (i - d.l1)] = acc;
          sb[q] += acc;
        }
      }
    }
  }
  block_sum4(sa, red);
  block_sum4(sb, red);
  float ma[PRO_CG], mb[PRO_CG], va[PRO_CG], vb[PRO_CG];
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) {
    ma[q] = sa[q] / (float)d.l1;
    mb[q] = sb[q] / (float)d.l2;
    va[q] = vb[q] = 0.f;
  }
  // two-pass variance: each thread re-reads only the entries it wrote
  for (int i = threadIdx.x; i < d.l1; i += blockDim.x)
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q)
      if (q < nc) {
        const float t = ta[q * stride + i] - ma[q];
        va[q] += t * t;
      }
  for (int j = threadIdx.x; j < d.l2; j += blockDim.x)
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q)
      if (q < nc) {
        const float t = tb[q * stride + j] - mb[q];
        vb[q] += t * t;
      }
  block_sum4(va, red);
  block_sum4(vb, red);
  float big[PRO_CG];
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) big[q] = 0.f;
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) {
    if (q >= nc) continue;
    const float var = va[q] / (float)d.l1 + vb[q] / (float)d.l2;
    const float s = gamma[c0 + q] / sqrtf(var + eps);
    const float bt = beta[c0 + q];
    float* a = ta + q * stride;
    float* b = tb + q * stride;
    float* ea = a + max_l1 + max_l2;
    float* eb = ea + max_l1;
    for (int i = threadIdx.x; i < d.l1; i += blockDim.x) {
      const float v = s * (a[i] - ma[q]) + bt;
      a[i] = v;
      ea[i] = expf(v);
      big[q] = fmaxf(big[q], fabsf(v));
    }
    for (int j = threadIdx.x; j < d.l2; j += blockDim.x) {
      const float v = s * (b[j] - mb[q]);
      b[j] = v;
      eb[j] = expf(v);
      big[q] = fmaxf(big[q], fabsf(v));
    }
  }
  // flag: any |a'|, |b'| beyond the exact-product range -> exact exp in the store stream
#pragma unroll
  for (int q = 0; q < PRO_CG; ++q) big[q] = big[q] > PRO_EXP_SAFE ? 1.f : 0.f;
  block_sum4(big, red);
  if (threadIdx.x == 0) {
    int* flags = reinterpret_cast<int*>(work + (int64_t)gridDim.x / groups * channels * stride);
#pragma unroll
    for (int q = 0; q < PRO_CG; ++q)
      if (q < nc) flags[(int64_t)cpx * channels + c0 + q] = big[q] > 0.f ? 1 : 0;
  }
}

template <typename T>
struct Pack16;
template <>
struct Pack16<float> {
  static constexpr int N = 4;
  __device__ static u32x4 pack(const float* v) {
    return (u32x4){__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                   __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3])};
  }
};
template <>
struct Pack16<u16> {
  static constexpr int N = 8;
  __device__ static u32x4 pack(const float* v) {
    return (u32x4){pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
  }
};

__device__ __forceinline__ float rdlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// ELU(a + b): exact (expm1f) or from the product e^a e^b (med3 form, see header)
template <bool PROD>
__device__ __forceinline__ float elu_ab(float a, float b, float ea, float eb) {
  const float x = a + b;
  if constexpr (PROD) return __builtin_amdgcn_fmed3f(x, fmaf(ea, eb, -1.0f), 0.f);
  else return x > 0.f ? x : expm1f(x);
}

// one wave: rows [r0, r1) (<= 64) of one output plane, segment-major
template <typename T, bool PROD>
__device__ __forceinline__ void pro_rows_wave(const float* __restrict__ ta, const float* __restrict__ tb,
                                              const float* __restrict__ tea, const float* __restrict__ teb,
                                              int r0, int r1, int nch, uint32_t pitch,
                                              __amdgpu_buffer_rsrc_t r) {
  constexpr int VEC = Pack16<T>::N;
  const int lane = threadIdx.x & 63;
  const float av = r0 + lane < r1 ? ta[r0 + lane] : 0.f;  // lane l: a' of row r0 + l
  const float eav = PROD && r0 + lane < r1 ? tea[r0 + lane] : 0.f;
  for (int seg = 0; seg < nch; seg += PRO_SEG) {
    const int k0 = seg + lane, k1 = seg + 64 + lane;
    const bool two = seg + 64 < nch;  // uniform
    float b0[VEC], b1[VEC], e0[VEC], e1[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      b0[e] = k0 < nch ? tb[k0 * VEC + e] : 0.f;
      b1[e] = two && k1 < nch ? tb[k1 * VEC + e] : 0.f;
      e0[e] = PROD && k0 < nch ? teb[k0 * VEC + e] : 0.f;
      e1[e] = PROD && two && k1 < nch ? teb[k1 * VEC + e] : 0.f;
    }
    for (int i = r0; i < r1; ++i) {
      const float a = rdlane(av, i - r0);
      const float ea = PROD ? rdlane(eav, i - r0) : 0.f;
      const int soff = (int)(i * pitch);
      float y[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) y[e] = elu_ab<PROD>(a, b0[e], ea, e0[e]);
      if (k0 < nch) __builtin_amdgcn_raw_buffer_store_b128(Pack16<T>::pack(y), r, k0 * 16, soff, 0);
      if (two) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) y[e] = elu_ab<PROD>(a, b1[e], ea, e1[e]);
        if (k1 < nch) __builtin_amdgcn_raw_buffer_store_b128(Pack16<T>::pack(y), r, k1 * 16, soff, 0);
      }
    }
  }
}

// Aligned path (L2 % VEC == 0, 16-B aligned outputs): work item = (complex, channel, 64 * waves
// rows); persistent grid-stride loop over items.
template <typename T>
__global__ __launch_bounds__(1024) void k_prologue_rows(const di_pair_desc* __restrict__ descs, int channels,
                                                        int max_l1, int max_l2, int rblocks, int items,
                                                        const float* __restrict__ work, T* __restrict__ out) {
  constexpr int VEC = Pack16<T>::N;
  const int rows_per_item = (int)blockDim.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = pro_table_stride(max_l1, max_l2);
  const int ncpx = items / (rblocks * channels);
  const int* flags = reinterpret_cast<const int*>(work + (int64_t)ncpx * channels * stride);
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int rb = item % rblocks;
    const int rest = item / rblocks;
    const int c = rest % channels;
    const int cpx = rest / channels;
    const di_pair_desc d = descs[cpx];
    const int r0 = rb * rows_per_item + 64 * wave;
    const int r1 = r0 + 64 < d.l1 ? r0 + 64 : d.l1;
    if (r0 >= r1) continue;  // uniform per wave
    const float* ta = work + ((int64_t)cpx * channels + c) * stride;
    const float* tb = ta + max_l1;
    const float* tea = tb + max_l2;
    const float* teb = tea + max_l1;
    const int nch = d.l2 / VEC;
    const uint32_t pitch = (uint32_t)d.l2 * sizeof(T);
    T* o = out + d.out_off + (int64_t)c * ((int64_t)d.l1 * d.l2);
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(o);
    if (sizeof(T) == 2 && __builtin_amdgcn_readfirstlane(flags[(int64_t)cpx * channels + c]) == 0)
      pro_rows_wave<T, true>(ta, tb, tea, teb, r0, r1, nch, pitch, r);
    else
      pro_rows_wave<T, false>(ta, tb, tea, teb, r0, r1, nch, pitch, r);
  }
}

// Generic path: one element per thread (exact exp).
template <typename T>
__global__ __launch_bounds__(PRO_THREADS) void k_prologue_flat(const di_pair_desc* __restrict__ descs, int channels,
                                                               int max_l1, int max_l2,
                                                               const float* __restrict__ work, T* __restrict__ out) {
  const int cpx = blockIdx.y;
  const di_pair_desc d = descs[cpx];
  const int64_t plane = (int64_t)d.l1 * d.l2;
  const int64_t n = plane * channels;
  const int64_t stride = pro_table_stride(max_l1, max_l2);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(q / plane);
    const int64_t p = q - c * plane;
    const int i = (int)(p / d.l2), j = (int)(p - (int64_t)i * d.l2);
    const float* ta = work + ((int64_t)cpx * channels + c) * stride;
    const float y = elu_ab<false>(ta[i], ta[max_l1 + j], 0.f, 0.f);
    if constexpr (sizeof(T) == 2) out[d.out_off + q] = (u16)(pack_bf16x2(y, 0.f) & 0xffffu);
    else out[d.out_off + q] = y;
  }
}

}  // namespace di

using namespace di;

// launch shape of the row-streaming store kernel: 512 resident 4-wave blocks
constexpr int PRO_ROW_BLOCKS = 512;
constexpr int PRO_ROW_WAVES = 4;

extern "C" int64_t di_head_prologue_work_bytes(int32_t num_complexes, int32_t max_l1, int32_t max_l2,
                                               int32_t channels) {
  if (num_complexes <= 0 || max_l1 <= 0 || max_l2 <= 0 || channels <= 0) return 0;
  const int64_t pc = (int64_t)num_complexes * channels;
  return pc * pro_table_stride(max_l1, max_l2) * (int64_t)sizeof(float) + pc * (int64_t)sizeof(int32_t);
}

extern "C" int di_head_prologue(di_dtype dt, const di_pair_desc* descs, int32_t num_complexes, int32_t max_l1,
                                int32_t max_l2, int32_t hidden, int32_t channels, int32_t aligned16, const void* h,
                                const float* conv_w, const float* conv_b, const float* in_gamma,
                                const float* in_beta, float eps, float* work, void* out, void* stream) {
  if (!descs || !h || !conv_w || !conv_b || !in_gamma || !in_beta || !work || !out || num_complexes <= 0 ||
      max_l1 <= 0 || max_l2 <= 0 || hidden <= 0 || hidden > 256 || hidden % 8 != 0 || channels <= 0 ||
      !(eps >= 0.f) || (dt != DI_BF16 && dt != DI_F32))
    return DI_EINVAL;
  if (((uintptr_t)h & 15) != 0) return DI_EINVAL;  // 16-B row loads in the table kernel
  if ((int64_t)max_l1 * max_l2 >= (1LL << 31) / (dt == DI_BF16 ? 2 : 4)) return DI_ERANGE;  // 32-bit row offsets
  hipStream_t s = (hipStream_t)stream;
  const int groups = (channels + PRO_CG - 1) / PRO_CG;
  const unsigned tgrid = (unsigned)num_complexes * (unsigned)groups;
  if (dt == DI_BF16)
    hipLaunchKernelGGL(k_prologue_tables<u16>, dim3(tgrid), dim3(PRO_TTHREADS), 0, s, descs, hidden, channels, max_l1,
                       max_l2, eps, (const u16*)h, conv_w, conv_b, in_gamma, in_beta, work);
  else
    hipLaunchKernelGGL(k_prologue_tables<float>, dim3(tgrid), dim3(PRO_TTHREADS), 0, s, descs, hidden, channels,
                       max_l1, max_l2, eps, (const float*)h, conv_w, conv_b, in_gamma, in_beta, work);
  if (aligned16) {
    const int rows = 64 * PRO_ROW_WAVES;
    const int rblocks = (max_l1 + rows - 1) / rows;
    const int64_t items64 = (int64_t)num_complexes * channels * rblocks;
    if (items64 > INT32_MAX) return DI_ERANGE;
    const int items = (int)items64;
    const unsigned grid = (unsigned)(items < PRO_ROW_BLOCKS ? items : PRO_ROW_BLOCKS);
    if (dt == DI_BF16)
      hipLaunchKernelGGL(k_prologue_rows<u16>, dim3(grid), dim3(rows), 0, s, descs, channels, max_l1, max_l2, rblocks,
                         items, (const float*)work, (u16*)out);
    else
      hipLaunchKernelGGL(k_prologue_rows<float>, dim3(grid), dim3(rows), 0, s, descs, channels, max_l1, max_l2,
                         rblocks, items, (const float*)work, (float*)out);
  } else {
    const int64_t per = (int64_t)channels * max_l1 * max_l2;
    const int64_t blocks = (per + PRO_THREADS - 1) / PRO_THREADS;
    dim3 grid((unsigned)(blocks < 4096 ? blocks : 4096), (unsigned)num_complexes);
    if (dt == DI_BF16)
      hipLaunchKernelGGL(k_prologue_flat<u16>, grid, dim3(PRO_THREADS), 0, s, descs, channels, max_l1, max_l2,
                         (const float*)work, (u16*)out);
    else
      hipLaunchKernelGGL(k_prologue_flat<float>, grid, dim3(PRO_THREADS), 0, s, descs, channels, max_l1, max_l2,
                         (const float*)work, (float*)out);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
