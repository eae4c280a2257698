// Building blocks of the module-level API (deepinteract_amd/layers.py): the reference's
// ConformationModule / MultiHeadGeometricAttentionLayer / GeometricTransformerModule can be called
// one module at a time, with the same weights and semantics as the fused layer kernels.
//
//   di_gemm_bias_act   y = res + act(W x + b): every Linear of those modules (BatchNorm folded
//                      into W, b on the host), deepinteract_modules.py:99-104, 696-723, 923-943
//   di_geo_attention   propagate_attention + h = wV / (z + 1e-6)       deepinteract_modules.py:76-121
//                      (edge UDFs graph_utils.py:21-63; gSpMM send_and_recv(u_mul_e/copy_e, sum))
//
// These are not on the benchmark path (there the same math runs inside the fused edge/node
// kernels); they are plain, correct MFMA / CSR kernels sized for module-at-a-time use.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"
#include "../../include/deepinteract_amd.h"

namespace di {

// ------------------------------------------------------------------ row-wise GEMM
// Rows on the MFMA column (lane & 15), output features on the accumulator rows, exactly as the
// fused kernels; x is read straight from memory, so the weights use the NATURAL k order:
//   bf16 block [lane][j]    = W[16bo + (lane&15)][32s + 8(lane>>4) + j]
//   f32  block [sub][lane]  = W[16bo + (lane&15)][32s + 4 sub + (lane>>4)]
// (packing.pack_matrix_natural). Grid: (row tiles of 64, output groups of 128 features).
struct GemmArgs {
  int rows, in_dim, out_dim, x_ld, y_ld, res_ld, act;
  const void* x;
  const void* w;
  const float* bias;
  const void* res;
  void* y;
};

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<u16>(const u16* p, int64_t i) {
  return __builtin_bit_cast(float, (uint32_t)p[i] << 16);
}

template <class DT>
__global__ __launch_bounds__(THREADS) void k_gemm_bias_act(GemmArgs a) {
  using T = typename DT::T;
  constexpr bool FAST = DT::kBF16;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int r0 = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6) * ROWS_PER_WAVE;
  const int row = r0 + (lane & 15);
  const bool valid = row < a.rows;
  const int rr = valid ? row : a.rows - 1;
  const int nob = a.out_dim / 16, ks = (a.in_dim + 31) / 32;
  const int ob0 = blockIdx.y * 8;
  const T* x = reinterpret_cast<const T*>(a.x) + (int64_t)rr * a.x_ld;
  const T* W = reinterpret_cast<const T*>(a.w);
  Act<8> acc;
  zero(acc);
  for (int s = 0; s < ks; ++s) {
    if constexpr (DT::kBF16) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * g + j;
        v[j] = k < a.in_dim ? ldf(x, k) : 0.f;
      }
      uint4 u;
      u.x = pack_bf16x2(v[0], v[1]);
      u.y = pack_bf16x2(v[2], v[3]);
      u.z = pack_bf16x2(v[4], v[5]);
      u.w = pack_bf16x2(v[6], v[7]);
      const bf16x8 bop = __builtin_bit_cast(bf16x8, u);
#pragma unroll
      for (int bo = 0; bo < 8; ++bo)
        if (ob0 + bo < nob) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(W + ((int64_t)(ob0 + bo) * ks + s) * BLK + lane * 8);
          acc.v[bo] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bop, acc.v[bo], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int sub = 0; sub < 8; ++sub) {
        const int k = 32 * s + 4 * sub + g;
        const float bv = k < a.in_dim ? ldf(x, k) : 0.f;
#pragma unroll
        for (int bo = 0; bo < 8; ++bo)
          if (ob0 + bo < nob) {
            const float av = W[((int64_t)(ob0 + bo) * ks + s) * BLK + sub * 64 + lane];
            acc.v[bo] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc.v[bo], 0, 0, 0);
          }
      }
    }
  }
  if (!valid) return;
  T* y = reinterpret_cast<T*>(a.y) + (int64_t)row * a.y_ld;
  const T* res = a.res ? reinterpret_cast<const T*>(a.res) + (int64_t)row * a.res_ld : nullptr;
#pragma unroll
  for (int bo = 0; bo < 8; ++bo) {
    if (ob0 + bo >= nob) break;
    const int o = 16 * (ob0 + bo) + 4 * g;
    floatx4 v = acc.v[bo];
    if (a.bias) v += ld4(a.bias + o);
    if (a.act == 1)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = silu<FAST>(v[q]);
    if (res) v += ld4(res + o);
    st4(y + o, v);
  }
}

// ------------------------------------------------------------------ attention
// Edge pass, one thread per (edge, head): score = clamp(K[src] * Q[dst] / sqrt(32), +-5) * P
// (elementwise, graph_utils.py:21-46), e_out = score (optional), alpha = exp(clamp(sum, +-5)).
template <class DT>
__global__ __launch_bounds__(256) void k_attn_edge(int Et, const int* __restrict__ src, const int* __restrict__ dst,
                                                   const typename DT::T* __restrict__ qkv,
                                                   const typename DT::T* __restrict__ proj,
                                                   typename DT::T* __restrict__ e_out, float* __restrict__ alpha) {
  using T = typename DT::T;
  constexpr bool FAST = DT::kBF16;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Et * 4) return;
  const int e = (int)(t >> 2), h = (int)(t & 3);
  const T* K = qkv + (int64_t)src[e] * 3 * HID + HID + 32 * h;
  const T* Q = qkv + (int64_t)dst[e] * 3 * HID + 32 * h;
  const T* P = proj + (int64_t)e * HID + 32 * h;
  const float scale = 5.656854249492381f;  // np.sqrt(32)
  float sum = 0.f;
  for (int d = 0; d < 32; d += 4) {
    const floatx4 k4 = ld4(K + d), q4 = ld4(Q + d), p4 = ld4(P + d);
    floatx4 s4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float sc = FAST ? (k4[q] * q4[q]) * (1.0f / scale) : (k4[q] * q4[q]) / scale;
      sc = fminf(fmaxf(sc, -5.f), 5.f) * p4[q];
      s4[q] = sc;
      sum += sc;
    }
    if (e_out) st4(e_out + (int64_t)e * HID + 32 * h + d, s4);
  }
  alpha[(int64_t)e * 4 + h] = expf_<FAST>(fminf(fmaxf(sum, -5.f), 5.f));
}

// Node pass, one thread per (node, 4 features): wV = sum_e alpha_e V[src_e], z = sum_e alpha_e
// over the node's in-edges (CSR by destination, edge-id order = DGL's reduction order),
// h = wV / (z + 1e-6).
template <class DT>
__global__ __launch_bounds__(256) void k_attn_node(int Nt, const int* __restrict__ src, const int* __restrict__ in_ptr,
                                                   const float* __restrict__ alpha,
                                                   const typename DT::T* __restrict__ qkv,
                                                   typename DT::T* __restrict__ h_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Nt * 32) return;
  const int n = (int)(t >> 5), c = 4 * (int)(t & 31), head = c >> 5;
  floatx4 wv = {0.f, 0.f, 0.f, 0.f};
  float z = 0.f;
  for (int e = in_ptr[n]; e < in_ptr[n + 1]; ++e) {
    const float al = alpha[(int64_t)e * 4 + head];
    wv += al * ld4(qkv + (int64_t)src[e] * 3 * HID + 2 * HID + c);
    z += al;
  }
  st4(h_out + (int64_t)n * HID + c, wv / (z + 1e-6f));
}

}  // namespace di

using namespace di;

static inline int mod_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_gemm_bias_act(di_dtype dt, int32_t rows, int32_t in_dim, int32_t out_dim, const void* x,
                                int32_t x_ld, const void* w_packed, const float* bias, int32_t act,
                                const void* res, int32_t res_ld, void* y, int32_t y_ld, void* stream) {
  if (!x || !w_packed || !y || rows <= 0 || in_dim <= 0 || out_dim <= 0 || out_dim % 16 || x_ld < in_dim ||
      y_ld < out_dim || y_ld % 4 || (res && (res_ld < out_dim || res_ld % 4)) || act < 0 || act > 1 ||
      (dt != DI_F32 && dt != DI_BF16))
    return DI_EINVAL;
  GemmArgs a{rows, in_dim, out_dim, x_ld, y_ld, res_ld, act, x, w_packed, bias, res, y};
  dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK, (out_dim / 16 + 7) / 8), block(THREADS);
  if (dt == DI_BF16) hipLaunchKernelGGL(k_gemm_bias_act<BF16T>, grid, block, 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(k_gemm_bias_act<F32T>, grid, block, 0, (hipStream_t)stream, a);
  return mod_status();
}

extern "C" int di_geo_attention(const di_graph* g, di_dtype dt, const void* qkv, const void* proj_e, void* e_out,
                                float* alpha_out, void* h_out, void* stream) {
  if (!g || !qkv || !proj_e || !alpha_out || !h_out || g->num_edges <= 0 || g->num_nodes <= 0 ||
      (dt != DI_F32 && dt != DI_BF16))
    return DI_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const unsigned ge = (unsigned)(((int64_t)g->num_edges * 4 + 255) / 256);
  const unsigned gn = (unsigned)(((int64_t)g->num_nodes * 32 + 255) / 256);
  if (dt == DI_BF16) {
    hipLaunchKernelGGL(k_attn_edge<BF16T>, dim3(ge), dim3(256), 0, s, g->num_edges, g->src, g->dst,
                       (const u16*)qkv, (const u16*)proj_e, (u16*)e_out, alpha_out);
    hipLaunchKernelGGL(k_attn_node<BF16T>, dim3(gn), dim3(256), 0, s, g->num_nodes, g->src, g->in_ptr,
                       (const float*)alpha_out, (const u16*)qkv, (u16*)h_out);
  } else {
    hipLaunchKernelGGL(k_attn_edge<F32T>, dim3(ge), dim3(256), 0, s, g->num_edges, g->src, g->dst,
                       (const float*)qkv, (const float*)proj_e, (float*)e_out, alpha_out);
    hipLaunchKernelGGL(k_attn_node<F32T>, dim3(gn), dim3(256), 0, s, g->num_nodes, g->src, g->in_ptr,
                       (const float*)alpha_out, (const float*)qkv, (float*)h_out);
  }
  return mod_status();
}
