// Diagnostic microbenchmark (NOT shipped): the compute core of the edge layers — a chain of
// 128x128 linear + SiLU stages with a residual every 3 stages (the ResBlock pattern), weights
// resident in LDS (no weight stream, no gathers) — in three MFMA shapes, to price the shape
// before restructuring k_edge_layer:
//   V0  v_mfma_f32_16x16x32_bf16, 16 rows per wave (k_edge_layer today)
//   V1  v_mfma_f32_16x16x32_bf16, two 16-row groups per wave sharing every LDS A fragment
//   V2  v_mfma_f32_32x32x16_bf16, 32 rows per wave (half the MFMA issues and A-fragment reads)
// Two 4-wave blocks per CU (240 VGPRs, as the edge kernels). Prints us per launch and the
// implied TFLOP/s for E rows x S stages x 128 x 128 MACs.
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_shape_bench tools/diag/mfma_shape_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

#ifndef DEPTH
#define DEPTH 4
#endif
constexpr int STAGES = 24;
constexpr int SLOT = 128 * 128;  // bf16 elements of one stage's weights (32 KiB)
constexpr int NSLOT = 2;         // 64 KiB per block, two blocks per CU

__device__ __forceinline__ uint32_t pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2){a, b}, bf16x2));
}
__device__ __forceinline__ float silu2(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x));
}
__device__ __forceinline__ bf16x8 pack8(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                        float a7) {
  uint4 u{pk(a0, a1), pk(a2, a3), pk(a4, a5), pk(a6, a7)};
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ void fill_lds(__bf16* lds, const __bf16* w) {
  for (int i = threadIdx.x * 8; i < NSLOT * SLOT; i += blockDim.x * 8)
    *reinterpret_cast<uint4*>(lds + i) = *reinterpret_cast<const uint4*>(w + i);
  __syncthreads();
}

// ---------------------------------------------------------------- V0 / V1: 16x16x32, G groups
template <int G, int ACT = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2), amdgpu_num_vgpr(120)))
void k16(const __bf16* __restrict__ w, const __bf16* __restrict__ xin, __bf16* __restrict__ xout, int E) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[NSLOT * SLOT];
  fill_lds(lds, w);
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int wave = threadIdx.x >> 6;
  floatx4 x[G][8];
  bf16x8 op[G][4];
  int row[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    row[q] = (blockIdx.x * 4 * G + q * 4 + wave) * 16 + (lane & 15);
    if (row[q] >= E) row[q] = E - 1;
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) x[q][b][r] = (float)xin[(size_t)row[q] * 128 + b * 16 + g * 4 + r];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      op[q][s] = pack8(x[q][2 * s][0], x[q][2 * s][1], x[q][2 * s][2], x[q][2 * s][3], x[q][2 * s + 1][0],
                       x[q][2 * s + 1][1], x[q][2 * s + 1][2], x[q][2 * s + 1][3]);
  }
#pragma unroll 1
  for (int st = 0; st < STAGES; ++st) {
    const __bf16* ws = lds + (st % NSLOT) * SLOT;
    floatx4 acc[G][8];
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[q][b] = (floatx4){0.f, 0.f, 0.f, 0.f};
    // fragment ring: step i -> (out block pair major, k-step); one A read per step feeds G MFMAs
    auto blk = [](int i) { return (i / 8) * 2 + (i % 2); };
    auto kst = [](int i) { return (i % 8) / 2; };
    bf16x8 fr[DEPTH];
#pragma unroll
    for (int i = 0; i < DEPTH; ++i)
      fr[i] = *reinterpret_cast<const bf16x8*>(ws + (blk(i) * 4 + kst(i)) * 512 + lane * 8);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < G; ++q)
        acc[q][blk(i)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i % DEPTH], op[q][kst(i)], acc[q][blk(i)], 0, 0, 0);
      if (i + DEPTH < 32)
        fr[i % DEPTH] = *reinterpret_cast<const bf16x8*>(ws + (blk(i + DEPTH) * 4 + kst(i + DEPTH)) * 512 + lane * 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool res = (st % 3) == 2;
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if constexpr (ACT == 0) {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[q][b][r] = silu2(acc[q][b][r]);
      }
      if (res) {
#pragma unroll
        for (int b = 0; b < 8; ++b) x[q][b] += 0.6931f * acc[q][b];
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[q][b] = x[q][b];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
        op[q][s] = pack8(acc[q][2 * s][0], acc[q][2 * s][1], acc[q][2 * s][2], acc[q][2 * s][3], acc[q][2 * s + 1][0],
                         acc[q][2 * s + 1][1], acc[q][2 * s + 1][2], acc[q][2 * s + 1][3]);
    }
  }
#pragma unroll
  for (int q = 0; q < G; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) xout[(size_t)row[q] * 128 + b * 16 + g * 4 + r] = (__bf16)x[q][b][r];
}

// ---------------------------------------------------------------- V2: 32x32x16, 32 rows per wave
// accumulator v of out block B: feature 32B + (v/4)*8 + h*4 + v%4 (h = lane/32), row = lane%32;
// B operand of k-step 2B+p = the accumulator values 8p..8p+7 packed (K order permuted on the host)
// ACT 0: fp32 SiLU, bf16 operands; 1: no activation (MFMA + pack core); 2: SiLU in packed f16
// (v_cvt_pk_f16_f32, SDWA v_exp_f16 / v_rcp_f16 per half, v_pk_add/mul_f16), f16 operands
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t silu2_pk_f16(float a, float b) {
  uint32_t p, e, d, r, y;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(p) : "v"(a), "v"(b));
  asm("v_exp_f16_sdwa %0, -%1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(e) : "v"(p));
  asm("v_exp_f16_sdwa %0, -%1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(e) : "v"(p));
  asm("v_pk_add_f16 %0, %1, 1.0 op_sel_hi:[1,0]" : "=v"(d) : "v"(e));
  asm("v_rcp_f16_sdwa %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(r) : "v"(d));
  asm("v_rcp_f16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(r) : "v"(d));
  asm("v_pk_mul_f16 %0, %1, %2" : "=v"(y) : "v"(p), "v"(r));
  return y;
}
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  uint32_t p;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(p) : "v"(a), "v"(b));
  return p;
}
template <int ACT>
__global__ __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2), amdgpu_num_vgpr(120)))
void k32(const __bf16* __restrict__ w, const __bf16* __restrict__ xin, __bf16* __restrict__ xout, int E) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[NSLOT * SLOT];
  fill_lds(lds, w);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = threadIdx.x >> 6;
  int row = (blockIdx.x * 4 + wave) * 32 + (lane & 31);
  if (row >= E) row = E - 1;
  floatx16 x[4];
  bf16x8 op[8];
#pragma unroll
  for (int B = 0; B < 4; ++B)
#pragma unroll
    for (int v = 0; v < 16; ++v) x[B][v] = (float)xin[(size_t)row * 128 + 32 * B + (v / 4) * 8 + h * 4 + v % 4];
#pragma unroll
  for (int B = 0; B < 4; ++B) {
    op[2 * B] = pack8(x[B][0], x[B][1], x[B][2], x[B][3], x[B][4], x[B][5], x[B][6], x[B][7]);
    op[2 * B + 1] = pack8(x[B][8], x[B][9], x[B][10], x[B][11], x[B][12], x[B][13], x[B][14], x[B][15]);
  }
#pragma unroll 1
  for (int st = 0; st < STAGES; ++st) {
    const __bf16* ws = lds + (st % NSLOT) * SLOT;
    floatx16 acc[4];
#pragma unroll
    for (int B = 0; B < 4; ++B)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[B][v] = 0.f;
    // step i -> (out block i / 8, k-step i % 8); A fragment (32 out x 16 K) = 1 KiB lane-linear
    bf16x8 fr[DEPTH];
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) fr[i] = *reinterpret_cast<const bf16x8*>(ws + i * 512 + lane * 8);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (ACT == 2)
        acc[i / 8] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, fr[i % DEPTH]),
                                                            __builtin_bit_cast(halfx8, op[i % 8]), acc[i / 8], 0, 0, 0);
      else
        acc[i / 8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[i % DEPTH], op[i % 8], acc[i / 8], 0, 0, 0);
      if (i + DEPTH < 32) fr[i % DEPTH] = *reinterpret_cast<const bf16x8*>(ws + (i + DEPTH) * 512 + lane * 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool res = (st % 3) == 2;
#pragma unroll
    for (int B = 0; B < 4; ++B) {
      if constexpr (ACT == 2) {
        if (!res) {
          uint4 u0, u1;
          u0.x = silu2_pk_f16(acc[B][0], acc[B][1]);
          u0.y = silu2_pk_f16(acc[B][2], acc[B][3]);
          u0.z = silu2_pk_f16(acc[B][4], acc[B][5]);
          u0.w = silu2_pk_f16(acc[B][6], acc[B][7]);
          u1.x = silu2_pk_f16(acc[B][8], acc[B][9]);
          u1.y = silu2_pk_f16(acc[B][10], acc[B][11]);
          u1.z = silu2_pk_f16(acc[B][12], acc[B][13]);
          u1.w = silu2_pk_f16(acc[B][14], acc[B][15]);
          op[2 * B] = __builtin_bit_cast(bf16x8, u0);
          op[2 * B + 1] = __builtin_bit_cast(bf16x8, u1);
          continue;
        }
      }
      if constexpr (ACT != 1) {
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[B][v] = silu2(acc[B][v]);
      }
      if (res) {
        x[B] += 0.6931f * acc[B];
        acc[B] = x[B];
      }
      if constexpr (ACT == 2) {
        uint4 u0{pk_f16(acc[B][0], acc[B][1]), pk_f16(acc[B][2], acc[B][3]), pk_f16(acc[B][4], acc[B][5]),
                 pk_f16(acc[B][6], acc[B][7])};
        uint4 u1{pk_f16(acc[B][8], acc[B][9]), pk_f16(acc[B][10], acc[B][11]), pk_f16(acc[B][12], acc[B][13]),
                 pk_f16(acc[B][14], acc[B][15])};
        op[2 * B] = __builtin_bit_cast(bf16x8, u0);
        op[2 * B + 1] = __builtin_bit_cast(bf16x8, u1);
      } else {
        op[2 * B] = pack8(acc[B][0], acc[B][1], acc[B][2], acc[B][3], acc[B][4], acc[B][5], acc[B][6], acc[B][7]);
        op[2 * B + 1] =
            pack8(acc[B][8], acc[B][9], acc[B][10], acc[B][11], acc[B][12], acc[B][13], acc[B][14], acc[B][15]);
      }
    }
  }
#pragma unroll
  for (int B = 0; B < 4; ++B)
#pragma unroll
    for (int v = 0; v < 16; ++v) xout[(size_t)row * 128 + 32 * B + (v / 4) * 8 + h * 4 + v % 4] = (__bf16)x[B][v];
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 327680;
  const int iters = 20;
  std::vector<__bf16> hw(NSLOT * SLOT), hx((size_t)E * 128);
  srand(1);
  for (auto& v : hw) v = (__bf16)((rand() / (float)RAND_MAX - 0.5f) * 0.18f);
  for (auto& v : hx) v = (__bf16)((rand() / (float)RAND_MAX - 0.5f) * 2.f);
  __bf16 *w, *xin, *xout;
  CHECK(hipMalloc(&w, hw.size() * 2));
  CHECK(hipMalloc(&xin, hx.size() * 2));
  CHECK(hipMalloc(&xout, hx.size() * 2));
  CHECK(hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(xin, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const double flop = 2.0 * E * STAGES * 128.0 * 128.0;
  __bf16* wh;  // f16 weights for ACT 2 (same magnitudes)
  {
    std::vector<_Float16> hh(NSLOT * SLOT);
    for (size_t i = 0; i < hh.size(); ++i) hh[i] = (_Float16)(float)hw[i];
    CHECK(hipMalloc(&wh, hh.size() * 2));
    CHECK(hipMemcpy(wh, hh.data(), hh.size() * 2, hipMemcpyHostToDevice));
  }
  for (int v = 0; v < 6; ++v) {
    const int rows_per_block = v == 0 || v == 5 ? 64 : 128;
    const int grid = (E + rows_per_block - 1) / rows_per_block;
    auto launch = [&]() {
      if (v == 0) k16<1><<<grid, 256>>>(w, xin, xout, E);
      else if (v == 1) k16<2><<<grid, 256>>>(w, xin, xout, E);
      else if (v == 2) k32<0><<<grid, 256>>>(w, xin, xout, E);
      else if (v == 3) k32<1><<<grid, 256>>>(w, xin, xout, E);
      else if (v == 4) k32<2><<<grid, 256>>>(wh, xin, xout, E);
      else k16<1, 1><<<grid, 256>>>(w, xin, xout, E);
    };
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("V%d  %s: %.1f us per launch (E=%d, %d stages) = %.0f TFLOP/s\n", v,
           v == 0 ? "16x16x32, 16 rows/wave, f32 SiLU    " : v == 1 ? "16x16x32, 2x16 rows, shared A       "
           : v == 2 ? "32x32x16, 32 rows/wave, f32 SiLU    " : v == 3 ? "32x32x16, no activation (core)      "
           : v == 4 ? "32x32x16 f16, SiLU in packed f16    " : "16x16x32, 16 rows, no activation    ",
           us, E, STAGES, flop / us / 1e6);
  }
  return 0;
}
