// Diagnostic microbenchmark (NOT shipped): where the edge layers' SiLU VALU work can go relative
// to their MFMAs. The compute core of k_edge_lean -- 24 chained 128x128 linear + SiLU stages with a
// residual every 3rd stage (the ResBlock pattern), two 16-row groups per wave sharing every LDS A
// fragment (v_mfma_f32_16x16x32_bf16), weights resident in LDS, two 4-wave blocks per CU at <= 240
// VGPRs -- in these schedules:
//   S0  stage-serial: all 64 MFMAs of a stage, then both groups' SiLU + pack (k_edge_lean, round 2)
//   S1  pair-pipelined: the SiLU + pack of output-block pair p-1 (both groups) is interleaved with
//       the 16 MFMAs of pair p by sched_group_barrier (1 MFMA : NV VALU); pair 3's tail after the loop
//   S2  as S1, and the tail (pair 3's SiLU) interleaved with the NEXT stage's k-steps 0-2 of pair 0
//       (pair 0 runs k-step major over its 3 ready operands first)
//   S3  no activation (MFMA + pack floor)
//   S4  SiLU + pack only, no MFMA (VALU floor)
// Prints us per launch, TFLOP/s and the max |difference| of S1/S2's output against S0's (the
// schedules compute identical arithmetic).
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/silu_overlap_bench tools/diag/silu_overlap_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
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

#ifndef NV
#define NV 4  // VALU instructions per MFMA in the interleave pattern
#endif
constexpr int STAGES = 24;
constexpr int SLOT = 128 * 128;  // bf16 elements of one stage's weights (32 KiB)
constexpr int NSLOT = 2;

__device__ __forceinline__ uint32_t pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2){a, b}, bf16x2));
}
__device__ __forceinline__ float silu2(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x));
}
__device__ __forceinline__ bf16x8 pack_pair(const floatx4& a, const floatx4& b) {
  uint4 u{pk(a[0], a[1]), pk(a[2], a[3]), pk(b[0], b[1]), pk(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ void fill_lds(__bf16* lds, const __bf16* w) {
  for (int i = threadIdx.x * 8; i < NSLOT * SLOT; i += blockDim.x * 8)
    *reinterpret_cast<uint4*>(lds + i) = *reinterpret_cast<const uint4*>(w + i);
  __syncthreads();
}

// A fragment of (output block bo, k-step s): 1 KiB lane-linear
__device__ __forceinline__ bf16x8 frag(const __bf16* ws, int bo, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(ws + (bo * 4 + s) * 512 + lane * 8);
}

// epilogue of one output-block pair p of group q: SiLU (or not), residual, pack into k-step p
template <int ACT, bool RES>
__device__ __forceinline__ void epi_pair(floatx4 (&acc)[8], floatx4 (&x)[8], bf16x8 (&op)[4], int p) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int b = 2 * p + h;
    if constexpr (ACT == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[b][r] = silu2(acc[b][r]);
    }
    if constexpr (RES) {
      x[b] += 0.6931f * acc[b];
      acc[b] = x[b];
    }
  }
  op[p] = pack_pair(acc[2 * p], acc[2 * p + 1]);
}

// one 128x128 stage for both row groups; RES: the ResBlock's residual (every third stage)
template <int SCHED, int ACT, bool RES, int DEPTH>
__device__ __forceinline__ void stage(const __bf16* ws, floatx4 (&x)[2][8], bf16x8 (&op)[2][4], int lane) {
  constexpr int G = 2;
  floatx4 acc[G][8];
#pragma unroll
  for (int q = 0; q < G; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[q][b] = (floatx4){0.f, 0.f, 0.f, 0.f};
  if constexpr (SCHED == 0 || SCHED == 3) {
    // fragment ring, pair major; then the whole epilogue
    auto blk = [](int i) { return (i / 8) * 2 + (i % 2); };
    auto kst = [](int i) { return (i % 8) / 2; };
    bf16x8 fr[DEPTH];
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) fr[i] = frag(ws, blk(i), kst(i), lane);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < G; ++q)
        acc[q][blk(i)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i % DEPTH], op[q][kst(i)], acc[q][blk(i)], 0, 0, 0);
      if (i + DEPTH < 32) fr[i % DEPTH] = frag(ws, blk(i + DEPTH), kst(i + DEPTH), lane);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p) epi_pair<SCHED == 3 ? 1 : 0, RES>(acc[q], x[q], op[q], p);
  } else {
    // pair-pipelined: pair p's 16 MFMAs (8 A fragments x 2 groups) carry the epilogue of pair
    // p-1; the new operands go to opn (the stage's MFMAs still read op)
    bf16x8 opn[G][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bf16x8 fr[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) fr[i] = frag(ws, 2 * p + (i & 1), i >> 1, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int b = 2 * p + (i & 1);
          acc[q][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i], op[q][i >> 1], acc[q][b], 0, 0, 0);
        }
      if (p > 0) {
#pragma unroll
        for (int q = 0; q < G; ++q) epi_pair<0, RES>(acc[q], x[q], opn[q], p - 1);
      }
      // interleave: 8 LDS reads first, then 16 x (1 MFMA, NV VALU)
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) epi_pair<0, RES>(acc[q], x[q], opn[q], 3);
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s) op[q][s] = opn[q][s];
  }
}

// clock probe (diagnostic only: the stamps go to their own buffer, nothing reads them in-kernel):
// lane 0 of wave 0 of every block records s_memtime / s_memrealtime around the stage loop
template <int SCHED, int ACT = 0, int DEPTH = 4>
__global__ __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2, 2), amdgpu_num_vgpr(120)))
void kcore(const __bf16* __restrict__ w, const __bf16* __restrict__ xin, __bf16* __restrict__ xout, int E,
           unsigned long long* __restrict__ stamps) {
  constexpr int G = 2;
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
    for (int s = 0; s < 4; ++s) op[q][s] = pack_pair(x[q][2 * s], x[q][2 * s + 1]);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (SCHED == 4) {
    // VALU floor: the same SiLU + pack work per stage, no MFMA (values chained through op)
#pragma unroll 1
    for (int st = 0; st < STAGES; ++st) {
#pragma unroll
      for (int q = 0; q < G; ++q) {
        floatx4 acc[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint4 u = __builtin_bit_cast(uint4, op[q][b >> 1]);
          const uint32_t lo = (b & 1) ? u.z : u.x, hi = (b & 1) ? u.w : u.y;
          acc[b] = (floatx4){__builtin_bit_cast(float, lo << 16), __builtin_bit_cast(float, lo & 0xffff0000u),
                             __builtin_bit_cast(float, hi << 16), __builtin_bit_cast(float, hi & 0xffff0000u)};
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) epi_pair<0, false>(acc, x[q], op[q], p);
      }
    }
  } else {
#pragma unroll 1
    for (int st = 0; st < STAGES; st += 3) {
      stage<SCHED, ACT, false, DEPTH>(lds + (st % NSLOT) * SLOT, x, op, lane);
      stage<SCHED, ACT, false, DEPTH>(lds + ((st + 1) % NSLOT) * SLOT, x, op, lane);
      stage<SCHED, ACT, true, DEPTH>(lds + ((st + 2) % NSLOT) * SLOT, x, op, lane);
    }
  }
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
#pragma unroll
  for (int q = 0; q < G; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) xout[(size_t)row[q] * 128 + b * 16 + g * 4 + r] = (__bf16)x[q][b][r];
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
  const int grid = (E + 127) / 128;
  std::vector<__bf16> ref((size_t)E * 128), got((size_t)E * 128);
  unsigned long long* stamps;
  CHECK(hipMalloc(&stamps, (size_t)grid * 2 * sizeof(unsigned long long)));
  std::vector<unsigned long long> hs((size_t)grid * 2);
  struct Var { const char* name; void (*k)(const __bf16*, const __bf16*, __bf16*, int, unsigned long long*); };
  const Var vars[] = {
      {"S0 stage-serial (round 2), depth 4 ", kcore<0, 0, 4>}, {"S0 stage-serial, depth 8           ", kcore<0, 0, 8>},
      {"S1 pair-pipelined (sched groups)   ", kcore<1, 0, 4>}, {"S3 no activation, depth 4          ", kcore<3, 1, 4>},
      {"S3 no activation, depth 8          ", kcore<3, 1, 8>}, {"S4 SiLU + pack only (VALU floor)   ", kcore<4, 0, 4>}};
  for (int v = 0; v < 6; ++v) {
    auto launch = [&]() { vars[v].k<<<grid, 256>>>(w, xin, xout, E, stamps); };
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    CHECK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int i = 0; i < grid; ++i)
      if (hs[2 * i + 1] > 0) clk.push_back((double)hs[2 * i] / (double)hs[2 * i + 1] * 100.0);  // MHz
    std::sort(clk.begin(), clk.end());
    const double mhz = clk.empty() ? 0.0 : clk[clk.size() / 2];
    double diff = 0.0;
    if (v == 0) CHECK(hipMemcpy(ref.data(), xout, ref.size() * 2, hipMemcpyDeviceToHost));
    if (v == 1 || v == 2) {
      CHECK(hipMemcpy(got.data(), xout, got.size() * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < got.size(); ++i) diff = fmax(diff, fabs((double)(float)got[i] - (double)(float)ref[i]));
    }
    printf("%s: %.1f us (E=%d, %d stages, NV=%d) = %.0f TFLOP/s, in-kernel clock %.0f MHz (%.0f%% of that clock's "
           "bf16 peak), max|vs S0| %.3g\n", vars[v].name, us, E, STAGES, NV, flop / us / 1e6, mhz,
           mhz > 0 ? 100.0 * flop / us / 1e6 / (2500.0 * mhz / 2400.0) : 0.0, diff);
  }
  return 0;
}
