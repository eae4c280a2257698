// Diagnostic microbenchmark (NOT shipped): vector-instruction issue cost on one SIMD, for the
// instructions a SiLU epilogue can be built from (f32 and packed-f16 forms). Each variant runs a
// loop of 16 independent instructions over 8 registers per iteration; lane 0 of every wave records
// s_memtime around the loop. Printed: shader cycles per instruction for ONE wave on a SIMD and the
// per-SIMD cycles per instruction with TWO waves on every SIMD (the edge kernels' occupancy).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/vib tools/diag/valu_issue_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int ITERS = 256;

#define OPS2(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define R8 "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])

#define E32(n) "v_exp_f32 %" #n ", -%" #n "\n"
#define RCP32(n) "v_rcp_f32 %" #n ", %" #n "\n"
#define ADD32(n) "v_add_f32 %" #n ", 1.0, %" #n "\n"
#define MUL32(n) "v_mul_f32 %" #n ", %" #n ", %" #n "\n"
#define E16(n) "v_exp_f16 %" #n ", -%" #n "\n"
#define RCP16(n) "v_rcp_f16 %" #n ", %" #n "\n"
#define E16HI(n) "v_exp_f16_sdwa %" #n ", -%" #n " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
#define PKADD16(n) "v_pk_add_f16 %" #n ", %" #n ", 1.0 op_sel_hi:[1,0]\n"
#define PKMUL16(n) "v_pk_mul_f16 %" #n ", %" #n ", %" #n "\n"
#define PKFMA16(n) "v_pk_fma_f16 %" #n ", %" #n ", %" #n ", %" #n "\n"
#define PKMUL32(n) "v_pk_mul_f32 %" #n ", %" #n ", %" #n "\n"
#define CVTRTZ(n) "v_cvt_pkrtz_f16_f32 %" #n ", %" #n ", %" #n "\n"
#define CVTBF(n) "v_cvt_pk_bf16_f32 %" #n ", %" #n ", %" #n "\n"
#define CVTF32F16(n) "v_cvt_f32_f16 %" #n ", %" #n "\n"

template <int V>
__device__ __forceinline__ void body(float (&r)[8]) {
  if constexpr (V == 0) asm volatile(OPS2(E32) : R8);
  if constexpr (V == 1) asm volatile(OPS2(RCP32) : R8);
  if constexpr (V == 2) asm volatile(OPS2(ADD32) : R8);
  if constexpr (V == 3) asm volatile(OPS2(E16) : R8);
  if constexpr (V == 4) asm volatile(OPS2(RCP16) : R8);
  if constexpr (V == 5) asm volatile(OPS2(E16HI) : R8);
  if constexpr (V == 6) asm volatile(OPS2(PKADD16) : R8);
  if constexpr (V == 7) asm volatile(OPS2(PKMUL16) : R8);
  if constexpr (V == 8) asm volatile(OPS2(PKFMA16) : R8);
  if constexpr (V == 9) asm volatile(OPS2(CVTRTZ) : R8);
  if constexpr (V == 10) asm volatile(OPS2(CVTBF) : R8);
  if constexpr (V == 11) asm volatile(OPS2(CVTF32F16) : R8);
  if constexpr (V == 12) asm volatile(OPS2(MUL32) : R8);
}
// packed-f32 needs 64-bit register pairs
template <int V>
__device__ __forceinline__ void body2(double (&d)[8]) {
  asm volatile(OPS2(PKMUL32) : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]),
               "+v"(d[7]));
}

template <int V>
__global__ __launch_bounds__(512) void kissue(unsigned long long* cyc, float* sink, float seed) {
  const int lane = threadIdx.x & 63;
  float r[8];
  double d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[i] = seed + 0.001f * (lane + i);
    d[i] = (double)r[i];
  }
  __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (V == 13) body2<V>(d);
    else body<V>(r);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += r[i] + (float)d[i];
  if (lane == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const char* names[] = {"v_exp_f32", "v_rcp_f32", "v_add_f32", "v_exp_f16", "v_rcp_f16", "v_exp_f16 sdwa hi",
                         "v_pk_add_f16", "v_pk_mul_f16", "v_pk_fma_f16", "v_cvt_pkrtz_f16_f32", "v_cvt_pk_bf16_f32",
                         "v_cvt_f32_f16", "v_mul_f32", "v_pk_mul_f32"};
  void (*ks[])(unsigned long long*, float*, float) = {kissue<0>, kissue<1>, kissue<2>,  kissue<3>,  kissue<4>,
                                                      kissue<5>, kissue<6>, kissue<7>,  kissue<8>,  kissue<9>,
                                                      kissue<10>, kissue<11>, kissue<12>, kissue<13>};
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned long long* cyc;
  float* sink;
  CHECK(hipMalloc(&cyc, (size_t)cus * 8 * 8));
  CHECK(hipMalloc(&sink, (size_t)cus * 512 * 4));
  std::vector<unsigned long long> h((size_t)cus * 8);
  const double ninst = 16.0 * ITERS;
  for (int v = 0; v < 14; ++v) {
    double res[2];
    for (int occ = 1; occ <= 2; ++occ) {
      // one block per CU: 4 waves (one per SIMD) or 8 waves (two per SIMD)
      const int threads = 256 * occ;
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(ks[v], dim3(cus), dim3(threads), 0, 0, cyc, sink, 0.5f);
        CHECK(hipDeviceSynchronize());
      }
      CHECK(hipMemcpy(h.data(), cyc, (size_t)cus * (threads / 64) * 8, hipMemcpyDeviceToHost));
      std::vector<double> c(h.begin(), h.begin() + (size_t)cus * (threads / 64));
      std::sort(c.begin(), c.end());
      // per-SIMD cycles per instruction: a wave's loop time / (instructions of the waves sharing its SIMD)
      res[occ - 1] = c[c.size() / 2] / (ninst * occ);
    }
    printf("%-22s one wave/SIMD %.2f cyc/inst, two waves/SIMD %.2f cyc/inst per SIMD\n", names[v], res[0], res[1]);
  }
  return 0;
}
