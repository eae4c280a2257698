// Shared device toolkit for the GeoT kernels (gfx950 / CDNA4).
//
// "Row-on-lane" activation engine
// -------------------------------
// Every GeoT kernel is a chain of small dense layers applied row-wise (one row = one edge or
// one node). A wave owns 16 rows: the row sits on the MFMA *column* (lane & 15) and the
// features sit in the accumulator registers, i.e. each activation is held TRANSPOSED, exactly
// as v_mfma_f32_16x16x{32_bf16,4_f32} writes its C/D tile (col = lane&15, row = 4*(lane>>4)+reg):
//
//     feature(block b, reg r, lane-group g = lane>>4) = 16*b + 4*g + r        (4 regs / block)
//
// A linear layer Y^T = W . X^T takes W as the A operand (streamed from LDS, packed on the host
// in fragment order) and the previous accumulator X^T directly as the B operand: no LDS round
// trip and no lane shuffles between chained layers (cdna_hip_programming.md §3, "An accumulator
// tile as the next MFMA's operand"). A 128-feature activation costs 32 VGPRs per lane.
// 16x16 tiles need twice the LDS weight bytes per MAC of 32x32 tiles (1 KiB of A per 8K MAC
// instead of 16K) but half the activation registers, which is what sets occupancy here; at full
// MFMA rate on 4 SIMDs that is 256 B/clk/CU, the ds_read_b128 peak.
//
// The k-permutation implied by using an accumulator as B is baked into the host-side packing
// (deepinteract_amd/packing.py). One packed block = 16 output rows x 32 input features =
// 512 elements for both dtypes:
//   bf16 16x16x32: [lane 0..63][j 0..7]          W[16bo + (lane&15)][32s + 16(j>>2) + 4(lane>>4) + (j&3)]
//   f32  16x16x4 : [sub 0..1][lane 0..63][r 0..3] W[16bo + (lane&15)][32s + 16 sub + 4(lane>>4) + r]
// Per-feature vectors (biases) are packed [b][g][r] (4 floats per lane group).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace di {

// Compute units of the CURRENT device (persistent grids), cached per device id: one attribute query
// per device and process, and a process driving several devices sizes each grid from its own device.
inline int device_cus() {
  constexpr int MAXDEV = 64;
  static std::atomic<int> cache[MAXDEV];  // 0: not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev < MAXDEV) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
  if (dev < MAXDEV) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16;

constexpr int HID = 128;          // num_gnn_hidden_channels
constexpr int NFEAT_E = 28;       // edge feature columns (FEATURE_INDICES)
constexpr int NFEAT_N = 113;      // node feature columns
constexpr int BLK = 512;          // elements per packed (16 out x 32 in) weight block
constexpr int MAT128 = 32;        // blocks of a 128x128 matrix
constexpr int ROWS_PER_WAVE = 16;
constexpr int WAVES = 4;
constexpr int ROWS_PER_BLOCK = ROWS_PER_WAVE * WAVES;
constexpr int THREADS = 64 * WAVES;

// ------------------------------------------------------------------ dtype traits
struct F32T {
  using T = float;
  static constexpr bool kBF16 = false;
};
struct BF16T {
  using T = u16;  // raw bf16 bits in memory
  static constexpr bool kBF16 = true;
};

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  bf16x2 v = __builtin_convertvector((floatx2){a, b}, bf16x2);
  return __builtin_bit_cast(uint32_t, v);
}

// 4 consecutive elements -> floatx4
__device__ __forceinline__ floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }
__device__ __forceinline__ floatx4 ld4(const u16* p) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  floatx4 r;
  r[0] = __builtin_bit_cast(float, u.x << 16);
  r[1] = __builtin_bit_cast(float, u.x & 0xffff0000u);
  r[2] = __builtin_bit_cast(float, u.y << 16);
  r[3] = __builtin_bit_cast(float, u.y & 0xffff0000u);
  return r;
}
__device__ __forceinline__ void st4(float* p, floatx4 v) { *reinterpret_cast<floatx4*>(p) = v; }
__device__ __forceinline__ void st4(u16* p, floatx4 v) {
  uint2 u;
  u.x = pack_bf16x2(v[0], v[1]);
  u.y = pack_bf16x2(v[2], v[3]);
  *reinterpret_cast<uint2*>(p) = u;
}
// non-temporal forms (write-once edge rows that do not fit in L2: kept from evicting weight stages)
__device__ __forceinline__ void st4_nt(float* p, floatx4 v) { __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p)); }
__device__ __forceinline__ void st4_nt(u16* p, floatx4 v) {
  typedef unsigned int uintx2 __attribute__((ext_vector_type(2)));
  const uintx2 u = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
  __builtin_nontemporal_store(u, reinterpret_cast<uintx2*>(p));
}

template <bool FAST>
__device__ __forceinline__ float expf_(float x) {
  if constexpr (FAST) return __expf(x);
  else return expf(x);
}
// SiLU. x * rcp(1 + exp(-x)) with the hardware v_exp_f32 / v_rcp_f32 (~1 ulp each): 5 VALU ops.
// The fp32 path (the reference's precision) uses it too: libm expf plus an IEEE division cost ~25
// VALU instructions per value, which made the fp32 edge layers issue-bound beside their MFMAs, and
// the hardware form stays a few ulp from the exact SiLU (fp32 outputs within ~1e-6 of the oracle;
// north_star's fp32 bound is 1e-4). DI_F32_FAST_SILU=0 restores the libm + division form for fp32.
#ifndef DI_F32_FAST_SILU
#define DI_F32_FAST_SILU 1
#endif
template <bool FAST>
__device__ __forceinline__ float silu(float x) {
  if constexpr (FAST || DI_F32_FAST_SILU) return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
  else return x / (1.0f + expf(-x));
}

// SiLU of a pre-activation held in log2 units (bf16 path): for a' = log2(e) * a,
// a' * rcp(1 + 2^-a') = log2(e) * silu(a) in 4 VALU ops (v_exp_f32 is 2^x; the negation is a free
// source modifier). The host packing scales the producing layer's weights and bias by log2(e) and
// the consuming layer's (or gate's) weights by ln(2) (packing.py, "log2-unit SiLU"); used where
// the SiLU output only feeds a linear layer or a gate. The fp32 path is unscaled: plain silu.
constexpr float LN2 = 0.6931471805599453f;
template <bool FAST>
constexpr float silu2_unit() { return FAST ? LN2 : 1.0f; }  // silu = silu2 * silu2_unit
template <bool FAST>
__device__ __forceinline__ float silu2(float x) {
  if constexpr (FAST) return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x));
  else return silu<false>(x);
}

// ------------------------------------------------------------------ activations
template <int NB>  // NB blocks of 16 features
struct Act {
  floatx4 v[NB];
};

template <int NB>
__device__ __forceinline__ void zero(Act<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] = (floatx4){0.f, 0.f, 0.f, 0.f};
}

// a = per-feature vector (packed [b][g][4], fp32)
template <int NB>
__device__ __forceinline__ void init_vec(Act<NB>& a, const float* vec, int g) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] = ld4(vec + (b * 4 + g) * 4);
}

// the same from LDS (vector staged with the layer's weights)
template <int NB>
__device__ __forceinline__ void init_vec_lds(Act<NB>& a, const float* vec, int g) {
  const __attribute__((address_space(3))) floatx4* p = (const __attribute__((address_space(3))) floatx4*)vec;
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] = p[b * 4 + g];
}

template <int NB>
__device__ __forceinline__ void add_vec(Act<NB>& a, const float* vec, int g) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] += ld4(vec + (b * 4 + g) * 4);
}

// row-major row (features 0 .. 16*NB-1) -> activation
template <int NB, typename T>
__device__ __forceinline__ void load_row(Act<NB>& a, const T* row, int g) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] = ld4(row + 16 * b + 4 * g);
}

template <int NB, typename T>
__device__ __forceinline__ void add_row(Act<NB>& a, const T* row, int g) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] += ld4(row + 16 * b + 4 * g);
}

template <int NB, typename T>
__device__ __forceinline__ void store_row(const Act<NB>& a, T* row, int g) {
#pragma unroll
  for (int b = 0; b < NB; ++b) st4(row + 16 * b + 4 * g, a.v[b]);
}
// edge-row outputs (F, Fn: 82 MB per C3 micro-batch each, re-read by the next kernel from HBM/MALL)
// keep the default store policy: non-temporal row stores measured slower beside the pair stream
// (7108-7150 vs 7438-7441 complexes/s, round 2)
template <int NB, typename T>
__device__ __forceinline__ void store_edge_row(const Act<NB>& a, T* row, int g) {
  store_row(a, row, g);
}

// A 128-feature row held in its STORAGE format (bf16: 16 VGPRs instead of 32), for prefetching
// gathered rows several MFMA chains ahead of their use.
template <typename T>
struct RawRow;
template <>
struct RawRow<u16> {
  uint2 u[8];
  __device__ __forceinline__ void load(const u16* row, int g) {
#pragma unroll
    for (int b = 0; b < 8; ++b) u[b] = *reinterpret_cast<const uint2*>(row + 16 * b + 4 * g);
  }
  __device__ __forceinline__ void to_act(Act<8>& a) const {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      a.v[b][0] = __builtin_bit_cast(float, u[b].x << 16);
      a.v[b][1] = __builtin_bit_cast(float, u[b].x & 0xffff0000u);
      a.v[b][2] = __builtin_bit_cast(float, u[b].y << 16);
      a.v[b][3] = __builtin_bit_cast(float, u[b].y & 0xffff0000u);
    }
  }
};
// Make the wave wait for a row's loads HERE (an empty asm that reads its registers): placed
// before a weight-stage DMA issue, it keeps a later use of the row from waiting for the whole
// in-flight stage (vmcnt retires in order; the compiler cannot count a runtime-length DMA loop).
__device__ __forceinline__ void settle(const RawRow<u16>& r) {
#pragma unroll
  for (int b = 0; b < 8; ++b) asm volatile("" ::"v"(r.u[b].x), "v"(r.u[b].y));
}
template <>
struct RawRow<float> {
  floatx4 v[8];
  __device__ __forceinline__ void load(const float* row, int g) {
#pragma unroll
    for (int b = 0; b < 8; ++b) v[b] = ld4(row + 16 * b + 4 * g);
  }
  __device__ __forceinline__ void to_act(Act<8>& a) const {
#pragma unroll
    for (int b = 0; b < 8; ++b) a.v[b] = v[b];
  }
};
__device__ __forceinline__ void settle(const RawRow<float>& r) {
#pragma unroll
  for (int b = 0; b < 8; ++b) asm volatile("" ::"v"(r.v[b]));
}

// edge feature row G [28] (fp32, 112-B rows) as a 32-feature activation, features 28..31 = 0
__device__ __forceinline__ void load_edge_geo(Act<2>& a, const float* row, int g) {
  a.v[0] = ld4(row + 4 * g);
  a.v[1] = g == 3 ? (floatx4){0.f, 0.f, 0.f, 0.f} : ld4(row + 16 + 4 * g);
}

template <int NB, bool FAST>
__device__ __forceinline__ void silu_(Act<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.v[b][r] = silu<FAST>(a.v[b][r]);
}

template <int NB, bool FAST>
__device__ __forceinline__ void silu2_(Act<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.v[b][r] = silu2<FAST>(a.v[b][r]);
}

// Pin an activation: an empty asm that reads and rewrites its registers, so every value is
// computed HERE. Without it the compiler may sink a chain of VALU work (a gate product, a running
// sum's terms) past later stages to its last use, keeping all the chain's inputs live meanwhile.
template <int NB>
__device__ __forceinline__ void pin(Act<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b) asm volatile("" : "+v"(a.v[b]));
}

// a += k * b (one v_fma per value: folds the ln(2) of a log2-unit SiLU output into a residual add)
template <int NB>
__device__ __forceinline__ void add_scaled_(Act<NB>& a, const Act<NB>& b_, float k) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] += k * b_.v[b];
}

template <int NB>
__device__ __forceinline__ void add_(Act<NB>& a, const Act<NB>& b_) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] += b_.v[b];
}
template <int NB>
__device__ __forceinline__ void mul_(Act<NB>& a, const Act<NB>& b_) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] *= b_.v[b];
}

// scheduling fence between row groups / phases (keeps the compiler from interleaving, and so
// doubling the live state of, independent groups). The memory clobber also keeps the groups'
// reads of the same LDS slot (A fragments, biases) from being merged into one live copy shared by
// both groups.
__device__ __forceinline__ void lean_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------------ MFMA operands
// NS = number of 32-feature k-steps (= NB / 2)
template <class DT, int NS>
struct Op;
template <int NS>
struct Op<BF16T, NS> {
  bf16x8 f[NS];
};
template <int NS>
struct Op<F32T, NS> {
  floatx4 f[2 * NS];
};

template <int NS>
__device__ __forceinline__ void pin(Op<BF16T, NS>& o) {
#pragma unroll
  for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(o.f[s]));
}
template <int NS>
__device__ __forceinline__ void make_op(Op<BF16T, NS>& o, const Act<2 * NS>& a) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    uint4 u;
    u.x = pack_bf16x2(a.v[2 * s][0], a.v[2 * s][1]);
    u.y = pack_bf16x2(a.v[2 * s][2], a.v[2 * s][3]);
    u.z = pack_bf16x2(a.v[2 * s + 1][0], a.v[2 * s + 1][1]);
    u.w = pack_bf16x2(a.v[2 * s + 1][2], a.v[2 * s + 1][3]);
    o.f[s] = __builtin_bit_cast(bf16x8, u);
  }
}
template <int NS>
__device__ __forceinline__ void make_op(Op<F32T, NS>& o, const Act<2 * NS>& a) {
#pragma unroll
  for (int b = 0; b < 2 * NS; ++b) o.f[b] = a.v[b];
}

// inverse of make_op for bf16 (exact: bf16 -> fp32)
template <int NS>
__device__ __forceinline__ void unpack_op(Act<2 * NS>& a, const Op<BF16T, NS>& o) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const uint4 u = __builtin_bit_cast(uint4, o.f[s]);
    a.v[2 * s][0] = __builtin_bit_cast(float, u.x << 16);
    a.v[2 * s][1] = __builtin_bit_cast(float, u.x & 0xffff0000u);
    a.v[2 * s][2] = __builtin_bit_cast(float, u.y << 16);
    a.v[2 * s][3] = __builtin_bit_cast(float, u.y & 0xffff0000u);
    a.v[2 * s + 1][0] = __builtin_bit_cast(float, u.z << 16);
    a.v[2 * s + 1][1] = __builtin_bit_cast(float, u.z & 0xffff0000u);
    a.v[2 * s + 1][2] = __builtin_bit_cast(float, u.w << 16);
    a.v[2 * s + 1][3] = __builtin_bit_cast(float, u.w & 0xffff0000u);
  }
}

constexpr int BUF_RSRC_W3 = 0x00020000;  // gfx9 raw buffer: DATA_FORMAT 32, no swizzle / stride

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* g) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(g), 0, 0x7fffffff, BUF_RSRC_W3);
}

// A fragments read MMA_DEPTH MFMAs ahead of their use through a register ring, with scheduling
// fences between steps, so at most MMA_DEPTH fragments (4 VGPRs each) are live: bounds register
// pressure for the two-waves-per-SIMD kernels (the compiler otherwise hoists most of a layer's
// ds_reads). Measured depth 3 / 6 vs 4 (C3, overlapped; rounds 2 and 4): noise.
constexpr int MMA_DEPTH = 4;
template <int NBO, int NS>
__device__ __forceinline__ void mma_ring(Act<NBO>& out, const Op<BF16T, NS>& op, const u16* w, int lane) {
  constexpr int G = NBO < 2 ? NBO : 2;
  constexpr int N = NBO * NS;
  constexpr int D = MMA_DEPTH < N ? MMA_DEPTH : N;
  // step i -> (output block, k-step), output-block-pair major
  auto blk = [](int i) { return (i / (G * NS)) * G + (i % G); };
  auto kst = [](int i) { return (i % (G * NS)) / G; };
  bf16x8 fr[D];
#pragma unroll
  for (int i = 0; i < D; ++i)
    fr[i] = *reinterpret_cast<const bf16x8*>(w + (blk(i) * NS + kst(i)) * BLK + lane * 8);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const int bo = blk(i), s = kst(i);
    out.v[bo] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i % D], op.f[s], out.v[bo], 0, 0, 0);
    if (i + D < N)
      fr[i % D] = *reinterpret_cast<const bf16x8*>(w + (blk(i + D) * NS + kst(i + D)) * BLK + lane * 8);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// out (NBO 16-row blocks) += W (NBO x NS packed blocks, in LDS) . op (NS 32-feature k-steps),
// output-block-pair major (a pair of output blocks completes early, so its epilogue can overlap)
template <int NBO, int NS>
__device__ __forceinline__ void mma(Act<NBO>& out, const Op<BF16T, NS>& op, const u16* w, int lane) {
  constexpr int G = NBO < 2 ? NBO : 2;
#pragma unroll
  for (int b0 = 0; b0 < NBO; b0 += G) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int bo = b0; bo < b0 + G; ++bo) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(w + (bo * NS + s) * BLK + lane * 8);
        out.v[bo] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, op.f[s], out.v[bo], 0, 0, 0);
      }
    }
  }
}
template <int NBO, int NS>
__device__ __forceinline__ void mma(Act<NBO>& out, const Op<F32T, NS>& op, const float* w, int lane) {
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int bo = 0; bo < NBO; ++bo) {
        const floatx4 a4 = *reinterpret_cast<const floatx4*>(w + (bo * NS + s) * BLK + sub * 256 + lane * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          out.v[bo] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[r], op.f[2 * s + sub][r], out.v[bo], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
}

// convenience: out += W . a   (a has 2*NS blocks)
template <class DT, int NBO, int NS>
__device__ __forceinline__ void linear(Act<NBO>& out, const Act<2 * NS>& a, const typename DT::T* w, int lane) {
  Op<DT, NS> op;
  make_op(op, a);
  mma<NBO, NS>(out, op, w, lane);
}

// ------------------------------------------------------------------ weight staging
// Completion of this wave's LDS-DMA pieces. buffer_load ... lds writes LDS asynchronously and is
// tracked by vmcnt only; a workgroup barrier does not wait for it, and hipcc does not reliably emit
// s_waitcnt vmcnt(0) in front of __syncthreads() (measured: C3 edge layers read stale weight
// stages under load). Every barrier that publishes a DMA'd stage to the other waves is preceded
// by this explicit wait (MI355X_MICROARCH.md, "Two waves per SIMD" item 7).
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Copy `nblk` packed blocks (512 elements each) from global memory to LDS with LDS-DMA
// (global_load_lds_dwordx4: 1 KiB per wave-instruction, lane-linear destination = the packed
// order). Issued by all NW waves of the block; completion is awaited by the next barrier.
// Issued as buffer_load_dwordx4 ... lds with an SGPR buffer resource and SGPR offset, and the
// wave index made wave-uniform (readfirstlane): per 1 KiB piece the loop is scalar except the
// load itself (s_mov m0, s_add, buffer_load; the lane offset is a loop-invariant VGPR).
template <int NW, typename T>
__device__ __forceinline__ void dma_blocks(T* lds, const T* g, int nblk) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int loff = (threadIdx.x & 63) * 16;
  const int nkib = nblk * BLK * (int)sizeof(T) / 1024;
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(g);
  for (int i = wave; i < nkib; i += NW)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r, (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(lds) + i * 1024), 16, loff, i * 1024, 0, 0);
}

// Copy `n512` 512-byte fp32 vector chunks (biases) to LDS: half-wave LDS-DMA pieces.
template <int NW>
__device__ __forceinline__ void dma_vec(float* lds, const float* g, int n512) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(g);
  if (lane < 32)
    for (int i = wave; i < n512; i += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(lds) + i * 512), 16, lane * 16, i * 512, 0, 0);
}

// Weight pipeline over one (DBUF=false) or two (DBUF=true) LDS slots, each holding CAP packed
// weight blocks plus VCAP fp32 vector elements (the stage's biases), for a block of NW waves.
//   issue(W_next, n, V_next, nv) starts the DMA of the NEXT layer's weights and biases; next()
//   waits for it (this wave's LDS-DMA via s_waitcnt vmcnt(0), every wave's via the barrier) and
//   makes it the current slot (w(), v()).
// With DBUF the DMA of layer i+1 runs under layer i's MFMAs; the slot it overwrites was last read
// in layer i-1, before the barrier inside next(). Call pattern per layer:
//     pipe.next(); pipe.issue(next layer); compute(pipe.w(), pipe.v());
// The DMA pieces of a stage are split over the NW waves by wave index: a block launched with a
// different wave count than NW would leave pieces unwritten (fewer waves) -- the kernels take NW
// and their launch shape from one geometry struct (KernelGeo below), never from two constants.
template <typename T, int NW, bool DBUF, int CAP, int VCAP = 0>
struct WPipe {
  static_assert(NW >= 1 && NW <= 16, "waves per block");
  static_assert((CAP * BLK * (int)sizeof(T)) % 1024 == 0, "a stage is whole 1-KiB LDS-DMA pieces");
  static_assert(VCAP % 128 == 0, "bias vectors are whole 512-B pieces");
  static constexpr int SLOT_BYTES = CAP * BLK * (int)sizeof(T) + VCAP * 4;
  char* base;
  int cur;
  const T* pend;
  int pend_n;
  const float* pendv;
  int pendv_n;
  __device__ explicit WPipe(void* lds)
      : base(reinterpret_cast<char*>(lds)), cur(0), pend(nullptr), pend_n(0), pendv(nullptr), pendv_n(0) {}
  __device__ __forceinline__ T* slot_w(int s) const { return reinterpret_cast<T*>(base + (DBUF ? s : 0) * SLOT_BYTES); }
  __device__ __forceinline__ float* slot_v(int s) const {
    return reinterpret_cast<float*>(base + (DBUF ? s : 0) * SLOT_BYTES + CAP * BLK * (int)sizeof(T));
  }
  __device__ __forceinline__ void issue(const T* g, int nblk, const float* gv = nullptr, int nvec = 0) {
    if constexpr (DBUF) {
      dma_blocks<NW>(slot_w(cur ^ 1), g, nblk);
      if (gv) dma_vec<NW>(slot_v(cur ^ 1), gv, nvec / 128);
    } else {
      pend = g;
      pend_n = nblk;
      pendv = gv;
      pendv_n = nvec;
    }
  }
  __device__ __forceinline__ const T* next() {
    if constexpr (DBUF) {
      lds_dma_wait();
      __syncthreads();
      cur ^= 1;
    } else {
      __syncthreads();
      dma_blocks<NW>(slot_w(0), pend, pend_n);
      if (pendv) dma_vec<NW>(slot_v(0), pendv, pendv_n / 128);
      lds_dma_wait();
      __syncthreads();
    }
    return slot_w(cur);
  }
  __device__ __forceinline__ const T* w() const { return slot_w(cur); }
  __device__ __forceinline__ const float* v() const { return slot_v(cur); }
};

// Launch geometry of a kernel: NW waves per block, ROWS_PER_WAVE rows per wave. The kernel's
// __launch_bounds__ / flat-work-group-size, its WPipe, its row index and the host launch all read
// THREADS / ROWS from the same struct.
template <int NW_>
struct KernelGeo {
  static_assert(NW_ >= 1 && NW_ <= 16, "waves per block");
  static constexpr int NW = NW_;
  static constexpr int THREADS = 64 * NW_;
  static constexpr int ROWS = ROWS_PER_WAVE * NW_;
};

// Single synchronous stage (kept for simple kernels).
template <typename T>
__device__ __forceinline__ void stage(T* lds, const T* g, int nblk) {
  __syncthreads();
  dma_blocks<WAVES>(lds, g, nblk);
  lds_dma_wait();
  __syncthreads();
}

// sum of the 32 features of head h (= blocks 2h, 2h+1) for this lane's row
template <int NB>
__device__ __forceinline__ float head_sum(const Act<NB>& a, int h) {
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) s += a.v[2 * h][r];
#pragma unroll
  for (int r = 0; r < 4; ++r) s += a.v[2 * h + 1][r];
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  return s;
}

}  // namespace di
