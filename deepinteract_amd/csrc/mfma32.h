// 32-row activation engine on v_mfma_f32_32x32x16_bf16 (gfx950), for the bf16 edge layers.
//
// The same "row-on-lane" idea as common.h, on the 32x32 tile: a wave owns 32 rows (edges), the
// row sits on the MFMA column (lane & 31) and the features in the 16 accumulator registers of
// each 32-feature block, i.e. every activation is held transposed, as v_mfma_f32_32x32x16_bf16
// writes its C/D tile (cdna_hip_programming.md §3):
//
//     feature(block b, reg k, lane half h = lane >> 5) = 32 b + 8 (k >> 2) + 4 h + (k & 3)
//
// A linear layer Y^T = W . X^T takes W as the A operand (32 output rows x 16 input features per
// packed 1-KiB block, streamed from LDS) and the previous accumulator as the B operand with no
// lane movement: registers 8t .. 8t+7 of block b, converted pairwise to bf16, are k-step
// s = 2b + t, whose element j in lane half h is input feature 16 s + 8 (j >> 2) + 4 h + (j & 3).
// The host packing (packing.pack_matrix32) bakes that k order into the weights:
//     block (ob, s), lane l, element j = W[32 ob + (l & 31)][16 s + 8 (j >> 2) + 4 (l >> 5) + (j & 3)]
//
// Why this shape for the edge layers: per 16K MAC the 32x32x16 instruction holds the
// SIMD's vector issue for 8 of its 32 cycles where two 16x16x32 hold it for 16 of 32, and the
// edge layers are bound by the SIMD's issue of their SiLU epilogues (two quarter-rate
// transcendentals per value) beside the MFMAs. One 1-KiB A fragment feeds 16K MAC (as the two
// 16-row groups of the 16x16 kernel sharing a fragment did), so the LDS traffic is unchanged.
// Bias / per-feature vectors stay in natural feature order: block b, quad q of lane half h is the
// float4 at index 8 b + 2 q + h.
#pragma once
#include "common.h"

namespace di {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// NB blocks of 32 features of a 32-row tile
template <int NB>
struct X32 {
  floatx16 v[NB];
};
// packed bf16 B operand: NS k-steps of 16 features
template <int NS>
struct P32 {
  bf16x8 f[NS];
};
// a row of NB*32 bf16 features in its storage format, laid out as the accumulator quads:
// u[4b + q] = features 32 b + 8 q + 4 h .. +3 (8 bytes)
template <int NB>
struct R32 {
  uint2 u[4 * NB];
  __device__ __forceinline__ void load(const u16* row, int h) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) u[4 * b + q] = *reinterpret_cast<const uint2*>(row + 32 * b + 8 * q + 4 * h);
  }
};

__device__ __forceinline__ floatx4 unpack4(uint2 u) {
  return (floatx4){__builtin_bit_cast(float, u.x << 16), __builtin_bit_cast(float, u.x & 0xffff0000u),
                   __builtin_bit_cast(float, u.y << 16), __builtin_bit_cast(float, u.y & 0xffff0000u)};
}
__device__ __forceinline__ floatx4 quad(const floatx16& v, int q) {
  return (floatx4){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}
__device__ __forceinline__ void set_quad(floatx16& v, int q, floatx4 x) {
  v[4 * q] = x[0];
  v[4 * q + 1] = x[1];
  v[4 * q + 2] = x[2];
  v[4 * q + 3] = x[3];
}

template <int NB>
__device__ __forceinline__ void zero(X32<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b) a.v[b] = (floatx16){};
}
// per-feature vector (natural order) from LDS / global memory
template <int NB>
__device__ __forceinline__ void init_vec32_lds(X32<NB>& a, const float* vec, int h) {
  const __attribute__((address_space(3))) floatx4* p = (const __attribute__((address_space(3))) floatx4*)vec;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(a.v[b], q, p[8 * b + 2 * q + h]);
}
template <int NB>
__device__ __forceinline__ void init_vec32(X32<NB>& a, const float* vec, int h) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(a.v[b], q, ld4(vec + 32 * b + 8 * q + 4 * h));
}
template <int NB>
__device__ __forceinline__ void to_x32(X32<NB>& a, const R32<NB>& r) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(a.v[b], q, unpack4(r.u[4 * b + q]));
}
template <int NB>
__device__ __forceinline__ void store_row32(const X32<NB>& a, u16* row, int h) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 x = quad(a.v[b], q);
      *reinterpret_cast<uint2*>(row + 32 * b + 8 * q + 4 * h) = (uint2){pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
    }
}

// k-steps 2b, 2b+1 of an operand from block b of an accumulator
__device__ __forceinline__ void pack_blk(bf16x8& f0, bf16x8& f1, const floatx16& v) {
  uint4 u0, u1;
  u0.x = pack_bf16x2(v[0], v[1]);
  u0.y = pack_bf16x2(v[2], v[3]);
  u0.z = pack_bf16x2(v[4], v[5]);
  u0.w = pack_bf16x2(v[6], v[7]);
  u1.x = pack_bf16x2(v[8], v[9]);
  u1.y = pack_bf16x2(v[10], v[11]);
  u1.z = pack_bf16x2(v[12], v[13]);
  u1.w = pack_bf16x2(v[14], v[15]);
  f0 = __builtin_bit_cast(bf16x8, u0);
  f1 = __builtin_bit_cast(bf16x8, u1);
}
template <int NB>
__device__ __forceinline__ void make_op32(P32<2 * NB>& o, const X32<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b) pack_blk(o.f[2 * b], o.f[2 * b + 1], a.v[b]);
}
// the raw bf16 row IS the packed operand (exact)
template <int NB>
__device__ __forceinline__ void raw_op32(P32<2 * NB>& o, const R32<NB>& r) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint2 lo = r.u[4 * b + 2 * t], hi = r.u[4 * b + 2 * t + 1];
      o.f[2 * b + t] = __builtin_bit_cast(bf16x8, (uint4){lo.x, lo.y, hi.x, hi.y});
    }
}

template <int NB>
__device__ __forceinline__ void pin(X32<NB>& a) {
#pragma unroll
  for (int b = 0; b < NB; ++b) asm volatile("" : "+v"(a.v[b]));
}
template <int NS>
__device__ __forceinline__ void pin(P32<NS>& o) {
#pragma unroll
  for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(o.f[s]));
}
template <int NB>
__device__ __forceinline__ void settle(const R32<NB>& r) {
#pragma unroll
  for (int i = 0; i < 4 * NB; ++i) asm volatile("" ::"v"(r.u[i].x), "v"(r.u[i].y));
}

__device__ __forceinline__ void silu2_blk(floatx16& v) {
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = silu2<true>(v[k]);
}
__device__ __forceinline__ void silu_blk(floatx16& v) {
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = silu<true>(v[k]);
}

__device__ __forceinline__ floatx16 mfma32(const bf16x8& a, const bf16x8& b, const floatx16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 afrag(const u16* w, int blk, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + blk * BLK + lane * 8);
}

// out (NBO 32-feature blocks) += W (NBO x NS packed blocks in LDS, block (ob, s) at ob*NS + s) . op,
// output-block major; A fragments read MMA_DEPTH MFMAs ahead through a register ring
template <int NBO, int NS>
__device__ __forceinline__ void mma32(X32<NBO>& out, const P32<NS>& op, const u16* w, int lane) {
  constexpr int N = NBO * NS;
  constexpr int D = MMA_DEPTH < N ? MMA_DEPTH : N;
  bf16x8 fr[D];
#pragma unroll
  for (int i = 0; i < D; ++i) fr[i] = afrag(w, i, lane);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    out.v[i / NS] = mfma32(fr[i % D], op.f[i % NS], out.v[i / NS]);
    if (i + D < N) fr[i % D] = afrag(w, i + D, lane);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// out = bias (or 0) + W . op over 4 output blocks, with epi(b) -- the epilogue of output block b
// (SiLU, pack, residual) -- issued between the MFMAs of block b + 1: PIPE32_NV VALU / transcendental
// instructions after each MFMA, then the step's LDS fragment read (sched_group_barrier). Block 3's
// epilogue follows the loop. A 32x32x16 MFMA leaves 24 of its 32 issue cycles to the wave's vector
// work (MI355X_MICROARCH.md, cycle constants). Measured (round 4): 4 / 12 VALU per MFMA and the first
// TWO MFMAs of block b + 1 ahead of epi(b) within noise of 8 and one.
constexpr int PIPE32_NV = 8;    // VALU / TRANS instructions per MFMA
constexpr int PIPE32_LEAD = 1;  // MFMAs of block b + 1 issued before epi(b)'s first VALU
template <int NS, class Epi>
__device__ __forceinline__ void lin32_pipe(X32<4>& out, const P32<NS>& op, const u16* w, const float* bias, int lane,
                                           int h, Epi&& epi) {
  constexpr int NBO = 4, N = NBO * NS, D = MMA_DEPTH < N ? MMA_DEPTH : N;
  if (bias) init_vec32_lds(out, bias, h);
  else zero(out);
  bf16x8 fr[D];
#pragma unroll
  for (int i = 0; i < D; ++i) fr[i] = afrag(w, i, lane);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ob = 0; ob < NBO; ++ob) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int i = ob * NS + s;
      out.v[ob] = mfma32(fr[i % D], op.f[s], out.v[ob]);
      if (i + D < N) fr[i % D] = afrag(w, i + D, lane);
    }
    if (ob > 0) epi(ob - 1);
    // the first PIPE32_LEAD MFMAs of block ob go out before any of epi(ob - 1)'s VALU, which reads
    // the accumulator block ob - 1's last MFMA is still writing
    __builtin_amdgcn_sched_group_barrier(0x008, PIPE32_LEAD, 0);  // MFMA
#pragma unroll
    for (int s = PIPE32_LEAD; s < NS + PIPE32_LEAD; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x402, PIPE32_NV, 0);  // VALU | TRANS
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);             // DS read
      if (s < NS) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  epi(NBO - 1);
}

}  // namespace di
