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
// Store cache policy of the row kernel's 16-B stores (gfx950 CPol bits: 2 = nt, 16 = sc1).
// Measured on the C3 pair tensor (4.1 GB per launch, alone): plain 681 us (6.0 TB/s), nt 875 us;
// sc1 / sc1+nt slowed the per-vector kernel by 15 % without speeding up the concurrent GeoT.
// The per-vector (legacy aligned) kernel keeps non-temporal stores.
#ifndef DI_PAIR_STORE
#define DI_PAIR_STORE 0
#endif
// ... and of the bounded row kernel that runs beside GeoT (kernel 3): non-temporal, so the store
// stream does not evict GeoT's L2-resident weight stages and rows. Measured beside GeoT (C3, 512
// complexes): nt 7472 vs plain 7002 complexes/s (GeoT edge layer 429 vs 471 us, pair 1045 vs
// 1082 us); sc0 7018, sc1 3818.
#ifndef DI_PAIR_STORE_BESIDE
#define DI_PAIR_STORE_BESIDE 2
#endif

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
                                                            T* __restrict__ out, int pace) {
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
#if !(DI_PAIR_STORE == 0 || DI_PAIR_STORE == 2)
      const __amdgpu_buffer_rsrc_t orsrc = buf_rsrc(o);  // plane base: q * sizeof(T) < 2^31
#endif
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
          if (q < q_end) {
#if DI_PAIR_STORE == 0 || DI_PAIR_STORE == 2
            __builtin_nontemporal_store(vals[u], reinterpret_cast<V*>(o + q));
#else
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, vals[u]), orsrc, (int)(q * sizeof(T)), 0,
                                                   DI_PAIR_STORE);
#endif
          }
        }
        for (int t = 0; t < pace; ++t) __builtin_amdgcn_s_sleep(1);  // store-rate pacing (di_pair_pace)
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

// Row-streaming form of the aligned path (every plane offset, L2 and chain-2 row 16-B aligned).
// A channel plane is L1 identical-shape rows of L2 elements: chain-2 rows are all the same vector
// hT[c - H, 0:L2], chain-1 row i is the constant h1[i, c]. A work item is (complex, channel,
// PAIR_ROWS rows); a wave owns a contiguous run of 64 of them (a cache line split between rows
// i and i+1 is completed by the same wave back to back). Per 128-chunk segment of the row it loads
// what its rows need ONCE (two 16-B row-vector pieces per lane, or one chain-1 value per row, one
// per lane, broadcast with readlane), then issues only stores: buffer_store_dwordx4 with a
// per-lane constant voffset and the row offset in an SGPR, so a 2-KB row costs two store
// instructions plus scalar address arithmetic, and no load sits between stores.
// <= 32 VGPRs: one wave per SIMD co-resides with the edge kernels (2 x 240 VGPRs).
// Block size is a launch parameter (di_pair_config): 4 waves x one block per CU when the kernel
// shares every CU with GeoT, 8 waves on a few dedicated CUs (CU-masked stream): 64 CUs alone
// store 5.6 TB/s, 32 CUs 3.4 TB/s (C3 micro-batch of 8 complexes).
// INFLIGHT = n > 0 (the "rows_bounded" kernel, di_pair_config kernel 3, the default beside GeoT):
// after every row the wave waits until at most n of its stores are outstanding. The per-CU
// vector-memory queue is in order, so a store-only wave that runs 60 stores ahead parks every
// load of the co-resident GeoT waves (weight-stage DMA, gathers) behind ~1k cycles of store drain;
// a bounded queue keeps GeoT's loads near the front. Measured beside GeoT (C3, 256 complexes,
// one 2-wave block per CU): n = 1/2/3/4/6 -> 5.14/5.53/5.50/5.37-5.61/5.23 k complexes/s, the
// unbounded rows kernel 5.01 k, the per-vector kernel 5.27-5.33 k; 4-wave blocks starve InitEdge.
#ifndef DI_PAIR_INFLIGHT
#define DI_PAIR_INFLIGHT 3
#endif
constexpr int PAIR_SEG = 128;  // 16-B chunks per row segment (2 per lane)
template <typename T, int INFLIGHT, int CPOL>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_vgpr(32)))
void k_pair_rows(const di_pair_desc* __restrict__ descs, int hidden, const T* __restrict__ h,
                 const T* __restrict__ hT, int nrows, int rblocks, int items, T* __restrict__ out, int pace) {
  using V = typename Vec16<T>::V;
  constexpr int VEC = Vec16<T>::N;
  const int PAIR_ROWS = (int)blockDim.x;  // rows per work item: 64 per wave
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int rb = item % rblocks;
    const int rest = item / rblocks;
    const int c = rest % (2 * hidden);
    const int cpx = rest / (2 * hidden);
    const di_pair_desc d = descs[cpx];
    const int r0 = rb * PAIR_ROWS + 64 * wave;  // this wave's rows [r0, r1)
    const int r1 = r0 + 64 < d.l1 ? r0 + 64 : d.l1;
    if (r0 >= r1) continue;  // uniform per wave
    const int nch = d.l2 / VEC;  // 16-B chunks per row
    const uint32_t pitch = (uint32_t)d.l2 * sizeof(T);
    T* o = out + d.out_off + (int64_t)c * ((int64_t)d.l1 * d.l2);
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(o);
    const bool second = c >= hidden;
    uint32_t hv = 0;  // chain 1: lane l holds the value of row r0 + l
    if (!second && r0 + lane < r1) {
      if constexpr (sizeof(T) == 2) {
        hv = h[(d.h1_row + r0 + lane) * hidden + c];
        hv |= hv << 16;
      } else {
        hv = __builtin_bit_cast(uint32_t, h[(d.h1_row + r0 + lane) * hidden + c]);
      }
    }
    const T* src = hT + (int64_t)(c - hidden) * nrows + d.h2_row;
    for (int seg = 0; seg < nch; seg += PAIR_SEG) {
      const int k0 = seg + lane, k1 = seg + 64 + lane;  // this lane's chunks of the segment
      const bool two = seg + 64 < nch;                  // uniform: the segment has a second piece
      V v0, v1;
      if (second) {
        if (k0 < nch) v0 = *reinterpret_cast<const V*>(src + k0 * VEC);
        if (k1 < nch) v1 = *reinterpret_cast<const V*>(src + k1 * VEC);
      }
      for (int i = r0; i < r1; ++i) {
        const int soff = (int)(i * pitch);
        if (!second) {
          const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)hv, i - r0);
          v0 = __builtin_bit_cast(V, (uintx4){b, b, b, b});
          v1 = v0;
        }
        if (k0 < nch)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, v0), r, k0 * 16, soff, CPOL);
        if (two && k1 < nch)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, v1), r, k1 * 16, soff, CPOL);
        if constexpr (INFLIGHT > 0)  // bound this wave's queued stores (see DI_PAIR_INFLIGHT)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
        for (int t = 0; t < pace; ++t) __builtin_amdgcn_s_sleep(1);  // store-rate pacing (di_pair_pace)
      }
    }
  }
}

}  // namespace di

using namespace di;

// resident grid of the persistent pair kernels and waves per row-kernel block (di_pair_config)
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
static int g_pair_blocks = env_int("DI_PAIR_BLOCKS", PAIR_MAX_BLOCKS);
static int g_pair_waves = env_int("DI_PAIR_WAVES", 4);
static int g_pair_kernel = env_int("DI_PAIR_KERNEL", 1);  // 1 row-streaming, 2 per-vector, 3 row-streaming
                                                          // with bounded in-flight stores (aligned path)
static int g_pair_pace = env_int("DI_PAIR_PACE", 0);      // s_sleep(1) (~64 clk) per row / per trip of stores

// Store-rate pacing of the aligned pair kernels when they share the GPU with GeoT: each wave
// sleeps `pace` x 64 clocks after every row (row kernel) or every PAIR_UNROLL-vector trip
// (vector kernel), so the store stream leaves the memory pipeline headroom for GeoT's loads.
extern "C" int di_pair_pace(int32_t pace) {
  if (pace < 0 || pace > 1000) return DI_EINVAL;
  g_pair_pace = pace;
  return DI_OK;
}

extern "C" int di_pair_config(int32_t blocks, int32_t waves_per_block, int32_t kernel) {
  if (blocks < 0 || waves_per_block < 0 || waves_per_block > 16 || kernel < 0 || kernel > 3) return DI_EINVAL;
  if (blocks > 0) g_pair_blocks = blocks;
  if (waves_per_block > 0) g_pair_waves = waves_per_block;
  if (kernel > 0) g_pair_kernel = kernel;
  return DI_OK;
}

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
  const int max_blocks = g_pair_blocks;
  const unsigned grid = (unsigned)(items < max_blocks ? items : max_blocks);
  hipStream_t s = (hipStream_t)stream;
  // aligned16: every channel plane (L1*L2), out_off, L2 and h2_row is a multiple of 16 bytes of
  // elements: 16-B vector loads and non-temporal 16-B stores.
  const int vec = dt == DI_BF16 ? 8 : 4;
#ifndef DI_PAIR_LEGACY
  if (aligned16 && (g_pair_kernel == 1 || g_pair_kernel == 3)) {
    const int rows = 64 * g_pair_waves;  // rows per work item
    const int rblocks = (max_l1 + rows - 1) / rows;
    const int64_t ritems64 = (int64_t)num_complexes * 2 * hidden * rblocks;
    if (ritems64 > INT32_MAX) return DI_ERANGE;
    const int ritems = (int)ritems64;
    const unsigned rgrid = (unsigned)(ritems < max_blocks ? ritems : max_blocks);
    const bool bounded = g_pair_kernel == 3;
    if (dt == DI_BF16 && bounded)
      hipLaunchKernelGGL((k_pair_rows<u16, DI_PAIR_INFLIGHT, DI_PAIR_STORE_BESIDE>), dim3(rgrid), dim3(rows), 0, s, descs, hidden,
                         (const u16*)h, (const u16*)hT, num_rows, rblocks, ritems, (u16*)out, g_pair_pace);
    else if (dt == DI_BF16)
      hipLaunchKernelGGL((k_pair_rows<u16, 0, DI_PAIR_STORE>), dim3(rgrid), dim3(rows), 0, s, descs, hidden, (const u16*)h,
                         (const u16*)hT, num_rows, rblocks, ritems, (u16*)out, g_pair_pace);
    else if (bounded)
      hipLaunchKernelGGL((k_pair_rows<float, DI_PAIR_INFLIGHT, DI_PAIR_STORE_BESIDE>), dim3(rgrid), dim3(rows), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, rblocks, ritems, (float*)out, g_pair_pace);
    else
      hipLaunchKernelGGL((k_pair_rows<float, 0, DI_PAIR_STORE>), dim3(rgrid), dim3(rows), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, rblocks, ritems, (float*)out, g_pair_pace);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DI_OK : (int)e;
  }
#endif
  if (dt == DI_BF16) {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<u16, true>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out, g_pair_pace);
    else
      hipLaunchKernelGGL((k_pair_tensor<u16, false>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out, g_pair_pace);
  } else {
    if (aligned16)
      hipLaunchKernelGGL((k_pair_tensor<float, true>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out, g_pair_pace);
    else
      hipLaunchKernelGGL((k_pair_tensor<float, false>), dim3(grid), dim3(PAIR_THREADS), 0, s, descs, hidden,
                         (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out, g_pair_pace);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
