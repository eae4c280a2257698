// L1 x L2 outer-concat interaction tensor (construct_interact_tensor, pad=False,
// deepinteract_utils.py:158-172):
//     T[c, i, j] = h1[i, c]          for c <  H
//     T[c, i, j] = h2[j, c - H]      for c >= H          (NCHW, [2H, L1, L2] per complex)
// The reference materialises it with two repeat_interleave tensors plus a cat (3x the output
// bytes); here every output byte is written exactly once: a pure HBM store stream (512 MB per
// 2x1000-residue complex in bf16).
//
// Kernels (di_pair_launch.kernel; all persistent, no LDS, so they co-reside with the GeoT kernels
// of the other stream, which hold the LDS):
//  * k_pair_lines (DI_PAIR_LINES, 128-B-aligned planes; measured slower, see di_pair_tensor): every store instruction
//    writes whole 128-B lines. A channel plane repeats with a period of p = 128 / gcd(row bytes,
//    128) rows (p <= 8; 2000-B rows: p = 8 rows = 125 lines), so line r + P t of the plane holds the
//    same bytes for every t (chain 2) or the same bytes of rows p t .. p t + p - 1 (chain 1). A wave
//    owns 8 line residues (8 lanes x 16 B each) and streams t = 0, 1, ...: per-lane constant data
//    and address, the period offset in an SGPR. Row-by-row streaming (k_pair_rows) splits the
//    128-B line at every row boundary between two partial writes (+2.9 % write traffic measured
//    at 2000-B rows).
//  * k_pair_rows (DI_PAIR_ROWS, the default): a wave owns 64 whole rows; the row vector (chain 2) / row value
//    (chain 1) is loaded once per 128-chunk segment, then only stores (16-B aligned planes).
//  * k_pair_vec (DI_PAIR_VECTOR): one 16-B load per 16-B store over flat plane positions.
//  * k_pair_flat: any shape / alignment, one element per thread and step.
// beside != 0 (the schedule beside GeoT): after every row / period the wave waits until at most
// PAIR_INFLIGHT of its stores are outstanding, and stores are non-temporal. The per-CU
// vector-memory queue is in order, so a store-only wave that runs 60 stores ahead parks every
// load of the co-resident GeoT waves (weight-stage DMA, gathers) behind ~1k cycles of store drain.
// Measured beside GeoT (C3, round 2): in-flight bound n = 1/2/3/4/6 -> 5.14/5.53/5.50/5.37-5.61/
// 5.23 k complexes/s (unbounded 5.01 k); nt stores 7472 vs plain 7002 complexes/s (sc0 7018,
// sc1 3818). Alone the plain policy is faster (row kernel 681 vs 875 us per 4.1 GB).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"
#include "pair_queue.h"
#include "../../include/deepinteract_amd.h"

namespace di {

constexpr int PAIR_THREADS = 256;   // k_pair_vec / k_pair_flat
constexpr int PAIR_CHUNK = 65536;   // elements per k_pair_vec / k_pair_flat work item
constexpr int PAIR_UNROLL = 4;
// stores in flight per wave beside GeoT (rounds 2-4: 2 / 4 / 5 slower or equal)
constexpr int PAIR_INFLIGHT = 3;
constexpr int PAIR_SEG = 128;       // 16-B chunks per row segment of k_pair_rows (2 per lane)
constexpr int PAIR_MAX_PLANE_ROWS = 1 << 20;  // k_pair_vec / k_pair_flat row index from an fp32 quotient

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

// store-queue bound of the beside-GeoT schedule (an immediate)
template <bool BESIDE>
__device__ __forceinline__ void pair_bound() {
  if constexpr (BESIDE) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PAIR_INFLIGHT) : "memory");
}
// CPol bits of the 16-B buffer stores: non-temporal (nt = 2) beside GeoT, plain alone. Measured beside
// GeoT (rounds 2-4): plain, sc0, sc1, sc0 sc1 and sc1 nt all slower than nt
template <bool BESIDE>
constexpr int pair_cpol() { return BESIDE ? 2 : 0; }

// (row, column) of flat plane position q: the fp32 quotient is within one of q / l2 for
// q / l2 < 2^20 (PAIR_MAX_PLANE_ROWS) and corrected with two selects; the remainder is exact
// in 64-bit arithmetic.
__device__ __forceinline__ void plane_rc(uint32_t q, uint32_t l2, float inv_l2, uint32_t& i, uint32_t& j) {
  int64_t ii = (int64_t)((float)q * inv_l2);
  int64_t jj = (int64_t)q - ii * (int64_t)l2;
  if (jj < 0) { --ii; jj += l2; }
  if (jj >= (int64_t)l2) { ++ii; jj -= l2; }
  i = (uint32_t)ii;
  j = (uint32_t)jj;
}

// ---- generic: any shape and alignment -------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(PAIR_THREADS) void k_pair_flat(const di_pair_desc* __restrict__ descs, int hidden,
                                                          const T* __restrict__ h, const T* __restrict__ hT,
                                                          int nrows, int chunks, int items, T* __restrict__ out) {
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int chunk = item % chunks;
    const int rest = item / chunks;
    const int c = rest % (2 * hidden);
    const di_pair_desc d = descs[rest / (2 * hidden)];
    const uint32_t l2 = (uint32_t)d.l2;
    const uint32_t plane = (uint32_t)d.l1 * l2;
    const uint32_t q_begin = (uint32_t)chunk * PAIR_CHUNK;
    if (q_begin >= plane) continue;  // uniform per block
    const uint32_t q_end = q_begin + PAIR_CHUNK < plane ? q_begin + PAIR_CHUNK : plane;
    const float inv_l2 = 1.0f / (float)l2;
    T* o = out + d.out_off + (int64_t)c * plane;
    const bool second = c >= hidden;
    const T* h1c = h + d.h1_row * hidden + c;
    const T* h2t = hT ? hT + (int64_t)(c - hidden) * nrows + d.h2_row : nullptr;
    const T* h2c = h + d.h2_row * hidden + (c - hidden);
    for (uint32_t q = q_begin + threadIdx.x; q < q_end; q += PAIR_THREADS) {
      uint32_t i, j;
      plane_rc(q, l2, inv_l2, i, j);
      o[q] = second ? (h2t ? h2t[j] : h2c[(int64_t)j * hidden]) : h1c[(int64_t)i * hidden];
    }
  }
}

// ---- 16-B aligned planes: one load per non-temporal 16-B store --------------------------------
template <typename T>
__global__ __launch_bounds__(PAIR_THREADS) void k_pair_vec(const di_pair_desc* __restrict__ descs, int hidden,
                                                         const T* __restrict__ h, const T* __restrict__ hT, int nrows,
                                                         int chunks, int items, T* __restrict__ out) {
  using V = typename Vec16<T>::V;
  constexpr int VEC = Vec16<T>::N;
  constexpr uint32_t STEP = PAIR_THREADS * VEC;
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int chunk = item % chunks;
    const int rest = item / chunks;
    const int c = rest % (2 * hidden);
    const di_pair_desc d = descs[rest / (2 * hidden)];
    const uint32_t l2 = (uint32_t)d.l2;
    const uint32_t plane = (uint32_t)d.l1 * l2;
    const uint32_t q_begin = (uint32_t)chunk * PAIR_CHUNK;
    if (q_begin >= plane) continue;
    const uint32_t q_end = q_begin + PAIR_CHUNK < plane ? q_begin + PAIR_CHUNK : plane;
    const float inv_l2 = 1.0f / (float)l2;
    T* o = out + d.out_off + (int64_t)c * plane;
    const bool second = c >= hidden;
    const T* h1c = h + d.h1_row * hidden + c;
    const T* h2t = hT + (int64_t)(c - hidden) * nrows + d.h2_row;
    // PAIR_UNROLL independent vectors per thread per trip: the trip's loads (L2 hits) are all in
    // flight before its stores
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
            const T v0 = h1c[(int64_t)i * hidden];
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
        if (q < q_end) __builtin_nontemporal_store(vals[u], reinterpret_cast<V*>(o + q));
      }
    }
  }
}

// broadcast a chain-1 value to a 16-B vector (bf16: two copies per dword)
template <typename T>
__device__ __forceinline__ uint32_t pair_bcast_bits(const T* p);
template <>
__device__ __forceinline__ uint32_t pair_bcast_bits<u16>(const u16* p) {
  const uint32_t v = *p;
  return v | (v << 16);
}
template <>
__device__ __forceinline__ uint32_t pair_bcast_bits<float>(const float* p) {
  return __builtin_bit_cast(uint32_t, *p);
}

// ---- 16-B aligned planes: row streaming ------------------------------------------------------
// One wave streams rows [r0, r1) (<= 64; none when r0 >= r1) of channel plane c of complex d. Per
// 128-chunk segment of the row it loads what its rows need ONCE -- two 16-B pieces of the chain-2 row
// vector hT[c - H, :] per lane, or one chain-1 value hT[c, h1_row + i] per row, one per lane (a
// coalesced 128-B load), broadcast with readlane -- then issues only stores: buffer_store_dwordx4 with
// a per-lane constant voffset and the row offset in an SGPR. hT is the transposed node-feature matrix
// [H, nrows] of di_node_layer's hT_out, bit-identical to h (the same bf16 rounding of the same value).
// hook(): called exactly once, unconditionally, after the first segment's loads have landed and before
// the first store (the queue kernel issues its next-ticket atomic there: behind the item's loads, ahead
// of all its stores). Returns the number of store instructions issued after hook().
template <typename T, bool BESIDE, class F>
__device__ __forceinline__ int pair_rows_item(const di_pair_desc& d, int c, int r0, int r1, int hidden,
                                              const T* __restrict__ hT, int nrows, T* __restrict__ out, int lane,
                                              F&& hook) {
  using V = typename Vec16<T>::V;
  constexpr int VEC = Vec16<T>::N;
  const int nch = d.l2 / VEC;  // 16-B chunks per row
  const uint32_t pitch = (uint32_t)d.l2 * sizeof(T);
  T* o = out + d.out_off + (int64_t)c * ((int64_t)d.l1 * d.l2);
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(o);
  const bool second = c >= hidden;
  const bool any = r0 < r1;  // uniform
  uint32_t hv = 0;           // chain 1: lane l holds the value of row r0 + l
  if (!second && r0 + lane < r1) hv = pair_bcast_bits<T>(hT + (int64_t)c * nrows + d.h1_row + r0 + lane);
  const T* src = hT + (int64_t)(c - hidden) * nrows + d.h2_row;
  V v0 = {}, v1 = {};
  if (second && any) {  // segment 0's chain-2 pieces
    if (lane < nch) v0 = *reinterpret_cast<const V*>(src + lane * VEC);
    if (64 + lane < nch) v1 = *reinterpret_cast<const V*>(src + (64 + lane) * VEC);
  }
  asm volatile("" ::"v"(hv), "v"(v0), "v"(v1));  // the loads land here, before hook()
  hook();
  int after = 0;
  for (int seg = 0; seg < nch; seg += PAIR_SEG) {
    const int k0 = seg + lane, k1 = seg + 64 + lane;  // this lane's chunks of the segment
    const bool two = seg + 64 < nch;                  // uniform: the segment has a second piece
    if (second && any && seg > 0) {
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
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, v0), r, k0 * 16, soff, pair_cpol<BESIDE>());
      if (two && k1 < nch)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, v1), r, k1 * 16, soff, pair_cpol<BESIDE>());
      pair_bound<BESIDE>();
      after += two ? 2 : 1;
    }
  }
  return after;
}

// A work item is (complex, channel, 64 x waves rows); a wave owns a contiguous run of 64 rows.
// <= 32 VGPRs: one wave per SIMD co-resides with the edge kernels (2 x 240 VGPRs).
template <typename T, bool BESIDE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_vgpr(32)))
void k_pair_rows(const di_pair_desc* __restrict__ descs, int hidden, const T* __restrict__ hT, int nrows, int rblocks,
                 int items, T* __restrict__ out) {
  const int rows_per_item = (int)blockDim.x;  // 64 per wave
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int rb = item % rblocks;
    const int rest = item / rblocks;
    const int c = rest % (2 * hidden);
    const di_pair_desc d = descs[rest / (2 * hidden)];
    const int r0 = rb * rows_per_item + 64 * wave;  // this wave's rows [r0, r1)
    const int r1 = r0 + 64 < d.l1 ? r0 + 64 : d.l1;
    if (r0 >= r1) continue;  // uniform per wave
    pair_rows_item<T, BESIDE>(d, c, r0, r1, hidden, hT, nrows, out, lane, [] {});
  }
}

// ---- the pair-tensor queue: the overlapped schedule's pair stream ---------------------------------
// Jobs (one micro-batch's pair tensors each, di_pair_job) are produced in order by the GeoT stream:
// di_pair_signal(job) after the job's final node layer raises the queue's READY word to job + 1 (the
// node layer's kernel end has written its hT back; the signal is a relaxed agent-scope atomic max).
// Items of job k = (complex, channel, 64-row block), ticket order = memory order of the planes.
//   k_pair_stream (the pair stream, beside GeoT): one persistent launch over jobs [begin, end); each
//     wave waits for READY > k (relaxed sc1 poll + s_sleep), acquires (buffer_inv sc1), then takes
//     tickets of job k until they run out. The next ticket's atomic is issued right after the first
//     row of the current item and read after its last row -- every row ends with s_waitcnt vmcnt(3),
//     so an atomic issued >= 4 stores earlier has returned and no wave ever waits for a ticket behind
//     its own store queue (the round-3 per-item ticket, waited at once, cost 45 % beside GeoT). A wave
//     that waits longer than `patience` for READY gives up (counted in the queue's GAVE_UP word):
//     progress never depends on this kernel running concurrently with the producer.
//   k_pair_help (the producer's stream): takes tickets of jobs [first, last] -- all produced, by stream
//     order -- with plain unbounded stores on the whole chip, then one wave waits until every item of
//     those jobs is DONE (items taken by the stream kernel included) and the launch ends. The producer
//     calls it before reusing an hT ring slot (its jobs' reads are over) and once at the end (drain):
//     every job is then complete whatever the stream kernel did. When the GeoT stream runs ahead, the
//     help launches convert its idle time into pair-tensor stores at the full-chip rate.
// Queue words: csrc/pair_queue.h. The producer signals job j with the standalone di_pair_signal launch,
// or (no launch of its own) at the start of its next launch: the node embedding / embedding + InitEdge
// of job j + 1 or a help launch (pq_signal_at_start) -- the kernel boundary has released hT.
// wave-uniform copies (readfirstlane): the compiler's divergence analysis treats every value downstream
// of an atomic as divergent and would wrap each buffer store in a waterfall loop over its resource
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
  const uint64_t u = (uint64_t)x;
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u));
}
template <typename P>
__device__ __forceinline__ P* uni(P* p) {
  return reinterpret_cast<P*>(uni((int64_t)reinterpret_cast<uintptr_t>(p)));
}
__device__ __forceinline__ di_pair_job uni(const di_pair_job& j) {
  di_pair_job u;
  u.hT = uni(j.hT);
  u.descs = uni(j.descs);
  u.out = uni(j.out);
  u.num_rows = uni(j.num_rows);
  u.num_complexes = uni(j.num_complexes);
  u.max_l1 = uni(j.max_l1);
  u.items = uni(j.items);
  return u;
}

__device__ __forceinline__ uint32_t pq_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0 takes the next ticket (returning atomic, waited here); uniform result
__device__ __forceinline__ uint32_t pq_take(uint32_t* tick, int lane) {
  uint32_t t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
}
// the same atomic issued with exec = lane 0 inside one asm statement and NOT waited for: the compiler
// sees a VALU-defined register and inserts no s_waitcnt; the caller reads it (pq_read) only once the
// wave's own in-order vmcnt has passed it. One statement (no branch) so no phi copy of the register
// can be placed between issue and return.
__device__ __forceinline__ uint32_t pq_take_async(uint32_t* tick) {
  uint32_t t;
  uint64_t save;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "global_atomic_add %0, %2, %3, off sc0\n\t"
      "s_mov_b64 exec, %1"
      : "=&v"(t), "=&s"(save)
      : "v"(tick), "v"(1u)
      : "memory");
  return t;
}
__device__ __forceinline__ uint32_t pq_read(uint32_t t, bool waited) {
  if (!waited) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(t));  // not read before the wait above
  return (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
}
// item t of job J -> (complex descriptor, channel, rows [r0, r1)); false: an empty item (r0 >= r1:
// a row block past a smaller complex's chain 1, or a ticket past the descriptors)
__device__ __forceinline__ bool pq_item(const di_pair_job& J, int hidden, uint32_t t, di_pair_desc& d, int& c, int& r0,
                                        int& r1) {
  const int rblocks = (J.max_l1 + 63) >> 6;
  const int rb = (int)(t % (uint32_t)rblocks);
  const int rest = (int)(t / (uint32_t)rblocks);
  c = rest % (2 * hidden);
  const int cx = rest / (2 * hidden);
  const bool in = cx < J.num_complexes;
  const di_pair_desc dd = J.descs[in ? cx : 0];
  d.h1_row = uni(dd.h1_row);
  d.h2_row = uni(dd.h2_row);
  d.out_off = uni(dd.out_off);
  d.l1 = uni(dd.l1);
  d.l2 = uni(dd.l2);
  c = uni(c);
  r0 = uni(rb * 64);
  r1 = uni(!in ? r0 : (r0 + 64 < d.l1 ? r0 + 64 : d.l1));
  return r0 < r1;
}
// wait until *p >= need, at most `patience` ticks of the 100-MHz realtime clock
__device__ __forceinline__ bool pq_wait(const uint32_t* p, uint32_t need, uint64_t patience) {
  if (pq_load(p) >= need) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (pq_load(p) < need) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > patience) return false;
  }
  return true;
}

template <typename T>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_vgpr(32)))
void k_pair_stream(const di_pair_job* __restrict__ jobs, int hidden, uint32_t* __restrict__ q, int job_begin,
                   int job_end, uint64_t patience) {
  const int lane = threadIdx.x & 63;
  for (int k = job_begin; k < job_end; ++k) {
    if (!pq_wait(q + PQ_READY, (uint32_t)k + 1, patience)) {
      if (lane == 0) __hip_atomic_fetch_add(q + PQ_GAVE_UP, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;  // the producer's help launches complete what is left
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // hT of job k as the producer wrote it
    const di_pair_job J = uni(jobs[k]);
    uint32_t* tick = pq_ticket(q, k);
    uint64_t bytes = 0;
    uint32_t done = 0, bad = 0;
    uint32_t t = pq_take(tick, lane);
    while (t < (uint32_t)J.items) {
      di_pair_desc d;
      int c = 0, r0 = 0, r1 = 0;
      pq_item(J, hidden, t, d, c, r0, r1);
      uint32_t tn = 0;
      const int after = pair_rows_item<T, true>(d, c, r0, r1, hidden, reinterpret_cast<const T*>(J.hT), J.num_rows,
                                                reinterpret_cast<T*>(J.out), lane, [&] { tn = pq_take_async(tick); });
      bytes += r1 > r0 ? (uint64_t)(r1 - r0) * d.l2 * sizeof(T) : 0;
      // >= PAIR_INFLIGHT + 1 stores after the atomic and a vmcnt(PAIR_INFLIGHT) after the last one
      const uint32_t next = pq_read(tn, after > PAIR_INFLIGHT);
      // tickets of one counter only grow: a repeated or smaller one means the asynchronous atomic's
      // register was read before its result landed (pq_take_async's contract broken by codegen)
      bad |= next <= t;
      t = next;
      ++done;
    }
    if (done) {
      // DONE counts items whose stores have completed (acknowledged by L2): the help launch that waits
      // for DONE and the kernel boundary after it then publish them to every later launch
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(pq_done(q, k), done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0 && bad) __hip_atomic_fetch_or(q + PQ_ERROR, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0 && bytes)
      __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(q + PQ_SBYTES), bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_vgpr(32)))
void k_pair_help(const di_pair_job* __restrict__ jobs, int hidden, uint32_t* __restrict__ q, int first, int last,
                 int signal_job, uint64_t patience) {
  pq_signal_at_start(q, signal_job);
  const int lane = threadIdx.x & 63;
  uint64_t bytes = 0;
  for (int k = first; k <= last; ++k) {
    const di_pair_job J = uni(jobs[k]);
    uint32_t* tick = pq_ticket(q, k);
    uint32_t done = 0;
    for (uint32_t t = pq_take(tick, lane); t < (uint32_t)J.items; t = pq_take(tick, lane)) {
      di_pair_desc d;
      int c = 0, r0 = 0, r1 = 0;
      if (pq_item(J, hidden, t, d, c, r0, r1)) {
        pair_rows_item<T, false>(d, c, r0, r1, hidden, reinterpret_cast<const T*>(J.hT), J.num_rows,
                                 reinterpret_cast<T*>(J.out), lane, [] {});
        bytes += (uint64_t)(r1 - r0) * d.l2 * sizeof(T);
      }
      ++done;
    }
    if (done) {  // as in k_pair_stream: DONE only for items whose stores have completed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(pq_done(q, k), done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (lane == 0 && bytes)
    __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(q + PQ_HBYTES), bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // one wave holds the launch open until every item of [first, last] is done (taken by either kernel)
  if (blockIdx.x != 0 || threadIdx.x >= 64) return;
  for (int k = first; k <= last; ++k) {
    if (!pq_wait(pq_done(q, k), (uint32_t)jobs[k].items, patience)) {
      if (lane == 0) __hip_atomic_fetch_or(q + PQ_ERROR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

__global__ void k_pair_signal(uint32_t* __restrict__ q, uint32_t ready) {
  if (threadIdx.x == 0) __hip_atomic_fetch_max(q + PQ_READY, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- 128-B aligned planes: whole-line streaming -------------------------------------------------
// Plane geometry (row bytes R, a multiple of 16): the plane repeats every p = 128 / gcd(R, 128) rows
// = P = p R / 128 lines (period bytes p R, a multiple of 128). Line residue r (0 <= r < P) holds
// chunks C = 8 r + s (s = 0..7, 16 B each) of the period: row dr = C / (R/16) of the period,
// chunk k = C % (R/16) of that row. The plane is q = L1 / p whole periods plus a tail of
// (L1 % p) R / 128 lines (the plane end is line aligned, so the tail is whole lines too).
// A work item is (complex, channel, group of 8 x waves residues); lane (wave w, l) stores residue
// r = group * 8 * waves + 8 w + l / 8, chunk s = l % 8, at voffset 128 r + 16 s and soffset t x
// period for t = 0 .. q (t = q: tail residues only):
//   chain 2: the value hT[c - H, 8k .. 8k + 7] is the same for every t (loaded once);
//   chain 1: the value h1[p t + dr, c]: rows t0 p .. t0 p + 63 are loaded one per lane for every
//            64 / p repeats and each lane picks its row by ds_bpermute.
template <typename T, bool BESIDE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_vgpr(32)))
void k_pair_lines(const di_pair_desc* __restrict__ descs, int hidden, const T* __restrict__ h,
                  const T* __restrict__ hT, int nrows, int groups, int items, T* __restrict__ out) {
  using V = typename Vec16<T>::V;
  constexpr int VEC = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = (int)(blockDim.x >> 6);
  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int grp = item % groups;
    const int rest = item / groups;
    const int c = rest % (2 * hidden);
    const di_pair_desc d = descs[rest / (2 * hidden)];
    const uint32_t R = (uint32_t)d.l2 * sizeof(T);
    const uint32_t low = R & (0u - R);                    // largest power of two dividing R (>= 16)
    const int p = 128 / (int)(low < 128u ? low : 128u);   // rows per period
    const uint32_t period = (uint32_t)p * R;              // bytes
    const int P = (int)(period >> 7);                     // lines per period
    const int rw = grp * 8 * nw + 8 * wave;               // this wave's first residue
    if (rw >= P) continue;  // uniform per wave
    const int r = rw + (lane >> 3), s = lane & 7;
    const int nq = d.l1 / p;                              // whole periods
    const int tail = (int)((uint32_t)(d.l1 - nq * p) * R >> 7);  // lines of the partial period
    const int nt = nq + (rw < tail ? 1 : 0);             // repeats this wave issues (uniform)
    const bool on = r < P;                               // lane's residue exists
    const int nch = (int)(R >> 4);
    const int C = 8 * r + s;
    const int dr = C / nch, k = C - dr * nch;
    T* o = out + d.out_off + (int64_t)c * ((int64_t)d.l1 * d.l2);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(o);
    const int voff = 128 * r + 16 * s;
    if (c >= hidden) {
      V v = {};
      if (on) v = *reinterpret_cast<const V*>(hT + (int64_t)(c - hidden) * nrows + d.h2_row + (int64_t)k * VEC);
      for (int t = 0; t < nt; ++t) {
        if (on && (t < nq || r < tail))
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4, v), rs, voff, (int)(t * period),
                                                 pair_cpol<BESIDE>());
        pair_bound<BESIDE>();
      }
    } else {
      const T* h1c = h + d.h1_row * hidden + c;
      const int G = 64 / p;  // repeats per 64 loaded rows
      for (int t0 = 0; t0 < nt; t0 += G) {
        const int row = t0 * p + lane;
        const uint32_t hv = row < d.l1 ? pair_bcast_bits<T>(h1c + (int64_t)row * hidden) : 0u;
        const int t1 = t0 + G < nt ? t0 + G : nt;
        for (int t = t0; t < t1; ++t) {
          const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * ((t - t0) * p + dr), (int)hv);
          if (on && (t < nq || r < tail))
            __builtin_amdgcn_raw_buffer_store_b128((uintx4){b, b, b, b}, rs, voff, (int)(t * period),
                                                   pair_cpol<BESIDE>());
          pair_bound<BESIDE>();
        }
      }
    }
  }
}

}  // namespace di

using namespace di;

// a * b <= limit for non-negative a, b, without forming the (possibly overflowing) product
static inline bool mul_le(int64_t a, int64_t b, int64_t limit) { return a == 0 || b <= limit / a; }

extern "C" int di_pair_tensor_check(int32_t num_complexes, int32_t max_l1, int32_t max_l2, int32_t hidden,
                                    int32_t elem_bytes, const di_pair_launch* launch) {
  if (num_complexes <= 0 || max_l1 <= 0 || max_l2 <= 0 || hidden <= 0 || (elem_bytes != 2 && elem_bytes != 4))
    return DI_EINVAL;
  if (launch) {
    if (launch->kernel < DI_PAIR_AUTO || launch->kernel > DI_PAIR_LINES || launch->blocks < 0 ||
        launch->waves_per_block < 0 || launch->waves_per_block > 16 || (launch->beside != 0 && launch->beside != 1))
      return DI_EINVAL;
  }
  // 32-bit byte offsets inside a channel plane (buffer stores: soffset / voffset < 2^31) and the
  // fp32-quotient row index of the flat kernels
  if (max_l1 > PAIR_MAX_PLANE_ROWS) return DI_ERANGE;
  const int64_t plane = (int64_t)max_l1 * max_l2;  // < 2^51
  if (plane * elem_bytes >= (1LL << 31)) return DI_ERANGE;
  // work items of any kernel: planes x (row blocks <= L1, residue groups <= L2, flat chunks)
  const int64_t chunks = (plane + PAIR_CHUNK - 1) / PAIR_CHUNK;
  int64_t per_plane = max_l1 > max_l2 ? max_l1 : max_l2;
  if (chunks > per_plane) per_plane = chunks;
  const int64_t planes = (int64_t)num_complexes * 2 * hidden;  // < 2^63
  if (!mul_le(planes, per_plane, INT32_MAX)) return DI_ERANGE;
  return DI_OK;
}

extern "C" int di_pair_tensor(di_dtype dt, const di_pair_desc* descs, int32_t num_complexes, int32_t max_l1,
                              int32_t max_l2, int32_t hidden, int32_t aligned, const void* h, const void* hT,
                              int32_t num_rows, const di_pair_launch* launch, void* out, void* stream) {
  if (!descs || !h || !out || aligned < 0 || aligned > 2 || (dt != DI_BF16 && dt != DI_F32)) return DI_EINVAL;
  if (aligned && !hT) return DI_EINVAL;
  const int esz = dt == DI_BF16 ? 2 : 4;
  const int rc = di_pair_tensor_check(num_complexes, max_l1, max_l2, hidden, esz, launch);
  if (rc != DI_OK) return rc;
  const di_pair_launch dflt = {DI_PAIR_AUTO, 0, 0, 0};
  const di_pair_launch& L = launch ? *launch : dflt;
  int kernel = L.kernel;
  // auto: row streaming for any aligned plane. Whole-line stores measured slower (C3, round 3): alone
  // 866 vs 751 us per 4.1 GB (4 waves), 774 vs 757 (8 waves); beside GeoT 7111-7257 vs 7425-7615
  // complexes/s -- each wave's 1-KiB stores stride by the 16-KB row period instead of streaming
  // contiguous rows, which costs more than the +2.9 % partial-line writes they remove. A third form
  // (round 3: row streaming's 64-row runs written as consecutive whole-line 1-KiB stores, chain-2
  // chunks from an LDS copy of the hT row, chain-1 values by ds_bpermute) was slower too: alone 770
  // vs 753 us, beside GeoT 5840-5937 vs 7320-7549 complexes/s (its per-store LDS reads queue behind
  // the edge kernels' fragment reads); removed
  if (kernel == DI_PAIR_AUTO) kernel = aligned >= 1 ? DI_PAIR_ROWS : 0;
  if (kernel == DI_PAIR_LINES && aligned < 2) return DI_EINVAL;  // whole-line stores need 128-B planes
  if ((kernel == DI_PAIR_ROWS || kernel == DI_PAIR_VECTOR) && aligned < 1) return DI_EINVAL;
  const int max_blocks = L.blocks > 0 ? L.blocks : device_cus();
  const int waves = L.waves_per_block > 0 ? L.waves_per_block : 4;
  const bool beside = L.beside != 0;
  hipStream_t s = (hipStream_t)stream;
  const int planes = num_complexes * 2 * hidden;
  auto grid_of = [&](int items) { return dim3((unsigned)(items < max_blocks ? items : max_blocks)); };
  if (kernel == DI_PAIR_LINES) {
    // residue groups per plane: the largest period (p = 8 rows) over every complex's plane
    const int64_t lines = ((int64_t)8 * max_l2 * esz) >> 7;
    const int groups = (int)((lines + 8 * waves - 1) / (8 * waves));
    const int items = planes * groups;
    const dim3 g = grid_of(items), b(64 * waves);
    if (dt == DI_BF16) {
      if (beside) hipLaunchKernelGGL((k_pair_lines<u16, true>), g, b, 0, s, descs, hidden, (const u16*)h, (const u16*)hT, num_rows, groups, items, (u16*)out);
      else hipLaunchKernelGGL((k_pair_lines<u16, false>), g, b, 0, s, descs, hidden, (const u16*)h, (const u16*)hT, num_rows, groups, items, (u16*)out);
    } else {
      if (beside) hipLaunchKernelGGL((k_pair_lines<float, true>), g, b, 0, s, descs, hidden, (const float*)h, (const float*)hT, num_rows, groups, items, (float*)out);
      else hipLaunchKernelGGL((k_pair_lines<float, false>), g, b, 0, s, descs, hidden, (const float*)h, (const float*)hT, num_rows, groups, items, (float*)out);
    }
  } else if (kernel == DI_PAIR_ROWS) {
    const int rows = 64 * waves;  // rows per work item
    const int rblocks = (max_l1 + rows - 1) / rows;
    const int items = planes * rblocks;
    const dim3 g = grid_of(items), b(rows);
    if (dt == DI_BF16) {
      if (beside) hipLaunchKernelGGL((k_pair_rows<u16, true>), g, b, 0, s, descs, hidden, (const u16*)hT, num_rows, rblocks, items, (u16*)out);
      else hipLaunchKernelGGL((k_pair_rows<u16, false>), g, b, 0, s, descs, hidden, (const u16*)hT, num_rows, rblocks, items, (u16*)out);
    } else {
      if (beside) hipLaunchKernelGGL((k_pair_rows<float, true>), g, b, 0, s, descs, hidden, (const float*)hT, num_rows, rblocks, items, (float*)out);
      else hipLaunchKernelGGL((k_pair_rows<float, false>), g, b, 0, s, descs, hidden, (const float*)hT, num_rows, rblocks, items, (float*)out);
    }
  } else {
    const int chunks = (int)(((int64_t)max_l1 * max_l2 + PAIR_CHUNK - 1) / PAIR_CHUNK);
    const int items = planes * chunks;
    const dim3 g = grid_of(items), b(PAIR_THREADS);
    if (kernel == DI_PAIR_VECTOR) {
      if (dt == DI_BF16) hipLaunchKernelGGL(k_pair_vec<u16>, g, b, 0, s, descs, hidden, (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out);
      else hipLaunchKernelGGL(k_pair_vec<float>, g, b, 0, s, descs, hidden, (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out);
    } else {
      if (dt == DI_BF16) hipLaunchKernelGGL(k_pair_flat<u16>, g, b, 0, s, descs, hidden, (const u16*)h, (const u16*)hT, num_rows, chunks, items, (u16*)out);
      else hipLaunchKernelGGL(k_pair_flat<float>, g, b, 0, s, descs, hidden, (const float*)h, (const float*)hT, num_rows, chunks, items, (float*)out);
    }
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

// ---- the pair-tensor queue (C ABI) ------------------------------------------------------------
static inline int64_t pq_bytes(int64_t jobs) { return 4 * (PQ_HEAD_WORDS + PQ_JOB_WORDS * jobs); }

extern "C" int64_t di_pair_queue_bytes(int32_t num_jobs) { return num_jobs > 0 ? pq_bytes(num_jobs) : -1; }

extern "C" int32_t di_pair_job_items(int32_t num_complexes, int32_t max_l1, int32_t hidden) {
  if (num_complexes <= 0 || max_l1 <= 0 || hidden <= 0) return DI_EINVAL;
  const int64_t n = (int64_t)num_complexes * 2 * hidden * ((max_l1 + 63) / 64);
  return n > INT32_MAX ? DI_ERANGE : (int32_t)n;
}

// ticks of the 100-MHz-class realtime clock (s_memrealtime) in `ms` milliseconds on this device
static uint64_t pq_ticks(double ms) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0)
    khz = 100000;
  return (uint64_t)(ms * khz);
}

extern "C" int di_pair_signal(void* queue, int32_t job, void* stream) {
  if (!queue || job < 0) return DI_EINVAL;
  hipLaunchKernelGGL(k_pair_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint32_t*)queue, (uint32_t)job + 1);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_pair_stream(di_dtype dt, const di_pair_job* jobs, int32_t job_begin, int32_t job_end, int32_t hidden,
                              void* queue, const di_pair_launch* launch, float patience_ms, void* stream) {
  if (!jobs || !queue || job_begin < 0 || job_end <= job_begin || hidden <= 0 || (dt != DI_BF16 && dt != DI_F32) ||
      !(patience_ms > 0.f))
    return DI_EINVAL;
  // default shape, bf16: one 2-wave block per CU (512 store waves on 256 CUs). Round 6, beside the
  // persistent edge ring and the weight-stationary node layers: 256 x 2 and 512 x 1 beat round 3's
  // 128 x 4 (4 waves on half the CUs) by 2 % on two boxes; more than 512 waves slow GeoT. fp32 keeps
  // 128 x 4 beside its 4-wave edge blocks (1831 / 1805 vs 1857 / 1851 complexes/s)
  const int cus = device_cus();
  const bool f32 = dt == DI_F32;
  const int blocks = launch && launch->blocks > 0 ? launch->blocks : (f32 ? (cus + 1) / 2 : cus);
  const int waves = launch && launch->waves_per_block > 0 ? launch->waves_per_block : (f32 ? 4 : 2);
  if (waves > 16) return DI_EINVAL;
  const dim3 g((unsigned)blocks), b((unsigned)(64 * waves));
  hipStream_t s = (hipStream_t)stream;
  const uint64_t pt = pq_ticks(patience_ms);
  if (dt == DI_BF16) hipLaunchKernelGGL(k_pair_stream<u16>, g, b, 0, s, jobs, hidden, (uint32_t*)queue, job_begin, job_end, pt);
  else hipLaunchKernelGGL(k_pair_stream<float>, g, b, 0, s, jobs, hidden, (uint32_t*)queue, job_begin, job_end, pt);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_pair_help(di_dtype dt, const di_pair_job* jobs, int32_t first_job, int32_t last_job, int32_t hidden,
                            void* queue, const di_pair_launch* launch, int32_t signal_job, void* stream) {
  if (!jobs || !queue || first_job < 0 || last_job < first_job || hidden <= 0 || (dt != DI_BF16 && dt != DI_F32))
    return DI_EINVAL;
  const int blocks = launch && launch->blocks > 0 ? launch->blocks : device_cus();
  const int waves = launch && launch->waves_per_block > 0 ? launch->waves_per_block : 8;
  if (waves > 16) return DI_EINVAL;
  const dim3 g((unsigned)blocks), b((unsigned)(64 * waves));
  hipStream_t s = (hipStream_t)stream;
  const uint64_t pt = pq_ticks(10000.0);  // a completion wait this long is an error (ERROR bit 0), never a hang
  if (dt == DI_BF16)
    hipLaunchKernelGGL(k_pair_help<u16>, g, b, 0, s, jobs, hidden, (uint32_t*)queue, first_job, last_job, signal_job, pt);
  else
    hipLaunchKernelGGL(k_pair_help<float>, g, b, 0, s, jobs, hidden, (uint32_t*)queue, first_job, last_job, signal_job, pt);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
