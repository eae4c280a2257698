// GeoT forward kernels for gfx950 (MI355X): node embedding, InitEdge, fused edge layer,
// fused node layer. Device engine: common.h ("row-on-lane" transposed activations,
// MFMA 16x16 chains with weights streamed through LDS by LDS-DMA).
//
// Reference semantics (paths relative to /root/reference/project/utils/):
//   node embedding            deepinteract_modules.py:1541-1543, 1663-1664
//   InitEdgeModule            deepinteract_modules.py:198-264
//   ConformationModule        deepinteract_modules.py:373-455 (+ ResBlock :458-497)
//   attention edge UDFs       deepinteract_modules.py:76-96, graph_utils.py:21-63
//   GT layer residual / FFN   deepinteract_modules.py:669-727 (intermediate), :892-946 (final)
// Algebraic rewrites (exact in real arithmetic, fp32-rounding-level differences only):
//   * eval BatchNorm folded into the following/preceding linear (host packing);
//   * nbr_linear applied once per edge (Fn = F W^T + b) and gathered, instead of per gathered row;
//   * two-stage geometric embeddings (W1 . W0 . g) pre-multiplied on the host;
//   * InitEdge's emb[src]/emb[dst] slots of combined_linear_0 precomputed per node position
//     (pos tables [2304,128]); the 4 final gates summed before multiplying (a*x+b*x = (a+b)*x).
#include <type_traits>
#include "common.h"
#include "layout.h"
#include "mfma32.h"
#include "pair_queue.h"
#include "../../include/deepinteract_amd.h"

namespace di {

struct EmbedArgs {
  int Nt;
  int in_dim;
  const float* node_f;
  const void* wmat;
  const float* wvec;
  void* h_out;
  void* qkv_out;
  uint32_t* sig_q;  // optional pair queue: raise its READY to sig_job + 1 at launch start (pair_queue.h)
  int sig_job;
};

struct InitArgs {
  int Et;
  const float* edge_f;
  const int* src;
  const int* dst;
  const int* node_pos;
  const void* wmat;
  const float* wvec;
  const float* pos_src;
  const float* pos_dst;
  void* f_out;
  void* fn_out;
};

struct EdgeArgs {
  int Et;
  const float* edge_f;
  const int* src;
  const int* dst;
  const int* nbr;
  const void* f_in;
  const void* fn_in;
  const void* qkv;
  const void* wmat;
  const float* wvec;
  float* alpha_out;
  void* f_out;
  void* fn_out;
  // di_edge_layer_attn (bf16): the attention aggregation folded into the epilogue (edge_attn_fold)
  float* attn_out = nullptr;
  float* attn_parts = nullptr;
  const int* in_ptr = nullptr;
};

struct NodeArgs {
  int Nt;
  const float* attn;  // optional [Nt, 128] aggregated attention rows (k_node_aggr); null: gather here
  void* hT_out;  // optional [128, Nt] transposed copy of h_out (pair-tensor input)
  const int* src;
  const int* in_ptr;
  const float* alpha;
  const void* h_in;
  const void* qkv;
  const void* wmat;
  const float* wvec;
  void* h_out;
  void* qkv_out;
  // with attn: di_edge_layer_attn's partial sums of the destinations split over edge tiles
  // (attn_row; in_ptr is then the CSR row pointer)
  const float* attn_parts = nullptr;
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// A bijection of [0, n) that turns slot j, run on XCD j mod 8 (blocks are dealt round-robin over
// the 8 XCDs: b and b + 8 share one -- speed only, correct under any placement), into
// base(j mod 8) + j / 8: the slots of one XCD cover one contiguous range, so neighbouring rows
// (a destination range's gathered K / Q / V rows) stay in that XCD's L2.
// (n = 8q + r: XCD y holds q + [y < r] slots, so base(x) = x q + min(x, r))
__device__ __forceinline__ int xcd_slot(int j, int n) {
  const int x = j & 7;
  return x * (n >> 3) + min(x, n & 7) + (j >> 3);
}
template <int NW>
__device__ __forceinline__ int row_id() {
  return blockIdx.x * (NW * ROWS_PER_WAVE) + (threadIdx.x >> 6) * ROWS_PER_WAVE + (threadIdx.x & 15);
}

// Launch geometry per storage dtype. bf16 (the benchmark path): 4-wave blocks, two per CU
// (2 x 80 KiB of LDS, <=256 VGPRs), each double-buffering its weight stages so the LDS-DMA of
// layer i+1 runs under layer i's MFMAs. Two independent blocks per CU matter: the waves of ONE
// block meet at every stage barrier in lockstep, so only waves of the other block can fill a
// SIMD's MFMA pipe while these run their SiLU VALU work (and vice versa). Measured alternatives
// (round 1-2): one 8-wave block per CU with or without a decoupled ring, persistent
// tiles, XCD-aware tile order, static wave priority, pumped DMA pieces -- all slower.
// fp32 (parity path; stages twice as large): same geometry, synchronous single-buffered stages.
template <class DT>
struct Geo : KernelGeo<4> {
  static constexpr bool DBUF = DT::kBF16;
  static constexpr int CAP = 40;  // blocks per weight stage buffer
};

// The edge's own input row F: bf16 path keeps it in registers as a packed MFMA operand (its
// stored values are bf16, so unpacking is exact); fp32 path re-reads it (L2) where needed.
template <class DT>
struct FRow;
template <>
struct FRow<BF16T> {
  Op<BF16T, 4> op;
  __device__ void load(const u16* row, int g) {
    Act<8> a;
    load_row(a, row, g);
    make_op(op, a);
  }
  // the raw row IS the packed operand: op.f[s] = {u[2s].x, u[2s].y, u[2s+1].x, u[2s+1].y}
  __device__ void set_raw(const RawRow<u16>& r) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      op.f[k] = __builtin_bit_cast(bf16x8, (uint4){r.u[2 * k].x, r.u[2 * k].y, r.u[2 * k + 1].x, r.u[2 * k + 1].y});
  }
  __device__ void act(Act<8>& a, const u16*, int) const { unpack_op(a, op); }
  __device__ const Op<BF16T, 4>& operand(const u16*, int) const { return op; }
};
template <>
struct FRow<F32T> {
  Op<F32T, 4> tmp;
  __device__ void load(const float*, int) {}
  __device__ void act(Act<8>& a, const float* row, int g) const { load_row(a, row, g); }
  __device__ const Op<F32T, 4>& operand(const float* row, int g) {
    Act<8> a;
    load_row(a, row, g);
    make_op(tmp, a);
    return tmp;
  }
};

// ================================================================ node embedding (+ Q/K/V of layer 0)
using EmbedGeo = KernelGeo<4>;
template <class DT>
__global__ __launch_bounds__(EmbedGeo::THREADS) void k_node_embed(EmbedArgs a) {
  pq_signal_at_start(a.sig_q, a.sig_job);
  using T = typename DT::T;
  __shared__ __attribute__((aligned(16))) T lds[2 * MAT128 * BLK];
  const int lane = lane_id(), g = lane >> 4;
  const int r = row_id<EmbedGeo::NW>();
  const bool valid = r < a.Nt;
  const int v = valid ? r : a.Nt - 1;
  const T* W = reinterpret_cast<const T*>(a.wmat);
  WPipe<T, EmbedGeo::NW, true, MAT128> pipe(lds);
  pipe.issue(W + EM_EMB * BLK, MAT128);

  Act<8> x;  // in_dim (113 raw DIPS-Plus + geometric features) input columns, zero padded to 128
  const float* row = a.node_f + (int64_t)v * a.in_dim;
#pragma unroll
  for (int b = 0; b < 8; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 16 * b + 4 * g + q;
      x.v[b][q] = f < a.in_dim ? row[f] : 0.f;
    }
  const T* w = pipe.next();
  pipe.issue(W + EM_Q * BLK, MAT128);
  Act<8> h;
  zero(h);
  linear<DT, 8, 4>(h, x, w, lane);
  if (valid) store_row(h, reinterpret_cast<T*>(a.h_out) + (int64_t)v * HID, g);
  T* qkv = reinterpret_cast<T*>(a.qkv_out);
#pragma unroll 1
  for (int q = 0; q < 3; ++q) {
    w = pipe.next();
    if (q < 2) pipe.issue(W + (EM_Q + MAT128 * (q + 1)) * BLK, MAT128);
    Act<8> t;
    init_vec(t, a.wvec + EMV_Q + 128 * q, g);
    linear<DT, 8, 4>(t, h, w, lane);
    if (valid) store_row(t, qkv + (int64_t)v * 3 * HID + q * HID, g);
  }
}

// ================================================================ InitEdgeModule (+ layer-0 nbr_linear)
// GC (DI_GRAPH_GEO_REF batches): the direction terms silu(dir_linear_{0,1}(0)) = 0 are skipped and
// the orientation terms are the packed constants IEV_ORC / IEV_OGATE; the layer-0
// silu(nbr_linear(F)) rows are only computed when fn_out is given (the grouped edge kernel does
// not gather them for such batches).
// Launch shape of the bf16 InitEdge: weights staged synchronously in one 40-KiB slot per block,
// so three blocks share a CU (the kernel holds 150 VGPRs) and cover each other's stage waits.
// Measured (C3 micro-batch, GEO_REF): alone 109 vs 118 us with two double-buffered blocks, beside
// the pair stream 168 vs 187 us; four blocks (128 VGPRs) spill: 130 / 206 us.
template <class DT>
struct InitGeo : Geo<DT> {
  static constexpr bool DBUF = false;
  static constexpr int WPE = DT::kBF16 ? 3 : 2;  // blocks (waves per SIMD) per CU
};
// The node embedding (+ layer-0 Q/K/V) as the first `embed_blocks` blocks of an InitEdge launch
// (di_embed_init_edge): same stages and arithmetic as k_node_embed<BF16T> through InitEdge's single
// 40-block LDS slot, so the two run side by side inside one launch instead of the embedding on a
// side stream (whose blocks find no LDS beside InitEdge's until its tail).
// (NW: the launch's waves per block, 16 rows each)
template <class DT, int NW = InitGeo<DT>::NW>
__device__ __forceinline__ void embed_block(const EmbedArgs& ea, WPipe<typename DT::T, NW, false, InitGeo<DT>::CAP>& pipe,
                                            int blk, int lane, int g) {
  using T = typename DT::T;
  const int r = blk * ROWS_PER_WAVE * NW + (threadIdx.x >> 6) * ROWS_PER_WAVE + (lane & 15);
  const bool valid = r < ea.Nt;
  const int v = valid ? r : ea.Nt - 1;
  const T* W = reinterpret_cast<const T*>(ea.wmat);
  pipe.issue(W + EM_EMB * BLK, MAT128);
  Act<8> x;
  const float* row = ea.node_f + (int64_t)v * ea.in_dim;
#pragma unroll
  for (int b = 0; b < 8; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 16 * b + 4 * g + q;
      x.v[b][q] = f < ea.in_dim ? row[f] : 0.f;
    }
  const T* w = pipe.next();
  Act<8> h;
  zero(h);
  // bf16: the fragment ring; fp32: the 16x16x4 chain of k_node_embed<F32T> (same operands, same order)
  auto mm = [&](Act<8>& out, const Op<DT, 4>& op, const T* wm) {
    if constexpr (DT::kBF16) mma_ring<8, 4>(out, op, wm, lane);
    else mma<8, 4>(out, op, wm, lane);
  };
  {
    Op<DT, 4> xop;
    make_op(xop, x);
    mm(h, xop, w);
  }
  if (valid) store_row(h, reinterpret_cast<T*>(ea.h_out) + (int64_t)v * HID, g);
  Op<DT, 4> hop;
  make_op(hop, h);
  T* qkv = reinterpret_cast<T*>(ea.qkv_out);
#pragma unroll 1
  for (int q = 0; q < 3; ++q) {
    pipe.issue(W + (EM_Q + MAT128 * q) * BLK, MAT128);
    w = pipe.next();
    Act<8> t;
    init_vec(t, ea.wvec + EMV_Q + 128 * q, g);
    mm(t, hop, w);
    if (valid) store_row(t, qkv + (int64_t)v * 3 * HID + q * HID, g);
  }
}

template <class DT, bool GC>
__global__ __attribute__((amdgpu_flat_work_group_size(1, InitGeo<DT>::THREADS),
                          amdgpu_waves_per_eu(InitGeo<DT>::WPE, InitGeo<DT>::WPE)))
void k_init_edge(InitArgs a, EmbedArgs ea, int embed_blocks) {
  pq_signal_at_start(ea.sig_q, ea.sig_job);
  using T = typename DT::T;
  using G = InitGeo<DT>;
  constexpr bool FAST = DT::kBF16;
  constexpr int CAP = G::CAP;
  __shared__ __attribute__((aligned(16))) T lds[(G::DBUF ? 2 : 1) * CAP * BLK];
  const int lane = lane_id(), g = lane >> 4;
  if constexpr (GC) {
    if ((int)blockIdx.x < embed_blocks) {  // uniform per block
      WPipe<T, G::NW, false, CAP> epipe(lds);
      embed_block<DT>(ea, epipe, blockIdx.x, lane, g);
      return;
    }
  }
  const int r = ((int)blockIdx.x - embed_blocks) * G::ROWS + (threadIdx.x >> 6) * ROWS_PER_WAVE + (lane & 15);
  const bool valid = r < a.Et;
  const int e = valid ? r : a.Et - 1;
  const T* W = reinterpret_cast<const T*>(a.wmat);
  WPipe<T, G::NW, G::DBUF, CAP> pipe(lds);
  pipe.issue(W + IE_T0 * BLK, 8);  // stage 0: the collapsed edge-message map (8 blocks)

  Act<2> geo;
  load_edge_geo(geo, a.edge_f + (int64_t)e * NFEAT_E, g);
  Op<DT, 1> gop;
  make_op(gop, geo);

  // combined_linear_0 over [emb[src], emb[dst], em0, silu(d0), silu(r0), silu(o0), silu(a0)]
  Act<8> acc;
  load_row(acc, a.pos_src + (int64_t)a.node_pos[a.src[e]] * HID, g);
  add_row(acc, a.pos_dst + (int64_t)a.node_pos[a.dst[e]] * HID, g);
  if constexpr (GC) add_vec(acc, a.wvec + IEV_ORC, g);  // orientation term (constant)
  // geometric terms t = 1..4 (dist, dir, orient, amide); GC: dist and amide only
  constexpr int NT = GC ? 2 : 4;
  auto geo_t = [](int i) { return GC ? (i == 0 ? 1 : 4) : i + 1; };
  {
    // t = 0: edge_messages_linear_0 and its combined_linear_0 slice, collapsed on the host into one
    // [128, 2] map of the message columns (no activation between them, :237-241)
    const T* w = pipe.next();
    pipe.issue(W + (IE_T0 + 40 * geo_t(0)) * BLK, 40);
    mma<8, 1>(acc, gop, w, lane);
  }
#pragma unroll 1
  for (int i = 0; i < NT; ++i) {
    const T* w = pipe.next();
    if (i + 1 < NT) pipe.issue(W + (IE_T0 + 40 * geo_t(i + 1)) * BLK, 40);
    else pipe.issue(W + IE_GEO1 * BLK, 40);
    Act<8> y;
    zero(y);
    mma<8, 1>(y, gop, w, lane);
    silu2_<8, FAST>(y);
    linear<DT, 8, 4>(acc, y, w + 8 * BLK, lane);
  }
  silu2_<8, FAST>(acc);  // combined_edge_logits (log2 units: feeds the gate product -> linear)
  // gating: (em1 + silu(d1) + silu(r1) + silu(o1) + silu(a1)) * c
  {
    const T* w = pipe.next();
    pipe.issue(W + IE_C1 * BLK, 16);
    Act<8> gs;
    if constexpr (GC) init_vec(gs, a.wvec + IEV_OGATE, g);  // silu(o1): constant; silu(r1) = 0
    else zero(gs);
#pragma unroll 1
    for (int t = 0; t < 5; ++t) {
      if (GC && (t == 2 || t == 3)) continue;
      Act<8> y;
      zero(y);
      mma<8, 1>(y, gop, w + 8 * t * BLK, lane);
      if (t > 0) silu2_<8, FAST>(y);
      add_(gs, y);
    }
    mul_(acc, gs);
  }
  const bool with_fn = a.fn_out != nullptr;  // uniform
  // combined_linear_2(combined_linear_1(.)) : 128 -> 28 (padded 32) -> 128
  Act<8> f;
  {
    const T* w = pipe.next();
    if (with_fn) pipe.issue(W + IE_NBR * BLK, MAT128);
    Act<2> z;
    zero(z);
    linear<DT, 2, 4>(z, acc, w, lane);
    zero(f);
    linear<DT, 8, 1>(f, z, w + 8 * BLK, lane);
  }
  if (valid) store_edge_row(f, reinterpret_cast<T*>(a.f_out) + (int64_t)e * HID, g);
  if (!with_fn) return;
  // layer-0 silu(nbr_linear(F)), applied once per edge and gathered by the conformation module
  // (silu(nbr_linear(F[ids])) == silu(nbr_linear(F))[ids], deepinteract_modules.py:386-390)
  {
    const T* w = pipe.next();
    Act<8> fn;
    init_vec(fn, a.wvec + IEV_NBR, g);
    linear<DT, 8, 4>(fn, f, w, lane);
    silu_<8, FAST>(fn);
    if (valid) store_edge_row(fn, reinterpret_cast<T*>(a.fn_out) + (int64_t)e * HID, g);
  }
}

// Resident InitEdge weights (k_init_res_x32): the 128 weight blocks the GEO_REF path reads, at these
// block offsets of the LDS copy
constexpr int IR_NBLK = 128;  // resident weight blocks
constexpr int IR_T0 = 0, IR_DIST = 8, IR_AMIDE = 48, IR_GATE = 88, IR_C = 112;

// ================================================================ InitEdgeModule on 32x32x16 MFMA (bf16)
// The arithmetic of k_init_edge<BF16T, GC> on 32-row tiles (csrc/mfma32.h): every 128-wide stage is
// half the MFMAs of the 16x16 form, so half the MFMA hold on the SIMD's vector issue the SiLU-heavy
// InitEdge is bound by (640 SiLU values per edge against 65,536 MAC). The bf16 init blob (kind 1) is
// packed in the 32x32 fragment order (di_blob_layout(1, bf16) == 32). Geometric terms and gates are
// produced one 32-feature block at a time (16 registers) and packed / multiplied straight away, so
// a 32-row tile fits three waves per SIMD (<= 168 VGPRs).
// Weight phases of one tile (GC: DI_GRAPH_GEO_REF batches):
//   T0 (collapsed edge-message map, [128x32] 8 blk) -> geometric terms (dist, [dir, orient,] amide:
//   [128x32] W_t0 + [128x128] combined_linear_0 slice, 40 blk each) -> gates (em1, dist1, [dir1,
//   orient1,] amide1: [128x32] each) -> combined_linear_1/2 (8 + 8 blk) -> [layer-0 nbr_linear, 32 blk]
constexpr int INIT_X32_NW = 4;  // waves per block (three waves per SIMD: 12 / NW blocks per CU)
struct InitX32Geo {
  static constexpr int NW = INIT_X32_NW, THREADS = 64 * NW, ROWS_PER_WAVE = 32, ROWS = ROWS_PER_WAVE * NW;
  static constexpr int EMBED_ROWS = 16 * NW;  // node rows of one embedding block of the same launch
};

// one 32-row tile of InitEdge; wt(phase) returns the phase's weight blocks (LDS) and gate_off(t) the
// block offset of gate t (0 em, 1 dist, 2 dir, 3 orient, 4 amide) inside the gates phase.
// acc enters holding emb[src] + emb[dst] slots (+ the orientation constant for GC).
template <bool GC, class WT, class GO>
__device__ __forceinline__ void init_tile_x32(X32<4>& acc, const P32<2>& gop, const float* wvec, int lane, int h,
                                              WT&& wt, GO&& gate_off, X32<4>& f) {
  mma32<4, 2>(acc, gop, wt(0), lane);  // t = 0: the collapsed [128, 2] edge-message map
  constexpr int NT = GC ? 2 : 4;
#pragma unroll 1
  for (int i = 0; i < NT; ++i) {
    const u16* w = wt(1 + i);
    // y = silu2(W_t0 . g), one 32-feature block at a time, packed as combined_linear_0's operand
    P32<8> yop;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      lean_fence();  // block by block: one block's fragments and values live at a time
      floatx16 y = {};
      y = mfma32(afrag(w, 2 * b, lane), gop.f[0], y);
      y = mfma32(afrag(w, 2 * b + 1, lane), gop.f[1], y);
      silu2_blk(y);
      pack_blk(yop.f[2 * b], yop.f[2 * b + 1], y);
      asm volatile("" : "+v"(yop.f[2 * b]), "+v"(yop.f[2 * b + 1]));
    }
    mma32<4, 8>(acc, yop, w + 8 * BLK, lane);
    pin(acc);
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) silu2_blk(acc.v[b]);  // combined_edge_logits (log2 units)
  pin(acc);  // computed here: sunk to their uses, x and rcp(1 + 2^-x) would both stay live
  // gating: (em1 + silu(d1) + silu(r1) + silu(o1) + silu(a1)) * c, block by block
  {
    const u16* w = wt(1 + NT);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      lean_fence();
      floatx16 gs = {};
      if constexpr (GC) {  // silu(o1): the packed constant IEV_OGATE (silu(r1) = 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) set_quad(gs, q, ld4(wvec + IEV_OGATE + 32 * b + 8 * q + 4 * h));
      }
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        if (GC && (t == 2 || t == 3)) continue;
        __builtin_amdgcn_sched_barrier(0);
        floatx16 y = {};
        const u16* wg = w + gate_off(t) * BLK;
        y = mfma32(afrag(wg, 2 * b, lane), gop.f[0], y);
        y = mfma32(afrag(wg, 2 * b + 1, lane), gop.f[1], y);
        if (t > 0) silu2_blk(y);
        gs += y;
      }
      acc.v[b] *= gs;
      asm volatile("" : "+v"(acc.v[b]));  // computed here (not sunk past the next stage barrier)
    }
  }
  // combined_linear_2(combined_linear_1(.)) : 128 -> 28 (padded 32) -> 128
  {
    const u16* w = wt(2 + NT);
    P32<8> aop;
    make_op32(aop, acc);
    X32<1> z;
    zero(z);
    mma32<1, 8>(z, aop, w, lane);
    P32<2> zop;
    make_op32(zop, z);
    zero(f);
    mma32<4, 2>(f, zop, w + 8 * BLK, lane);
  }
}

// acc = pos_src[node_pos[src]] + pos_dst[node_pos[dst]] (the orientation constant of GEO_REF batches
// arrives through the collapsed message map: geo_op32<true>)
__device__ __forceinline__ void init_acc_x32(X32<4>& acc, const InitArgs& a, int ps, int pd, int h) {
  const float* rs = a.pos_src + (int64_t)ps * HID;
  const float* rd = a.pos_dst + (int64_t)pd * HID;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 32 * b + 8 * q + 4 * h;
      set_quad(acc.v[b], q, ld4(rs + f) + ld4(rd + f));
    }
}

// the edge's geometric features [28] as a 32-feature operand; ONE: features 28 and 29 = 1 (the
// bf16 hi / lo columns of the orientation constant in the 32x32 init blob's message map), else 0
template <bool ONE = false>
__device__ __forceinline__ void geo_op32(P32<2>& gop, const float* edge_f, int e, int h) {
  const float* grow = edge_f + (int64_t)e * NFEAT_E;
  X32<1> geo;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = 8 * q + 4 * h;
    set_quad(geo.v[0], q, f < NFEAT_E ? ld4(grow + f) : (ONE ? (floatx4){1.f, 1.f, 0.f, 0.f} : (floatx4){0.f, 0.f, 0.f, 0.f}));
  }
  make_op32(gop, geo);
}

// staged weights (one 40-block slot per block, three blocks per CU, as k_init_edge); the first
// embed_blocks blocks run the node embedding (16x16 k_node_embed arithmetic, kind-0 blob)
// <= 160 VGPRs (amdgpu_num_vgpr counts register pairs): three waves per SIMD hold 480 of the 512
// registers, leaving exactly one 32-register pair-tensor wave room beside them. At 161 (168 allocated)
// the pair kernel's persistent blocks found no SIMD with room while InitEdge ran and the overlapped
// pair tensor slowed from ~1050 to ~1540 us per micro-batch (round 4)
template <bool GC>
__global__ __attribute__((amdgpu_flat_work_group_size(1, InitX32Geo::THREADS), amdgpu_waves_per_eu(3, 3),
                          amdgpu_num_vgpr(80)))
void k_init_x32(InitArgs a, EmbedArgs ea, int embed_blocks) {
  pq_signal_at_start(ea.sig_q, ea.sig_job);
  using G = InitGeo<BF16T>;
  constexpr int NW = InitX32Geo::NW;
  __shared__ __attribute__((aligned(16))) u16 lds[G::CAP * BLK];
  const int lane = lane_id();
  if ((int)blockIdx.x < embed_blocks) {  // uniform per block
    WPipe<u16, NW, false, G::CAP> epipe(lds);
    embed_block<BF16T, NW>(ea, epipe, blockIdx.x, lane, lane >> 4);
    return;
  }
  const int h = lane >> 5;
  const int r = ((int)blockIdx.x - embed_blocks) * InitX32Geo::ROWS + (threadIdx.x >> 6) * InitX32Geo::ROWS_PER_WAVE +
                (lane & 31);
  const bool valid = r < a.Et;
  const int e = valid ? r : a.Et - 1;
  const u16* W = reinterpret_cast<const u16*>(a.wmat);
  WPipe<u16, NW, false, G::CAP> pipe(lds);
  pipe.issue(W + IE_T0 * BLK, 8);
  P32<2> gop;
  geo_op32<GC>(gop, a.edge_f, e, h);
  X32<4> acc;
  init_acc_x32(acc, a, a.node_pos[a.src[e]], a.node_pos[a.dst[e]], h);
  const bool with_fn = a.fn_out != nullptr;  // uniform
  constexpr int NT = GC ? 2 : 4;
  auto geo_t = [](int i) { return GC ? (i == 0 ? 1 : 4) : i + 1; };
  // phase p's weights: wait for its stage, issue the next one
  auto wt = [&](int p) -> const u16* {
    const u16* w = pipe.next();
    if (p == 0) pipe.issue(W + (IE_T0 + 40 * geo_t(0)) * BLK, 40);
    else if (p < NT) pipe.issue(W + (IE_T0 + 40 * geo_t(p)) * BLK, 40);
    else if (p == NT) pipe.issue(W + IE_GEO1 * BLK, 40);
    else if (p == NT + 1) pipe.issue(W + IE_C1 * BLK, 16);
    else if (with_fn) pipe.issue(W + IE_NBR * BLK, MAT128);
    return w;
  };
  X32<4> f;
  init_tile_x32<GC>(acc, gop, a.wvec, lane, h, wt, [](int t) { return 8 * t; }, f);
  if (valid) store_row32(f, reinterpret_cast<u16*>(a.f_out) + (int64_t)e * HID, h);
  if (!with_fn) return;
  // layer-0 silu(nbr_linear(F)), applied once per edge and gathered by the conformation module
  const u16* w = pipe.next();
  P32<8> fop;
  make_op32(fop, f);
  X32<4> fn;
  init_vec32(fn, a.wvec + IEV_NBR, h);
  mma32<4, 8>(fn, fop, w, lane);
#pragma unroll
  for (int b = 0; b < 4; ++b) silu_blk(fn.v[b]);
  if (valid) store_row32(fn, reinterpret_cast<u16*>(a.fn_out) + (int64_t)e * HID, h);
}

// resident weights (DI_GRAPH_GEO_REF, no Fn): the path's 128 blocks loaded once per CU into LDS
// (block offsets IR_*), one 12-wave block per CU, waves striding over 32-edge tiles with the
// next tile's src/dst -> node_pos chain issued a tile ahead
constexpr int IRX_NW = 12;
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * IRX_NW), amdgpu_waves_per_eu(IRX_NW / 4, IRX_NW / 4)))
void k_init_res_x32(InitArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) u16 w[IR_NBLK * BLK];
  const u16* W = reinterpret_cast<const u16*>(a.wmat);
  dma_blocks<IRX_NW>(w + IR_T0 * BLK, W + IE_T0 * BLK, 8);
  dma_blocks<IRX_NW>(w + IR_DIST * BLK, W + (IE_T0 + 40 * 1) * BLK, 40);
  dma_blocks<IRX_NW>(w + IR_AMIDE * BLK, W + (IE_T0 + 40 * 4) * BLK, 40);
  dma_blocks<IRX_NW>(w + IR_GATE * BLK, W + IE_GEO1 * BLK, 16);               // em1, dist1
  dma_blocks<IRX_NW>(w + (IR_GATE + 16) * BLK, W + (IE_GEO1 + 32) * BLK, 8);  // amide1
  dma_blocks<IRX_NW>(w + IR_C * BLK, W + IE_C1 * BLK, 16);                    // combined_linear_1, _2
  lds_dma_wait();
  __syncthreads();
  const int lane = lane_id(), h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int stride = gridDim.x * IRX_NW;
  auto edge_of = [&](int t) {
    const int r = t * 32 + (lane & 31);
    return r < a.Et ? r : a.Et - 1;
  };
  int tile = blockIdx.x * IRX_NW + wave;
  int ps = 0, pd = 0;
  if (tile < ntiles) {
    const int e = edge_of(tile);
    ps = a.node_pos[a.src[e]];
    pd = a.node_pos[a.dst[e]];
  }
  auto wt = [&](int p) -> const u16* {
    return w + (p == 0 ? IR_T0 : p == 1 ? IR_DIST : p == 2 ? IR_AMIDE : p == 3 ? IR_GATE : IR_C) * BLK;
  };
  auto gate_off = [](int t) { return t == 0 ? 0 : (t == 1 ? 8 : 16); };  // em1, dist1, amide1
#pragma unroll 1
  for (; tile < ntiles; tile += stride) {
    const int r = tile * 32 + (lane & 31);
    const bool valid = r < a.Et;
    const int e = valid ? r : a.Et - 1;
    P32<2> gop;
    geo_op32<true>(gop, a.edge_f, e, h);
    X32<4> acc;
    init_acc_x32(acc, a, ps, pd, h);
    const bool more = tile + stride < ntiles;  // uniform
    if (more) {  // the next tile's positional-row indices
      const int en = edge_of(tile + stride);
      ps = a.node_pos[a.src[en]];
      pd = a.node_pos[a.dst[en]];
    }
    X32<4> f;
    init_tile_x32<true>(acc, gop, a.wvec, lane, h, wt, gate_off, f);
    if (valid) store_row32(f, reinterpret_cast<u16*>(a.f_out) + (int64_t)e * HID, h);
  }
}

// ================================================================ fused edge layer
// Weight stage order of the edge layer: block offsets / sizes (csrc/layout.h) and the fp32
// vector (bias) staged with each layer (-1: none).
__constant__ int EL_ORDER[25] = {
    EL_S0, EL_UP, EL_OM,
    EL_RES + 0 * MAT128, EL_RES + 1 * MAT128, EL_RES + 2 * MAT128,
    EL_RES + 3 * MAT128, EL_RES + 4 * MAT128, EL_RES + 5 * MAT128,
    EL_RC,
    EL_RES + 6 * MAT128, EL_RES + 7 * MAT128, EL_RES + 8 * MAT128,
    EL_RES + 9 * MAT128, EL_RES + 10 * MAT128, EL_RES + 11 * MAT128,
    EL_FG, EL_F, EL_P,
    EL_OE, EL_F1, EL_F2, EL_F1 + MAT128, EL_F2 + MAT128, EL_NN};
__constant__ int EL_SIZE[25] = {36, 16, 32, 32, 32, 32, 32, 32, 32, 32, 32, 32, 32,
                                32, 32, 32, 8, 32, 32, 32, 32, 32, 32, 32, 32};
__constant__ int EL_VEC[25] = {-1, ELV_OM, -1,
                               ELV_RES + 0 * 128, ELV_RES + 1 * 128, ELV_RES + 2 * 128,
                               ELV_RES + 3 * 128, ELV_RES + 4 * 128, ELV_RES + 5 * 128,
                               ELV_RC,
                               ELV_RES + 6 * 128, ELV_RES + 7 * 128, ELV_RES + 8 * 128,
                               ELV_RES + 9 * 128, ELV_RES + 10 * 128, ELV_RES + 11 * 128,
                               -1, ELV_F, ELV_P,
                               ELV_OE, ELV_F1, -1, ELV_F1 + 128, -1, ELV_NN};
constexpr int EL_NSTAGE_CONF = 18, EL_NSTAGE_FINAL = 19, EL_NSTAGE = 25;
constexpr int EL_CAP = 36;

// k_edge_layer: 16 rows per wave, 4-wave blocks, two blocks per CU: the fp32 edge layers (the
// reference's precision; the bf16 layers are k_edge_x32_ring below) and the conformation module
// alone (di_conformation, both dtypes).
template <class DT>
using EdgePipe = WPipe<typename DT::T, Geo<DT>::NW, Geo<DT>::DBUF, EL_CAP, 128>;

// MODE: 0 intermediate layer, 1 final layer, 2 conformation module alone (di_conformation)
template <int MODE>
constexpr int edge_nstage() { return MODE == 2 ? EL_NSTAGE_CONF : (MODE == 1 ? EL_NSTAGE_FINAL : EL_NSTAGE); }

// The weight-stage sequence of one tile: next() makes the next stage current (its weights w(),
// its bias vector v()) and issues the DMA of the one after it.
// GC (DI_GRAPH_GEO_REF batches, layer modes 0/1): the sequence starts at orig_msg_linear, which
// then carries the orig_msg_linear bias, and (intermediate layers) ends before nbr_linear
template <class DT, int MODE, bool GC = false>
struct EdgeStages {
  using T = typename DT::T;
  static constexpr int NS = edge_nstage<MODE>() - (GC ? (MODE == 1 ? 2 : 3) : 0);
  EdgePipe<DT>& pipe;
  const T* W;
  const float* V;
  int gi;  // index of the next stage to make current
  __device__ void issue(int s0) {
    const int s = GC ? s0 + 2 : s0;
    const int vo = (GC && s0 == 0) ? ELV_OM : EL_VEC[s];
    pipe.issue(W + EL_ORDER[s] * BLK, EL_SIZE[s], vo >= 0 ? V + vo : nullptr, 128);
  }
  __device__ void begin() { issue(0); }
  __device__ const T* next() {
    const int i = gi++;
    const T* w = pipe.next();
    if (i + 1 < NS) issue(i + 1);
    return w;
  }
  __device__ const float* v() const { return pipe.v(); }
};

template <class DT, int MODE, bool GC>
__device__ __forceinline__ void res_block(Act<8>& x, EdgeStages<DT, MODE, GC>& st, int lane, int g) {
  constexpr bool FAST = DT::kBF16;
  Act<8> y = x;
#pragma unroll 1
  for (int l = 0; l < 3; ++l) {
    const typename DT::T* w = st.next();
    Act<8> t;
    init_vec_lds(t, st.v(), g);
    linear<DT, 8, 4>(t, y, w, lane);
    silu2_<8, FAST>(t);  // log2 units: folded into the next linear / the residual fma
    y = t;
  }
  add_scaled_(x, y, silu2_unit<FAST>());
}

// Two 4-wave blocks per CU, each wave capped at 240 VGPRs (amdgpu_num_vgpr counts the unified
// VGPR+AGPR file in pairs on gfx950): 2 x 240 + 32 = 512 leaves one pair-tensor wave per SIMD
// co-resident. One 64-row tile per block.
// GC (DI_GRAPH_GEO_REF, modes 0/1): the neighbour-message stages are skipped (exactly zero) and no
// silu(nbr_linear(F)) rows are gathered or written.
template <class DT, int MODE, bool GC = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, Geo<DT>::THREADS), amdgpu_waves_per_eu(2, 2),
                          amdgpu_num_vgpr(120)))
void k_edge_layer(EdgeArgs a) {
  constexpr bool FINAL = MODE == 1, CONF = MODE == 2;
  using T = typename DT::T;
  using G = Geo<DT>;
  constexpr bool FAST = DT::kBF16;
  __shared__ __attribute__((aligned(16))) char lds[(G::DBUF ? 2 : 1) * EdgePipe<DT>::SLOT_BYTES];
  const int lane = lane_id(), g = lane >> 4;
  const int r = row_id<G::NW>();
  const bool valid = r < a.Et;
  const int e = valid ? r : a.Et - 1;
  const T* W = reinterpret_cast<const T*>(a.wmat);
  const T* fn_in = reinterpret_cast<const T*>(a.fn_in);
  const T* qkv = reinterpret_cast<const T*>(a.qkv);
  const T* f_row = reinterpret_cast<const T*>(a.f_in) + (int64_t)e * HID;

  EdgePipe<DT> pipe(lds);
  EdgeStages<DT, MODE, GC> st{pipe, W, a.wvec, 0};
  st.begin();
  int4 nb = {0, 0, 0, 0};
  if constexpr (!GC) nb = *reinterpret_cast<const int4*>(a.nbr + (int64_t)e * 4);
  Op<DT, 1> gop;
  {
    Act<2> geo;
    load_edge_geo(geo, a.edge_f + (int64_t)e * NFEAT_E, g);
    make_op(gop, geo);
  }
  FRow<DT> fr;
  if constexpr (DT::kBF16) {
    RawRow<T> fraw;
    fraw.load(f_row, g);
    fr.set_raw(fraw);
  }

  const T* w;
  Act<8> x;
  if constexpr (GC) {
    // DI_GRAPH_GEO_REF: the neighbour messages are multiplied by dir_linear_1(dir_linear_0(0)) = 0
    // (:408): x = orig_msg_linear(F) + b exactly
    w = st.next();  // orig_msg_linear (+ its bias)
    init_vec_lds(x, st.v(), g);
  } else {
    // ---- neighbour-edge messages (conformation_module_message_func :384-418)
    RawRow<T> xn;
    xn.load(fn_in + (int64_t)nb.x * HID, g);
    w = st.next();  // stage 0: geometric gates + downward_proj
    Act<4> gate;    // dir . orient . amide embeddings (64)
    {
      Act<4> t1;
      zero(gate);
      mma<4, 1>(gate, gop, w + 8 * BLK, lane);
      zero(t1);
      mma<4, 1>(t1, gop, w + 12 * BLK, lane);
      mul_(gate, t1);
      zero(t1);
      mma<4, 1>(t1, gop, w + 16 * BLK, lane);
      mul_(gate, t1);
    }
    Act<4> s;
    zero(s);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      Act<8> xa;
      xn.to_act(xa);
      if (j < 3) {  // prefetch the next neighbour row under this one's MFMAs
        const int nx = j == 0 ? nb.y : (j == 1 ? nb.z : nb.w);
        xn.load(fn_in + (int64_t)nx * HID, g);
      }
      // dist_linear_1(dist_linear_0(dist)), recomputed per neighbour (8 MFMAs) rather than held
      // live across the loop: the memory clobber stops the compiler from hoisting it (32 VGPRs)
      asm volatile("" ::: "memory");
      Act<8> dg;
      zero(dg);
      mma<8, 1>(dg, gop, w, lane);
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) xa.v[b][q] *= dg.v[b][q];  // gathered rows are silu(nbr_linear(F))
      Act<4> y;
      zero(y);
      linear<DT, 4, 4>(y, xa, w + 20 * BLK, lane);  // downward_proj
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) s.v[b][q] += silu2<FAST>(y.v[b][q]) * gate.v[b][q];
    }
    w = st.next();  // stage 1: upward_proj (+ orig_msg_linear bias)
    zero(x);
    linear<DT, 8, 2>(x, s, w, lane);
    silu2_<8, FAST>(x);
    {
      Act<8> bo;
      init_vec_lds(bo, st.v(), g);
#pragma unroll
      for (int b = 0; b < 8; ++b) x.v[b] = silu2_unit<FAST>() * x.v[b] + bo.v[b];
    }
    w = st.next();  // stage 2: orig_msg_linear(res) + nbr
  }
  mma<8, 4>(x, fr.operand(f_row, g), w, lane);
  res_block<DT, MODE, GC>(x, st, lane, g);
  res_block<DT, MODE, GC>(x, st, lane, g);
  {
    w = st.next();  // res_connect_linear
    Act<8> y;
    init_vec_lds(y, st.v(), g);
    linear<DT, 8, 4>(y, x, w, lane);
    silu2_<8, FAST>(y);
    fr.act(x, f_row, g);
    add_scaled_(x, y, silu2_unit<FAST>());
  }
  res_block<DT, MODE, GC>(x, st, lane, g);
  res_block<DT, MODE, GC>(x, st, lane, g);
  {
    w = st.next();  // final geometric gate
    Act<8> fg;
    zero(fg);
    mma<8, 1>(fg, gop, w, lane);
    mul_(x, fg);
    w = st.next();  // final_linear
    Act<8> y;
    init_vec_lds(y, st.v(), g);
    linear<DT, 8, 4>(y, x, w, lane);
    silu2_<8, FAST>(y);
    fr.act(x, f_row, g);
    add_scaled_(x, y, silu2_unit<FAST>());  // conformation output
  }
  if constexpr (CONF) {
    if (valid) store_row(x, reinterpret_cast<T*>(a.f_out) + (int64_t)e * HID, g);
    return;
  } else {
    // ---- attention scores (propagate_attention :76-91)
    const int sn = a.src[e], dn = a.dst[e];
    RawRow<T> kr, qr;  // K[src], Q[dst] in flight under the projection's MFMAs
    kr.load(qkv + (int64_t)sn * 3 * HID + HID, g);
    qr.load(qkv + (int64_t)dn * 3 * HID, g);
    w = st.next();  // edge_feats_projection(BN1e(conf))
    Act<8> p;
    init_vec_lds(p, st.v(), g);
    linear<DT, 8, 4>(p, x, w, lane);
    {
      Act<8> kq, qd;
      kr.to_act(kq);
      qr.to_act(qd);
      const float scale = 5.656854249492381f;  // np.sqrt(32)
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float sc = FAST ? (kq.v[b][q] * qd.v[b][q]) * (1.0f / scale) : (kq.v[b][q] * qd.v[b][q]) / scale;
          sc = fminf(fmaxf(sc, -5.f), 5.f);
          p.v[b][q] = sc * p.v[b][q];  // score = e_out
        }
    }
    floatx4 al;
#pragma unroll
    for (int h = 0; h < 4; ++h) al[h] = expf_<FAST>(fminf(fmaxf(head_sum(p, h), -5.f), 5.f));
    if (valid && g == 0) st4(a.alpha_out + (int64_t)e * 4, al);

    if constexpr (!FINAL) {
      // ---- edge output: e = in + O_e(e_out); e = e + FFN(BN2e(e)) (:697-724)
      w = st.next();  // O_edge_feats
      Act<8> e1;
      init_vec_lds(e1, st.v(), g);
      linear<DT, 8, 4>(e1, p, w, lane);
      {
        Act<8> fa;
        fr.act(fa, f_row, g);
        add_(e1, fa);
      }
      Act<8> o;
      zero(o);
#pragma unroll 1
      for (int half = 0; half < 2; ++half) {
        w = st.next();  // edge_feats_MLP.0 (BN2e folded), hidden half
        Act<8> t;
        init_vec_lds(t, st.v(), g);
        linear<DT, 8, 4>(t, e1, w, lane);
        silu2_<8, FAST>(t);
        w = st.next();  // edge_feats_MLP.3, input half
        linear<DT, 8, 4>(o, t, w, lane);
      }
      add_(e1, o);
      if (valid) store_edge_row(e1, reinterpret_cast<T*>(a.f_out) + (int64_t)e * HID, g);
      if constexpr (GC) return;  // no silu(nbr_linear(F)) rows for the next layer
      w = st.next();  // next layer's silu(nbr_linear(.))
      Act<8> fn;
      init_vec_lds(fn, st.v(), g);
      linear<DT, 8, 4>(fn, e1, w, lane);
      silu_<8, FAST>(fn);
      if (valid) store_edge_row(fn, reinterpret_cast<T*>(a.fn_out) + (int64_t)e * HID, g);
    }
  }
}

// ================================================================ fused edge layer on 32x32x16 MFMA (bf16)
// The stage sequence and arithmetic of k_edge_layer<BF16T, MODE, GC>, with each wave's 32 rows as ONE
// 32x32 tile (csrc/mfma32.h): a 128x128 linear is 32 v_mfma_f32_32x32x16_bf16 per wave. Weight stages
// weight stages on an 8-wave LDS ring (k_edge_x32_ring below); the weight blobs are packed in the 32x32
// fragment order (packing.pack_matrix32, di_blob_layout() == 32).

// x through one ResBlock: two silu2(W . + b) layers packed as the next operand, then x += ln2 * silu2(W . + b)
template <class ST>
__device__ __forceinline__ void x32_res_block(X32<4>& x, ST& st, int lane, int h) {
  P32<8> op;
  make_op32(op, x);
#pragma unroll 1
  for (int l = 0; l < 2; ++l) {
    const u16* w = st.next();
    X32<4> t;
    P32<8> opn;
    lin32_pipe<8>(t, op, w, st.v(), lane, h, [&](int b) {
      silu2_blk(t.v[b]);
      pack_blk(opn.f[2 * b], opn.f[2 * b + 1], t.v[b]);
    });
    op = opn;
    pin(op);
  }
  const u16* w = st.next();
  X32<4> t;
  lin32_pipe<8>(t, op, w, st.v(), lane, h, [&](int b) {
    silu2_blk(t.v[b]);
    x.v[b] += silu2_unit<true>() * t.v[b];
  });
  pin(x);
}

// x = F + ln2 * silu2(W x + b)  (res_connect_linear / final_linear residual; F the edge's bf16 row)
__device__ __forceinline__ void x32_f_residual(X32<4>& x, const u16* w, const float* v, const R32<4>& fr, int lane,
                                               int h) {
  P32<8> op;
  make_op32(op, x);
  X32<4> y;
  lin32_pipe<8>(y, op, w, v, lane, h, [&](int b) {
    silu2_blk(y.v[b]);
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(x.v[b], q, unpack4(fr.u[4 * b + q]) + silu2_unit<true>() * quad(y.v[b], q));
  });
  pin(x);
}

// ---- the node layer's attention aggregation folded into the edge layer (di_edge_layer_attn)
// h_attn[v] = sum_{e in in(v)} alpha[e, head] * V[src e] / (sum_e alpha[e, head] + 1e-6)
// (send_and_recv(u_mul_e('V_h','score'), sum), (copy_e('score'), sum), wV / (z + 1e-6):
// deepinteract_modules.py:93-96, 116). Edges are destination-major, so a destination's in-edges are
// consecutive rows: a wave's 32 rows hold whole destinations plus at most one continuing from the
// previous 32-row tile and one continuing into the next. Each lane forms alpha * V[src] for its row
// (the 64 features of its lane half, in the accumulator quads) and alpha itself; a segmented
// inclusive scan over the 32 rows -- DPP row shifts by 1, 2, 4, 8 inside each 16-lane row, then the
// first row's last lane broadcast into the second -- leaves every destination's sums in the lane of
// its last row here. That lane writes attn[v] = wV / (z + 1e-6) when all of v's in-edges are in this
// tile, else the partial sums to attn_parts[tile][slot] (slot 1: v continues into the next tile;
// slot 0: v continues from the previous one); attn_row (the node update) adds a split
// destination's partials. Summation order: a tree over each tile's rows, then tile by tile.
constexpr int FOLD_ROWS = 32;   // edges per tile of attn_parts (one wave's rows)
constexpr int FOLD_PART = 132;  // floats per partial: 128 wV, then z of the 4 heads

// one scan step: lanes whose DPP source row has the same destination add its sums
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void fold_step(X32<4>& s, floatx4& z, int d) {
  const bool same = __builtin_amdgcn_update_dpp(-2, d, CTRL, ROW_MASK, 0xf, false) == d;
  auto mv = [](float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROW_MASK, 0xf,
                                                                  false));
  };
#pragma unroll
  for (int b = 0; b < 4; ++b) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float t = mv(s.v[b][k]);
      s.v[b][k] += same ? t : 0.f;
    }
    const float t = mv(z[b]);
    z[b] += same ? t : 0.f;
  }
}

// d: the row's destination, vr: its V[src] row, ip: in_ptr[d], in_ptr[d + 1] (loaded with K / Q)
__device__ __forceinline__ void edge_attn_fold(const EdgeArgs& a, int e, bool valid, int lane, int h, floatx4 al,
                                               int d, const R32<4>& vr, int2 ip) {
  if (!valid) {  // rows past the end: their own (empty) segment
    d = -1;
    al = (floatx4){0.f, 0.f, 0.f, 0.f};
  }
  X32<4> s;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(s.v[b], q, al[b] * unpack4(vr.u[4 * b + q]));
  floatx4 z = al;
  fold_step<0x111, 0xf>(s, z, d);  // row_shr:1
  fold_step<0x112, 0xf>(s, z, d);  // row_shr:2
  fold_step<0x114, 0xf>(s, z, d);  // row_shr:4
  fold_step<0x118, 0xf>(s, z, d);  // row_shr:8
  fold_step<0x142, 0xa>(s, z, d);  // row_bcast:15 into rows 1 and 3 (each lane half's second 16 rows)
  const int dnext = __shfl_down(d, 1, 32);
  if (!valid || ((lane & 31) != 31 && dnext == d)) return;
  const int t = e / FOLD_ROWS, t0 = ip.x / FOLD_ROWS, t1 = (ip.y - 1) / FOLD_ROWS;
  if (t0 == t1) {
    float* row = a.attn_out + (int64_t)d * HID;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const float den = z[b] + 1e-6f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 x = quad(s.v[b], q);
        st4(row + 32 * b + 8 * q + 4 * h, (floatx4){x[0] / den, x[1] / den, x[2] / den, x[3] / den});
      }
    }
  } else {
    float* p = a.attn_parts + ((int64_t)t * 2 + (t == t0 ? 1 : 0)) * FOLD_PART;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) st4(p + 32 * b + 8 * q + 4 * h, quad(s.v[b], q));
    if (h == 0) st4(p + HID, z);
  }
}

// One 32-row tile per wave through the whole edge layer: the stage sequence `st` (the 8-wave ring's
// RingStages) hands out each weight stage in order (next(): its weights, v(): its bias).
template <int MODE, bool GC, class ST>
__device__ __forceinline__ void edge_x32_tile(const EdgeArgs& a, ST& st, int e, bool valid, int lane, int h) {
  constexpr bool FINAL = MODE == 1;
  const u16* f_row = reinterpret_cast<const u16*>(a.f_in) + (int64_t)e * HID;
  const u16* qkv = reinterpret_cast<const u16*>(a.qkv);

  // the edge's geometric features [28] (fp32 row) as a 32-feature operand, features 28..31 = 0
  P32<2> gop;
  {
    const float* grow = a.edge_f + (int64_t)e * NFEAT_E;
    X32<1> geo;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 8 * q + 4 * h;
      set_quad(geo.v[0], q, f < NFEAT_E ? ld4(grow + f) : (floatx4){0.f, 0.f, 0.f, 0.f});
    }
    make_op32(gop, geo);
  }
  X32<4> x;
  R32<4> fr;  // the edge's own row F, re-read (L2) before each use: the stages have no room to hold it
  const u16* w;
  if constexpr (GC) {
    // DI_GRAPH_GEO_REF: the neighbour messages are multiplied by dir_linear_1(dir_linear_0(0)) = 0
    // (:408), so x = orig_msg_linear(F) + b exactly; no gathered rows, no stages 0-1
    fr.load(f_row, h);
    w = st.next([&] { settle(fr); });  // orig_msg_linear (+ its bias)
    init_vec32_lds(x, st.v(), h);
  } else {
    // ---- neighbour-edge messages (conformation_module_message_func :384-418)
    const u16* fn_in = reinterpret_cast<const u16*>(a.fn_in);
    const int4 nb = *reinterpret_cast<const int4*>(a.nbr + (int64_t)e * 4);
    R32<4> xn;  // the gathered silu(nbr_linear(F)) row in flight
    xn.load(fn_in + (int64_t)nb.x * HID, h);
    w = st.next();  // stage 0: geometric gates (dist [4x2] blocks 0-7, dir / orient / amide [2x2] at 8 / 12 / 16)
                    // + downward_proj [2x8] at 20
    X32<2> gate;
    {
      X32<2> t1;
      zero(gate);
      mma32<2, 2>(gate, gop, w + 8 * BLK, lane);
      zero(t1);
      mma32<2, 2>(t1, gop, w + 12 * BLK, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) gate.v[b] *= t1.v[b];
      zero(t1);
      mma32<2, 2>(t1, gop, w + 16 * BLK, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) gate.v[b] *= t1.v[b];
      pin(gate);
    }
    X32<2> s;
    zero(s);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // x = silu(nbr_linear(F))[nbr_j] * dist gate, packed block by block (the dist gate recomputed
      // per neighbour: 2 MFMAs per block instead of 64 live registers)
      P32<8> xop;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        asm volatile("" ::: "memory");
        floatx16 dg = {};
        dg = mfma32(afrag(w, 2 * b, lane), gop.f[0], dg);
        dg = mfma32(afrag(w, 2 * b + 1, lane), gop.f[1], dg);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          asm volatile("" : "+v"(xn.u[4 * b + 2 * t]), "+v"(xn.u[4 * b + 2 * t + 1]));
          const floatx4 lo = unpack4(xn.u[4 * b + 2 * t]) * quad(dg, 2 * t);
          const floatx4 hi = unpack4(xn.u[4 * b + 2 * t + 1]) * quad(dg, 2 * t + 1);
          const uint4 u = {pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]), pack_bf16x2(hi[0], hi[1]),
                           pack_bf16x2(hi[2], hi[3])};
          xop.f[2 * b + t] = __builtin_bit_cast(bf16x8, u);
        }
      }
      if (j < 3) {  // the next gathered row, in flight under this one's downward_proj
        const int nx = j == 0 ? nb.y : (j == 1 ? nb.z : nb.w);
        xn.load(fn_in + (int64_t)nx * HID, h);
      }
      X32<2> y;
      zero(y);
      mma32<2, 8>(y, xop, w + 20 * BLK, lane);  // downward_proj
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int k = 0; k < 16; ++k) s.v[b][k] += silu2<true>(y.v[b][k]) * gate.v[b][k];
      pin(s);
    }
    w = st.next();  // stage 1: upward_proj [4x4] (+ orig_msg_linear bias)
    {
      P32<4> sop;
      make_op32(sop, s);
      zero(x);
      mma32<4, 4>(x, sop, w, lane);
      X32<4> bo;
      init_vec32_lds(bo, st.v(), h);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        silu2_blk(x.v[b]);
        x.v[b] = silu2_unit<true>() * x.v[b] + bo.v[b];
      }
      pin(x);
    }
    fr.load(f_row, h);
    w = st.next([&] { settle(fr); });  // stage 2: orig_msg_linear(res) + nbr
  }
  {
    P32<8> fop;
    raw_op32(fop, fr);
    mma32<4, 8>(x, fop, w, lane);
    pin(x);
  }
  x32_res_block(x, st, lane, h);
  x32_res_block(x, st, lane, h);
  // F rows are loaded BEFORE the stage's barrier and DMA issue: vmcnt retires in order, so a load
  // issued after the stage's LDS-DMA pieces would make its use wait for the whole weight stage
  fr.load(f_row, h);
  w = st.next([&] { settle(fr); });  // res_connect_linear: x = F + silu(rc(x))
  x32_f_residual(x, w, st.v(), fr, lane, h);
  x32_res_block(x, st, lane, h);
  x32_res_block(x, st, lane, h);
  w = st.next();  // final geometric gate [4x2]
  {
    X32<4> fg;
    zero(fg);
    mma32<4, 2>(fg, gop, w, lane);
#pragma unroll
    for (int b = 0; b < 4; ++b) x.v[b] *= fg.v[b];
    pin(x);
  }
  fr.load(f_row, h);
  w = st.next([&] { settle(fr); });  // final_linear: x = F + silu(final(x)) = conformation output
  x32_f_residual(x, w, st.v(), fr, lane, h);

  // ---- attention scores (propagate_attention :76-91): head hd = features 32 hd .. 32 hd + 31 = block hd
  R32<4> kr, qr;  // K[src], Q[dst], issued before the stage barrier
  const int sn = a.src[e], dn = a.dst[e];
  kr.load(qkv + (int64_t)sn * 3 * HID + HID, h);
  qr.load(qkv + (int64_t)dn * 3 * HID, h);
  // the fold's V[src] row and the destination's in-edge range, in flight with K / Q (GEO_REF kernels;
  // the general path's extra live rows leave no room: loaded at the fold)
  const bool fold = a.attn_out != nullptr;  // uniform
  R32<4> vr;
  int2 ip = {0, 0};
  auto fold_loads = [&] {
    vr.load(qkv + (int64_t)sn * 3 * HID + 2 * HID, h);
    ip = *reinterpret_cast<const int2*>(a.in_ptr + dn);
  };
  if (GC && fold) fold_loads();
  w = st.next([&] {
    settle(kr);
    settle(qr);
    if (GC && fold) {
      settle(vr);
      asm volatile("" ::"v"(ip.x), "v"(ip.y));
    }
  });  // edge_feats_projection(BN1e(conf))
  X32<4> p;
  {
    P32<8> xop;
    make_op32(xop, x);
    init_vec32_lds(p, st.v(), h);
    mma32<4, 8>(p, xop, w, lane);
  }
  floatx4 al;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 kq = unpack4(kr.u[4 * b + q]), qd = unpack4(qr.u[4 * b + q]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sc = (kq[i] * qd[i]) * (1.0f / 5.656854249492381f);  // / np.sqrt(32)
        sc = fminf(fmaxf(sc, -5.f), 5.f);
        const float pv = sc * p.v[b][4 * q + i];  // score = e_out
        p.v[b][4 * q + i] = pv;
        sum += pv;
      }
    }
    sum += __shfl_xor(sum, 32);  // the head's other 16 features: the same row in the other lane half
    al[b] = expf_<true>(fminf(fmaxf(sum, -5.f), 5.f));
  }
  if (valid && h == 0 && a.alpha_out != nullptr) st4(a.alpha_out + (int64_t)e * 4, al);
  if (!GC && fold) fold_loads();
  if constexpr (FINAL) {
    if (fold) edge_attn_fold(a, e, valid, lane, h, al, dn, vr, ip);
  } else {
    // ---- edge output: e = in + O_e(e_out); e = e + FFN(BN2e(e)) (:697-724)
    P32<8> pop;
    make_op32(pop, p);
    pin(pop);
    if (fold) edge_attn_fold(a, e, valid, lane, h, al, dn, vr, ip);  // p is packed: room for the scan
    fr.load(f_row, h);                 // O_edge: re-read
    w = st.next([&] { settle(fr); });  // O_edge_feats
    X32<4> e1;
    init_vec32_lds(e1, st.v(), h);
    mma32<4, 8>(e1, pop, w, lane);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) set_quad(e1.v[b], q, quad(e1.v[b], q) + unpack4(fr.u[4 * b + q]));
    pin(e1);
    P32<8> eop;
    make_op32(eop, e1);
    pin(eop);
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      w = st.next();  // edge_feats_MLP.0 (BN2e folded), hidden half
      X32<4> t;
      P32<8> top;
      lin32_pipe<8>(t, eop, w, st.v(), lane, h, [&](int b) {
        silu2_blk(t.v[b]);
        pack_blk(top.f[2 * b], top.f[2 * b + 1], t.v[b]);
      });
      pin(top);
      w = st.next();  // edge_feats_MLP.3, input half: accumulated into the residual
      mma32<4, 8>(e1, top, w, lane);
      pin(e1);
    }
    if (valid) store_row32(e1, reinterpret_cast<u16*>(a.f_out) + (int64_t)e * HID, h);
    if constexpr (GC) return;  // the next layer gathers no silu(nbr_linear(F)) rows
    make_op32(eop, e1);
    w = st.next();  // next layer's silu(nbr_linear(.))
    X32<4> fn;
    init_vec32_lds(fn, st.v(), h);
    mma32<4, 8>(fn, eop, w, lane);
#pragma unroll
    for (int b = 0; b < 4; ++b) silu_blk(fn.v[b]);
    if (valid) store_row32(fn, reinterpret_cast<u16*>(a.fn_out) + (int64_t)e * HID, h);
  }
}

// ================================================================ the bf16 edge layers on an 8-wave weight ring
// One persistent 8-wave block per CU (2 waves per SIMD, <= 240 VGPRs), a 4-slot ring of
// 36-block weight stages in LDS (150 KB): every stage is DMA'd ONCE per 256 edges (8 waves x 32 rows)
// instead of once per 128 -- half the L2 -> LDS weight stream of round 4's two 4-wave blocks per CU,
// the traffic that competes with the pair-tensor stores beside it -- and there is no
// block-wide barrier per stage. Per slot two LDS counters, both monotonic: FULL counts publications of
// the slot's stages (the owner waits its vmcnt, then adds), FREE the waves done reading it. A wave entering global stage g (stages run on across the block's tiles, so the
// next tile's first stages are in flight under the current tile's last ones):
//   releases stage g - 1 (FREE += 1); if it owns a stage it issued earlier (stage s is loaded by wave
//   s % 8), waits for its own loads (vmcnt(0)) and publishes it (FULL += 1); if it owns stage g + 2,
//   issues it into the slot of stage g - 2 once all 8 waves have released that one; then waits until
//   stage g is published. No block-wide barrier: a wave waits only for the owner of the stage it needs
//   and, once in 8 stages, for the slowest wave two stages back.
constexpr int RING_NW = 8, RING_SLOTS = 4, RING_AHEAD = 2;
using RingSlot = WPipe<u16, RING_NW, true, EL_CAP, 128>;  // slot geometry only (SLOT_BYTES)
struct EdgeRingGeo {
  static constexpr int NW = RING_NW, THREADS = 64 * NW, ROWS_PER_WAVE = 32, ROWS = ROWS_PER_WAVE * NW;
};
static_assert(EdgeRingGeo::ROWS_PER_WAVE == FOLD_ROWS, "a fold tile is one wave's rows");

// The ring's LDS counters are read and added with explicit ds_ instructions: through C++ atomics the
// compiler cannot tell them from the weight slots the in-flight LDS-DMA writes and puts an
// s_waitcnt vmcnt(0) in front of every poll, which would drain the prefetch at every stage.
__device__ __forceinline__ uint32_t lds_off(const uint32_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_off(p)) : "memory");
  return v;
}
// +1 per WAVE (one lane; LDS operations of a wave execute in order, so the add follows the wave's
// earlier reads of the slot)
__device__ __forceinline__ void lds_add(uint32_t* p) {
  asm volatile(
      "s_mov_b64 s[0:1], exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %0, %1\n\t"
      "s_mov_b64 exec, s[0:1]" ::"v"(lds_off(p)), "v"(1u)
      : "memory", "s0", "s1");
}
// spin until *p >= v (s_sleep between LDS polls)
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t v) {
  while (lds_ld(p) < v) __builtin_amdgcn_s_sleep(1);
}

// raw buffer descriptor (as buf_rsrc: stride 0, num_records 0x7fffffff, DATA_FORMAT 32) in SGPRs
typedef uint32_t rsrc4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ rsrc4 rsrc_of(const void* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return (rsrc4){(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a),
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) & 0xffffu, 0x7fffffffu,
                 (uint32_t)BUF_RSRC_W3};
}
// one 1-KiB LDS-DMA piece: 16 B per lane from rsrc + voff + soff to LDS byte address lds + 16 * lane
__device__ __forceinline__ void dma_piece(rsrc4 r, uint32_t lds, int voff, int soff) {
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(__builtin_amdgcn_readfirstlane((int)lds)),
      "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(soff))
      : "memory", "m0");
}

// What one ring stage loads: up to three runs of packed 512-element blocks (laid out back to back in
// the slot) and an optional bias vector (128 floats, after the slot's blocks).
struct RingPieces {
  const u16* w;  // blob base
  int off[3], n[3];
  int np;
  const float* v;  // bias vector or null
};
// the bf16 edge layer's stages (EL_ORDER / EL_SIZE / EL_VEC): one run each
template <int NS, bool GC>
struct EdgeRingSrc {
  const u16* W;
  const float* V;
  __device__ RingPieces operator()(int gs) const {
    const int s = gs % NS;
    const int si = GC ? s + 2 : s;
    const int vo = (GC && s == 0) ? ELV_OM : EL_VEC[si];
    return {W, {EL_ORDER[si], 0, 0}, {EL_SIZE[si], 0, 0}, 1, vo >= 0 ? V + vo : nullptr};
  }
};

template <class SRC, int NW = RING_NW>
struct RingStagesT {
  char* base;          // RING_SLOTS x RingSlot::SLOT_BYTES
  uint32_t* full;      // [RING_SLOTS]: stage uses published (1 per use)
  uint32_t* freec;     // [RING_SLOTS]: wave releases (NW per use)
  SRC src;             // global stage -> its weight runs and bias
  int wave;
  int total;           // global stages of this block
  int g = 0;           // next stage to consume
  int issued = 0;      // stages [0, issued) are issued (by their owners)
  int pending = -1;    // a stage this wave issued and has not published yet
  int cur = 0;         // slot of the stage being consumed
  __device__ u16* slot_w(int sl) const { return reinterpret_cast<u16*>(base + sl * RingSlot::SLOT_BYTES); }
  __device__ float* slot_v(int sl) const {
    return reinterpret_cast<float*>(base + sl * RingSlot::SLOT_BYTES + EL_CAP * BLK * 2);
  }
  // global stage gs is loaded and published by ONE wave, gs % NW (its owner): all its 1-KiB
  // LDS-DMA pieces and the bias vector. Issued by inline asm: the compiler's waitcnt pass cannot tell a
  // ring slot (runtime index) from the one being read and would wait for every piece before the next
  // ds_read -- completion is what FULL tracks (the owner's vmcnt(0), then its publish).
  __device__ void issue_one(int gs) {
    const RingPieces p = src(gs);
    const int sl = gs % RING_SLOTS;
    uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)slot_w(sl);
    const int loff = (threadIdx.x & 63) * 16;
    for (int k = 0; k < p.np; ++k) {
      const rsrc4 r = rsrc_of(p.w + p.off[k] * BLK);
      for (int i = 0; i < p.n[k]; ++i) dma_piece(r, dst + i * 1024, loff, i * 1024);  // 1 KiB per block
      dst += p.n[k] * 1024;
    }
    if (p.v && (threadIdx.x & 63) < 32)
      dma_piece(rsrc_of(p.v), (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)slot_v(sl), loff, 0);
    pending = gs;
  }
  // stages issued ahead of the one consumed, owners' slots permitting
  __device__ void issue_ahead() {
    for (; issued <= g + RING_AHEAD && issued < total; ++issued) {
      if (issued % NW != wave) continue;
      const int prev = issued - RING_SLOTS;  // the stage that used this slot last
      if (prev >= 0) lds_wait_ge(freec + issued % RING_SLOTS, (uint32_t)(NW * (prev / RING_SLOTS + 1)));
      issue_one(issued);
    }
  }
  __device__ void fill() {
    for (; issued < RING_AHEAD && issued < total; ++issued)
      if (issued % NW == wave) issue_one(issued);
  }
  // settle(): an empty asm reading the rows the caller loaded just before this call (F rows, K / Q):
  // the compiler then waits for them HERE, after the vmcnt(0) that has landed them anyway -- not after
  // the asm-issued DMA below, which it cannot see and would otherwise wait for at their first use
  template <class F>
  __device__ const u16* next(F&& settle) {
    asm volatile("" ::: "memory");
    if (g > 0) lds_add(freec + (g - 1) % RING_SLOTS);  // done reading stage g - 1 (its reads are in order before)
    lds_dma_wait();  // this wave's loads (rows, and the pieces of a stage it owns) have landed
    settle();
    if (pending >= 0) {
      lds_add(full + pending % RING_SLOTS);
      pending = -1;
    }
    issue_ahead();
    lds_wait_ge(full + g % RING_SLOTS, (uint32_t)(g / RING_SLOTS + 1));
    asm volatile("" ::: "memory");
    cur = g % RING_SLOTS;
    ++g;
    return slot_w(cur);
  }
  __device__ const u16* next() {
    return next([] {});
  }
  __device__ const float* v() const { return slot_v(cur); }
};
template <int NS, bool GC>
using RingStages = RingStagesT<EdgeRingSrc<NS, GC>>;

template <int MODE, bool GC>
__global__ __attribute__((amdgpu_flat_work_group_size(1, EdgeRingGeo::THREADS), amdgpu_waves_per_eu(2, 2),
                          amdgpu_num_vgpr(120)))
void k_edge_x32_ring(EdgeArgs a, int ntiles) {
  constexpr bool FINAL = MODE == 1;
  constexpr int NS = (FINAL ? EL_NSTAGE_FINAL : EL_NSTAGE) - (GC ? (FINAL ? 2 : 3) : 0);
  __shared__ __attribute__((aligned(16))) char lds[RING_SLOTS * RingSlot::SLOT_BYTES];
  __shared__ uint32_t counters[2 * RING_SLOTS];
  const int lane = lane_id(), h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int my_tiles = ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (threadIdx.x < 2 * RING_SLOTS) counters[threadIdx.x] = 0;
  __syncthreads();
  RingStages<NS, GC> st{lds, counters, counters + RING_SLOTS, {reinterpret_cast<const u16*>(a.wmat), a.wvec}, wave,
                        my_tiles * NS};
  st.fill();
#pragma unroll 1
  for (int i = 0; i < my_tiles; ++i) {
    // slot j = b + i G: with G a multiple of 8, slot j runs on block b's XCD (j mod 8), and
    // xcd_slot gives each XCD one contiguous eighth of the edges (every block keeps its tile count)
    const int j = (int)blockIdx.x + i * (int)gridDim.x;
    const int tile = (gridDim.x & 7) == 0 ? xcd_slot(j, ntiles) : j;
    const int r = tile * EdgeRingGeo::ROWS + wave * EdgeRingGeo::ROWS_PER_WAVE + (lane & 31);
    const bool valid = r < a.Et;
    const int e = valid ? r : a.Et - 1;
    edge_x32_tile<MODE, GC>(a, st, e, valid, lane, h);
  }
}

// ================================================================ node aggregation (CSR segment sum)
// h_attn[v] = sum_{e in in(v)} alpha[e, head] * V[src e]  /  (sum_e alpha[e, head] + 1e-6)
// (send_and_recv(u_mul_e('V_h','score'), sum) and (copy_e('score'), sum), then wV / (z + 1e-6):
// deepinteract_modules.py:93-96, 116). Edges are destination-major (CSR in_ptr), so a node's
// in-edges are one contiguous range.
// 16 lanes per destination, 8 features (16 B of bf16) per lane: a gathered V row is one coalesced
// 256-B access. In-edges go in chunks of U: the chunk's source ids arrive with ONE coalesced load
// (lane j of the node's 16 reads src[e0 + j], broadcast by ds_bpermute) and the next chunk's ids are
// in flight while this chunk's alphas and V rows land, so a chunk costs one memory latency; U rows
// per lane in flight and 16 nodes per 256-thread block (grid = Nt / 16, several blocks per CU) hide
// it. The products are added one edge at a time in edge order with the same fused multiply-adds as
// the fused node kernel, so h_attn is bit-identical to what k_node_layer computes internally.
constexpr int AGG_NODES = 16;  // destinations per block (16 lanes each)
template <class DT>
struct AggrCfg {
  static constexpr int U = DT::kBF16 ? 16 : 8;  // in-edges per chunk (V bytes in flight per lane: U x 16/32)
};
struct AggrArgs {
  int Nt;
  const int* src;
  const int* in_ptr;
  const float* alpha;
  const void* qkv;
  float* attn;
};

template <class DT>
__global__ __launch_bounds__(16 * AGG_NODES) void k_node_aggr(AggrArgs a) {
  using T = typename DT::T;
  constexpr int U = AggrCfg<DT>::U;
  constexpr int FPL = 8;  // features per lane
  const int j = threadIdx.x & 15;
  const int v = blockIdx.x * AGG_NODES + (threadIdx.x >> 4);
  if (v >= a.Nt) return;  // whole 16-lane groups exit together (shuffles stay within a group)
  const int head = (FPL * j) >> 5;
  const T* vbase = reinterpret_cast<const T*>(a.qkv) + 2 * HID + FPL * j;
  const int e0 = a.in_ptr[v], e1 = a.in_ptr[v + 1];
  float acc[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) acc[f] = 0.f;
  float z = 0.f;
  const int lane_base = threadIdx.x & 48;  // first lane of this node's 16 (within the wave)
  int id_next = e0 + j < e1 ? a.src[e0 + j] : 0;
#pragma unroll 1
  for (int c = e0; c < e1; c += U) {
    const int n = min(U, e1 - c);
    // this chunk's ids (lanes 0..n-1 of the group hold them) and alphas / V rows in flight
    const int id_cur = id_next;
    int ids[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ids[u] = __shfl(id_cur, lane_base + (u & 15), 64);
    float al[U];
    T vv[U][FPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
        al[u] = a.alpha[(int64_t)(c + u) * 4 + head];
        const T* row = vbase + (int64_t)ids[u] * 3 * HID;
        if constexpr (DT::kBF16) {
          *reinterpret_cast<uint4*>(vv[u]) = *reinterpret_cast<const uint4*>(row);
        } else {
          *reinterpret_cast<float4*>(vv[u]) = *reinterpret_cast<const float4*>(row);
          *reinterpret_cast<float4*>(vv[u] + 4) = *reinterpret_cast<const float4*>(row + 4);
        }
      }
    }
    // ids of the next chunk (U <= 16 lanes of the group)
    if (c + U < e1) id_next = c + U + j < e1 && j < U ? a.src[c + U + j] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
#pragma unroll
        for (int f = 0; f < FPL; ++f) {
          float x;
          if constexpr (DT::kBF16) x = __builtin_bit_cast(float, (uint32_t)vv[u][f] << 16);
          else x = vv[u][f];
          acc[f] = __builtin_fmaf(al[u], x, acc[f]);
        }
        z += al[u];
      }
    }
  }
  const float d = z + 1e-6f;
  float4 o0, o1;
  o0.x = acc[0] / d; o0.y = acc[1] / d; o0.z = acc[2] / d; o0.w = acc[3] / d;
  o1.x = acc[4] / d; o1.y = acc[5] / d; o1.z = acc[6] / d; o1.w = acc[7] / d;
  float* out = a.attn + (int64_t)v * HID + FPL * j;
  *reinterpret_cast<float4*>(out) = o0;
  *reinterpret_cast<float4*>(out + 4) = o1;
}

// The attention row of node v from precomputed aggregates: di_node_aggregate's rows, or
// di_edge_layer_attn's (attn_parts != null): complete rows for destinations whose in-edges lie in
// one fold tile, partial sums for the others (edge_attn_fold), zero for a node without in-edges
// (wV / (z + 1e-6) = 0 there).
__device__ __forceinline__ void attn_row(Act<8>& wv, const NodeArgs& a, int v, int g) {
  if (a.attn_parts == nullptr) {
    load_row(wv, a.attn + (int64_t)v * HID, g);
    return;
  }
  const int e0 = a.in_ptr[v], e1 = a.in_ptr[v + 1];
  const int t0 = e0 / FOLD_ROWS, t1 = (e1 - 1) / FOLD_ROWS;
  if (e1 <= e0) {
    zero(wv);
  } else if (t0 == t1) {
    load_row(wv, a.attn + (int64_t)v * HID, g);
  } else {
    const float* p = a.attn_parts + ((int64_t)t0 * 2 + 1) * FOLD_PART;
    load_row(wv, p, g);
    floatx4 z = ld4(p + HID);
#pragma unroll 1
    for (int t = t0 + 1; t <= t1; ++t) {
      p = a.attn_parts + (int64_t)t * 2 * FOLD_PART;
      add_row(wv, p, g);
      z += ld4(p + HID);
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float d = z[b >> 1] + 1e-6f;
#pragma unroll
      for (int q = 0; q < 4; ++q) wv.v[b][q] = wv.v[b][q] / d;
    }
  }
}

// The CSR segment sum of one node held in the MFMA layout (wv[b][q] = feature 16b + 4g + q of node
// v): wV / (z + 1e-6) with wV = sum alpha * V[src], z = sum alpha over v's in-edges
// (deepinteract_modules.py:93-96, 116). Shared by the fused node layers (k_node_layer,
// k_node_update_ring with attn == NULL); k_node_aggr computes the same products in the same order.
template <class DT>
__device__ __forceinline__ void node_gather(Act<8>& wv, const NodeArgs& a, int v, int g) {
  using T = typename DT::T;
  const T* qkv = reinterpret_cast<const T*>(a.qkv);
  zero(wv);
  floatx4 z = {0.f, 0.f, 0.f, 0.f};
  // In-edges in groups of UNR: the group's source ids, alphas and V[src] rows are all in flight
  // before the first product (one latency per group instead of two dependent ones per edge); the
  // products are still added one edge at a time in edge order (the reference's summation order).
  constexpr int UNR = DT::kBF16 ? 4 : 2;
  const int e0 = a.in_ptr[v], e1 = a.in_ptr[v + 1];
  int e = e0;
#pragma unroll 1
  for (; e + UNR <= e1; e += UNR) {
    int sid[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) sid[u] = a.src[e + u];
    floatx4 al[UNR];
    RawRow<T> vr[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      al[u] = ld4(a.alpha + (int64_t)(e + u) * 4);
      vr[u].load(qkv + (int64_t)sid[u] * 3 * HID + 2 * HID, g);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      Act<8> vv;
      vr[u].to_act(vv);
#pragma unroll
      for (int b = 0; b < 8; ++b) wv.v[b] = __builtin_elementwise_fma((floatx4)al[u][b >> 1], vv.v[b], wv.v[b]);
      z += al[u];
    }
  }
#pragma unroll 1
  for (; e < e1; ++e) {
    const floatx4 al = ld4(a.alpha + (int64_t)e * 4);
    Act<8> vv;
    load_row(vv, qkv + (int64_t)a.src[e] * 3 * HID + 2 * HID, g);
#pragma unroll
    for (int b = 0; b < 8; ++b) wv.v[b] = __builtin_elementwise_fma((floatx4)al[b >> 1], vv.v[b], wv.v[b]);
    z += al;
  }
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const float d = z[b >> 1] + 1e-6f;
#pragma unroll
    for (int q = 0; q < 4; ++q) wv.v[b][q] = wv.v[b][q] / d;
  }
}

// ================================================================ node update (bf16), 4-slot weight ring
// O_node + residual + FFN (+ next layer's Q/K/V, + hT) from the aggregated rows of k_node_aggr.
// Nt / 64 blocks is one block per CU, so a stage's 32 MFMAs per wave (~0.3 us) are far shorter than
// an LDS-DMA stage's landing latency (~1 us): the double-buffered pipe of k_node_layer waits on
// every stage. Here ALL the layer's biases land once at entry and the 32-KiB stages stream through
// a 4-slot ring, three stages ahead: entering stage s the wave waits only for its own pieces of
// stage s (s_waitcnt vmcnt(8 x stages issued after it): each wave issues exactly 8 one-KiB pieces
// per stage, and every other vector-memory operation is older than them: outputs are held in
// registers and stored at the end), then a barrier publishes the stage and frees the slot of
// stage s-1 for stage s+3. Arithmetic identical to k_node_layer (same operands, same order).
constexpr int NU_SLOTS = 4;
constexpr int NU_STAGE = MAT128;  // blocks per stage
__device__ __forceinline__ void nu_wait_younger(int n_stages_younger) {
  // vmcnt takes an immediate: the three counts this ring can need
  if (n_stages_younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n_stages_younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// each of the 4 waves issues exactly NU_STAGE * BLK * 2 / 1024 / 4 = 8 one-KiB pieces per stage:
// the vmcnt immediates of nu_wait_younger assume that split
using NodeRingGeo = KernelGeo<4>;
static_assert(NU_STAGE * BLK * 2 / 1024 / NodeRingGeo::NW == 8, "nu_wait_younger counts 8 pieces per wave");
template <bool FINAL>
__global__ __launch_bounds__(NodeRingGeo::THREADS, 1) void k_node_update_ring(NodeArgs a) {
  constexpr int NS = FINAL ? 5 : 8;
  constexpr int NVEC = FINAL ? NLV_N_FINAL : NLV_N;
  // one LDS object: [4 ring slots | all biases]
  __shared__ __attribute__((aligned(16))) char lds[NU_SLOTS * NU_STAGE * BLK * 2 + NLV_N * 4];
  u16* wring = reinterpret_cast<u16*>(lds);
  float* vlds = reinterpret_cast<float*>(lds + NU_SLOTS * NU_STAGE * BLK * 2);
  const int lane = lane_id(), g = lane >> 4;
  const int r = row_id<NodeRingGeo::NW>();
  const bool valid = r < a.Nt;
  const int v = valid ? r : a.Nt - 1;
  const u16* W = reinterpret_cast<const u16*>(a.wmat);
  // stage s -> first packed block
  auto stage_blk = [](int s) {
    return s == 0 ? NL_ON : (s == 1 ? NL_F1 : (s == 2 ? NL_F2 : (s == 3 ? NL_F1 + MAT128 : (s == 4 ? NL_F2 + MAT128 : NL_Q + MAT128 * (s - 5)))));
  };
  auto issue = [&](int s) { dma_blocks<NodeRingGeo::NW>(wring + (s % NU_SLOTS) * NU_STAGE * BLK, W + stage_blk(s) * BLK, NU_STAGE); };
  // biases and stage 0, then this node's rows, landed here (the compiler cannot count the DMA
  // loops, so a row used later would make it wait for every stage in flight), then stages 1-2
  dma_vec<NodeRingGeo::NW>(vlds, a.wvec, NVEC / 128);
  issue(0);
  RawRow<u16> hin;
  hin.load(reinterpret_cast<const u16*>(a.h_in) + (int64_t)v * HID, g);
  Act<8> wv;
  attn_row(wv, a, v, g);
  settle(hin);
#pragma unroll
  for (int b = 0; b < 8; ++b) asm volatile("" ::"v"(wv.v[b]));
  issue(1);
  issue(2);
  auto enter = [&](int s) -> const u16* {
    nu_wait_younger(min(2, NS - 1 - s));
    // a bare s_barrier: __syncthreads()' workgroup fence would wait for every outstanding
    // vector-memory operation, i.e. also for the stages in flight behind this one
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 3 < NS) issue(s + 3);
    return wring + (s % NU_SLOTS) * NU_STAGE * BLK;
  };
  // n = in1 + O_node(h)
  const u16* w = enter(0);
  Act<8> n;
  init_vec_lds(n, vlds + NLV_ON, g);
  {
    Act<8> hv;
    hin.to_act(hv);
    add_(n, hv);
  }
  linear<BF16T, 8, 4>(n, wv, w, lane);
  // n = n + W2 silu(W1 BN2(n))
  Act<8> o;
  zero(o);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    w = enter(1 + 2 * half);
    Act<8> t;
    init_vec_lds(t, vlds + NLV_F1 + 128 * half, g);
    linear<BF16T, 8, 4>(t, n, w, lane);
    silu2_<8, true>(t);
    w = enter(2 + 2 * half);
    linear<BF16T, 8, 4>(o, t, w, lane);
  }
  add_(n, o);
  if constexpr (FINAL) {
    if (valid) store_row(n, reinterpret_cast<u16*>(a.h_out) + (int64_t)v * HID, g);
    if (a.hT_out != nullptr && valid) {
      u16* hT = reinterpret_cast<u16*>(a.hT_out);
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          hT[(int64_t)(16 * b + 4 * g + q) * a.Nt + v] = (u16)(pack_bf16x2(n.v[b][q], 0.f) & 0xffffu);
    }
  } else {
    Op<BF16T, 4> nop;
    make_op(nop, n);  // bf16 bits of n: the h_out row and the Q/K/V operand
    Op<BF16T, 4> qkv_rows[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      w = enter(5 + q);
      Act<8> t;
      init_vec_lds(t, vlds + NLV_Q + 128 * q, g);
      mma<8, 4>(t, nop, w, lane);
      make_op(qkv_rows[q], t);
    }
    if (valid) {
      // packed operand -> row-major bf16: f[s] = {blk 2s regs 0-3, blk 2s+1 regs 0-3} = 4+4 features
      auto store_op = [&](const Op<BF16T, 4>& op, u16* row) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint4 u = __builtin_bit_cast(uint4, op.f[s]);
          *reinterpret_cast<uint2*>(row + 16 * (2 * s) + 4 * g) = (uint2){u.x, u.y};
          *reinterpret_cast<uint2*>(row + 16 * (2 * s + 1) + 4 * g) = (uint2){u.z, u.w};
        }
      };
      store_op(nop, reinterpret_cast<u16*>(a.h_out) + (int64_t)v * HID);
      u16* qo = reinterpret_cast<u16*>(a.qkv_out) + (int64_t)v * 3 * HID;
#pragma unroll
      for (int q = 0; q < 3; ++q) store_op(qkv_rows[q], qo + q * HID);
    }
  }
}

// The CSR segment sum of ONE destination by its 16-lane group (lane j: features 8j .. 8j + 7, head
// j / 4): acc = sum_e alpha[e, head] * V[src e], z = sum_e alpha[e, head] over e in [e0, e1), edge by
// edge in order -- k_node_aggr's products and order, so the row is bit-identical to it for any chunk
// size U. Every product is added with an explicit fused multiply-add (here, in k_node_aggr and in
// node_gather): a plain a += w * x is llvm.fmuladd, which the backend may fuse in one kernel and split
// into a multiply and an add in another (round 6: a build with specialised aggregation waves differed
// from the split form by one bf16 ulp on 1 row in 96 until its sums were explicit FMAs). Every load of a chunk is issued unconditionally (a slot past e1 re-reads edge c's alpha and
// a valid V row and adds it with weight 0, which is exact), so a chunk is one batch of buffer loads
// (32-bit offsets from SGPR descriptors) and one wait, with no per-edge branch. A chunk's source ids
// arrive as two per-lane registers (lane j of the group: src[c + j] and src[c + 16 + j], 0 past e1),
// loaded one chunk ahead; on entry (ida, idb) hold chunk e0's.
template <int U>
__device__ __forceinline__ void seg_ids(const int* __restrict__ src, int c, int e1, int j, int& ida, int& idb) {
  ida = c + j < e1 && j < U ? src[c + j] : 0;
  if constexpr (U > 16) idb = c + 16 + j < e1 && 16 + j < U ? src[c + 16 + j] : 0;
}
template <int U>
__device__ __forceinline__ void seg_sum16(__amdgpu_buffer_rsrc_t vr, __amdgpu_buffer_rsrc_t ar, const int* __restrict__ src,
                                          int e0, int e1, int j, int lane_base, int ida, int idb, float (&acc)[8],
                                          float& z) {
  static_assert(U >= 1 && U <= 32, "a chunk's ids come from two registers of the group's 16 lanes");
  const int head = j >> 2;
#pragma unroll 1
  for (int c = e0; c < e1; c += U) {
    const int n = min(U, e1 - c);
    const int id_a = ida, id_b = idb;
    float al[U];
    uint4 vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int id = __shfl(u < 16 ? id_a : id_b, lane_base + (u & 15), 64);
      const int eu = u < n ? c + u : c;
      al[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ar, (eu * 4 + head) * 4, 0, 0));
      vv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vr, id * (3 * HID * 2) + 16 * j, 0, 0));
    }
    if (c + U < e1) seg_ids<U>(src, c + U, e1, j, ida, idb);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float w = u < n ? al[u] : 0.f;
      const uint32_t x[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const uint32_t b = f & 1 ? (x[f >> 1] & 0xffff0000u) : (x[f >> 1] << 16);
        acc[f] = __builtin_fmaf(w, __builtin_bit_cast(float, b), acc[f]);
      }
      z += w;
    }
  }
}

constexpr int SEG_U = 10;     // k_node_fast (<= 120 VGPRs): k = 20 in-edges are two chunks
// k_node_ws: chunks of 10 as well. One chunk of 20 (one memory latency per tile) spills 5 VGPRs at
// the 240 cap and measured slower: node layers beside the pair stream 47 / 27-29 vs 43 / 26-29 us,
// 7953 / 7918 vs 8038 / 7993 complexes/s (round 6, tools/sessions/r6_05_wsu.sh)
constexpr int SEG_U_WS = 10;
// LDS row strides of the node kernels' exchange buffers, padded for the banking of the instructions
// that touch them (MI355X_MICROARCH.md §LDS): the fp32 aggregated rows are read by ds_read_b128 (four
// 16-lane groups, bank = word mod 64) -- a 136-word stride puts every group's 16 lanes (rows r, lane
// groups g) on distinct bank quads; the bf16 operand rows are read by ds_read2_b64 and written by
// ds_write_b64 (16 contiguous lanes per access, bank = word mod 32, 2 words per lane) -- 66 / 130-word
// strides put 16 rows on 32 distinct banks. Unpadded (128 / 64 / 128 words) every row starts on bank
// 0: 16-way conflicts on each exchange access (round 6, first k_node_ws build: 2x slower).
constexpr int LDS_ATTN = HID + 8;       // fp32 aggregated rows: 136 words
constexpr int LDS_N = HID + 4;          // bf16 n / h rows: 66 words
constexpr int LDS_T = 2 * HID + 4;      // bf16 FFN-hidden rows: 130 words
template <int U>
__device__ __forceinline__ void seg_sum16(__amdgpu_buffer_rsrc_t vr, __amdgpu_buffer_rsrc_t ar, const int* __restrict__ src,
                                          int e0, int e1, int j, int lane_base, int id_first, float (&acc)[8], float& z) {
  static_assert(U >= 1 && U <= 16, "a chunk's ids come from the group's 16 lanes");
  const int head = j >> 2;
  int id_next = id_first;
#pragma unroll 1
  for (int c = e0; c < e1; c += U) {
    const int n = min(U, e1 - c);
    const int id_cur = id_next;
    float al[U];
    uint4 vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int id = __shfl(id_cur, lane_base + u, 64);
      const int eu = u < n ? c + u : c;
      al[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ar, (eu * 4 + head) * 4, 0, 0));
      vv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vr, id * (3 * HID * 2) + 16 * j, 0, 0));
    }
    if (c + U < e1) id_next = c + U + j < e1 && j < U ? src[c + U + j] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float w = u < n ? al[u] : 0.f;
      const uint32_t x[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const uint32_t b = f & 1 ? (x[f >> 1] & 0xffff0000u) : (x[f >> 1] << 16);
        acc[f] = __builtin_fmaf(w, __builtin_bit_cast(float, b), acc[f]);
      }
      z += w;
    }
  }
}

// ================================================================ node layer at full occupancy (bf16)
// The bf16 di_node_layer (the overlapped schedule's node layer, round 5). k_node_layer runs 16
// destinations per wave and one 4-wave block per CU (a C3 micro-batch's 16 k nodes are 250 blocks):
// one latency-bound chain per CU -- in-edge gathers, then eight dependent weight stages. Here a
// 256-thread block owns 16 destinations and splits BOTH halves of the layer over its threads:
//   1. the CSR segment sum, 16 lanes per destination, exactly as k_node_aggr (same products, same
//      order, same division: bit-identical rows), into LDS;
//   2. O_node + residual, the node FFN and the next layer's Q/K/V with the OUTPUT features split
//      over the 4 waves (wave w: features 32w..32w+31 of O and of the FFN output, 64w..64w+63 of the
//      FFN hidden layer, 96w..96w+95 of Q|K|V), each wave reading its A fragments straight from L2
//      (a wave's slice of a 128x128 matrix is 8 KiB: no LDS weight stages, no stage waits), the
//      activations between the linears exchanged through LDS as the bf16 operand the MFMAs read.
// 4x the blocks of k_node_layer (1000 per C3 micro-batch, four per CU): the latency of one block's
// chain is covered by the others. Per output element the arithmetic is k_node_layer<BF16T>'s (the
// same bias + residual initial value, the same k-steps in the same order, the same bf16 operands),
// so h / Q,K,V / hT are bit-identical to di_node_layer's fused and split forms.
// NG node groups of 16 destinations per block and 4 NG waves: every wave computes its output blocks
// for ALL the block's groups, so one A-fragment load from L2 feeds NG MFMAs (NG = 2 halves the L2
// weight stream per node). Blocks per wave: O / FFN output 8 / (4 NG), hidden 16 / (4 NG),
// Q|K|V 24 / (4 NG).
constexpr int NF_NODES = 16;  // destinations per node group (16 lanes each in the aggregation)
constexpr int NF_GROUPS = 1;  // node groups per block (the launch; 2 measured slower: each wave's chain doubles)
template <bool FINAL, int NG>
// <= 120 VGPRs (amdgpu_num_vgpr counts register pairs): four waves per SIMD leave one pair-stream
// wave room beside them
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256 * NG), amdgpu_waves_per_eu(4), amdgpu_num_vgpr(60)))
void k_node_fast(NodeArgs a) {
  constexpr int NWV = 4 * NG, BO = 8 / NWV, BH = 16 / NWV, BQ = 24 / NWV;
  static_assert(8 % NWV == 0 && BQ >= 1, "node groups per block: 1 or 2");
  __shared__ __attribute__((aligned(16))) float s_attn[NG * NF_NODES * LDS_ATTN];  // aggregated rows (fp32)
  __shared__ __attribute__((aligned(16))) u16 s_n[NG * NF_NODES * LDS_N];       // n as a bf16 operand
  __shared__ __attribute__((aligned(16))) u16 s_t[NG * NF_NODES * LDS_T];   // FFN hidden (bf16)
  const int vb = (int)blockIdx.x * NG * NF_NODES;  // the block's first destination
  // ---- 1. wV / (z + 1e-6), 16 lanes per destination (k_node_aggr<BF16T>'s loop)
  {
    constexpr int FPL = 8;
    const int j = threadIdx.x & 15, nl = threadIdx.x >> 4;  // nl: the block's destination 0 .. 16 NG - 1
    const int v = vb + nl;
    float acc[FPL];
#pragma unroll
    for (int f = 0; f < FPL; ++f) acc[f] = 0.f;
    float z = 0.f;
    if (v < a.Nt) {  // uniform per 16-lane group (the shuffles stay inside the group)
      const int e0 = a.in_ptr[v], e1 = a.in_ptr[v + 1];
      int ida = 0, idb = 0;
      seg_ids<SEG_U>(a.src, e0, e1, j, ida, idb);
      seg_sum16<SEG_U>(buf_rsrc(reinterpret_cast<const u16*>(a.qkv) + 2 * HID), buf_rsrc(a.alpha), a.src, e0, e1, j,
                       threadIdx.x & 48, ida, idb, acc, z);
    }
    const float d = z + 1e-6f;
    float* out = s_attn + nl * LDS_ATTN + FPL * j;
    st4(out, (floatx4){acc[0] / d, acc[1] / d, acc[2] / d, acc[3] / d});
    st4(out + 4, (floatx4){acc[4] / d, acc[5] / d, acc[6] / d, acc[7] / d});
  }
  // ---- 2. the update: wave w computes its output blocks for every node group
  const int lane = lane_id(), g = lane >> 4, r = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  int vq[NG];
  bool valid[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    vq[q] = vb + q * NF_NODES + r;
    valid[q] = vq[q] < a.Nt;
  }
  const u16* W = reinterpret_cast<const u16*>(a.wmat);
  const float* V = a.wvec;
  // A fragment (output block bo, k-step s) of the 128x128 matrix at packed block m, from L2
  auto frag = [&](int m, int bo, int s) {
    return *reinterpret_cast<const bf16x8*>(W + (m + bo * 4 + s) * BLK + lane * 8);
  };
  // the bf16 operand of group q's 16 rows stored row-major in LDS (make_op's packing of blocks 2s, 2s+1)
  auto lds_op = [&](const u16* rows, int stride, int q, int f0) {
    Op<BF16T, 4> o;
    const u16* row = rows + (q * NF_NODES + r) * stride + f0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint2 lo = *reinterpret_cast<const uint2*>(row + 32 * s + 4 * g);
      const uint2 hi = *reinterpret_cast<const uint2*>(row + 32 * s + 16 + 4 * g);
      o.f[s] = __builtin_bit_cast(bf16x8, (uint4){lo.x, lo.y, hi.x, hi.y});
    }
    return o;
  };
  auto put_slice = [&](u16* rows, int stride, int q, int f, floatx4 x) {
    *reinterpret_cast<uint2*>(rows + (q * NF_NODES + r) * stride + f + 4 * g) =
        (uint2){pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
  };
  // n = b_O + h_in + O(attn): output blocks BO w .. BO w + BO - 1
  Act<BO> n[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q)
#pragma unroll
    for (int b = 0; b < BO; ++b) {
      const int ob = BO * w + b;
      const int vc = valid[q] ? vq[q] : a.Nt - 1;
      n[q].v[b] = ld4(V + NLV_ON + 16 * ob + 4 * g) +
                  ld4(reinterpret_cast<const u16*>(a.h_in) + (int64_t)vc * HID + 16 * ob + 4 * g);
    }
  bf16x8 fo[BO][4];
#pragma unroll
  for (int b = 0; b < BO; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s) fo[b][s] = frag(NL_ON, BO * w + b, s);
  __syncthreads();  // the aggregated rows
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    Act<8> wv;
#pragma unroll
    for (int b = 0; b < 8; ++b)
      wv.v[b] = *reinterpret_cast<const floatx4*>(s_attn + (q * NF_NODES + r) * LDS_ATTN + 16 * b + 4 * g);
    Op<BF16T, 4> op;
    make_op(op, wv);
#pragma unroll
    for (int b = 0; b < BO; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) n[q].v[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fo[b][s], op.f[s], n[q].v[b], 0, 0, 0);
#pragma unroll
    for (int b = 0; b < BO; ++b) put_slice(s_n, LDS_N, q, 16 * (BO * w + b), n[q].v[b]);
  }
  // FFN hidden: blocks hb = BH w + b of the 16 (half hb / 8, output block hb % 8 of that half)
  bf16x8 f1[BH][4];
#pragma unroll
  for (int b = 0; b < BH; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int hb = BH * w + b;
      f1[b][s] = frag(NL_F1 + MAT128 * (hb >> 3), hb & 7, s);
    }
  __syncthreads();  // n, all 128 features of every group
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const Op<BF16T, 4> nop = lds_op(s_n, LDS_N, q, 0);
    Act<BH> tq;
#pragma unroll
    for (int b = 0; b < BH; ++b) tq.v[b] = ld4(V + NLV_F1 + 16 * (BH * w + b) + 4 * g);
#pragma unroll
    for (int b = 0; b < BH; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) tq.v[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[b][s], nop.f[s], tq.v[b], 0, 0, 0);
    silu2_<BH, true>(tq);
#pragma unroll
    for (int b = 0; b < BH; ++b) put_slice(s_t, LDS_T, q, 16 * (BH * w + b), tq.v[b]);
  }
  // FFN output (blocks BO w ..): both hidden halves in order, as k_node_layer
  bf16x8 f2[2][BO][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < BO; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) f2[h][b][s] = frag(NL_F2 + MAT128 * h, BO * w + b, s);
  __syncthreads();  // the hidden layer, all 256 features (and every wave is past its n operands)
  // the first half of this wave's Q | K | V fragments, in flight across the h exchange below
  constexpr int BQP = (BQ + 1) / 2;
  bf16x8 fq[BQP][4];
  if constexpr (!FINAL) {
#pragma unroll
    for (int b = 0; b < BQP; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) fq[b][s] = frag(NL_Q + MAT128 * ((BQ * w + b) >> 3), (BQ * w + b) & 7, s);
  }
  // the second half, issued as soon as the last group's FFN-output MFMAs no longer need f2's
  // registers: in flight across the h stores and the exchange barrier (global loads are not
  // moved across s_barrier by the compiler)
  bf16x8 fq2[BQ - BQP][4];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    Act<BO> o;
    zero(o);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const Op<BF16T, 4> top = lds_op(s_t, LDS_T, q, HID * h);
#pragma unroll
      for (int b = 0; b < BO; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s) o.v[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f2[h][b][s], top.f[s], o.v[b], 0, 0, 0);
    }
    if constexpr (!FINAL) {
      if (q == NG - 1) {
#pragma unroll
        for (int b = BQP; b < BQ; ++b)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            fq2[b - BQP][s] = frag(NL_Q + MAT128 * ((BQ * w + b) >> 3), (BQ * w + b) & 7, s);
      }
    }
    add_(n[q], o);
    if (valid[q]) {
      u16* hrow = reinterpret_cast<u16*>(a.h_out) + (int64_t)vq[q] * HID;
#pragma unroll
      for (int b = 0; b < BO; ++b) st4(hrow + 16 * (BO * w + b) + 4 * g, n[q].v[b]);
    }
    if constexpr (FINAL) {
      if (a.hT_out != nullptr && valid[q]) {
        u16* hT = reinterpret_cast<u16*>(a.hT_out);
#pragma unroll
        for (int b = 0; b < BO; ++b)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            hT[(int64_t)(16 * (BO * w + b) + 4 * g + k) * a.Nt + vq[q]] = (u16)(pack_bf16x2(n[q].v[b][k], 0.f) & 0xffffu);
      }
    } else {
#pragma unroll
      for (int b = 0; b < BO; ++b) put_slice(s_n, LDS_N, q, 16 * (BO * w + b), n[q].v[b]);
    }
  }
  if constexpr (!FINAL) {
    // next layer's Q | K | V from the new h: this wave's BQ output blocks of the 24 (Q 0-7, K 8-15, V 16-23)
    __syncthreads();  // the new h, all 128 features (s_n's previous readers finished before the last barrier)
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const Op<BF16T, 4> hop = lds_op(s_n, LDS_N, q, 0);
      u16* qo = reinterpret_cast<u16*>(a.qkv_out) + (int64_t)vq[q] * 3 * HID;
#pragma unroll
      for (int b = 0; b < BQ; ++b) {
        const int ob = BQ * w + b;
        floatx4 x = ld4(V + NLV_Q + 16 * ob + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b < BQP ? fq[b][s] : fq2[b - BQP][s], hop.f[s], x, 0, 0, 0);
        if (valid[q]) st4(qo + 16 * ob + 4 * g, x);
      }
    }
  }
}

// ================================================================ node layer, weights stationary (bf16)
// The bf16 di_node_layer since round 6. k_node_fast streams the whole layer's weights (256 KiB) from
// L2 into every 16-destination block: 1000 blocks, 256 MB of L2 -> CU fragment traffic per C3
// micro-batch, each wave's chain waiting on its fragment loads, beside a pair stream that pushes
// ~4 TB/s of stores through the same L2s. Here the weights are loaded ONCE per CU and stay:
//   * one persistent 8-wave block per CU (two waves per SIMD) walks tiles of 32 destinations
//     (XCD-contiguous tile order, as the edge ring);
//   * wave w keeps its slice of O (output block w), the FFN hidden layer (blocks 2w, 2w+1 of 16) and
//     the FFN output (block w, both K halves) in registers for the whole launch (80 VGPRs), and the
//     next layer's Q|K|V (96 KiB) sits in LDS, DMA'd once at entry (wave w: blocks 3w..3w+2 of 24);
//   * per tile: (1) the CSR segment sum, 16 lanes per destination, exactly k_node_fast's loop (same
//     products, same order: bit-identical rows) into LDS -- 32 destinations x 16 lanes = the block;
//     (2) O_node + residual, FFN, Q|K|V as two 16-destination MFMA column groups, every register
//     fragment feeding both groups, activations exchanged through LDS as bf16 operands.
// Per output element the arithmetic is k_node_fast's (the same bias + residual initial value, the
// same k-steps in the same order, the same bf16 operands): h / Q,K,V / hT are bit-identical.
constexpr int NWS_NW = 8;        // waves per block
constexpr int NWS_TILE = 32;     // destinations per tile (2 MFMA column groups of 16)
static_assert(NWS_TILE * 16 == 64 * NWS_NW, "16 aggregation lanes per destination of a tile");
// <= 240 VGPRs (amdgpu_num_vgpr counts register pairs): two waves per SIMD leave a pair-stream wave
// (32 VGPRs) room beside them, as the edge ring
template <bool FINAL>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * NWS_NW), amdgpu_waves_per_eu(2, 2),
                          amdgpu_num_vgpr(120)))
void k_node_ws(NodeArgs a, int ntiles) {
  constexpr int NG = NWS_TILE / 16;
  __shared__ __attribute__((aligned(16))) float s_attn[NWS_TILE * LDS_ATTN];  // aggregated rows (fp32), 16 KiB
  __shared__ __attribute__((aligned(16))) u16 s_n[NWS_TILE * LDS_N];       // n / new h as a bf16 operand, 8 KiB
  __shared__ __attribute__((aligned(16))) u16 s_t[NWS_TILE * LDS_T];   // FFN hidden (bf16), 16 KiB
  __shared__ __attribute__((aligned(16))) u16 s_q[FINAL ? 8 : 3 * MAT128 * BLK];  // Q|K|V weights, 96 KiB
  const int lane = lane_id(), g = lane >> 4, r = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const u16* W = reinterpret_cast<const u16*>(a.wmat);
  const float* V = a.wvec;
  if constexpr (!FINAL) dma_blocks<NWS_NW>(s_q, W + NL_Q * BLK, 3 * MAT128);
  // this wave's register-resident weights (A fragments: output block bo, k-step s of a 128x128 matrix)
  auto frag = [&](int m, int bo, int s) {
    return *reinterpret_cast<const bf16x8*>(W + (m + bo * 4 + s) * BLK + lane * 8);
  };
  bf16x8 fo[4], f1[2][4], f2[2][4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    fo[s] = frag(NL_ON, w, s);
#pragma unroll
    for (int b = 0; b < 2; ++b) f1[b][s] = frag(NL_F1 + MAT128 * ((2 * w + b) >> 3), (2 * w + b) & 7, s);
#pragma unroll
    for (int h = 0; h < 2; ++h) f2[h][s] = frag(NL_F2 + MAT128 * h, w, s);
  }
  auto lds_op = [&](const u16* rows, int stride, int q, int f0) {
    Op<BF16T, 4> o;
    const u16* row = rows + (q * 16 + r) * stride + f0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint2 lo = *reinterpret_cast<const uint2*>(row + 32 * s + 4 * g);
      const uint2 hi = *reinterpret_cast<const uint2*>(row + 32 * s + 16 + 4 * g);
      o.f[s] = __builtin_bit_cast(bf16x8, (uint4){lo.x, lo.y, hi.x, hi.y});
    }
    return o;
  };
  auto put_slice = [&](u16* rows, int stride, int q, int f, floatx4 x) {
    *reinterpret_cast<uint2*>(rows + (q * 16 + r) * stride + f + 4 * g) =
        (uint2){pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
  };
  bool qkv_landed = FINAL;
  const int j = threadIdx.x & 15, nl = threadIdx.x >> 4;  // aggregation: destination nl of the tile, lane j
  auto tile_of = [&](int i) { return (gridDim.x & 7) == 0 ? xcd_slot(i, ntiles) : i; };
  // this lane's CSR range and first source id of a tile's destination (issued a tile ahead)
  int e0 = 0, e1 = 0, ida = 0, idb = 0;
  auto seg_head = [&](int i) {
    const int v = tile_of(i) * NWS_TILE + nl;
    e0 = e1 = 0;
    if (i < ntiles && v < a.Nt) {
      e0 = a.in_ptr[v];
      e1 = a.in_ptr[v + 1];
    }
  };
  auto seg_id0 = [&]() { seg_ids<SEG_U_WS>(a.src, e0, e1, j, ida, idb); };
  seg_head((int)blockIdx.x);
  seg_id0();
#pragma unroll 1
  for (int i = (int)blockIdx.x; i < ntiles; i += (int)gridDim.x) {
    const int vb = tile_of(i) * NWS_TILE;
    // ---- 1. wV / (z + 1e-6), 16 lanes per destination (k_node_fast's sums)
    {
      constexpr int FPL = 8;
      float acc[FPL];
#pragma unroll
      for (int f = 0; f < FPL; ++f) acc[f] = 0.f;
      float z = 0.f;
      // empty past Nt (e0 == e1): the shuffles stay inside the 16-lane group
      seg_sum16<SEG_U_WS>(buf_rsrc(reinterpret_cast<const u16*>(a.qkv) + 2 * HID), buf_rsrc(a.alpha), a.src, e0, e1, j,
                          threadIdx.x & 48, ida, idb, acc, z);
      seg_head(i + (int)gridDim.x);  // the next tile's CSR range, in flight under this tile's update
      const float d = z + 1e-6f;
      float* out = s_attn + nl * LDS_ATTN + FPL * j;
      st4(out, (floatx4){acc[0] / d, acc[1] / d, acc[2] / d, acc[3] / d});
      st4(out + 4, (floatx4){acc[4] / d, acc[5] / d, acc[6] / d, acc[7] / d});
    }
    // ---- 2. the update: wave w's output blocks for both column groups
    int vq[NG];
    bool valid[NG];
    Act<1> n[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      vq[q] = vb + q * 16 + r;
      valid[q] = vq[q] < a.Nt;
      const int vc = valid[q] ? vq[q] : a.Nt - 1;
      n[q].v[0] = ld4(V + NLV_ON + 16 * w + 4 * g) + ld4(reinterpret_cast<const u16*>(a.h_in) + (int64_t)vc * HID + 16 * w + 4 * g);
    }
    __syncthreads();  // the aggregated rows (and, tile > 0, every wave past the previous tile's reads)
    // n = b_O + h_in + O(attn)
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      Act<8> wv;
#pragma unroll
      for (int b = 0; b < 8; ++b)
        wv.v[b] = *reinterpret_cast<const floatx4*>(s_attn + (q * 16 + r) * LDS_ATTN + 16 * b + 4 * g);
      Op<BF16T, 4> op;
      make_op(op, wv);
#pragma unroll
      for (int s = 0; s < 4; ++s) n[q].v[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fo[s], op.f[s], n[q].v[0], 0, 0, 0);
      put_slice(s_n, LDS_N, q, 16 * w, n[q].v[0]);
    }
    floatx4 b1[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) b1[b] = ld4(V + NLV_F1 + 16 * (2 * w + b) + 4 * g);
    seg_id0();  // the next tile's first source ids
    __syncthreads();  // n, all 128 features of both groups
    // FFN hidden: blocks 2w, 2w + 1 of the 16
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const Op<BF16T, 4> nop = lds_op(s_n, LDS_N, q, 0);
      Act<2> tq;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        tq.v[b] = b1[b];
#pragma unroll
        for (int s = 0; s < 4; ++s) tq.v[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[b][s], nop.f[s], tq.v[b], 0, 0, 0);
      }
      silu2_<2, true>(tq);
#pragma unroll
      for (int b = 0; b < 2; ++b) put_slice(s_t, LDS_T, q, 16 * (2 * w + b), tq.v[b]);
    }
    __syncthreads();  // the hidden layer, all 256 features (and every wave is past its n operands)
    // FFN output block w: both hidden halves in order, as k_node_fast
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      Act<1> o;
      zero(o);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const Op<BF16T, 4> top = lds_op(s_t, LDS_T, q, HID * h);
#pragma unroll
        for (int s = 0; s < 4; ++s) o.v[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f2[h][s], top.f[s], o.v[0], 0, 0, 0);
      }
      add_(n[q], o);
      if (valid[q]) st4(reinterpret_cast<u16*>(a.h_out) + (int64_t)vq[q] * HID + 16 * w + 4 * g, n[q].v[0]);
      if constexpr (FINAL) {
        if (a.hT_out != nullptr && valid[q]) {
          u16* hT = reinterpret_cast<u16*>(a.hT_out);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            hT[(int64_t)(16 * w + 4 * g + k) * a.Nt + vq[q]] = (u16)(pack_bf16x2(n[q].v[0][k], 0.f) & 0xffffu);
        }
      } else {
        put_slice(s_n, LDS_N, q, 16 * w, n[q].v[0]);
      }
    }
    if constexpr (!FINAL) {
      floatx4 bq[3];
#pragma unroll
      for (int b = 0; b < 3; ++b) bq[b] = ld4(V + NLV_Q + 16 * (3 * w + b) + 4 * g);
      if (!qkv_landed) {  // first tile only: this wave's pieces of the Q|K|V weights, before the barrier
        lds_dma_wait();
        qkv_landed = true;
      }
      __syncthreads();  // the new h, all 128 features (s_n's previous readers finished before the last barrier)
      // next layer's Q | K | V: blocks 3w .. 3w + 2 of the 24 (Q 0-7, K 8-15, V 16-23)
      bf16x8 fq[3][4];
#pragma unroll
      for (int b = 0; b < 3; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ob = 3 * w + b;
          fq[b][s] = *reinterpret_cast<const bf16x8*>(s_q + (MAT128 * (ob >> 3) + (ob & 7) * 4 + s) * BLK + lane * 8);
        }
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        const Op<BF16T, 4> hop = lds_op(s_n, LDS_N, q, 0);
        u16* qo = reinterpret_cast<u16*>(a.qkv_out) + (int64_t)vq[q] * 3 * HID;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          floatx4 x = bq[b];
#pragma unroll
          for (int s = 0; s < 4; ++s) x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fq[b][s], hop.f[s], x, 0, 0, 0);
          if (valid[q]) st4(qo + 16 * (3 * w + b) + 4 * g, x);
        }
      }
    }
  }
}

// ================================================================ fused node layer
// Every bias vector rides in its stage's LDS slot (init_vec_lds) and the node's own input row is
// added right after the stage barrier, before the next stage's DMA is issued: a global load
// consumed after a DMA issue makes the wave wait for the whole in-flight weight stage (vmcnt
// counts in order, and the compiler cannot count a runtime-length DMA loop), which exposed the
// DMA latency at every stage.
// Launch geometry of k_node_layer (di_node_layer, and di_node_update's fp32 path): DI_NODE_NW
// waves (16 nodes each) per block. Round 2's 2-wave build faulted (code 719) because
// di_node_update's fp32 launch kept a hard-coded 256-thread block while the kernel had been
// compiled for 128 (__launch_bounds__(64 * 2)): every launch site now takes its shape from
// NodeGeo. A C3 micro-batch has 16k nodes: 4-wave blocks give 250 blocks, 2-wave blocks 500
// (measured beside the pair stream 58 vs 55 us per launch, so 4 is the default; the 2-wave build
// is a tested variant, tools/build_variants.py "node2").
#ifndef DI_NODE_NW
#define DI_NODE_NW 4
#endif
using NodeGeo = KernelGeo<DI_NODE_NW>;
template <class DT, bool FINAL>
__global__ __launch_bounds__(NodeGeo::THREADS, 2) void k_node_layer(NodeArgs a) {
  using T = typename DT::T;
  constexpr bool FAST = DT::kBF16;
  constexpr bool DB = DT::kBF16;
  using Pipe = WPipe<T, NodeGeo::NW, DB, MAT128, 128>;
  __shared__ __attribute__((aligned(16))) char lds[(DB ? 2 : 1) * Pipe::SLOT_BYTES];
  const int lane = lane_id(), g = lane >> 4;
  const int r = row_id<NodeGeo::NW>();
  const bool valid = r < a.Nt;
  const int v = valid ? r : a.Nt - 1;
  const T* W = reinterpret_cast<const T*>(a.wmat);
  const float* V = a.wvec;
  const T* qkv = reinterpret_cast<const T*>(a.qkv);
  Pipe pipe(lds);
  pipe.issue(W + NL_ON * BLK, MAT128, V + NLV_ON, 128);
  RawRow<T> hin;  // in1 of the residual, consumed after the O stage barrier
  hin.load(reinterpret_cast<const T*>(a.h_in) + (int64_t)v * HID, g);

  // send_and_recv(u_mul_e('V_h','score'), sum) and (copy_e('score'), sum); h = wV / (z + 1e-6)
  Act<8> wv;
  if (a.attn != nullptr) attn_row(wv, a, v, g);  // k_node_aggr (same products, order, division) or the fold
  else node_gather<DT>(wv, a, v, g);
  // n = in1 + O_node(h)
  const T* w = pipe.next();
  settle(hin);  // landed with the O stage (the barrier drained vmcnt); no wait on the F1 DMA later
  pipe.issue(W + NL_F1 * BLK, MAT128, V + NLV_F1, 128);
  Act<8> n;
  init_vec_lds(n, pipe.v(), g);
  {
    Act<8> hv;
    hin.to_act(hv);
    add_(n, hv);
  }
  linear<DT, 8, 4>(n, wv, w, lane);
  // n = n + W2 silu(W1 BN2(n))
  Act<8> o;
  zero(o);
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    w = pipe.next();
    pipe.issue(W + (NL_F2 + MAT128 * half) * BLK, MAT128);
    Act<8> t;
    init_vec_lds(t, pipe.v(), g);
    linear<DT, 8, 4>(t, n, w, lane);
    silu2_<8, FAST>(t);
    w = pipe.next();
    if (half == 0) pipe.issue(W + (NL_F1 + MAT128) * BLK, MAT128, V + NLV_F1 + 128, 128);
    else if (!FINAL) pipe.issue(W + NL_Q * BLK, MAT128, V + NLV_Q, 128);
    linear<DT, 8, 4>(o, t, w, lane);
  }
  add_(n, o);
  if (valid) store_row(n, reinterpret_cast<T*>(a.h_out) + (int64_t)v * HID, g);
  if (a.hT_out != nullptr && valid) {  // 16 lanes (nodes) store 32 contiguous bytes per feature
    T* hT = reinterpret_cast<T*>(a.hT_out);
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float x = n.v[b][q];
        if constexpr (DT::kBF16) hT[(int64_t)(16 * b + 4 * g + q) * a.Nt + v] = (u16)(pack_bf16x2(x, 0.f) & 0xffffu);
        else hT[(int64_t)(16 * b + 4 * g + q) * a.Nt + v] = x;
      }
  }
  if constexpr (!FINAL) {
    T* qo = reinterpret_cast<T*>(a.qkv_out);
#pragma unroll 1
    for (int q = 0; q < 3; ++q) {
      w = pipe.next();
      if (q < 2) pipe.issue(W + (NL_Q + MAT128 * (q + 1)) * BLK, MAT128, V + NLV_Q + 128 * (q + 1), 128);
      Act<8> t;
      init_vec_lds(t, pipe.v(), g);
      linear<DT, 8, 4>(t, n, w, lane);
      if (valid) store_row(t, qo + (int64_t)v * 3 * HID + q * HID, g);
    }
  }
}

}  // namespace di

// ================================================================ C ABI
using namespace di;

// grid / block of a launch, both from the kernel's geometry struct
template <class Geom>
static inline dim3 grid_of(int n) { return dim3((unsigned)((n + Geom::ROWS - 1) / Geom::ROWS)); }
template <class Geom>
static inline dim3 block_of() { return dim3(Geom::THREADS); }

static inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

static inline bool dtype_ok(di_dtype dt) { return dt == DI_BF16 || dt == DI_F32; }

extern "C" int di_abi_version(void) { return DI_ABI_VERSION; }

extern "C" int64_t di_blob_bytes(int kind, di_dtype dtype, int vec) {
  if (!dtype_ok(dtype)) return -1;
  const int64_t esz = dtype == DI_BF16 ? 2 : 4;
  int64_t blk = 0, nvec = 0;
  switch (kind) {
    case 0: blk = EM_NBLK; nvec = EMV_N; break;
    case 1: blk = IE_NBLK; nvec = IEV_N; break;
    case 2: blk = EL_NBLK; nvec = ELV_N; break;
    case 3: blk = EL_NBLK_FINAL; nvec = ELV_N_FINAL; break;
    case 4: blk = NL_NBLK; nvec = NLV_N; break;
    case 5: blk = NL_NBLK_FINAL; nvec = NLV_N_FINAL; break;
    case 6: blk = EL_NBLK_CONF; nvec = ELV_N_CONF; break;
    default: return -1;
  }
  return vec ? nvec * 4 : blk * BLK * esz;
}

extern "C" int di_blob_layout(int kind, di_dtype dtype) {
  if (!dtype_ok(dtype) || kind < 0 || kind > 6) return -1;
  if (dtype != DI_BF16) return 16;
  if (kind == 1 || kind == 2 || kind == 3) return 32;  // k_init_x32 / k_init_res_x32 / k_edge_x32_ring
  return 16;
}

extern "C" int di_node_embed(const di_graph* g, di_dtype dt, int32_t in_dim, const float* node_f, const void* wmat,
                             const float* wvec, void* h_out, void* qkv_out, void* queue, int32_t signal_job,
                             void* stream) {
  if (!g || !node_f || !wmat || !wvec || !h_out || !qkv_out || g->num_nodes <= 0 || in_dim <= 0 || in_dim > HID ||
      !dtype_ok(dt))
    return DI_EINVAL;
  EmbedArgs a{g->num_nodes, in_dim, node_f, wmat, wvec, h_out, qkv_out, (uint32_t*)queue, signal_job};
  hipStream_t s = (hipStream_t)stream;
  if (dt == DI_BF16)
    hipLaunchKernelGGL(k_node_embed<BF16T>, grid_of<EmbedGeo>(a.Nt), block_of<EmbedGeo>(), 0, s, a);
  else
    hipLaunchKernelGGL(k_node_embed<F32T>, grid_of<EmbedGeo>(a.Nt), block_of<EmbedGeo>(), 0, s, a);
  return launch_status();
}

extern "C" int di_init_edge(const di_graph* g, di_dtype dt, const float* edge_f, const void* wmat,
                            const float* wvec, const float* pos_src_tab, const float* pos_dst_tab,
                            void* f_out, void* fn_out, void* stream) {
  const bool gc = (g ? g->flags : 0) & DI_GRAPH_GEO_REF;
  if (!g || !edge_f || !wmat || !wvec || !pos_src_tab || !pos_dst_tab || !f_out || (!fn_out && !gc) ||
      g->num_edges <= 0 || !dtype_ok(dt))
    return DI_EINVAL;
  InitArgs a{g->num_edges, edge_f, g->src, g->dst, g->node_pos, wmat, wvec, pos_src_tab, pos_dst_tab,
             f_out, fn_out};
  hipStream_t s = (hipStream_t)stream;
  const dim3 gf = grid_of<InitGeo<F32T>>(a.Et), bf = block_of<InitGeo<F32T>>();
  const EmbedArgs ne{};
  const dim3 gx((unsigned)((a.Et + InitX32Geo::ROWS - 1) / InitX32Geo::ROWS)), bx(InitX32Geo::THREADS);
  if (dt == DI_BF16 && gc) hipLaunchKernelGGL((k_init_x32<true>), gx, bx, 0, s, a, ne, 0);
  else if (dt == DI_BF16) hipLaunchKernelGGL((k_init_x32<false>), gx, bx, 0, s, a, ne, 0);
  else if (gc) hipLaunchKernelGGL((k_init_edge<F32T, true>), gf, bf, 0, s, a, ne, 0);
  else hipLaunchKernelGGL((k_init_edge<F32T, false>), gf, bf, 0, s, a, ne, 0);
  return launch_status();
}

template <class DT>
static void launch_embed_init(const InitArgs& a, const EmbedArgs& ea, hipStream_t s) {
  using G = InitGeo<DT>;
  if constexpr (DT::kBF16) {
    const int eb = (ea.Nt + InitX32Geo::EMBED_ROWS - 1) / InitX32Geo::EMBED_ROWS;
    const int ib = (a.Et + InitX32Geo::ROWS - 1) / InitX32Geo::ROWS;
    hipLaunchKernelGGL((k_init_x32<true>), dim3((unsigned)(eb + ib)), dim3(InitX32Geo::THREADS), 0, s, a, ea, eb);
    return;
  }
  const int eb = (ea.Nt + G::ROWS - 1) / G::ROWS;
  const int ib = (a.Et + G::ROWS - 1) / G::ROWS;
  hipLaunchKernelGGL((k_init_edge<DT, true>), dim3((unsigned)(eb + ib)), block_of<G>(), 0, s, a, ea, eb);
}

extern "C" int di_embed_init_edge(const di_graph* g, di_dtype dt, int32_t in_dim, const float* node_f,
                                  const void* embed_wmat, const float* embed_wvec, void* h_out, void* qkv_out,
                                  const float* edge_f, const void* init_wmat, const float* init_wvec,
                                  const float* pos_src_tab, const float* pos_dst_tab, void* f_out, void* queue,
                                  int32_t signal_job, void* stream) {
  if (!g || !(g->flags & DI_GRAPH_GEO_REF) || !g->src || !g->dst || !g->node_pos || g->num_nodes <= 0 ||
      g->num_edges <= 0 || in_dim <= 0 || in_dim > HID || !node_f || !embed_wmat || !embed_wvec || !h_out ||
      !qkv_out || !edge_f || !init_wmat || !init_wvec || !pos_src_tab || !pos_dst_tab || !f_out || !dtype_ok(dt))
    return DI_EINVAL;
  EmbedArgs ea{g->num_nodes, in_dim, node_f, embed_wmat, embed_wvec, h_out, qkv_out, (uint32_t*)queue, signal_job};
  InitArgs a{g->num_edges, edge_f, g->src, g->dst, g->node_pos, init_wmat, init_wvec, pos_src_tab, pos_dst_tab,
             f_out, nullptr};
  if (dt == DI_BF16) launch_embed_init<BF16T>(a, ea, (hipStream_t)stream);
  else launch_embed_init<F32T>(a, ea, (hipStream_t)stream);
  return launch_status();
}

extern "C" int di_init_edge_resident(const di_graph* g, const float* edge_f, const void* wmat, const float* wvec,
                                     const float* pos_src_tab, const float* pos_dst_tab, void* f_out, void* stream) {
  if (!g || !(g->flags & DI_GRAPH_GEO_REF) || !g->src || !g->dst || !g->node_pos || !edge_f || !wmat || !wvec ||
      !pos_src_tab || !pos_dst_tab || !f_out || g->num_edges <= 0)
    return DI_EINVAL;
  InitArgs a{g->num_edges, edge_f, g->src, g->dst, g->node_pos, wmat, wvec, pos_src_tab, pos_dst_tab, f_out, nullptr};
  // one block per CU holding the path's weights; never more blocks than the tiles need
  const int cus = device_cus();
  const int ntiles = (a.Et + 31) / 32;
  const int need = (ntiles + IRX_NW - 1) / IRX_NW;
  hipLaunchKernelGGL(k_init_res_x32, dim3((unsigned)(need < cus ? need : cus)), dim3(64 * IRX_NW), 0,
                     (hipStream_t)stream, a, ntiles);
  return launch_status();
}

static int edge_layer(const di_graph* g, di_dtype dt, int final_layer, const float* edge_f, const void* f_in,
                      const void* fn_in, const void* qkv, const void* wmat, const float* wvec, float* alpha_out,
                      void* f_out, void* fn_out, float* attn_out, float* attn_parts, void* stream) {
  // DI_GRAPH_GEO_REF: the neighbour-message branch is skipped (exactly zero), fn_in is not read and
  // fn_out not written (every edge-layer kernel; di_conformation computes the branch)
  const bool gc = g && (g->flags & DI_GRAPH_GEO_REF);
  const bool fold = attn_out != nullptr;
  if (!g || !edge_f || !f_in || (!fn_in && !gc) || !qkv || !wmat || !wvec || (!alpha_out && !fold) ||
      g->num_edges <= 0 || !dtype_ok(dt))
    return DI_EINVAL;
  if (fold && (dt != DI_BF16 || !attn_parts || !g->in_ptr || !g->src || !g->dst)) return DI_EINVAL;
  if (!final_layer && (!f_out || (!fn_out && !gc))) return DI_EINVAL;
  EdgeArgs a{g->num_edges, edge_f, g->src, g->dst, g->nbr, f_in, fn_in, qkv, wmat, wvec, alpha_out,
             f_out, fn_out, attn_out, attn_parts, g->in_ptr};
  hipStream_t s = (hipStream_t)stream;
  if (dt == DI_BF16) {
    // persistent 8-wave blocks on the weight ring, one per CU (k_edge_x32_ring)
    const int ntiles = (a.Et + EdgeRingGeo::ROWS - 1) / EdgeRingGeo::ROWS;
    const int cus = device_cus();
    const dim3 grid((unsigned)(ntiles < cus ? ntiles : cus)), block(EdgeRingGeo::THREADS);
    if (final_layer && gc) hipLaunchKernelGGL((k_edge_x32_ring<1, true>), grid, block, 0, s, a, ntiles);
    else if (final_layer) hipLaunchKernelGGL((k_edge_x32_ring<1, false>), grid, block, 0, s, a, ntiles);
    else if (gc) hipLaunchKernelGGL((k_edge_x32_ring<0, true>), grid, block, 0, s, a, ntiles);
    else hipLaunchKernelGGL((k_edge_x32_ring<0, false>), grid, block, 0, s, a, ntiles);
  } else {
    const dim3 grid = grid_of<Geo<F32T>>(a.Et), block = block_of<Geo<F32T>>();
    if (final_layer && gc) hipLaunchKernelGGL((k_edge_layer<F32T, 1, true>), grid, block, 0, s, a);
    else if (final_layer) hipLaunchKernelGGL((k_edge_layer<F32T, 1>), grid, block, 0, s, a);
    else if (gc) hipLaunchKernelGGL((k_edge_layer<F32T, 0, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_edge_layer<F32T, 0>), grid, block, 0, s, a);
  }
  return launch_status();
}

extern "C" int di_edge_layer(const di_graph* g, di_dtype dt, int final_layer, const float* edge_f,
                             const void* f_in, const void* fn_in, const void* qkv, const void* wmat,
                             const float* wvec, float* alpha_out, void* f_out, void* fn_out,
                             void* stream) {
  return edge_layer(g, dt, final_layer, edge_f, f_in, fn_in, qkv, wmat, wvec, alpha_out, f_out, fn_out, nullptr,
                    nullptr, stream);
}

extern "C" int64_t di_attn_parts_bytes(int32_t num_edges) {
  if (num_edges <= 0) return DI_EINVAL;
  return (int64_t)((num_edges + FOLD_ROWS - 1) / FOLD_ROWS) * 2 * FOLD_PART * (int64_t)sizeof(float);
}

extern "C" int di_edge_layer_attn(const di_graph* g, di_dtype dt, int final_layer, const float* edge_f,
                                  const void* f_in, const void* fn_in, const void* qkv, const void* wmat,
                                  const float* wvec, float* alpha_out, void* f_out, void* fn_out, float* attn_out,
                                  float* attn_parts, void* stream) {
  if (!attn_out) return DI_EINVAL;
  return edge_layer(g, dt, final_layer, edge_f, f_in, fn_in, qkv, wmat, wvec, alpha_out, f_out, fn_out, attn_out,
                    attn_parts, stream);
}

extern "C" int di_conformation(const di_graph* g, di_dtype dt, const float* edge_f, const void* f_in,
                               const void* fn_in, const void* wmat, const float* wvec, void* conf_out,
                               void* stream) {
  if (!g || !edge_f || !f_in || !fn_in || !wmat || !wvec || !conf_out || g->num_edges <= 0 || !dtype_ok(dt))
    return DI_EINVAL;
  EdgeArgs a{g->num_edges, edge_f, g->src, g->dst, g->nbr, f_in, fn_in, nullptr, wmat, wvec, nullptr,
             conf_out, nullptr};
  hipStream_t s = (hipStream_t)stream;
  if (dt == DI_BF16)
    hipLaunchKernelGGL((k_edge_layer<BF16T, 2>), grid_of<Geo<BF16T>>(a.Et), block_of<Geo<BF16T>>(), 0, s, a);
  else
    hipLaunchKernelGGL((k_edge_layer<F32T, 2>), grid_of<Geo<F32T>>(a.Et), block_of<Geo<F32T>>(), 0, s, a);
  return launch_status();
}

extern "C" int di_node_layer(const di_graph* g, di_dtype dt, int final_layer, const float* alpha,
                             const void* h_in, const void* qkv, const void* wmat, const float* wvec,
                             void* h_out, void* qkv_out, void* hT_out, void* stream) {
  if (!g || !alpha || !h_in || !qkv || !wmat || !wvec || !h_out || g->num_nodes <= 0 || !dtype_ok(dt))
    return DI_EINVAL;
  if (!final_layer && !qkv_out) return DI_EINVAL;
  NodeArgs a{g->num_nodes, nullptr, hT_out, g->src, g->in_ptr, alpha, h_in, qkv, wmat, wvec, h_out, qkv_out};
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid = grid_of<NodeGeo>(a.Nt), block = block_of<NodeGeo>();
  if (dt == DI_BF16) {
    // persistent weight-stationary blocks, one per CU, 32-destination tiles (k_node_ws)
    if (!g->src || !g->in_ptr) return DI_EINVAL;
    // the segment sums address V rows and alphas by 32-bit buffer offsets
    if ((int64_t)a.Nt * 3 * HID * 2 >= (1LL << 31) || (int64_t)g->num_edges * 16 >= (1LL << 31)) return DI_ERANGE;
    const int ntiles = (a.Nt + NWS_TILE - 1) / NWS_TILE;
    const int cus = device_cus();
    const dim3 gw((unsigned)(ntiles < cus ? ntiles : cus)), bw(64 * NWS_NW);
    if (final_layer) hipLaunchKernelGGL((k_node_ws<true>), gw, bw, 0, s, a, ntiles);
    else hipLaunchKernelGGL((k_node_ws<false>), gw, bw, 0, s, a, ntiles);
  } else {
    if (final_layer) hipLaunchKernelGGL((k_node_layer<F32T, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_node_layer<F32T, false>), grid, block, 0, s, a);
  }
  return launch_status();
}

extern "C" int di_node_aggregate(const di_graph* g, di_dtype dt, const float* alpha, const void* qkv, float* attn_out,
                                 void* stream) {
  if (!g || !alpha || !qkv || !attn_out || !g->src || !g->in_ptr || g->num_nodes <= 0 || !dtype_ok(dt))
    return DI_EINVAL;
  AggrArgs a{g->num_nodes, g->src, g->in_ptr, alpha, qkv, attn_out};
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((a.Nt + AGG_NODES - 1) / AGG_NODES)), block(16 * AGG_NODES);
  if (dt == DI_BF16) hipLaunchKernelGGL(k_node_aggr<BF16T>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(k_node_aggr<F32T>, grid, block, 0, s, a);
  return launch_status();
}

static int node_update(const di_graph* g, di_dtype dt, int final_layer, const float* attn, const float* attn_parts,
                       const void* h_in, const void* wmat, const float* wvec, void* h_out, void* qkv_out, void* hT_out,
                       void* stream) {
  if (!g || !attn || !h_in || !wmat || !wvec || !h_out || g->num_nodes <= 0 || !dtype_ok(dt)) return DI_EINVAL;
  if (!final_layer && !qkv_out) return DI_EINVAL;
  if (attn_parts && !g->in_ptr) return DI_EINVAL;
  NodeArgs a{g->num_nodes, attn, hT_out, nullptr, attn_parts ? g->in_ptr : nullptr, nullptr, h_in, nullptr, wmat,
             wvec, h_out, qkv_out, attn_parts};
  hipStream_t s = (hipStream_t)stream;
  if (dt == DI_BF16) {
    const dim3 grid = grid_of<NodeRingGeo>(a.Nt), block = block_of<NodeRingGeo>();
    if (final_layer) hipLaunchKernelGGL((k_node_update_ring<true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_node_update_ring<false>), grid, block, 0, s, a);
  } else {
    const dim3 grid = grid_of<NodeGeo>(a.Nt), block = block_of<NodeGeo>();
    if (final_layer) hipLaunchKernelGGL((k_node_layer<F32T, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_node_layer<F32T, false>), grid, block, 0, s, a);
  }
  return launch_status();
}

extern "C" int di_node_update(const di_graph* g, di_dtype dt, int final_layer, const float* attn, const void* h_in,
                              const void* wmat, const float* wvec, void* h_out, void* qkv_out, void* hT_out,
                              void* stream) {
  return node_update(g, dt, final_layer, attn, nullptr, h_in, wmat, wvec, h_out, qkv_out, hT_out, stream);
}

extern "C" int di_node_update_folded(const di_graph* g, di_dtype dt, int final_layer, const float* attn,
                                     const float* attn_parts, const void* h_in, const void* wmat, const float* wvec,
                                     void* h_out, void* qkv_out, void* hT_out, void* stream) {
  if (!attn_parts) return DI_EINVAL;
  return node_update(g, dt, final_layer, attn, attn_parts, h_in, wmat, wvec, h_out, qkv_out, hT_out, stream);
}
