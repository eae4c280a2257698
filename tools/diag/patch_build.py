"""Timing-diagnostic builds of the library from PATCHED COPIES of csrc/ (never -D knobs in the
product sources): each diagnostic is a list of exact text substitutions applied to a copy of
deepinteract_amd/csrc + include/, built into deepinteract_amd/lib/variants/diag_<name>/ and loaded
with bench.py --lib. Every diagnostic computes WRONG results on purpose (timing only), except the
A/B variants marked as such (one-line launch / pipeline changes measured against the product).

usage: python tools/diag/patch_build.py nosilu nosync w0 initnopos initnostore initw0 ...
"""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from deepinteract_amd import build  # noqa: E402

DIAGS = {
    # the edge layers' SiLU epilogues as a plain multiply (no transcendentals): how much of the step a
    # faster GeoT converts into throughput
    "nosilu": [("mfma32.h", "for (int k = 0; k < 16; ++k) v[k] = silu2<true>(v[k]);",
                "for (int k = 0; k < 16; ++k) v[k] = v[k] * 0.5f;", 1)],
    # the double-buffered weight stages switch without waiting for their LDS-DMA or a barrier
    "nosync": [("common.h", """    if constexpr (DBUF) {
      lds_dma_wait();
      __syncthreads();
      cur ^= 1;""", """    if constexpr (DBUF) {
      cur ^= 1;""", 1)],
    # every bf16 edge-layer weight stage DMA'd from the blob's first blocks: the weight stream always
    # hits L2 (same bytes, same instruction count; wrong weights)
    "w0": [("geot_kernels.hip", "    pipe.issue(W + EL_ORDER[si] * BLK, EL_SIZE[si], vo >= 0 ? V + vo : nullptr, 128);\n  }\n  __device__ const u16* next() {",
            "    pipe.issue(W, EL_SIZE[si], vo >= 0 ? V : nullptr, 128);\n  }\n  __device__ const u16* next() {", 1)],
    # InitEdge (k_init_x32) without the positional-table gathers: acc starts at zero
    "initnopos": [("geot_kernels.hip", "  init_acc_x32(acc, a, a.node_pos[a.src[e]], a.node_pos[a.dst[e]], h);\n  const bool with_fn",
                   "  zero(acc);\n  const bool with_fn", 1)],
    # InitEdge without its F row stores (kept alive by a never-true condition)
    "initnostore": [("geot_kernels.hip", "  if (valid) store_row32(f, reinterpret_cast<u16*>(a.f_out) + (int64_t)e * HID, h);\n  if (!with_fn) return;",
                     "  if (valid && f.v[0][0] == 1.2345e30f) store_row32(f, reinterpret_cast<u16*>(a.f_out) + (int64_t)e * HID, h);\n  if (!with_fn) return;", 1)],
    # InitEdge's weight phases all DMA'd from the blob's first blocks (L2-resident; wrong weights)
    "initw0": [("geot_kernels.hip", """    if (p == 0) pipe.issue(W + (IE_T0 + 40 * geo_t(0)) * BLK, 40);
    else if (p < NT) pipe.issue(W + (IE_T0 + 40 * geo_t(p)) * BLK, 40);
    else if (p == NT) pipe.issue(W + IE_GEO1 * BLK, 40);
    else if (p == NT + 1) pipe.issue(W + IE_C1 * BLK, 16);""", """    if (p == 0) pipe.issue(W, 40);
    else if (p < NT) pipe.issue(W, 40);
    else if (p == NT) pipe.issue(W, 40);
    else if (p == NT + 1) pipe.issue(W, 16);""", 1)],
    # A/B variants with CORRECT results (timing comparisons of one-line changes, never shipped):
    # the edge ring issuing each weight stage three stages ahead (two in the product)
    "ahead3": [("geot_kernels.hip", "constexpr int RING_NW = 8, RING_SLOTS = 4, RING_AHEAD = 2;",
                "constexpr int RING_NW = 8, RING_SLOTS = 4, RING_AHEAD = 3;", 1)],
    # InitEdge (k_init_x32) in 6-wave blocks, two per CU (four-wave blocks, three per CU, in the
    # product): 192 instead of 128 edges per weight pass
    "init6": [("geot_kernels.hip", "constexpr int INIT_X32_NW = 4;", "constexpr int INIT_X32_NW = 6;", 1)],
    # the persistent edge ring on 8 CUs fewer than the device has: room for a collective's blocks
    # beside it (the chunked gather's exposure)
    "ring248": [("geot_kernels.hip", "const dim3 grid((unsigned)(ntiles < cus ? ntiles : cus)), block(EdgeRingGeo::THREADS);",
                 "const dim3 grid((unsigned)(ntiles < cus - 8 ? ntiles : cus - 8)), block(EdgeRingGeo::THREADS);", 1)],
    # k_node_fast's second half of Q|K|V fragments loaded inside the Q|K|V loop (after the last
    # barrier) instead of right after the FFN-output MFMAs
    "qkvjit": [("geot_kernels.hip", """    if constexpr (!FINAL) {
      if (q == NG - 1) {
#pragma unroll
        for (int b = BQP; b < BQ; ++b)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            fq2[b - BQP][s] = frag(NL_Q + MAT128 * ((BQ * w + b) >> 3), (BQ * w + b) & 7, s);
      }
    }
    add_(n[q], o);""", """    add_(n[q], o);""", 1),
               ("geot_kernels.hip", "b < BQP ? fq[b][s] : fq2[b - BQP][s], hop.f[s], x, 0, 0, 0);",
                "b < BQP ? fq[b][s] : frag(NL_Q + MAT128 * (ob >> 3), ob & 7, s), hop.f[s], x, 0, 0, 0);", 1)],
    # round 6: the bf16 node layer as k_node_fast (16-destination blocks streaming the weights from L2)
    # instead of the weight-stationary k_node_ws
    "nodefast": [("geot_kernels.hip", """    if (final_layer) hipLaunchKernelGGL((k_node_ws<true>), gw, bw, 0, s, a, ntiles);
    else hipLaunchKernelGGL((k_node_ws<false>), gw, bw, 0, s, a, ntiles);""", """    (void)gw; (void)bw;
    const dim3 gf((unsigned)((a.Nt + NF_NODES - 1) / NF_NODES)), bf(256);
    if (final_layer) hipLaunchKernelGGL((k_node_fast<true, 1>), gf, bf, 0, s, a);
    else hipLaunchKernelGGL((k_node_fast<false, 1>), gf, bf, 0, s, a);""", 1)],
    # k_node_ws's segment sums in one chunk of 20 in-edges (one memory latency per tile; 5 VGPRs
    # spilled) instead of two chunks of 10 (round 6: slower, tools/sessions/r6_05_wsu.sh)
    "wsu20": [("geot_kernels.hip", "constexpr int SEG_U_WS = 10;", "constexpr int SEG_U_WS = 20;", 1)],
    # the pair stream's blocks on the first N XCDs only (block b runs on XCD b mod 8; the others exit at
    # once): can a few XCDs' L2s and fabric links carry the store stream? (round-5 verdict item 4)
    **{f"pairxcd{n}": [("pair_tensor.hip", """  const int lane = threadIdx.x & 63;
  for (int k = job_begin; k < job_end; ++k) {
    if (!pq_wait(q + PQ_READY, (uint32_t)k + 1, patience)) {""", f"""  const int lane = threadIdx.x & 63;
  if ((int)(blockIdx.x & 7) >= {n}) return;
  for (int k = job_begin; k < job_end; ++k) {{
    if (!pq_wait(q + PQ_READY, (uint32_t)k + 1, patience)) {{""", 1)] for n in (1, 2, 3, 4, 6)},
    # the LDS-resident InitEdge capped at 160 VGPRs (three waves per SIMD + one pair-stream wave fit;
    # uncapped it allocates 168, so a CU hosting a pair-stream block cannot take its 12-wave block)
    "initres160": [("geot_kernels.hip", """__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * IRX_NW), amdgpu_waves_per_eu(IRX_NW / 4, IRX_NW / 4)))
void k_init_res_x32(InitArgs a, int ntiles) {""", """__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * IRX_NW), amdgpu_waves_per_eu(IRX_NW / 4, IRX_NW / 4),
                          amdgpu_num_vgpr(80)))
void k_init_res_x32(InitArgs a, int ntiles) {""", 1)],
    # the node kernels' LDS exchange rows at round 6's first padding (132 / 68 / 132 words: 2-way
    # conflicts left) instead of the conflict-free 136 / 66 / 130
    "ldspad4": [("geot_kernels.hip", """constexpr int LDS_ATTN = HID + 8;       // fp32 aggregated rows: 136 words
constexpr int LDS_N = HID + 4;          // bf16 n / h rows: 66 words
constexpr int LDS_T = 2 * HID + 4;      // bf16 FFN-hidden rows: 130 words""", """constexpr int LDS_ATTN = HID + 4;
constexpr int LDS_N = HID + 8;
constexpr int LDS_T = 2 * HID + 8;""", 1)],
    # the beside store window: four stores in flight per pair wave (three in the product)
    "inflight4": [("pair_tensor.hip", "constexpr int PAIR_INFLIGHT = 3;", "constexpr int PAIR_INFLIGHT = 4;", 1)],
    "inflight2": [("pair_tensor.hip", "constexpr int PAIR_INFLIGHT = 3;", "constexpr int PAIR_INFLIGHT = 2;", 1)],
    "inflight6": [("pair_tensor.hip", "constexpr int PAIR_INFLIGHT = 3;", "constexpr int PAIR_INFLIGHT = 6;", 1)],
    # round 6, static issue priority (MI355X_MICROARCH.md, two waves per SIMD, item 4): the edge ring's
    # second-dispatched half (waves 4-7) at s_setprio 1 for the whole launch / the first half instead
    "prio47": [("geot_kernels.hip", "  st.fill();\n#pragma unroll 1\n", "  if (wave >= 4) __builtin_amdgcn_s_setprio(1);\n  st.fill();\n#pragma unroll 1\n", 1)],
    "prio03": [("geot_kernels.hip", "  st.fill();\n#pragma unroll 1\n", "  if (wave < 4) __builtin_amdgcn_s_setprio(1);\n  st.fill();\n#pragma unroll 1\n", 1)],
    # the edge ring's waves 4-7 start ~512 cycles late (a stagger against lockstep SIMD partners, item 9)
    "stag": [("geot_kernels.hip", "  st.fill();\n#pragma unroll 1\n", "  st.fill();\n  if (wave >= 4) __builtin_amdgcn_s_sleep(8);\n#pragma unroll 1\n", 1)],
    # k_node_ws's waves 4-7 at s_setprio 1
    "nodeprio": [("geot_kernels.hip", "  if constexpr (!FINAL) dma_blocks<NWS_NW>(s_q, W + NL_Q * BLK, 3 * MAT128);\n  // this wave's",
                  "  if (w >= 4) __builtin_amdgcn_s_setprio(1);\n  if constexpr (!FINAL) dma_blocks<NWS_NW>(s_q, W + NL_Q * BLK, 3 * MAT128);\n  // this wave's", 1)],
    # the pair stream's waves at s_setprio 2: their store instructions win issue over the GeoT waves
    # sharing their SIMD
    "pairprio": [("pair_tensor.hip", """  const int lane = threadIdx.x & 63;
  for (int k = job_begin; k < job_end; ++k) {
    if (!pq_wait(q + PQ_READY, (uint32_t)k + 1, patience)) {""", """  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_s_setprio(2);
  for (int k = job_begin; k < job_end; ++k) {
    if (!pq_wait(q + PQ_READY, (uint32_t)k + 1, patience)) {""", 1)],
    # InitEdge's positional rows read at half their bytes (features 0..63 twice: the traffic a bf16
    # copy of the fp32 tables would gather; timing only)
    "posh": [("geot_kernels.hip", """      const int f = 32 * b + 8 * q + 4 * h;
      set_quad(acc.v[b], q, ld4(rs + f) + ld4(rd + f));""", """      const int f = 32 * (b & 1) + 8 * q + 4 * h;
      set_quad(acc.v[b], q, ld4(rs + f) + ld4(rd + f));""", 1)],
    # CU-level spatial split of the two dedicated streams (environment-driven, diagnostic only):
    # DI_DIAG_GMASK=m takes m CUs per XCD away from the GeoT stream (and sizes its persistent grids to
    # the CUs left), DI_DIAG_PMASK=m puts the pair stream on exactly those m CUs per XCD (0: all CUs).
    # The set is balanced per XCD whether mask bit c maps to XCD c % 8 or to XCD c / 32: bit
    # c = 32 x + 8 j + y is in it iff (y - x) mod 8 < m / 4.
    "cusplit": [("streams.hip", """  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c >> 5] |= 1u << (c & 31);""", """  static int calls = 0;
  const int which = calls++ & 1;  // 0: the GeoT stream, 1: the pair stream (schedule_streams order)
  const char* ev = getenv(which ? "DI_DIAG_PMASK" : "DI_DIAG_GMASK");
  const int m = ev ? atoi(ev) : 0;
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) {
    const bool in = m > 0 && ((((c & 7) - (c >> 5)) & 7) < m / 4);
    if (which ? (m == 0 || in) : !in) mask[(size_t)c >> 5] |= 1u << (c & 31);
  }""", 1),
                ("geot_kernels.hip", "const int cus = device_cus();",
                 'const int cus = device_cus() - 8 * (getenv("DI_DIAG_GMASK") ? atoi(getenv("DI_DIAG_GMASK")) : 0);', 3)],
    # the edge ring's three re-reads of the edge's own F row (res_connect, final_linear, O_edge) from
    # rows 0..31 instead (always L2-hot): the most keeping F on chip could buy (timing only)
    "reread0": [("geot_kernels.hip", "  const u16* f_row = reinterpret_cast<const u16*>(a.f_in) + (int64_t)e * HID;\n  const u16* qkv",
                 "  const u16* f_row = reinterpret_cast<const u16*>(a.f_in) + (int64_t)e * HID;\n"
                 "  const u16* f_row0 = reinterpret_cast<const u16*>(a.f_in) + (int64_t)(e & 31) * HID;\n  const u16* qkv", 1),
                ("geot_kernels.hip", "  fr.load(f_row, h);\n  w = st.next([&] { settle(fr); });  // res_connect_linear",
                 "  fr.load(f_row0, h);\n  w = st.next([&] { settle(fr); });  // res_connect_linear", 1),
                ("geot_kernels.hip", "  fr.load(f_row, h);\n  w = st.next([&] { settle(fr); });  // final_linear",
                 "  fr.load(f_row0, h);\n  w = st.next([&] { settle(fr); });  // final_linear", 1),
                ("geot_kernels.hip", "    fr.load(f_row, h);                 // O_edge: re-read",
                 "    fr.load(f_row0, h);                 // O_edge: re-read", 1)],
    # the edge ring's weight stages DMA'd at half their blocks (the slot's second half keeps stale
    # weights; timing only): how much of the edge layers' cost to the pair stream is their L2 -> LDS
    # weight stream (~16 TB/s of L2 reads chip-wide while the ring runs)
    "whalf": [("geot_kernels.hip", "    return {W, {EL_ORDER[si], 0, 0}, {EL_SIZE[si], 0, 0}, 1, vo >= 0 ? V + vo : nullptr};",
               "    return {W, {EL_ORDER[si], 0, 0}, {EL_SIZE[si] / 2, 0, 0}, 1, vo >= 0 ? V + vo : nullptr};", 1)],
    # the edge ring's weight stages all DMA'd from the blob's first blocks (same bytes, a 36-KiB
    # footprint that always hits L2; timing only): separates the stream's L2 misses from its bytes
    "ringw0": [("geot_kernels.hip", "    return {W, {EL_ORDER[si], 0, 0}, {EL_SIZE[si], 0, 0}, 1, vo >= 0 ? V + vo : nullptr};",
                "    return {W, {0, 0, 0}, {EL_SIZE[si], 0, 0}, 1, vo >= 0 ? V + vo : nullptr};", 1)],
    # the edge ring's blocks of one XCD kept in step: after each tile (but a block's last ones), wave 0
    # adds to its XCD's counter and waits (<= 20 us) until every block of the XCD has finished that
    # tile, so the 32 blocks stay within one tile of each other and fewer of the layer's weight stages
    # are live in the XCD's L2 at once (the stream's L2 misses). Results
    # unchanged (A/B variant, correct outputs)
    "xcdbar": [("geot_kernels.hip", """  const int* in_ptr = nullptr;
};

struct NodeArgs {""", """  const int* in_ptr = nullptr;
  uint32_t* xbar = nullptr;  // diag xcdbar: per-XCD tile counters (16 words apart)
};

struct NodeArgs {""", 1),
               ("geot_kernels.hip", """    edge_x32_tile<MODE, GC>(a, st, e, valid, lane, h);
  }
}""", """    edge_x32_tile<MODE, GC>(a, st, e, valid, lane, h);
    const int G = (int)gridDim.x, x = (int)(blockIdx.x & 7);
    if (a.xbar && wave == 0 && (G & 7) == 0 && i + 1 < ntiles / G) {
      uint32_t* c = a.xbar + 16 * x;
      const uint32_t need = (uint32_t)((i + 1) * (G / 8));
      if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need &&
             __builtin_amdgcn_s_memrealtime() - t0 < 2000)
        __builtin_amdgcn_s_sleep(2);
    }
  }
}""", 1),
               ("geot_kernels.hip", """    const dim3 grid((unsigned)(ntiles < cus ? ntiles : cus)), block(EdgeRingGeo::THREADS);
    if (final_layer && gc) hipLaunchKernelGGL((k_edge_x32_ring<1, true>), grid, block, 0, s, a, ntiles);""",
                """    const dim3 grid((unsigned)(ntiles < cus ? ntiles : cus)), block(EdgeRingGeo::THREADS);
    static uint32_t* xbar = nullptr;
    if (!xbar && hipMalloc(&xbar, 8 * 16 * sizeof(uint32_t)) != hipSuccess) xbar = nullptr;
    if (xbar && hipMemsetAsync(xbar, 0, 8 * 16 * sizeof(uint32_t), s) == hipSuccess) a.xbar = xbar;
    if (final_layer && gc) hipLaunchKernelGGL((k_edge_x32_ring<1, true>), grid, block, 0, s, a, ntiles);""", 1)],
}
# combinations (every substitution of each part)
DIAGS["prio47node"] = DIAGS["prio47"] + DIAGS["nodeprio"]
DIAGS["prio47pair"] = DIAGS["prio47"] + DIAGS["pairprio"]


def build_diag(name):
    tmp = tempfile.mkdtemp(prefix=f"di_diag_{name}_")
    try:
        src = os.path.join(tmp, "deepinteract_amd", "csrc")
        shutil.copytree(build.CSRC, src)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        for fname, old, new, count in DIAGS[name]:
            p = os.path.join(src, fname)
            text = open(p).read()
            if text.count(old) != count:
                raise SystemExit(f"diag {name}: pattern found {text.count(old)}x in {fname}, expected {count}")
            open(p, "w").write(text.replace(old, new))
        out = os.path.join(build.LIBDIR, "variants", f"diag_{name}", "libdeepinteract_amd.so")
        saved = build.CSRC, build.CFLAGS
        build.CSRC = src
        build.CFLAGS = [f for f in build.CFLAGS if not f.startswith("-I")] + [f"-I{os.path.join(tmp, 'include')}"]
        try:
            return build.build(force=True, defines=[f"DI_TIMING_DIAG_{name.upper()}=1"], out=out)
        finally:
            build.CSRC, build.CFLAGS = saved
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(DIAGS):
        print(build_diag(n))
