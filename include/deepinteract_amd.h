/*
 * deepinteract_amd — C ABI of the MI355X (gfx950) GeoT hot path.
 *
 * Plain pointers and sizes only: every pointer argument is a DEVICE pointer unless stated;
 * every call is asynchronous on `stream` (a hipStream_t passed as void*); no call allocates
 * device memory; every call returns 0 or a hipError_t code (>0) or a negative DI_E* code.
 *
 * Each entry point replaces one piece of the reference's DGL/ATen hot path (file:line cited
 * relative to /root/reference/project/utils/):
 *
 *   di_node_embed   LitGINI.gnn_forward node_in_embedding            deepinteract_modules.py:1663-1664
 *                   + layer-0 Q/K/V of MultiHeadGeometricAttention   deepinteract_modules.py:101-103
 *   di_init_edge    InitEdgeModule.forward / message UDF             deepinteract_modules.py:198-264
 *   di_edge_layer   ConformationModule (:373-455) + attention edge UDFs (:76-91, graph_utils.py:21-63)
 *                   + O_edge/edge FFN of GeometricTransformerModule  deepinteract_modules.py:669-727
 *   di_node_layer   send_and_recv(u_mul_e/copy_e, sum) gSpMM         deepinteract_modules.py:93-96,116
 *   di_edge_layer_attn / di_node_update_folded: the same gSpMM folded into the edge layer (bf16)
 *                   + O_node / node FFN                               deepinteract_modules.py:696-723, 923-943
 *   di_pair_tensor  construct_interact_tensor (pad=False)            deepinteract_utils.py:158-172
 *   di_pair_stream / di_pair_help / di_pair_signal: the same, per micro-batch, as a device queue beside
 *                   the GeoT stream (lit_model_predict.py:236 calls it once per complex)
 *   di_head_prologue  ELU(inorm_1(conv2d_1(T))) of the head, T never materialised
 *                                                                    deepinteract_modules.py:1181-1184, 1228-1232
 *   di_inorm_elu    ELU(InstanceNorm2d(x)) of the head's ResNet blocks deepinteract_modules.py:1016-1030,1075-1095
 *   di_se_scale_add conv bias + SEBlock gate + residual add          deepinteract_modules.py:954-970, 1095
 *   di_channel_mean SEBlock squeeze (channel mean)                   deepinteract_modules.py:966
 *   di_knn_topk     dgl.knn_graph + topk(pairwise_squared_distance)  graph_utils.py:107-108
 *   di_knn_graph    knn_graph's edge list / in-edge CSR (src, dst)   graph_utils.py:107, deepinteract_utils.py:442-443
 *   di_geo_feats    GeometricProteinFeatures('full') + edge/node feature assembly
 *                                                                    protein_feature_utils.py:322-377,
 *                                                                    deepinteract_utils.py:474-530
 *   di_build_nbr_ids  per-edge neighbour-edge ids                    deepinteract_utils.py:534-553
 *   di_build_nbr_ids_torch  the same, bit-exact with torch.randperm  deepinteract_utils.py:539-546
 *
 * Module-at-a-time entry points (deepinteract_amd/layers.py; same math as the fused kernels):
 *   di_conformation   ConformationModule.forward                      deepinteract_modules.py:373-455
 *   di_gemm_bias_act  nn.Linear (+ folded BatchNorm, + SiLU, + residual) of the GeoT modules
 *                                                                    deepinteract_modules.py:99-104, 696-723
 *   di_geo_attention  MultiHeadGeometricAttentionLayer.propagate_attention + h = wV/(z+1e-6)
 *                                                                    deepinteract_modules.py:76-121
 */
#ifndef DEEPINTERACT_AMD_H
#define DEEPINTERACT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DI_ABI_VERSION 8

/* activation / weight storage type of the GeoT kernels (accumulation is always fp32). A plain
 * int32 (not a C enum type): a foreign caller may pass any value, and every entry point refuses
 * values other than DI_F32 / DI_BF16 with DI_EINVAL (a C++ enum holding 5 would be undefined
 * behaviour before the check could run; found by the host UBSan build). */
enum { DI_F32 = 0, DI_BF16 = 1 };
typedef int32_t di_dtype;

enum {
  DI_OK = 0,
  DI_EINVAL = -1,   /* bad shape / null pointer / unsupported config */
  DI_ERANGE = -2,   /* a size beyond the kernels' index range (see each entry point) */
};

/* A batch of residue graphs (one graph per chain, concatenated). Edges are destination-major:
 * the in-edges of node v are edge ids in_ptr[v] .. in_ptr[v+1]-1. All ids are GLOBAL to the batch. */
typedef struct {
  int32_t num_nodes;        /* Nt */
  int32_t num_edges;        /* Et */
  const int32_t* src;       /* [Et] source node of each edge */
  const int32_t* dst;       /* [Et] destination node of each edge */
  const int32_t* nbr;       /* [Et,4] src_nbr_e_ids[0:2], dst_nbr_e_ids[0:2] */
  const int32_t* node_pos;  /* [Nt] node index inside its chain (positional-embedding row) */
  const int32_t* in_ptr;    /* [Nt+1] CSR row pointer of in-edges by destination */
  int32_t flags;            /* DI_GRAPH_* properties of the batch's edge features (0: none known) */
} di_graph;

/* di_graph.flags bit: every edge's direction columns edge_f[:, 20:23] are 0 and its orientation
 * columns edge_f[:, 23:27] are (0, 0, 0, 1) -- what the reference featuriser produces for every
 * kNN graph (GeometricProteinFeatures is called with E_idx = the destination node itself,
 * deepinteract_utils.py:474-477, so dU = normalize(0) = 0 and the relative rotation is the
 * identity quaternion). With all direction features zero, the conformation module's neighbour
 * messages are multiplied by dir_linear_1(dir_linear_0(0)) = 0 (both bias-free,
 * deepinteract_modules.py:301-302, :408), so that branch is exactly zero and the gathered
 * silu(nbr_linear(F)) rows are never needed; InitEdge's direction terms are silu(0) = 0 and its
 * orientation terms are per-model constants. With this flag:
 *   di_init_edge  skips the direction terms, adds the orientation terms as packed constants, and
 *                 writes fn_out only when fn_out != NULL;
 *   di_edge_layer skips the neighbour-message branch: fn_in is not read and fn_out is not
 *                 written (both may be NULL).
 * di_conformation ignores the flag (it computes the branch, which is exactly zero). */
#define DI_GRAPH_GEO_REF 1

/* one complex of a pair-tensor launch (host-built array copied to the device) */
typedef struct {
  int64_t h1_row;   /* first node row of chain 1 in the node-feature matrix */
  int64_t h2_row;   /* first node row of chain 2 */
  int64_t out_off;  /* element offset of this complex's [2H, L1, L2] block in `out` */
  int32_t l1, l2;
} di_pair_desc;

int di_abi_version(void);
/* bytes of the packed weight blobs a kernel expects: kind = 0 embed, 1 init_edge,
 * 2 edge_layer(non-final), 3 edge_layer(final), 4 node_layer(non-final), 5 node_layer(final).
 * `vec` selects the fp32 vector blob (biases) instead of the matrix blob. */
int64_t di_blob_bytes(int kind, di_dtype dtype, int vec);
/* MFMA fragment order of a kind's matrix blob (ABI 5): 16 = blocks of 16 output rows x 32 input
 * features (v_mfma_f32_16x16x32_bf16 / 16x16x4_f32 A fragments), 32 = blocks of 32 output rows x 16
 * input features (v_mfma_f32_32x32x16_bf16: the bf16 InitEdge and edge-layer blobs, kinds 1, 2 and 3;
 * the kind-1 32 order also carries the DI_GRAPH_GEO_REF orientation constant as a bf16 hi/lo pair in
 * columns 28/29 of the collapsed message map); -1 for an unknown kind or dtype. Both orders hold the
 * same number of 512-element blocks at the same block offsets (deepinteract_amd/packing.py:
 * pack_matrix / pack_matrix32, init_blob / edge_blob with layout = di_blob_layout(kind, dtype)). */
int di_blob_layout(int kind, di_dtype dtype);

/* in_dim: width of node_f rows (113 for LitGINI's raw node features; 128 with an identity
 * embedding when DGLGeometricTransformer is used standalone on already-embedded features).
 * queue / signal_job (ABI 6; NULL / -1: none): a pair-queue signal carried by this launch -- at its
 * start it marks job signal_job ready, i.e. what di_pair_signal(queue, signal_job) issued just before
 * it on `stream` would do, without that launch (the producer of signal_job's hT must precede this
 * launch on `stream`). Same pair on di_embed_init_edge and di_pair_help. */
int di_node_embed(const di_graph* g, di_dtype dt, int32_t in_dim, const float* node_f /*[Nt,in_dim]*/,
                  const void* wmat, const float* wvec,
                  void* h_out /*[Nt,128]*/, void* qkv_out /*[Nt,384]*/, void* queue, int32_t signal_job,
                  void* stream);

int di_init_edge(const di_graph* g, di_dtype dt, const float* edge_f /*[Et,28]*/,
                 const void* wmat, const float* wvec,
                 const float* pos_src_tab /*[2304,128]*/, const float* pos_dst_tab /*[2304,128]*/,
                 void* f_out /*[Et,128]*/, void* fn_out /*[Et,128]*/, void* stream);
/* The same InitEdge for bf16 DI_GRAPH_GEO_REF batches without layer-0 Fn rows, with the 128 KiB of
 * weight blocks that path reads resident in LDS (one block per CU; waves stride over 16-edge tiles):
 * F bit-identical to di_init_edge. A scheduling choice of this build: faster alone, but its block
 * holds 128 KiB of a CU's 160 KiB LDS, so LDS-staged kernels of other streams (the node embedding)
 * cannot run beside it. DI_EINVAL for batches without DI_GRAPH_GEO_REF. */
int di_init_edge_resident(const di_graph* g, const float* edge_f /*[Et,28]*/, const void* wmat /*bf16 blob*/,
                          const float* wvec, const float* pos_src_tab, const float* pos_dst_tab,
                          void* f_out /*[Et,128] bf16*/, void* stream);
/* di_node_embed + di_init_edge (DI_GRAPH_GEO_REF, no Fn) as ONE launch: the embedding runs as the
 * launch's first blocks, beside InitEdge's, through the same LDS slot -- instead of on a side
 * stream. h_out / qkv_out / f_out bit-identical to the two separate calls. 0 < in_dim <= 128.
 * ABI 5: any dtype (fp32 added: the embedding of the reference's precision inside the launch). */
int di_embed_init_edge(const di_graph* g, di_dtype dt, int32_t in_dim, const float* node_f /*[Nt,in_dim]*/,
                       const void* embed_wmat, const float* embed_wvec, void* h_out /*[Nt,128]*/,
                       void* qkv_out /*[Nt,384]*/, const float* edge_f, const void* init_wmat, const float* init_wvec,
                       const float* pos_src_tab, const float* pos_dst_tab, void* f_out /*[Et,128]*/, void* queue,
                       int32_t signal_job, void* stream);

int di_edge_layer(const di_graph* g, di_dtype dt, int final_layer, const float* edge_f,
                  const void* f_in, const void* fn_in, const void* qkv,
                  const void* wmat, const float* wvec,
                  float* alpha_out /*[Et,4]*/, void* f_out, void* fn_out, void* stream);

/* hT_out (optional, may be NULL): also write h_out transposed, [128, Nt] (pair-tensor input).
 * bf16: DI_ERANGE when Nt * 768 or Et * 16 reaches 2^31 (the segment sums use 32-bit byte offsets;
 * split such a batch, or use di_node_aggregate + di_node_update). */
int di_node_layer(const di_graph* g, di_dtype dt, int final_layer, const float* alpha,
                  const void* h_in, const void* qkv, const void* wmat, const float* wvec,
                  void* h_out, void* qkv_out, void* hT_out, void* stream);
/* The node layer in two launches (what GeoTEngine runs): the attention aggregation as a CSR
 * segment reduction over each node's in-edges (replaces send_and_recv(u_mul_e, sum) +
 * (copy_e, sum) + wV / (z + 1e-6), deepinteract_modules.py:93-96, 116):
 *   attn_out[v, :] = sum_{e: dst(e) = v} alpha[e, head] * V[src(e), :] / (sum_e alpha[e, head] + 1e-6)
 * (fp32 [Nt, 128]; V = columns 256..383 of qkv), then O_node + residual + FFN (+ next layer's
 * Q/K/V, + optional transposed copy) from those rows. Bit-identical to di_node_layer: the same
 * products added one in-edge at a time in edge order (16 lanes per destination). */
int di_node_aggregate(const di_graph* g, di_dtype dt, const float* alpha /*[Et,4]*/, const void* qkv /*[Nt,384]*/,
                      float* attn_out /*[Nt,128]*/, void* stream);
int di_node_update(const di_graph* g, di_dtype dt, int final_layer, const float* attn /*[Nt,128]*/,
                   const void* h_in, const void* wmat, const float* wvec, void* h_out, void* qkv_out,
                   void* hT_out, void* stream);
/* ABI 7: the same aggregation folded into the bf16 edge layer's epilogue (no alpha round trip, no
 * gather launch). di_edge_layer_attn = di_edge_layer (alpha_out may be NULL: not written) + the
 * segment sums of its edges: the kernel's waves each hold 32 consecutive (destination-major) edges,
 * "fold tile" t = edges 32t .. 32t+31; for every destination v
 *   all in-edges in one fold tile:  attn_out[v, :] = wV / (z + 1e-6)  (fp32 [Nt,128], as di_node_aggregate)
 *   in-edges over tiles t0 < .. < t1: attn_parts[t0][1] holds tile t0's partial sums (wV[128], z[4]),
 *                                     attn_parts[t][0] tile t's for t0 < t <= t1
 * attn_parts: di_attn_parts_bytes(num_edges) bytes (fp32 [ceil(Et/32)][2][132]); rows of nodes
 * without in-edges are not written. dt must be DI_BF16 and g->in_ptr set (DI_EINVAL otherwise).
 * Summation order: a tree over a tile's rows, then tile by tile (di_node_aggregate adds in edge
 * order; both within the bf16 path's bound). di_node_update_folded = di_node_update on those
 * outputs: split destinations add their partials, nodes without in-edges get 0. */
int64_t di_attn_parts_bytes(int32_t num_edges);
int di_edge_layer_attn(const di_graph* g, di_dtype dt, int final_layer, const float* edge_f,
                       const void* f_in, const void* fn_in, const void* qkv, const void* wmat, const float* wvec,
                       float* alpha_out, void* f_out, void* fn_out, float* attn_out /*[Nt,128]*/,
                       float* attn_parts, void* stream);
int di_node_update_folded(const di_graph* g, di_dtype dt, int final_layer, const float* attn,
                          const float* attn_parts, const void* h_in, const void* wmat, const float* wvec,
                          void* h_out, void* qkv_out, void* hT_out, void* stream);

/* Pair-tensor kernel of a di_pair_tensor call (di_pair_launch.kernel). Scheduling choice of this
 * build, not a reference interface; every kernel writes the same bytes. */
enum {
  DI_PAIR_AUTO = 0,    /* ROWS for aligned >= 1, the generic kernel otherwise */
  DI_PAIR_ROWS = 1,    /* a wave streams 64 whole rows (needs aligned >= 1) */
  DI_PAIR_VECTOR = 2,  /* one 16-B load per 16-B store over flat plane positions (aligned >= 1) */
  DI_PAIR_LINES = 3,   /* every store writes whole 128-B lines (aligned == 2) */
};
/* Launch of one di_pair_tensor call (host struct; NULL = all defaults). */
typedef struct {
  int32_t kernel;           /* DI_PAIR_* */
  int32_t blocks;           /* resident blocks of the persistent grid; 0 = one per CU */
  int32_t waves_per_block;  /* ROWS / LINES: 1..16 waves per block; 0 = 4 */
  int32_t beside;           /* 1: the schedule beside a concurrent GeoT stream: at most 3 stores in
                               flight per wave (its loads do not queue behind a store backlog) and
                               non-temporal stores; 0: plain stores, unbounded */
} di_pair_launch;

/* h [Nt, hidden] node features; hT (optional for aligned == 0) the same transposed [hidden, Nt]
 * (di_node_layer's hT_out), which turns chain-2 column reads into 16-B vector loads.
 * aligned: 0 none; 1 promises every L2, out_off and h2_row is a multiple of 16 bytes worth of
 * elements and `out` is 16-B aligned (vector stores); 2 additionally promises every channel plane
 * starts on a 128-B line (out 128-B aligned, out_off * elem and L1 * L2 * elem multiples of 128).
 * Limits: L1 * L2 * elem < 2^31 bytes per plane, L1 <= 2^20 (di_pair_tensor_check). */
int di_pair_tensor(di_dtype dt, const di_pair_desc* descs /*device [B]*/, int32_t num_complexes,
                   int32_t max_l1, int32_t max_l2, int32_t hidden, int32_t aligned, const void* h,
                   const void* hT, int32_t num_rows, const di_pair_launch* launch, void* out, void* stream);
/* The shape / launch validation di_pair_tensor applies before launching (host only): DI_OK,
 * DI_EINVAL or DI_ERANGE. elem_bytes: 2 (bf16) or 4 (fp32). */
int di_pair_tensor_check(int32_t num_complexes, int32_t max_l1, int32_t max_l2, int32_t hidden, int32_t elem_bytes,
                         const di_pair_launch* launch);

/* ---- pair-tensor queue (ABI 6): the overlapped schedule's pair stream -----------------------------
 * A job is one micro-batch's pair tensors (construct_interact_tensor of each complex,
 * deepinteract_utils.py:158-172), produced by the GeoT stream in job order. The producer stream signals
 * each job after its final node layer (hT written): with di_pair_signal, or carried by its next launch
 * (the signal_job argument of di_node_embed / di_embed_init_edge / di_pair_help); it calls
 * di_pair_help before it reuses a job's hT buffer and once at the end of a run (drain). di_pair_stream is one persistent launch
 * on its own stream over a range of jobs, beside the producer: its waves wait for each job's signal and
 * take the job's items (complex, channel, 64-row block) from the queue's per-job ticket counter, with
 * the bounded non-temporal stores of di_pair_launch.beside. di_pair_help takes the remaining items of
 * its jobs with plain stores on the whole chip and returns (on the device) once every item of them is
 * done, whoever took it: a wave counts its items DONE only after its stores have completed, so every
 * launch ordered after a help launch on its stream reads the jobs' final bytes. Completion never depends on di_pair_stream running concurrently: a stream
 * wave that waits longer than patience_ms for a signal gives up and the help launches do the rest. The
 * bytes written are those of di_pair_tensor(aligned = 1) for the same descriptors.
 * Preconditions (the kernels cannot check device-resident jobs): every job's descs are 16-B aligned
 * planes (L2 and out_off multiples of 16 bytes of the dtype, h2_row too), hT 16-B aligned, items =
 * di_pair_job_items(num_complexes, max_l1, hidden), and max_l1 >= every descs[i].l1. */
typedef struct {
  const void* hT;             /* [hidden, num_rows] transposed final node features (di_node_layer hT_out) */
  const di_pair_desc* descs;  /* [num_complexes] (device) */
  void* out;                  /* base of the job's pair tensors (descs[i].out_off elements from here) */
  int32_t num_rows;           /* columns of hT: node rows of the micro-batch */
  int32_t num_complexes;
  int32_t max_l1;             /* largest chain-1 length of the job */
  int32_t items;              /* di_pair_job_items(num_complexes, max_l1, hidden) */
} di_pair_job;
/* device bytes of a queue for jobs 0 .. num_jobs-1 (zero it before first use; -1 for num_jobs <= 0).
 * Words (uint32): [0] jobs signalled, [32] error bits (1: a help launch's completion wait timed out,
 * 2: a stream wave read a non-increasing ticket),
 * [33] stream waves that gave up waiting, [40..41] / [42..43] bytes written by stream / help launches
 * (uint64), then 256 B per job (ticket, arrive, done; csrc/pair_queue.h). */
int64_t di_pair_queue_bytes(int32_t num_jobs);
/* items of a job: num_complexes * 2 * hidden * ceil(max_l1 / 64); DI_EINVAL / DI_ERANGE */
int32_t di_pair_job_items(int32_t num_complexes, int32_t max_l1, int32_t hidden);
/* the job's hT is complete (stream order of `stream`): raises the queue's signalled count to job + 1 */
int di_pair_signal(void* queue, int32_t job, void* stream);
/* persistent pair stream over jobs [job_begin, job_end) (jobs: device array indexed by job number);
 * launch: blocks (0: one per CU; fp32: half the CUs), waves_per_block (0: 2; fp32: 4); always the beside
 * store policy */
int di_pair_stream(di_dtype dt, const di_pair_job* jobs, int32_t job_begin, int32_t job_end, int32_t hidden,
                   void* queue, const di_pair_launch* launch, float patience_ms, void* stream);
/* complete jobs [first_job, last_job] (all produced before this call in `stream` order); launch:
 * blocks (0: one per CU), waves_per_block (0: 8); signal_job >= 0: also marks that job ready at the
 * launch's start (as di_node_embed's signal) */
int di_pair_help(di_dtype dt, const di_pair_job* jobs, int32_t first_job, int32_t last_job, int32_t hidden,
                 void* queue, const di_pair_launch* launch, int32_t signal_job, void* stream);

/* ---- streams of the overlapped schedule (ABI 8; host calls, synchronous) ---------------------------
 * di_pair_stream waits on the device for signals that launches on the producer's stream raise, so the
 * two streams must reach the GPU through DIFFERENT hardware queues. HIP multiplexes a process's
 * streams onto at most GPU_MAX_HW_QUEUES in-order queues per priority (least-used first once the pool
 * is full), so which queue an ordinary stream gets depends on every stream created before it (an RCCL
 * communicator creates several); two streams on one queue run one after the other and every stream
 * wave waits out its patience.
 * di_stream_create_dedicated: a normal-priority stream whose CU mask covers every CU -- the runtime
 * gives each CU-masked stream a hardware queue of its own, never shared with another stream. Like every
 * stream created with default flags it synchronises with the legacy NULL stream: issue nothing on the
 * NULL stream while a pair-stream launch is in flight.
 * di_streams_concurrent: measures the property: a one-wave kernel on `a` waits (at most patience_ms,
 * <= 10000) for a word that a kernel on `b`, issued after it, raises; *concurrent (host) = 1 if it saw
 * it, else 0. work: >= 256 device bytes, overwritten. Synchronises both streams. */
int di_stream_create_dedicated(void** stream);
int di_stream_destroy(void* stream);
int di_streams_concurrent(void* a, void* b, void* work, float patience_ms, int32_t* concurrent);

/* Fused head prologue: x = ELU(InstanceNorm2d(conv2d_1(T))) of the contact
 * head (ResNet2DInputWithOptAttention.forward, deepinteract_modules.py:1181-1184, 1228-1232) for a
 * batch of complexes WITHOUT materialising the pair tensor T: the 1x1 conv of the outer concat
 * separates into W[:, :H] h1[i] + W[:, H:] h2[j] + b and the InstanceNorm statistics of that
 * separable sum are analytic. h: [rows, hidden] node features in `dt` (16-B aligned, hidden a
 * multiple of 8, <= 256); conv_w [channels, 2*hidden], conv_b, in_gamma, in_beta [channels] fp32;
 * work: device scratch of di_head_prologue_work_bytes() bytes; out: per complex [channels, L1, L2]
 * in `dt` at descs[i].out_off (elements). aligned16: every L2 and out_off a multiple of 16 bytes
 * of `dt` (row-streaming store kernel). */
int di_head_prologue(di_dtype dt, const di_pair_desc* descs /*device [B]*/, int32_t num_complexes, int32_t max_l1,
                     int32_t max_l2, int32_t hidden, int32_t channels, int32_t aligned16, const void* h,
                     const float* conv_w, const float* conv_b, const float* in_gamma, const float* in_beta,
                     float eps, float* work, void* out, void* stream);
int64_t di_head_prologue_work_bytes(int32_t num_complexes, int32_t max_l1, int32_t max_l2, int32_t channels);

/* ---- contact-head body (convolutions stay on MIOpen) --------------------- */
/* y = ELU(InstanceNorm2d(x)) of one [channels, hw] NCHW image (batch 1): biased variance, eps,
 * affine gamma/beta [channels] fp32; fp64 statistics. Replaces the `inorm_i` + `F.elu` pair of
 * every inorm ResNet block (ResNet.forward, deepinteract_modules.py:1075-1095; the modules
 * :1016-1030) and of the head prologue (:1231-1232). x, y: 16-B aligned, `dt` storage (y may
 * alias x); work: di_inorm_work_bytes() bytes of device scratch. */
int di_inorm_elu(di_dtype dt, const void* x, int32_t channels, int64_t hw, const float* gamma,
                 const float* beta, float eps, void* work, void* y, void* stream);
int64_t di_inorm_work_bytes(int32_t channels, int64_t hw);
/* y = (x + bias[c]) * scale[c] + res: the ResNet block's last conv bias (nullable), SEBlock's
 * channel gate (deepinteract_modules.py:954-970) and the block's residual add (:1095); each step
 * is rounded to `dt`, as torch's separate kernels do. x, res, y: [channels, hw], 16-B aligned (y
 * may alias x or res); scale, bias [channels] fp32. */
int di_se_scale_add(di_dtype dt, const void* x, const float* scale, const float* bias, const void* res,
                    int32_t channels, int64_t hw, void* y, void* stream);
/* mean[c] = mean over hw of x[c] (+ bias[c], nullable): SEBlock's x.mean(dim=(2, 3))
 * (:966) of a conv output whose bias is deferred to di_se_scale_add. fp64 accumulation;
 * work: di_inorm_work_bytes() bytes. */
int di_channel_mean(di_dtype dt, const void* x, int32_t channels, int64_t hw, const float* bias, void* work,
                    float* mean, void* stream);

/* ---- graph builder ----------------------------------------------------------------------- */
/* Cα kNN per chain: idx_out [Nt,k] chain-local neighbour ids (ascending squared distance,
 * self first), d2_out [Nt,k] the expansion-formula squared distances. node_off [G+1] device. */
int di_knn_topk(int32_t num_graphs, const int32_t* node_off, const float* ca /*[Nt,3]*/, int32_t k,
                int32_t max_nodes, int32_t* idx_out, float* d2_out, void* stream);

/* kNN graph topology of every chain from di_knn_topk's idx ([DGL-ASSUMPTION] DGL 0.6 knn_graph
 * edge order, graph_utils.py:107): edge e = v*k + r has src = idx[v,r] + node_off[g] and dst = v
 * (global ids); in_ptr_out [Nt+1] = v*k; node_pos_out [Nt] = v - node_off[g]. */
int di_knn_graph(int32_t num_graphs, const int32_t* node_off, int32_t k, const int32_t* knn_idx,
                 int32_t num_nodes, int32_t* src_out, int32_t* dst_out, int32_t* in_ptr_out,
                 int32_t* node_pos_out, void* stream);

typedef struct {
  int32_t num_graphs, k, max_nodes;
  const int32_t* node_off;   /* [G+1] */
  const float* backbone;     /* [Nt,4,3] N, CA, C, O */
  const float* amide_norm;   /* [Nt,3] */
  const float* dips;         /* [Nt,106] DIPS-Plus residue features */
  const int32_t* knn_idx;    /* [Nt,k] chain-local (di_knn_topk) */
  const float* knn_d2;       /* [Nt,k] */
  float* node_f;             /* out [Nt,113] */
  float* edge_f;             /* out [Nt*k,28] */
  float* stats;              /* workspace [G,4] */
} di_geo_args;
int di_geo_feats(const di_geo_args* args, void* stream);

/* neighbour-edge ids: 2 distinct in-edges of src(e) and of dst(e), uniform, counter-based RNG
 * (seed, e); nbr_out [Et,4] global edge ids in the di_graph.nbr layout. */
int di_build_nbr_ids(int32_t num_edges, const int32_t* src, const int32_t* dst, const int32_t* in_ptr,
                     uint64_t seed, int32_t* nbr_out, void* stream);

/* neighbour-edge ids bit-exact with the reference's torch.randperm draws
 * (deepinteract_utils.py:539-546): chain g's ids are those convert_df_to_dgl_graph produces right
 * after torch.manual_seed(seeds[g]) (torch CPU generator = mt19937; randperm = Fisher-Yates, E src
 * calls then E dst calls). kNN graphs only (uniform in-degree k, dst-major edges, k >= 3).
 * node_off [G+1], seeds [G] (device); num_nodes = node_off[G]; src/dst [Et = num_nodes*k] global
 * node ids; nbr_out [Et,4] global ids. Two launches: the per-chain mt19937 streams (one wave per
 * chain) write the kept in-edge positions, then every id gets its endpoint's in-edge base.
 * DI_ERANGE when 2 * num_nodes * k * (k-1) exceeds INT32_MAX (a chain's draw count is int32). */
int di_build_nbr_ids_torch(int32_t num_graphs, const int32_t* node_off, int32_t k, const uint64_t* seeds,
                           int32_t num_nodes, const int32_t* src, const int32_t* dst, int32_t* nbr_out, void* stream);

/* ---- module-at-a-time API ---------------------------------------------------------------- */
/* ConformationModule alone (kind-6 blob): conf_out [Et,128] = F + SiLU(final_linear(...)), from the
 * current edge features f_in [Et,128] and fn_in = SiLU(nbr_linear(f_in)) [Et,128]. */
int di_conformation(const di_graph* g, di_dtype dt, const float* edge_f /*[Et,28]*/, const void* f_in,
                    const void* fn_in, const void* wmat, const float* wvec, void* conf_out, void* stream);

/* y[r,:] = res[r,:] + act(W x[r,:] + bias) for r < rows; W packed in the natural-k fragment order
 * (packing.pack_matrix_natural: out_dim % 16 == 0, in_dim padded to 32). act: 0 none, 1 SiLU.
 * bias / res may be NULL. x, res, y in the storage dtype; bias fp32. */
int di_gemm_bias_act(di_dtype dt, int32_t rows, int32_t in_dim, int32_t out_dim, const void* x, int32_t x_ld,
                     const void* w_packed, const float* bias, int32_t act, const void* res, int32_t res_ld,
                     void* y, int32_t y_ld, void* stream);

/* qkv [Nt,384] = Q|K|V, proj_e [Et,128]: e_out [Et,128] (NULL: not produced), alpha_out [Et,4]
 * (fp32, exp(clamp(sum score))), h_out [Nt,128] = sum alpha V[src] / (sum alpha + 1e-6). */
int di_geo_attention(const di_graph* g, di_dtype dt, const void* qkv, const void* proj_e, void* e_out,
                     float* alpha_out, void* h_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DEEPINTERACT_AMD_H */
