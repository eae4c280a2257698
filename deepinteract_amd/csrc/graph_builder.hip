// On-device residue-graph builder: Cα kNN, geometric node/edge features, neighbour-edge ids.
//
// Reference (paths relative to /root/reference/project/utils/):
//   kNN            graph_utils.py:107-108 (dgl.knn_graph bruteforce-blas + topk of
//                  pairwise_squared_distance). [DGL-ASSUMPTION, DGL 0.6] edge e = i*k + r has
//                  src = idx[i, r], dst = i.
//   featuriser     deepinteract_utils.py:460-530 + protein_feature_utils.py:82-101, 201-320
//   nbr edge ids   deepinteract_utils.py:534-553
//
// kNN ranks the reference's EXPANSION-formula fp32 distances  D = (|xi|^2 + |xj|^2) - 2 xi.xj
// (including its ~1e-3 non-zero diagonal) with ties broken by the smaller index, so the
// neighbour indices reproduce the CPU reference bit for bit except at exact value ties.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "../../include/deepinteract_amd.h"

// hipcc contracts a*b + c into an FMA by default (-ffp-contract=fast); the reference computes these
// features on the CPU without contraction, so contraction is off for this file and the one FMA the
// CPU sgemm does use (the K=3 dot product) is written explicitly.
#pragma clang fp contract(off)

namespace di {

constexpr int KNN_WAVES = 4;
constexpr int KNN_MAX_N = 4096;

// ------------------------------------------------------------------ exact torch.topk tie order
// torch.topk(largest=False) on the CPU (ATen TopKImpl) selects with libstdc++:
//   k * 64 <= n : std::partial_sort(q, q + k, q + n)                      (heap select + sort_heap)
//   otherwise   : std::nth_element(q, q + k - 1, q + n); std::sort(q, q + k - 1)
// over (value, index) pairs in index order with comparator  x.v < y.v  (NaN ordered last).
// Exactly tied distances are therefore ordered by the algorithms' swap history, not by index.
// This is a restatement of those published algorithms (GCC libstdc++ bits/stl_algo.h,
// bits/stl_heap.h) on an LDS array, run by one lane for the rare rows whose top-(k+1) contains
// an exact tie; rows without ties take the parallel path, whose result is then unique.
struct Seq {
  float* v;
  uint16_t* ix;
  __device__ bool lt(int a, int b) const { return lt_val(v[a], v[b]); }
  __device__ static bool lt_val(float x, float y) { return (!isnan(x) && isnan(y)) || x < y; }
  __device__ void swp(int a, int b) const {
    float t = v[a]; v[a] = v[b]; v[b] = t;
    uint16_t u = ix[a]; ix[a] = ix[b]; ix[b] = u;
  }
  __device__ void mov(int dst, int src) const { v[dst] = v[src]; ix[dst] = ix[src]; }
  __device__ void put(int dst, float val, uint16_t i) const { v[dst] = val; ix[dst] = i; }
};

__device__ inline int lg2i(int n) { return 31 - __clz(n); }

__device__ void ins_sort(const Seq& A, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i < last; ++i) {
    const float val = A.v[i];
    const uint16_t vi = A.ix[i];
    if (Seq::lt_val(val, A.v[first])) {
      for (int j = i; j > first; --j) A.mov(j, j - 1);
      A.put(first, val, vi);
    } else {
      int j = i, nx = i - 1;
      while (Seq::lt_val(val, A.v[nx])) { A.mov(j, nx); j = nx; --nx; }
      A.put(j, val, vi);
    }
  }
}

__device__ void unguarded_lin_insert(const Seq& A, int last) {
  const float val = A.v[last];
  const uint16_t vi = A.ix[last];
  int nx = last - 1;
  while (Seq::lt_val(val, A.v[nx])) { A.mov(last, nx); last = nx; --nx; }
  A.put(last, val, vi);
}

__device__ void median_to_first(const Seq& A, int result, int a, int b, int c) {
  if (A.lt(a, b)) {
    if (A.lt(b, c)) A.swp(result, b);
    else if (A.lt(a, c)) A.swp(result, c);
    else A.swp(result, a);
  } else if (A.lt(a, c)) A.swp(result, a);
  else if (A.lt(b, c)) A.swp(result, c);
  else A.swp(result, b);
}

__device__ int unguarded_part(const Seq& A, int first, int last, int pivot) {
  while (true) {
    while (A.lt(first, pivot)) ++first;
    --last;
    while (A.lt(pivot, last)) --last;
    if (!(first < last)) return first;
    A.swp(first, last);
    ++first;
  }
}

__device__ int part_pivot(const Seq& A, int first, int last) {
  const int mid = first + (last - first) / 2;
  median_to_first(A, first, first + 1, mid, last - 1);
  return unguarded_part(A, first + 1, last, first);
}

__device__ void adjust_heap(const Seq& A, int first, int hole, int len, float val, uint16_t vi) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (A.lt(first + second, first + second - 1)) --second;
    A.mov(first + hole, first + second);
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    A.mov(first + hole, first + second - 1);
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && Seq::lt_val(A.v[first + parent], val)) {
    A.mov(first + hole, first + parent);
    hole = parent;
    parent = (hole - 1) / 2;
  }
  A.put(first + hole, val, vi);
}

__device__ void make_heap_(const Seq& A, int first, int last) {
  const int n = last - first;
  if (n < 2) return;
  for (int parent = (n - 2) / 2;; --parent) {
    adjust_heap(A, first, parent, n, A.v[first + parent], A.ix[first + parent]);
    if (parent == 0) return;
  }
}

__device__ void pop_heap_(const Seq& A, int first, int last, int result) {
  const float val = A.v[result];
  const uint16_t vi = A.ix[result];
  A.mov(result, first);
  adjust_heap(A, first, 0, last - first, val, vi);
}

__device__ void heap_select(const Seq& A, int first, int middle, int last) {
  make_heap_(A, first, middle);
  for (int i = middle; i < last; ++i)
    if (A.lt(i, first)) pop_heap_(A, first, middle, i);
}

__device__ void sort_heap_(const Seq& A, int first, int last) {
  while (last - first > 1) {
    --last;
    pop_heap_(A, first, last, last);
  }
}

__device__ void introselect(const Seq& A, int first, int nth, int last, int depth) {
  while (last - first > 3) {
    if (depth == 0) {
      heap_select(A, first, nth + 1, last);
      A.swp(first, nth);
      return;
    }
    --depth;
    const int cut = part_pivot(A, first, last);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  ins_sort(A, first, last);
}

__device__ void std_sort(const Seq& A, int first, int last) {
  if (first == last) return;
  // introsort loop; the recursion touches disjoint ranges, so an explicit stack in any order
  // produces the same array
  int st_f[48], st_l[48], st_d[48], sp = 0;
  st_f[sp] = first; st_l[sp] = last; st_d[sp] = 2 * lg2i(last - first); ++sp;
  while (sp > 0) {
    --sp;
    int f = st_f[sp], l = st_l[sp], d = st_d[sp];
    while (l - f > 16) {
      if (d == 0) {
        heap_select(A, f, l, l);
        sort_heap_(A, f, l);
        break;
      }
      --d;
      const int cut = part_pivot(A, f, l);
      st_f[sp] = cut; st_l[sp] = l; st_d[sp] = d; ++sp;
      l = cut;
    }
  }
  if (last - first > 16) {
    ins_sort(A, first, first + 16);
    for (int i = first + 16; i < last; ++i) unguarded_lin_insert(A, i);
  } else {
    ins_sort(A, first, last);
  }
}

__device__ void torch_topk_smallest(const Seq& A, int n, int k) {
  if (k * 64 <= n) {
    heap_select(A, 0, k, n);
    sort_heap_(A, 0, k);
  } else {
    introselect(A, 0, k - 1, n, 2 * lg2i(n));
    std_sort(A, 0, k - 1);
  }
}

// no FMA contraction: elementwise products / sums as separate roundings, like torch's
// x * x followed by a sum over the last dim (x2s, graph_utils.py:108 / DGL factory)
__device__ __forceinline__ float sq3(float a, float b, float c) { return (a * a + b * b) + c * c; }
// x . y with K = 3 as the CPU sgemm micro-kernel computes it: an explicit fma chain
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
  return fmaf(a2, b2, fmaf(a1, b1, a0 * b0));
}

__device__ __forceinline__ float knn_dist(const float* ca, int n0, int j, float x0, float x1, float x2, float ni) {
  const float* xj = ca + (int64_t)(n0 + j) * 3;
  const float y0 = xj[0], y1 = xj[1], y2 = xj[2];
  const float nj = sq3(y0, y1, y2);
  return (ni + nj) - 2.f * dot3(x0, x1, x2, y0, y1, y2);
}

// LDS sized to the batch's largest chain (stride S = max_nodes rounded up to 64 per wave): at
// 1000-node chains 24 KiB per block, so six blocks (24 waves) share a CU instead of one.
__global__ __launch_bounds__(64 * KNN_WAVES) void k_knn(const int* __restrict__ node_off,
                                                          const float* __restrict__ ca, int k, int S,
                                                          int* __restrict__ idx_out, float* __restrict__ d2_out) {
  extern __shared__ __attribute__((aligned(16))) char knn_lds[];
  const int gph = blockIdx.y;
  const int n0 = node_off[gph], n = node_off[gph + 1] - n0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * KNN_WAVES + wave;
  if (i >= n || n > S) return;  // wave-uniform; no block barrier below (n > S: max_nodes too small)
  const float* xi = ca + (int64_t)(n0 + i) * 3;
  const float x0 = xi[0], x1 = xi[1], x2 = xi[2];
  const float ni = sq3(x0, x1, x2);
  float* d = reinterpret_cast<float*>(knn_lds) + wave * S;
  for (int j = lane; j < n; j += 64) d[j] = knn_dist(ca, n0, j, x0, x1, x2, ni);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // parallel selection of the k+1 smallest (value, index); lane 0 keeps the list
  const int kk = k + 1 <= n ? k + 1 : k;
  float prev_v = 0.f;
  bool tie = false;
  for (int r = 0; r < kk; ++r) {
    float bv = INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
      const float v = d[j];
      if (v < bv || (v == bv && j < bi)) {
        bv = v;
        bi = j;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int oi = __shfl_xor(bi, off);
      if (ov < bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (r > 0 && bv == prev_v) tie = true;
    prev_v = bv;
    if (lane == 0) {
      if (r < k) {
        idx_out[(int64_t)(n0 + i) * k + r] = bi;
        d2_out[(int64_t)(n0 + i) * k + r] = bv;
      }
      d[bi] = NAN;  // removed: NaN fails every '<' above
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  if (!tie) return;  // wave-uniform (every lane reduced the same values)
  // exact-tie row: replay torch's CPU selection on the full row
  uint16_t* ix = reinterpret_cast<uint16_t*>(knn_lds + (size_t)KNN_WAVES * S * 4) + wave * S;
  for (int j = lane; j < n; j += 64) {
    d[j] = knn_dist(ca, n0, j, x0, x1, x2, ni);
    ix[j] = (uint16_t)j;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane == 0) {
    Seq A{d, ix};
    torch_topk_smallest(A, n, k);
    for (int r = 0; r < k; ++r) {
      idx_out[(int64_t)(n0 + i) * k + r] = ix[r];
      d2_out[(int64_t)(n0 + i) * k + r] = d[r];
    }
  }
}

// ------------------------------------------------------------------ featuriser helpers
struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 ld3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ float dotf3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ f3 normalize3(f3 a) {  // F.normalize: x / max(||x||, 1e-12)
  const float nrm = fmaxf(sqrtf(dotf3(a, a)), 1e-12f);
  return {a.x / nrm, a.y / nrm, a.z / nrm};
}
__device__ __forceinline__ float signf_(float v) { return (float)((v > 0.f) - (v < 0.f)); }

// dihedral t of the flattened N,CA,C atom chain (protein_feature_utils.py:276-298), t in [0, 3N-4]
__device__ float dihedral(const float* bb, int t) {
  auto atom = [&](int m) { return ld3(bb + (int64_t)(m / 3) * 12 + (m % 3) * 3); };
  const f3 u2 = normalize3(sub3(atom(t + 1), atom(t)));
  const f3 u1 = normalize3(sub3(atom(t + 2), atom(t + 1)));
  const f3 u0 = normalize3(sub3(atom(t + 3), atom(t + 2)));
  const f3 n2 = normalize3(cross3(u2, u1));
  const f3 n1 = normalize3(cross3(u1, u0));
  const float eps = 1e-7f;
  const float cosd = fminf(fmaxf(dotf3(n2, n1), -1.f + eps), 1.f - eps);
  return signf_(dotf3(u2, n1)) * acosf(cosd);
}

// amide-plane angle of an edge (deepinteract_utils.py:520-523): NaN for zero normals
__device__ __forceinline__ float amide_angle(const float* am, int a, int b) {
  const f3 v1 = ld3(am + (int64_t)a * 3), v2 = ld3(am + (int64_t)b * 3);
  return acosf(dotf3(v1, v2) / (sqrtf(dotf3(v1, v1)) * sqrtf(dotf3(v2, v2))));
}

// pass 1: per chain min/max of the raw edge weight and of the (NaN-zeroed) amide angle
__global__ __launch_bounds__(256) void k_geo_stats(di_geo_args a) {
  const int gph = blockIdx.x;
  const int n0 = a.node_off[gph], n = a.node_off[gph + 1] - n0;
  const int k = a.k;
  float wmin = INFINITY, wmax = -INFINITY, amin = INFINITY, amax = -INFINITY;
  for (int q = threadIdx.x; q < n * k; q += 256) {
    const int i = q / k;
    const int src = a.knn_idx[(int64_t)(n0 + i) * k + (q - i * k)];
    const f3 cs = ld3(a.backbone + (int64_t)(n0 + src) * 12 + 3), cd = ld3(a.backbone + (int64_t)(n0 + i) * 12 + 3);
    const f3 dd = sub3(cs, cd);
    const float wr = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
    float ang = amide_angle(a.amide_norm + (int64_t)n0 * 3, i, src);
    if (isnan(ang)) ang = 0.f;
    wmin = fminf(wmin, wr);
    wmax = fmaxf(wmax, wr);
    amin = fminf(amin, ang);
    amax = fmaxf(amax, ang);
  }
  __shared__ float red[4][256];
  red[0][threadIdx.x] = wmin;
  red[1][threadIdx.x] = wmax;
  red[2][threadIdx.x] = amin;
  red[3][threadIdx.x] = amax;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] = fminf(red[0][threadIdx.x], red[0][threadIdx.x + s]);
      red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + s]);
      red[2][threadIdx.x] = fminf(red[2][threadIdx.x], red[2][threadIdx.x + s]);
      red[3][threadIdx.x] = fmaxf(red[3][threadIdx.x], red[3][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) a.stats[gph * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// pass 2: node features [N,113] and edge features [E,28]
__global__ __launch_bounds__(256) void k_geo_feats(di_geo_args a) {
  const int gph = blockIdx.y;
  const int n0 = a.node_off[gph], n = a.node_off[gph + 1] - n0;
  const int k = a.k;
  const float* st = a.stats + gph * 4;
  const float wmin = st[0], wrng = st[1] - st[0], amin = st[2], arng = st[3] - st[2];
  const float* bb = a.backbone + (int64_t)n0 * 12;
  // torch.linspace(0, 20, 18) (float32, symmetric evaluation) and sigma = 20/18
  const float step = 20.f / 17.f;
  const float sigma = 20.f / 18.f;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < n * k; q += gridDim.x * 256) {
    const int i = q / k, r = q - i * k;
    const int64_t e = (int64_t)(n0 + i) * k + r;  // global edge id (uniform in-degree k)
    const int src = a.knn_idx[e];
    float* out = a.edge_f + e * 28;
    out[0] = sinf((float)(src - i));                                         // :504
    const f3 dd = sub3(ld3(bb + (int64_t)src * 12 + 3), ld3(bb + (int64_t)i * 12 + 3));
    out[1] = ((dd.x * dd.x + dd.y * dd.y + dd.z * dd.z) - wmin) / wrng;        // :506
    const float d2 = a.knn_d2[e];
#pragma unroll
    for (int j = 0; j < 18; ++j) {                                             // RBF of d^2 (:82-101)
      const float mu = j < 9 ? (float)j * step : 20.f - (float)(17 - j) * step;
      const float z = (d2 - mu) / sigma;
      out[2 + j] = expf(-(z * z));
    }
    // orientation features: under DGL 0.6's dst-major edge order the featuriser is called with
    // E_idx = dst = i (deepinteract_utils.py:476), so every "neighbour" frame is the node's own:
    // dU = normalize(O_i . 0) = 0 and R = O_i^T O_i is symmetric -> quaternion (0, 0, 0, 1).
    out[20] = 0.f;
    out[21] = 0.f;
    out[22] = 0.f;
    out[23] = 0.f;
    out[24] = 0.f;
    out[25] = 0.f;
    out[26] = 1.f;
    float ang = amide_angle(a.amide_norm + (int64_t)n0 * 3, i, src);         // plane1 = dst, plane2 = src
    if (isnan(ang)) ang = 0.f;
    float an = (ang - amin) / arng;
    if (isnan(an)) an = 0.f;
    out[27] = an;
  }
  // node features
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float* out = a.node_f + (int64_t)(n0 + i) * 113;
    out[0] = n > 1 ? (float)i / (float)(n - 1) : 0.f;                        // :494
    // D_pad[3i + c] = D[3i + c - 1] for 0 <= 3i+c-1 <= 3n-4 (phi[0], psi[-1], omega[-1] = 0)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int t = 3 * i + c - 1;
      const float dih = (t >= 0 && t <= 3 * n - 4) ? dihedral(bb, t) : 0.f;
      out[1 + c] = cosf(dih);
      out[4 + c] = sinf(dih);
    }
    const float* dp = a.dips + (int64_t)(n0 + i) * 106;
    for (int c = 0; c < 106; ++c) out[7 + c] = dp[c];
  }
}

// ------------------------------------------------------------------ neighbour-edge ids
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// For edge e: 2 distinct in-edges of src(e) and 2 distinct in-edges of dst(e), drawn uniformly
// (the first two entries of a uniform random permutation, deepinteract_utils.py:539-546).
__global__ __launch_bounds__(256) void k_nbr_ids(int Et, const int* __restrict__ src, const int* __restrict__ dst,
                                                 const int* __restrict__ in_ptr, uint64_t seed, int* __restrict__ nbr) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Et) return;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const int v = side == 0 ? src[e] : dst[e];
    const int base = in_ptr[v], deg = in_ptr[v + 1] - base;
    const uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)e << 1) | (uint64_t)side));
    const uint32_t r1 = (uint32_t)h, r2 = (uint32_t)(h >> 32);
    const int p0 = deg > 0 ? (int)(((uint64_t)r1 * (uint64_t)deg) >> 32) : 0;
    int p1 = p0;
    if (deg > 1) {
      p1 = (int)(((uint64_t)r2 * (uint64_t)(deg - 1)) >> 32);
      p1 += p1 >= p0;
    }
    nbr[(int64_t)e * 4 + 2 * side + 0] = base + p0;
    nbr[(int64_t)e * 4 + 2 * side + 1] = base + p1;
  }
}

// ------------------------------------------------------------------ torch-seeded neighbour ids
// Bit-exact restatement of the reference's draw (deepinteract_utils.py:539-546): with the torch
// CPU generator seeded by torch.manual_seed(seed) just before convert_df_to_dgl_graph, the loop
// calls torch.randperm(k) once per edge for the src side (E calls), then once per edge for the
// dst side (E calls). torch's CPU randperm (ATen randperm_cpu) is Fisher-Yates over mt19937:
//   r = 0..k-1; for i in 0..k-2: z = mt() % (k - i); swap(r[i], r[i + z])
// so every call consumes k-1 consecutive 32-bit mt19937 outputs and only the first two (the two
// entries kept, geo_nbrhd_size = 2, :545-546) matter:
//   pi[0] = z0 = u0 % k;   pi[1] = (1 + z1 == z0) ? 0 : 1 + z1,  z1 = u1 % (k - 1).
// The [DGL-ASSUMPTION] in-edge order (in_edges(v) = edge ids v*k .. v*k+k-1) makes the kept edge
// id node*k + pi (global ids: every chain has uniform in-degree k, so its edge offset is k times
// its node offset). mt19937 (MT19937RNGEngine.h: init_with_uint32, standard twist/tempering) is
// serial per chain: one workgroup per chain generates the stream 624 words at a time, the twist in
// three data-parallel phases ([0,227) reads only old words, [227,454) reads the words phase 1
// wrote, [454,624) those of phase 2 and word 0).
constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_A = 0x9908b0dfu, MT_UP = 0x80000000u, MT_LO = 0x7fffffffu;

__device__ __forceinline__ uint32_t mt_next(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & MT_UP) | (nxt & MT_LO);
  return far ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}

// One wave per chain (wave-synchronous: LDS ordering by wave barriers, no workgroup barrier in the
// 624-word loop); the kept draws are extracted per randperm call, not per stream position.
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__global__ __launch_bounds__(64) void k_nbr_ids_torch(const int* __restrict__ node_off, int k,
                                                      const uint64_t* __restrict__ seeds, int* __restrict__ nbr) {
  __shared__ uint32_t st[MT_N];
  __shared__ uint32_t out[MT_N];
  constexpr int P1 = MT_N - MT_M, P2 = 2 * (MT_N - MT_M);  // 227, 454
  const int g = blockIdx.x, lane = threadIdx.x;
  const int n0 = node_off[g], n = node_off[g + 1] - n0;
  const int E = n * k, e0 = n0 * k, km1 = k - 1;
  const int total = 2 * E * km1;  // draws of the 2E randperm(k) calls (int32: di_build_nbr_ids_torch checks)
  if (lane == 0) {                // init_with_uint32(seed)
    uint32_t s = (uint32_t)(seeds[g] & 0xffffffffull);
    st[0] = s;
    for (int i = 1; i < MT_N; ++i) {
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
      st[i] = s;
    }
  }
  wave_sync_lds();
  uint32_t prev_last = 0u;  // last tempered word of the previous 624-word block (wave-uniform)
  for (int base = 0; base < total; base += MT_N) {
    uint32_t v[4];
    // twist, phase 1: i in [0, 227) from old words only
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = lane + 64 * q;
      if (i < P1) v[q] = mt_next(st[i], st[i + 1], st[i + MT_M]);
    }
    wave_sync_lds();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = lane + 64 * q;
      if (i < P1) st[i] = v[q];
    }
    wave_sync_lds();
    // phase 2: i in [227, 454): far word i-227 is new (phase 1); i+1 <= 454 is still old
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = P1 + lane + 64 * q;
      if (i < P2) v[q] = mt_next(st[i], st[i + 1], st[i - P1]);
    }
    wave_sync_lds();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = P1 + lane + 64 * q;
      if (i < P2) st[i] = v[q];
    }
    wave_sync_lds();
    // phase 3: i in [454, 624): far word i-227 from phase 2; word 623 wraps to the new word 0
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int i = P2 + lane + 64 * q;
      if (i < MT_N) v[q] = mt_next(st[i], st[i + 1 < MT_N ? i + 1 : 0], st[i - P1]);
    }
    wave_sync_lds();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int i = P2 + lane + 64 * q;
      if (i < MT_N) st[i] = v[q];
    }
    wave_sync_lds();
    // tempering
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int i = lane + 64 * q;
      if (i < MT_N) {
        uint32_t y = st[i];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        out[i] = y;
      }
    }
    wave_sync_lds();
    // the kept draws (positions 0 and 1 of a call) that fall in this block: calls c with
    // c*km1 in [base - 1, base + 624)
    const int c_lo = base / km1, c_hi = min((base + MT_N - 1) / km1, 2 * E - 1);
    for (int c = c_lo + lane; c <= c_hi; c += 64) {
      const int t0 = c * km1 - base;  // block offset of the call's first draw
      if (t0 < -1) continue;          // both kept draws were in the previous block
      const int side = c >= E;
      const int e = e0 + (side ? c - E : c);
      const uint32_t u0 = t0 >= 0 ? out[t0] : prev_last;
      const int z0 = (int)(u0 % (uint32_t)k);
      // positions only: the endpoint's in-edge base is added by k_nbr_base (no dependent global
      // load on the stream's critical path)
      if (t0 >= 0) nbr[(int64_t)e * 4 + 2 * side] = z0;
      if (t0 + 1 < MT_N) {
        const int z1 = (int)(out[t0 + 1] % (uint32_t)km1);
        nbr[(int64_t)e * 4 + 2 * side + 1] = (1 + z1 == z0) ? 0 : 1 + z1;
      }
    }
    prev_last = out[MT_N - 1];
    wave_sync_lds();  // every lane's reads of out[] before the next block's tempering
  }
}

// kept in-edge positions -> edge ids: nbr[e][2*side + j] = endpoint * k + position
__global__ __launch_bounds__(256) void k_nbr_base(int Et, int k, const int* __restrict__ src,
                                                  const int* __restrict__ dst, int* __restrict__ nbr) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Et) return;
  int4 p = reinterpret_cast<const int4*>(nbr)[e];
  const int bs = src[e] * k, bd = dst[e] * k;
  p.x += bs;
  p.y += bs;
  p.z += bd;
  p.w += bd;
  reinterpret_cast<int4*>(nbr)[e] = p;
}

// ------------------------------------------------------------------ kNN graph topology
// [DGL-ASSUMPTION, DGL 0.6 knn_graph] edge e = v*k + r of chain g: src = idx[v, r] (chain-local)
// + node_off[g], dst = v; in-edges of v are v*k .. v*k+k-1 (CSR row pointer v*k); node_pos = the
// node's index inside its chain (InitEdge positional row). One thread per node.
__global__ __launch_bounds__(256) void k_knn_graph(int num_graphs, const int* __restrict__ node_off, int k,
                                                   const int* __restrict__ idx, int Nt, int* __restrict__ src,
                                                   int* __restrict__ dst, int* __restrict__ in_ptr,
                                                   int* __restrict__ node_pos) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v > Nt) return;
  in_ptr[v] = v * k;
  if (v == Nt) return;
  int lo = 0, hi = num_graphs - 1;  // last g with node_off[g] <= v
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (node_off[mid] <= v) lo = mid;
    else hi = mid - 1;
  }
  const int n0 = node_off[lo];
  node_pos[v] = v - n0;
  for (int r = 0; r < k; ++r) {
    const int64_t e = (int64_t)v * k + r;
    src[e] = idx[e] + n0;
    dst[e] = v;
  }
}

}  // namespace di

using namespace di;

extern "C" int di_knn_graph(int32_t num_graphs, const int32_t* node_off, int32_t k, const int32_t* knn_idx,
                            int32_t num_nodes, int32_t* src_out, int32_t* dst_out, int32_t* in_ptr_out,
                            int32_t* node_pos_out, void* stream) {
  if (num_graphs <= 0 || !node_off || k <= 0 || !knn_idx || num_nodes <= 0 || !src_out || !dst_out ||
      !in_ptr_out || !node_pos_out || (int64_t)num_nodes * k > INT32_MAX)
    return DI_EINVAL;
  hipLaunchKernelGGL(k_knn_graph, dim3(num_nodes / 256 + 1), dim3(256), 0, (hipStream_t)stream, num_graphs,
                     node_off, k, knn_idx, num_nodes, src_out, dst_out, in_ptr_out, node_pos_out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_build_nbr_ids_torch(int32_t num_graphs, const int32_t* node_off, int32_t k, const uint64_t* seeds,
                                      int32_t num_nodes, const int32_t* src, const int32_t* dst, int32_t* nbr_out,
                                      void* stream) {
  // k_nbr_ids_torch counts a chain's mt19937 draws, 2 n k (k-1), in int32: bounded through the
  // batch total (every chain's n <= num_nodes), checked here on the host
  if (num_graphs <= 0 || num_graphs > 65535 || !node_off || k < 3 || k > 256 || !seeds || num_nodes <= 0 ||
      !src || !dst || !nbr_out)
    return DI_EINVAL;
  if (2LL * num_nodes * k * (k - 1) > INT32_MAX) return DI_ERANGE;
  const int num_edges = num_nodes * k;
  hipLaunchKernelGGL(k_nbr_ids_torch, dim3(num_graphs), dim3(64), 0, (hipStream_t)stream, node_off, k, seeds,
                     nbr_out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_nbr_base, dim3((num_edges + 255) / 256), dim3(256), 0, (hipStream_t)stream, num_edges, k, src,
                     dst, nbr_out);
  e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_knn_topk(int32_t num_graphs, const int32_t* node_off, const float* ca, int32_t k,
                           int32_t max_nodes, int32_t* idx_out, float* d2_out, void* stream) {
  if (num_graphs <= 0 || !node_off || !ca || !idx_out || !d2_out || k <= 0 || max_nodes < k ||
      max_nodes > KNN_MAX_N || num_graphs > 65535)
    return DI_EINVAL;
  dim3 grid((max_nodes + KNN_WAVES - 1) / KNN_WAVES, num_graphs);
  const int S = (max_nodes + 63) & ~63;
  hipLaunchKernelGGL(k_knn, grid, dim3(64 * KNN_WAVES), (size_t)KNN_WAVES * S * 6, (hipStream_t)stream, node_off, ca,
                     k, S, idx_out, d2_out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_geo_feats(const di_geo_args* args, void* stream) {
  if (!args || args->num_graphs <= 0 || args->k <= 0 || !args->node_off || !args->backbone ||
      !args->amide_norm || !args->dips || !args->knn_idx || !args->knn_d2 || !args->node_f ||
      !args->edge_f || !args->stats || args->num_graphs > 65535)
    return DI_EINVAL;
  const di_geo_args a = *args;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_geo_stats, dim3(a.num_graphs), dim3(256), 0, s, a);
  const int per = (a.max_nodes * a.k + 255) / 256;
  dim3 grid(per < 64 ? (per > 0 ? per : 1) : 64, a.num_graphs);
  hipLaunchKernelGGL(k_geo_feats, grid, dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_build_nbr_ids(int32_t num_edges, const int32_t* src, const int32_t* dst, const int32_t* in_ptr,
                                uint64_t seed, int32_t* nbr_out, void* stream) {
  if (num_edges <= 0 || !src || !dst || !in_ptr || !nbr_out) return DI_EINVAL;
  hipLaunchKernelGGL(k_nbr_ids, dim3((num_edges + 255) / 256), dim3(256), 0, (hipStream_t)stream, num_edges, src,
                     dst, in_ptr, seed, nbr_out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DI_OK : (int)e;
}
