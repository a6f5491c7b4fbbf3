// gtr_lap.hip — sparse kernels of the GPU Laplacian positional-encoding precompute
// (etpgt/encodings/laplacian_pe.py:19-66: k+1 smallest eigenvectors of the
// sym-normalised Laplacian L = I - D^-1/2 A D^-1/2 of PyG get_laplacian).
//
//   k_lap_build: CSR values of L from a symmetric adjacency in CSR (self loops dropped,
//     deg = row counts, off-diagonal -deg_r^-1/2 deg_c^-1/2, unit diagonal; duplicate
//     edges summed as to_scipy_sparse_matrix does, since each occurrence adds its value).
//   gtr_lap_plan (host): an nnz-balanced work list -- rows of <= chunk nonzeros are one
//     item, longer rows are cut into chunk-sized items whose partial rows are summed in
//     order afterwards.
//   k_spmm_items / k_spmm_split: Y = alpha * (L X) + beta * X for a block of b vectors
//     (X, Y [n, b] row-major): a wave per item, lanes over the b columns, so each nonzero's
//     X row is one coalesced read (the solver's only O(nnz) work; bound by the X-row
//     gathers, which hit L2/MALL for catalogue-sized n).
// The eigen-solver itself (block LOBPCG: orthonormalisation + Rayleigh-Ritz on [n, 3b]
// blocks) runs in etpgt.encodings.laplacian_gpu on top of these kernels.

#include <algorithm>
#include <climits>

#include "gtr_common.cuh"

namespace {

using namespace gtr;

// deg[r] = number of off-diagonal entries of row r; dis = deg^-1/2 (0 for isolated rows).
__global__ __launch_bounds__(256) void k_lap_dis(const int32_t* ptr, const int32_t* col, int n, float* dis) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  int d = 0;
  for (int e = ptr[r]; e < ptr[r + 1]; ++e) d += col[e] != r;
  dis[r] = d > 0 ? 1.0f / sqrtf((float)d) : 0.0f;
}

// Off-diagonal values -dis[r] * dis[c] (self loops: 0, the unit diagonal is implicit).
__global__ __launch_bounds__(256) void k_lap_vals(const int32_t* ptr, const int32_t* col, int n, const float* dis,
                                                  float* val) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const float dr = dis[r];
  for (int e = ptr[r]; e < ptr[r + 1]; ++e) {
    const int c = col[e];
    val[e] = c == r ? 0.0f : -(dr * dis[c]);
  }
}

// Y = alpha * (I + offdiag) X + beta * X over an nnz-balanced work list: a wave per item
// (row, e0, e1, part), each item at most `chunk` nonzeros of one row, so a hub row
// (the co-occurrence graph's most popular item has ~33k neighbours) is spread over many
// waves instead of serialising one.  The wave splits into 64/BP groups of BP column
// lanes; group g takes nonzeros e0+g, e0+g+G, ... (4 in flight per lane), the groups are
// summed by xor-shuffles, and group 0 writes Y (single-item rows) or the item's partial
// row part[p] (split rows, summed in order by k_spmm_split: deterministic).
template <int BP>
__global__ __launch_bounds__(256) void k_spmm_items(const int4* items, int64_t n_items, const int32_t* col,
                                                    const float* val, int b, const float* X, float* Y,
                                                    float* part, float alpha, float beta) {
  constexpr int G = 64 / BP;
  const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (it >= n_items) return;
  const int lane = threadIdx.x & 63;
  const int g = lane / BP, cl = lane % BP;
  const int4 w = items[it];
  for (int c0 = 0; c0 < b; c0 += BP) {
    const int c = c0 + cl;
    const bool on = c < b;
    float acc = 0.0f;
    int e = w.y + g;
    for (; e + 3 * G < w.z; e += 4 * G) {
      const int j0 = col[e], j1 = col[e + G], j2 = col[e + 2 * G], j3 = col[e + 3 * G];
      const float v0 = val[e], v1 = val[e + G], v2 = val[e + 2 * G], v3 = val[e + 3 * G];
      if (on) {
        const float x0 = X[(size_t)j0 * b + c], x1 = X[(size_t)j1 * b + c];
        const float x2 = X[(size_t)j2 * b + c], x3 = X[(size_t)j3 * b + c];
        acc += v0 * x0;
        acc += v1 * x1;
        acc += v2 * x2;
        acc += v3 * x3;
      }
    }
    for (; e < w.z; e += G)
      if (on) acc += val[e] * X[(size_t)col[e] * b + c];
#pragma unroll
    for (int o = BP; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    if (g == 0 && on) {
      if (w.w < 0) {
        const float x = X[(size_t)w.x * b + c];
        Y[(size_t)w.x * b + c] = alpha * (x + acc) + beta * x;  // unit diagonal
      } else {
        part[(size_t)w.w * b + c] = acc;
      }
    }
  }
}

// Split rows: Y = alpha * (x + sum of the row's item partials, in item order) + beta * x.
__global__ __launch_bounds__(256) void k_spmm_split(const int4* splits, int64_t n_splits, int b, const float* X,
                                                    float* Y, const float* part, float alpha, float beta) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n_splits) return;
  const int4 w = splits[s];
  for (int c = threadIdx.x & 63; c < b; c += 64) {
    float acc = 0.0f;
    for (int p = w.y; p < w.z; ++p) acc += part[(size_t)p * b + c];
    const float x = X[(size_t)w.x * b + c];
    Y[(size_t)w.x * b + c] = alpha * (x + acc) + beta * x;
  }
}

// Gram matrices of the block eigen-solver, S^T S and S^T Y for tall-skinny S, Y [n, m]
// (m <= 64), accumulated in fp64: workgroup p takes rows [p*rows, (p+1)*rows), stages
// GRAM_TR rows of S and Y in LDS and each thread accumulates 16 entries of each 64x64
// product (entry e = tid + 256k: row i = e / 64 is uniform across a wave, so the S[.][i]
// read is a broadcast); k_gram_reduce sums the partials in workgroup order.
#define GRAM_TR 32
__global__ __launch_bounds__(256) void k_gram_part(const float* S, const float* Y, int n, int m, int rows,
                                                   double* part) {
  __shared__ float sS[GRAM_TR][64];
  __shared__ float sY[GRAM_TR][64];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * rows, r1 = min(n, r0 + rows);
  double g[16], h[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { g[k] = 0.0; h[k] = 0.0; }
  for (int rb = r0; rb < r1; rb += GRAM_TR) {
    for (int idx = tid; idx < GRAM_TR * 64; idx += 256) {
      const int rr = idx >> 6, c = idx & 63, r = rb + rr;
      const bool in = r < r1 && c < m;
      sS[rr][c] = in ? S[(size_t)r * m + c] : 0.0f;
      sY[rr][c] = in ? Y[(size_t)r * m + c] : 0.0f;
    }
    __syncthreads();
    for (int rr = 0; rr < GRAM_TR; ++rr) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e = tid + 256 * k;
        const double si = (double)sS[rr][e >> 6];
        g[k] += si * (double)sS[rr][e & 63];
        h[k] += si * (double)sY[rr][e & 63];
      }
    }
    __syncthreads();
  }
  double* out = part + (size_t)blockIdx.x * 8192;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    out[tid + 256 * k] = g[k];
    out[4096 + tid + 256 * k] = h[k];
  }
}

__global__ __launch_bounds__(256) void k_gram_reduce(const double* part, int P, double* out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 8192) return;
  double acc = 0.0;
  for (int p = 0; p < P; ++p) acc += part[(size_t)p * 8192 + e];
  out[e] = acc;
}

}  // namespace

extern "C" int gtr_lap_gram(const float* S, const float* Y, int n, int m, double* part, int P, double* out,
                            gtr_stream_t stream) {
  if (!S || !Y || !part || !out || n <= 0 || m <= 0 || m > 64 || P <= 0) {
    set_error("gtr_lap_gram: bad arguments (m <= 64, P >= 1)");
    return GTR_E_ARG;
  }
  const int rows = (n + P - 1) / P;
  const int grid = (n + rows - 1) / rows;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_gram_part, dim3(grid), dim3(256), 0, s, S, Y, n, m, rows, part);
  GTR_HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_gram_reduce, dim3(32), dim3(256), 0, s, part, grid, out);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_lap_build(const int32_t* ptr, const int32_t* col, int n, float* dis, float* val,
                             gtr_stream_t stream) {
  if (!ptr || !col || !dis || !val || n <= 0) { set_error("gtr_lap_build: bad arguments"); return GTR_E_ARG; }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_lap_dis, dim3((n + 255) / 256), dim3(256), 0, s, ptr, col, n, dis);
  GTR_HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_lap_vals, dim3((n + 255) / 256), dim3(256), 0, s, ptr, col, n, dis, val);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_lap_plan(const int32_t* ptr, int n, int chunk, int32_t* items, int64_t* n_items,
                            int32_t* splits, int64_t* n_splits, int64_t* n_parts) {
  if (!ptr || n <= 0 || chunk <= 0 || !n_items || !n_splits || !n_parts) {
    set_error("gtr_lap_plan: bad arguments");
    return GTR_E_ARG;
  }
  int64_t ni = 0, ns = 0, np = 0;
  for (int r = 0; r < n; ++r) {
    const int e0 = ptr[r], e1 = ptr[r + 1];
    if (e1 < e0) { set_error("gtr_lap_plan: ptr not monotone"); return GTR_E_ARG; }
    if (e1 - e0 <= chunk) {
      if (items) { int32_t* q = items + 4 * ni; q[0] = r; q[1] = e0; q[2] = e1; q[3] = -1; }
      ++ni;
      continue;
    }
    const int nch = (int)(((int64_t)(e1 - e0) + chunk - 1) / chunk);
    if (np + nch >= INT32_MAX) { set_error("gtr_lap_plan: too many partial rows"); return GTR_E_ARG; }
    if (splits) { int32_t* q = splits + 4 * ns; q[0] = r; q[1] = (int32_t)np; q[2] = (int32_t)(np + nch); q[3] = 0; }
    ++ns;
    for (int i = 0; i < nch; ++i, ++ni) {
      if (!items) continue;
      int32_t* q = items + 4 * ni;
      q[0] = r;
      q[1] = e0 + i * chunk;
      q[2] = (int)std::min<int64_t>((int64_t)e0 + (int64_t)(i + 1) * chunk, e1);
      q[3] = (int32_t)(np + i);
    }
    np += nch;
  }
  *n_items = ni;
  *n_splits = ns;
  *n_parts = np;
  return GTR_OK;
}

extern "C" int gtr_lap_spmm(const int32_t* col, const float* val, int n, int b, const int32_t* items, int64_t n_items,
                            const int32_t* splits, int64_t n_splits, float* part, const float* X, float* Y,
                            float alpha, float beta, gtr_stream_t stream) {
  if (!col || !val || !items || !X || !Y || n <= 0 || b <= 0 || b > 256 || X == Y || n_items <= 0 ||
      n_splits < 0 || (n_splits > 0 && (!splits || !part))) {
    set_error("gtr_lap_spmm: bad arguments (1 <= b <= 256, X != Y, a plan from gtr_lap_plan)");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((n_items + 3) / 4));
  const int4* it = (const int4*)items;
  if (b <= 16)
    hipLaunchKernelGGL(k_spmm_items<16>, grid, dim3(256), 0, s, it, n_items, col, val, b, X, Y, part, alpha, beta);
  else if (b <= 32)
    hipLaunchKernelGGL(k_spmm_items<32>, grid, dim3(256), 0, s, it, n_items, col, val, b, X, Y, part, alpha, beta);
  else
    hipLaunchKernelGGL(k_spmm_items<64>, grid, dim3(256), 0, s, it, n_items, col, val, b, X, Y, part, alpha, beta);
  GTR_HIP_CHECK_LAUNCH();
  if (n_splits > 0) {
    hipLaunchKernelGGL(k_spmm_split, dim3((unsigned)((n_splits + 3) / 4)), dim3(256), 0, s, (const int4*)splits,
                       n_splits, b, X, Y, part, alpha, beta);
    GTR_HIP_CHECK_LAUNCH();
  }
  return GTR_OK;
}
