// gtr_wgrad.cuh — weight gradients of the dense parameters (lin_{query,key,value,skip}
// weight + bias, lin_beta, the LapPE projection) as jobs of 64 x 64 output tiles summed
// over a node-row range.  Two users:
//   k_wgrad (gtr_bwd.hip): split-K partial slabs over P row chunks, summed by the
//     optimizer (large batches);
//   k_step_tail_wgrad (gtr_opt.hip): small batches, ONE chunk over all rows computed
//     inside the step tail and applied by AdamW directly -- the same loop, so the
//     gradients are bitwise those of k_wgrad with P = 1 + the tail's one-partial sum.
#pragma once

#include "gtr_common.cuh"

namespace gtr {

enum { WJ_MM = 0, WJ_GATE = 1, WJ_COLSUM = 2 };

struct WJob {
  int type, M1, M2, lda, ldb, tn, nt, blk0;
  const float* A;
  const float* B;
  const int32_t* bidx;
  const float* agg;
  const float* s;   // skip rows (qkvs + 3D), row stride lda
  float* outW;      // slab destinations (k_wgrad)
  float* outB;
  int64_t fW, fB;   // flat-buffer offsets of the same outputs (fused tail), -1: none
};

#define GTR_MAX_WJOBS 16

struct WgradK {
  const int32_t* hdr;
  int P, njobs, D, pad0;
  int64_t stride;
  WJob jobs[GTR_MAX_WJOBS];
};

// Tile `tile` of job J summed over node rows [t0, t1); emit(which, idx, value) for each
// output (which 0: W element idx, 1: bias element idx).  Whole block (GTR_BLOCK threads).
template <class Emit>
__device__ __forceinline__ void wgrad_tile(const WJob& J, int tile, int t0, int t1, int D, Emit&& emit) {
  constexpr int TK = 32;  // node rows staged per round
  __shared__ __attribute__((aligned(16))) float As[TK][64];
  __shared__ __attribute__((aligned(16))) float Bs[TK][64];
  const int tid = threadIdx.x;
  if (J.type == WJ_GATE) {
    const int j = tile * GTR_BLOCK + tid;
    if (j >= 3 * D) return;
    float acc = 0.0f;
#pragma unroll 4
    for (int t = t0; t < t1; ++t) {
      const float u = J.A[t];
      float f;
      if (j < D) f = J.agg[(size_t)t * D + j];
      else if (j < 2 * D) f = J.s[(size_t)t * J.lda + (j - D)];
      else f = J.agg[(size_t)t * D + (j - 2 * D)] - J.s[(size_t)t * J.lda + (j - 2 * D)];
      acc += u * f;
    }
    emit(0, j, acc);
    return;
  }
  if (J.type == WJ_COLSUM) {  // bias gradient: column sums of A over the rows
    const int j = tile * GTR_BLOCK + tid;
    if (j >= J.M1) return;
    float acc = 0.0f;
#pragma unroll 8
    for (int t = t0; t < t1; ++t) acc += J.A[(size_t)t * J.lda + j];
    emit(1, j, acc);
    return;
  }
  const int tm = tile / J.tn, tq = tile - tm * J.tn;
  const int m0 = tm * 64, n0 = tq * 64;
  const int ty = tid >> 4, tx = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[i][k] = 0.0f;
  // rows of round r + 1 are loaded into registers while round r is multiplied out of LDS
  constexpr int NQ = TK * 64 / GTR_BLOCK;
  float av[NQ], bv[NQ];
  auto load = [&](int tb) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = tid + q * GTR_BLOCK;
      const int i = idx >> 6, c = idx & 63;
      const int t = tb + i;
      av[q] = 0.0f;
      bv[q] = 0.0f;
      if (t < t1) {
        if (m0 + c < J.M1) av[q] = J.A[(size_t)t * J.lda + m0 + c];
        const int col = n0 + c;
        if (col < J.M2) {
          const float* brow = J.bidx ? J.B + (size_t)J.bidx[t] * J.ldb : J.B + (size_t)t * J.ldb;
          bv[q] = brow[col];
        } else if (col == J.M2) {
          bv[q] = 1.0f;
        }
      }
    }
  };
  if (t0 < t1) load(t0);
  for (int tb = t0; tb < t1; tb += TK) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = tid + q * GTR_BLOCK;
      As[idx >> 6][idx & 63] = av[q];
      Bs[idx >> 6][idx & 63] = bv[q];
    }
    __syncthreads();
    if (tb + TK < t1) load(tb + TK);
#pragma unroll 8
    for (int k = 0; k < TK; ++k) {
      const float4 a4 = *reinterpret_cast<const float4*>(&As[k][ty * 4]);
      const float4 b4 = *reinterpret_cast<const float4*>(&Bs[k][tx * 4]);
      const float ar[4] = {a4.x, a4.y, a4.z, a4.w};
      const float br[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] += ar[i] * br[q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= J.M1) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nn = n0 + tx * 4 + q;
      if (nn < J.M2) emit(0, (int64_t)m * J.M2 + nn, acc[i][q]);
      else if (nn == J.M2) emit(1, m, acc[i][q]);
    }
  }
}

// Host: the job list of layers [l_begin, l_end) (+ the LapPE projection when l_begin == 0
// and cfg->pe_k > 0).  Slab destinations layer_slab[l] / pe_slab (k_wgrad) and/or flat
// offsets layer_flat[l] = {w_all, b_all, w_beta} / pe_flat = {pe.w, pe.b} (fused tail);
// `blocks` = workgroups for n_chunks row chunks.
inline int build_wjobs(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, const float* dx0,
                       const float* pe_tab, float* const* layer_slab, float* pe_slab, const int64_t* layer_flat,
                       const int64_t* pe_flat, int n_chunks, int l_begin, int l_end, WJob* jobs, int& nj,
                       int& blocks) {
  const int D = cfg->dim;
  nj = 0;
  blocks = 0;
  for (int l = l_begin; l < l_end; ++l) {
    const gtr_layer& L = layers[l];
    float* base = layer_slab ? layer_slab[l] : nullptr;
    const int64_t* fl = layer_flat ? layer_flat + 3 * l : nullptr;
    WJob& w = jobs[nj++];
    w = WJob{};
    w.type = WJ_MM; w.M1 = 4 * D; w.M2 = D; w.lda = 4 * D; w.ldb = D;
    // the bias rides as a ones-column in the last tile when it fits there (D = 32); for
    // D a multiple of 64 it would need a tile column of its own (1/3 more tiles at
    // D = 128), so it is a column-sum job instead
    w.tn = (D + 63) / 64; w.nt = ((4 * D + 63) / 64) * w.tn; w.blk0 = blocks;
    w.A = L.dqkvs; w.B = L.xin; w.bidx = nullptr;
    w.outW = base; w.outB = base ? base + (size_t)4 * D * D : nullptr;
    w.fW = fl ? fl[0] : -1; w.fB = fl ? fl[1] : -1;
    blocks += w.nt * n_chunks;
    if (D % 64 == 0) {
      WJob& c = jobs[nj++];
      c = WJob{};
      c.type = WJ_COLSUM; c.M1 = 4 * D; c.lda = 4 * D; c.tn = 1; c.nt = (4 * D + GTR_BLOCK - 1) / GTR_BLOCK;
      c.blk0 = blocks; c.A = L.dqkvs; c.outB = base ? base + (size_t)4 * D * D : nullptr;
      c.fW = -1; c.fB = fl ? fl[1] : -1;
      blocks += c.nt * n_chunks;
    }
    WJob& q = jobs[nj++];
    q = WJob{};
    q.type = WJ_GATE; q.M1 = 1; q.M2 = 3 * D; q.lda = 4 * D; q.tn = 1; q.nt = (3 * D + GTR_BLOCK - 1) / GTR_BLOCK;
    q.blk0 = blocks; q.A = L.du; q.agg = L.agg; q.s = L.qkvs + 3 * D;
    q.outW = base ? base + (size_t)4 * D * D + 4 * D : nullptr;
    q.fW = fl ? fl[2] : -1; q.fB = -1;
    blocks += q.nt * n_chunks;
  }
  if (cfg->pe_k > 0 && (pe_slab || pe_flat) && l_begin == 0) {
    if (!dx0 || (!pe_tab && !bt->node_pe)) { set_error("gtr_wgrad: PE gradient needs dx0 and PE rows"); return GTR_E_ARG; }
    const int K = cfg->pe_k;
    WJob& w = jobs[nj++];
    w = WJob{};
    w.type = WJ_MM; w.M1 = D; w.M2 = K; w.lda = D; w.ldb = K;
    w.tn = (K + 1 + 63) / 64; w.nt = ((D + 63) / 64) * w.tn; w.blk0 = blocks;
    w.A = dx0;
    if (bt->node_pe) { w.B = bt->node_pe; w.bidx = nullptr; }
    else { w.B = pe_tab; w.bidx = bt->node_item; }
    w.outW = pe_slab; w.outB = pe_slab ? pe_slab + (size_t)D * K : nullptr;
    w.fW = pe_flat ? pe_flat[0] : -1; w.fB = pe_flat ? pe_flat[1] : -1;
    blocks += w.nt * n_chunks;
  }
  return GTR_OK;
}

}  // namespace gtr
