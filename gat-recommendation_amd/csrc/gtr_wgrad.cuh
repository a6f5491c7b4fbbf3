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

#include <type_traits>

namespace gtr {

enum { WJ_MM = 0, WJ_GATE = 1, WJ_COLSUM = 2 };

struct WJob {
  int type, M1, M2, lda, ldb, tn, nt, blk0;
  int mfma, wm, wn, fold_bias;  // WJ_MM on MFMA tiles (wgrad_tile_mfma): wm x wn waves of 64 x 64;
                                 // fold_bias: the bias gradient from the same A loads
  const float* A;
  const float* B;
  const int32_t* bidx;
  const float* agg;
  const float* s;   // skip rows (qkvs + 3D), row stride lda
  float* outW;      // slab destinations (k_wgrad)
  float* outB;
  int64_t fW, fB;   // flat-buffer offsets of the same outputs (fused tail), -1: none
  int tile0, pad_t; // first arrival counter of the job's tiles (fused tail)
};

#define GTR_MAX_WJOBS 16

#ifndef GTR_WGRAD_MFMA_ROWS
#define GTR_WGRAD_MFMA_ROWS 128  // rows per split-K chunk from which the QKVS job runs on MFMA
#endif

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
  if (J.type == WJ_GATE || J.type == WJ_COLSUM) {
    // 64 columns per block as 16 float4 lanes x 16 row phases (4 per wave: each wave load
    // instruction reads 4 rows x 256 B); the phases are summed in order through LDS.
    // GATE: lin_beta weight u . [agg, s, agg - s] -- columns c of agg and s are read once
    // for all three segments (outputs c, D + c, 2D + c); COLSUM: column sums of A.
    constexpr int PH = GTR_BLOCK / 16;
    __shared__ float4 part[3][PH][16];
    const int c16 = tid & 15, ph = tid >> 4;
    const int col = tile * 64 + c16 * 4;
    const bool gate = J.type == WJ_GATE;
    const int ncol = gate ? D : J.M1;  // multiples of 4
    float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0, g2 = g0;
    if (col < ncol) {
      if (gate) {
        const float* ag = J.agg + col;
        const float* sk = J.s + col;
#pragma unroll 4
        for (int t = t0 + ph; t < t1; t += PH) {
          const float u = J.A[t];
          const float4 x = *reinterpret_cast<const float4*>(ag + (size_t)t * D);
          const float4 y = *reinterpret_cast<const float4*>(sk + (size_t)t * J.lda);
          g0.x += u * x.x; g0.y += u * x.y; g0.z += u * x.z; g0.w += u * x.w;
          g1.x += u * y.x; g1.y += u * y.y; g1.z += u * y.z; g1.w += u * y.w;
          g2.x += u * (x.x - y.x); g2.y += u * (x.y - y.y); g2.z += u * (x.z - y.z); g2.w += u * (x.w - y.w);
        }
      } else {
        const float* cp = J.A + col;
#pragma unroll 4
        for (int t = t0 + ph; t < t1; t += PH) {
          const float4 x = *reinterpret_cast<const float4*>(cp + (size_t)t * J.lda);
          g0.x += x.x; g0.y += x.y; g0.z += x.z; g0.w += x.w;
        }
      }
    }
    part[0][ph][c16] = g0;
    if (gate) {
      part[1][ph][c16] = g1;
      part[2][ph][c16] = g2;
    }
    __syncthreads();
    const int nseg = gate ? 3 : 1;
    if (tid < 64 * nseg) {
      const int sg = tid >> 6, cl = tid & 63, cc = cl >> 2, comp = cl & 3;
      const int j = tile * 64 + cl;
      float g = 0.0f;
#pragma unroll
      for (int q = 0; q < PH; ++q) {
        const float4 v = part[sg][q][cc];
        g += comp == 0 ? v.x : comp == 1 ? v.y : comp == 2 ? v.z : v.w;
      }
      if (j < ncol) {
        if (gate) emit(0, sg * D + j, g);
        else emit(1, j, g);
      }
    }
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

// MFMA form of a WJ_MM tile for long row ranges (k_wgrad at large batches):
// out[m][n] = sum_t A[t][m] * B[t][n] with v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate).
// The block's wm x wn waves each own a 64-row output block, the other waves
// (kw = GTR_WAVES / (wm * wn) > 1) split the rows and are summed through LDS in split
// order.  Lane l takes row t + (l >> 4) of a k-step and loads ONE float4 of A (columns
// m0 + 4(l & 15) .. +3); MFMA tile mt uses its component mt, so C row i is output row
// m0 + 4i + mt.  Operands come straight from global memory (each row segment a 256 B
// coalesced run), two k-steps in flight ahead of the MFMAs.
//  * wide (QKVS weight, M2 a multiple of 64): 64 x 64 per wave; B also one float4 per lane
//    and tile (mt, nt) has C[i][j] = out[m0 + 4i + mt][n0 + 4j + nt], so a lane's four nt
//    tiles of one C row are four consecutive n: one float4 store per (mt, reg);
//  * NARROW (LapPE projection, M2 + 1 <= 32 with the bias as a ones column at M2, rows of
//    B gathered through bidx): 64 x 32 per wave, B as two scalars per lane, C[i][j] of
//    tile (mt, nt) = out[m0 + 4i + mt][16 nt + j].
// emit(which, idx, value) as wgrad_tile; emit4(idx, float4): W elements idx .. idx + 3.
template <bool NARROW, class Emit, class Emit4>
__device__ __forceinline__ void wgrad_tile_mfma(const WJob& J, int tile, int t0, int t1, Emit&& emit, Emit4&& emit4) {
  constexpr int NT = NARROW ? 2 : 4;
  __shared__ f32x4 red[GTR_WAVES][4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = J.wm * J.wn, kw = GTR_WAVES / nw;
  const int wt = wave % nw, ks = wave / nw;
  const int tm = tile / J.tn, tq = tile - tm * J.tn;
  const int m0 = (tm * J.wm + wt % J.wm) * 64, n0 = (tq * J.wn + wt / J.wm) * 64;
  const int len = t1 - t0, per = (((len + kw - 1) / kw) + 3) & ~3;
  const int r0 = min(t1, t0 + ks * per), r1 = min(t1, r0 + per);
  const int kq = lane >> 4, c4 = (lane & 15) * 4, j16 = lane & 15;
  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* Ap = J.A + m0 + c4;
  // Loads are unconditional: a row past the range reads the range's last row (row 0 for
  // an empty range) and is zeroed where it is used.  A load under a lane-dependent branch
  // is skipped when no lane takes it, so the compiler cannot count it and waits for
  // vmcnt(0) -- every row in flight -- before the next use.
  const int rlast = max(0, r1 - 1);
  const int jb0 = min(j16, J.M2 - 1), jb1 = min(16 + j16, J.M2 - 1);
  // NARROW rows of B gathered through bidx: the row ids are loaded 24 rows (three
  // k-steps) before the row itself (ring ri below), so a gathered row's load does not
  // wait on an id requested just before it -- with in-order returns that wait was a
  // vmcnt(0) per k-step (the LapPE job: 14 us of the C3 B = 8192 launch).
  // (the id is loaded unconditionally -- from A's words when there is no bidx, unused --
  // so the load is counted: a load under the bidx branch made the loop wait vmcnt(0))
  const int32_t* ib = J.bidx ? J.bidx : reinterpret_cast<const int32_t*>(J.A);
  auto idx = [&](int t) -> int {
    const int tc = min(t, rlast);
    const int v = __builtin_nontemporal_load(ib + tc);
    return J.bidx ? v : tc;
  };
  auto ld = [&](int t, int bi, float4& a, float4& b) {
    const int tc = min(t, rlast);
    a = *reinterpret_cast<const float4*>(Ap + (size_t)tc * J.lda);
    if (NARROW) {
      const float* brow = J.B + (size_t)bi * J.ldb;
      b.x = brow[jb0];
      b.y = brow[jb1];
    } else {
      b = *reinterpret_cast<const float4*>(J.B + (size_t)tc * J.ldb + n0 + c4);
    }
  };
  // the operands of row t as the MFMAs take them: zero past the range; NARROW columns
  // past M2 are the bias's ones column (at M2) or zero
  auto fix = [&](int t, float4& a, float4& b) {
    if (t >= r1) {
      a = make_float4(0.f, 0.f, 0.f, 0.f);
      b = a;
    } else if (NARROW) {
      if (j16 >= J.M2) b.x = j16 == J.M2 ? 1.0f : 0.0f;
      if (16 + j16 >= J.M2) b.y = 16 + j16 == J.M2 ? 1.0f : 0.0f;
    }
  };
  auto mma = [&](float4 a4, float4 b4, int t) {
    fix(t, a4, b4);
    const float av[4] = {a4.x, a4.y, a4.z, a4.w};
    const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], bv[nt], acc[mt][nt], 0, 0, 0);
  };
  // wide tiles with n0 == 0 also sum the A columns (the bias gradient: a ones column of B)
  const bool colsum = !NARROW && n0 == 0;
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  // rows 16 ahead in flight (4 row quads): at 2 waves per SIMD one 8-row round of MFMAs
  // (~1k cycles) is shorter than a load's latency from MALL under a full-chip stream.
  // Round 5: a ring of three register sets of 8 rows, the loop unrolled by three so that
  // no set is ever COPIED (a copy of an in-flight load is a use whose wait -- vector
  // loads retire in order -- drained the 16 rows in flight at every step).
  float4 ra[3][2], rb[3][2];
  int ri[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // NARROW: ids of the rows set n loads next
  if (NARROW) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      ri[q][0] = idx(r0 + 8 * q + kq);
      ri[q][1] = idx(r0 + 8 * q + 4 + kq);
    }
  }
  ld(r0 + kq, ri[0][0], ra[0][0], rb[0][0]);
  ld(r0 + 4 + kq, ri[0][1], ra[0][1], rb[0][1]);
  ld(r0 + 8 + kq, ri[1][0], ra[1][0], rb[1][0]);
  ld(r0 + 12 + kq, ri[1][1], ra[1][1], rb[1][1]);
  if (NARROW) {
    ri[0][0] = idx(r0 + 24 + kq); ri[0][1] = idx(r0 + 28 + kq);
    ri[1][0] = idx(r0 + 32 + kq); ri[1][1] = idx(r0 + 36 + kq);
  }
  auto stepk = [&](auto S, int t) {
    constexpr int c = decltype(S)::value, n = (c + 2) % 3;
    ld(t + 16 + kq, ri[n][0], ra[n][0], rb[n][0]);
    ld(t + 20 + kq, ri[n][1], ra[n][1], rb[n][1]);
    if (NARROW) {  // set n's next rows (three k-steps on)
      ri[n][0] = idx(t + 40 + kq);
      ri[n][1] = idx(t + 44 + kq);
    }
    mma(ra[c][0], rb[c][0], t + kq);
    mma(ra[c][1], rb[c][1], t + 4 + kq);
    if (colsum) {
      const float4 a0 = t + kq < r1 ? ra[c][0] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 a1 = t + 4 + kq < r1 ? ra[c][1] : make_float4(0.f, 0.f, 0.f, 0.f);
      cs.x += a0.x; cs.y += a0.y; cs.z += a0.z; cs.w += a0.w;
      cs.x += a1.x; cs.y += a1.y; cs.z += a1.z; cs.w += a1.w;
    }
  };
  for (int t = r0; t < r1; t += 24) {
    stepk(std::integral_constant<int, 0>{}, t);
    if (t + 8 >= r1) break;
    stepk(std::integral_constant<int, 1>{}, t + 8);
    if (t + 16 >= r1) break;
    stepk(std::integral_constant<int, 2>{}, t + 16);
  }
  if (colsum) {  // the four row lanes of a column, then the row splits in order
    cs.x = bfly_add<32>(bfly_add<16>(cs.x)); cs.y = bfly_add<32>(bfly_add<16>(cs.y));
    cs.z = bfly_add<32>(bfly_add<16>(cs.z)); cs.w = bfly_add<32>(bfly_add<16>(cs.w));
  }
  for (int s = 1; s < kw; ++s) {
    if (colsum && ks == s) red[wt][0][lane] = f32x4{cs.x, cs.y, cs.z, cs.w};
    __syncthreads();
    if (colsum && ks == 0) {
      const f32x4 v = red[wt][0][lane];
      cs.x += v[0]; cs.y += v[1]; cs.z += v[2]; cs.w += v[3];
    }
    __syncthreads();
  }
  if (colsum && ks == 0 && kq == 0 && J.fold_bias) {
    emit(1, m0 + c4, cs.x);
    emit(1, m0 + c4 + 1, cs.y);
    emit(1, m0 + c4 + 2, cs.z);
    emit(1, m0 + c4 + 3, cs.w);
  }
  // row splits: split 0 adds splits 1, 2, .. in order, one mt at a time through LDS
  for (int mt = 0; mt < 4; ++mt) {
    for (int s = 1; s < kw; ++s) {
      if (ks == s) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[wt][nt][lane] = acc[mt][nt];
      }
      __syncthreads();
      if (ks == 0) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += red[wt][nt][lane];
      }
      __syncthreads();
    }
  }
  if (ks != 0) return;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 16 * kq + 4 * r + mt;
      if (m >= J.M1) continue;
      if (NARROW) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int nn = 16 * nt + j16;
          if (nn < J.M2) emit(0, (int64_t)m * J.M2 + nn, acc[mt][nt][r]);
          else if (nn == J.M2) emit(1, m, acc[mt][nt][r]);
        }
      } else {
        emit4((int64_t)m * J.M2 + n0 + c4, make_float4(acc[mt][0][r], acc[mt][1][r], acc[mt][2][r], acc[mt][3][r]));
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
                       int& blocks, bool mfma = false) {
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
    if (mfma && D % 64 == 0) {  // MFMA tiles: wm x wn waves per block, 64 x 64 each
      w.mfma = 1;
      w.wn = D / 64 >= 2 ? 2 : 1;
      w.wm = GTR_WAVES / w.wn < 4 * D / 64 ? GTR_WAVES / w.wn : 4 * D / 64;
      w.tn = D / (64 * w.wn);
      w.nt = (4 * D / (64 * w.wm)) * w.tn;
      w.fold_bias = 1;
    }
    w.A = L.dqkvs; w.B = L.xin; w.bidx = nullptr;
    w.outW = base; w.outB = base ? base + (size_t)4 * D * D : nullptr;
    w.fW = fl ? fl[0] : -1; w.fB = fl ? fl[1] : -1;
    blocks += w.nt * n_chunks;
    if (D % 64 == 0 && !w.mfma) {  // (MFMA tiles fold the column sums into the A loads)
      WJob& c = jobs[nj++];
      c = WJob{};
      c.type = WJ_COLSUM; c.M1 = 4 * D; c.lda = 4 * D; c.tn = 1; c.nt = (4 * D + 63) / 64;
      c.blk0 = blocks; c.A = L.dqkvs; c.outB = base ? base + (size_t)4 * D * D : nullptr;
      c.fW = -1; c.fB = fl ? fl[1] : -1;
      blocks += c.nt * n_chunks;
    }
    WJob& q = jobs[nj++];
    q = WJob{};
    q.type = WJ_GATE; q.M1 = 1; q.M2 = 3 * D; q.lda = 4 * D; q.tn = 1; q.nt = (D + 63) / 64;
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
    if (mfma && D % 64 == 0 && K + 1 <= 32) {  // narrow MFMA tiles (64 x 32 per wave)
      w.mfma = 2;
      w.wn = 1;
      w.wm = 1;  // the other waves split the rows: this job is load-latency bound
      w.tn = 1;
      w.nt = D / 64;
    }
    blocks += w.nt * n_chunks;
  }
  return GTR_OK;
}

}  // namespace gtr
