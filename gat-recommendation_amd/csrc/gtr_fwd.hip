// gtr_fwd.hip — forward kernels of the GraphTransformer hot path (gfx950).
//
// k_conv_fwd<D>: one TransformerConv layer + the previous layer's BatchNorm /
//   residual / dropout, fused.  Reference: graph_transformer.py:140-152 (layer 0
//   prologue: item_embedding + LapPE), :171-177 (conv -> bn -> +res -> dropout) and
//   PyG TransformerConv.
//   Work unit = a row group: every session whose first node falls in [g*R,(g+1)*R)
//   (ranges precomputed in the batch image).  Sessions are independent subgraphs
//   (dataloader.py:157-202), so one workgroup owns every source of every destination
//   it processes: projection, attention and gate need no inter-workgroup exchange.
//   Only BatchNorm couples sessions: each group writes (count, mean, M2) partials which
//   the CONSUMING kernel reduces in its prologue (consumer_reduce) or the last arriving
//   group combines (large grids).
//
// k_readout<D>: last layer's BN/residual/dropout + mean readout (base.py:136-155)
//   + scoring loss fwd/bwd (base.py:80-113, losses.py:8-164) + readout backward and
//   the last BatchNorm's backward partial sums.

#include "gtr_layer.cuh"

namespace {

using namespace gtr;

GTR_PH_DECL

struct ConvFwdK {
  gtr_batch bt;
  int H, C, first, train, layer, pe_k, cred, pad0;
  float sqrt_c, bn_eps, bn_mom, scale;
  uint32_t seed, thresh;
  int drop_on, pad1;
  const uint32_t* rng_ctr;
  const float* table;
  const float* pe_tab;
  const float* wpe;
  const float* bpe;
  const float* p_out;
  const float* p_xin;
  float* p_stats;        // previous layer's finalized stats (read, or written by block 0 when cred)
  const float* p_part;   // previous layer's forward partials (cred)
  const float* p_gamma;
  const float* p_beta;
  float* p_rmean;
  float* p_rvar;
  int64_t* p_nbt;
  const float* w_all;
  const float* b_all;
  const float* w_beta;
  float* xin;
  float* qkvs;
  float* alpha;
  float* agg;
  float* gate;
  float* out;
  float* bn_part;
  uint32_t* cnt;
  float* bn_stats;
  float* bn_rmean;
  float* bn_rvar;
  int64_t* bn_nbt;
};

// Block prologue shared by k_conv_fwd (previous layer) and k_readout (last layer):
// BatchNorm mean/rstd of the layer feeding this kernel into s_mean/s_rstd.
//   eval: running stats; train + cred: reduce the producer's partials (block 0 also
//   publishes the stats and updates running_mean/var/num_batches_tracked);
//   train, producer-finalised: read the stats.
template <int D, int BLK>
__device__ __forceinline__ void prev_bn_stats(int train, int cred, int G, const float* part, float* stats,
                                              float* rmean, float* rvar, int64_t* nbt, float eps, float mom,
                                              float* s_mean, float* s_rstd, float* s_uvar, float* scr) {
  if (!train) {
    for (int j = threadIdx.x; j < D; j += BLK) {
      s_mean[j] = rmean[j];
      s_rstd[j] = 1.0f / sqrtf(rvar[j] + eps);
    }
  } else if (cred) {
    bn_stats_from_parts<D, BLK>(part, G, eps, s_mean, s_rstd, s_uvar, scr);
    if (blockIdx.x == 0) {
      for (int j = threadIdx.x; j < D; j += BLK) {
        stats[j] = s_mean[j];
        stats[D + j] = s_rstd[j];
        rmean[j] = (1.0f - mom) * rmean[j] + mom * s_mean[j];
        rvar[j] = (1.0f - mom) * rvar[j] + mom * s_uvar[j];
      }
      if (threadIdx.x == 0 && nbt) *nbt += 1;
    }
  } else {
    for (int j = threadIdx.x; j < D; j += BLK) {
      s_mean[j] = stats[j];
      s_rstd[j] = stats[D + j];
    }
  }
}

// Attention + gate of one destination row (wave per row).  QB/SB/KB/VB: row bases
// with stride ST (LDS on the fast path, global qkvs otherwise); EP/ES: CSR of the rows
// (local indices on the fast path); eoff: offset of EP's edge indices in alpha.
template <int D>
__device__ __forceinline__ void attn_row(const ConvFwdK& a, int t, int tl, const float* QB, const float* SB,
                                         const float* KB, const float* VB, int ST, const int* EP, const int* ES,
                                         int eoff, int lane, const Drop& dr, uint32_t st_attn,
                                         const float (&w1)[LayerGeom<D>::VPL], const float (&w2)[LayerGeom<D>::VPL],
                                         const float (&w3)[LayerGeom<D>::VPL], float* xo_row) {
  constexpr int VPL = LayerGeom<D>::VPL;
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int GL = C / VPL;
  const int head = act ? d0 / C : 0;
  const bool leader = act && ((lane & (GL - 1)) == 0);
  float q[VPL], s[VPL], ag[VPL];
  load_vec<VPL>(q, QB + (size_t)tl * ST + d0, act);
  load_vec<VPL>(s, SB + (size_t)tl * ST + d0, act);
#pragma unroll
  for (int v = 0; v < VPL; ++v) ag[v] = 0.0f;
  const int e0 = EP[tl], e1 = EP[tl + 1];
  float m = -INFINITY, z = 0.0f;
  for (int e = e0; e < e1; ++e) {
    float kv[VPL];
    load_vec<VPL>(kv, KB + (size_t)ES[e] * ST + d0, act);
    float dt = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dt += q[v] * kv[v];
    const float l = group_sum(dt, GL) / a.sqrt_c;
    const float mn = fmaxf(m, l);
    z = z * expf(m - mn) + expf(l - mn);
    m = mn;
  }
  const float zd = z + 1e-16f;
  for (int e = e0; e < e1; ++e) {
    const int src = ES[e];
    float kv[VPL], vv[VPL];
    load_vec<VPL>(kv, KB + (size_t)src * ST + d0, act);
    load_vec<VPL>(vv, VB + (size_t)src * ST + d0, act);
    float dt = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dt += q[v] * kv[v];
    const float l = group_sum(dt, GL) / a.sqrt_c;
    const float al = expf(l - m) / zd;
    const int eg = e + eoff;
    if (leader) a.alpha[(size_t)eg * H + head] = al;
    const float ad = al * dr.mul(st_attn, (uint32_t)(eg * H + head));
#pragma unroll
    for (int v = 0; v < VPL; ++v) ag[v] += ad * vv[v];
  }
  float u = 0.0f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) u += w1[v] * ag[v] + w2[v] * s[v] + w3[v] * (ag[v] - s[v]);
  u = wave_sum(u);
  const float beta = 1.0f / (1.0f + expf(-u));
  float o[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) o[v] = beta * s[v] + (1.0f - beta) * ag[v];
  store_vec<VPL>(a.agg + (size_t)t * D + d0, ag, act);
  store_vec<VPL>(a.out + (size_t)t * D + d0, o, act);
  if (xo_row) store_vec<VPL>(xo_row + d0, o, act);
  if (lane == 0) a.gate[t] = beta;
}

template <int D>
__global__ __launch_bounds__(CONV_BLOCK) void k_conv_fwd(ConvFwdK a) {
  using G = LayerGeom<D>;
  constexpr int VPL = G::VPL, RMAX = G::RMAX, XS = G::XS, KPE = G::KPE, TPR = G::TPR, CH = G::CH;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* XO = sm + G::F_XO;
  float* KVs = sm + G::F_KV;
  float* QSs = sm + G::F_QS;
  float* PEs = sm + G::F_PE;
  float* LOG = sm + G::F_LOG;
  float* s_bn = sm + G::F_BN;
  int* items = reinterpret_cast<int*>(sm + G::F_ITEMS);
  int* iptr = reinterpret_cast<int*>(sm + G::F_IPTR);
  int* isrc = reinterpret_cast<int*>(sm + G::F_ISRC);
  int* edst = reinterpret_cast<int*>(sm + G::F_EDST);
  int* s_flag = reinterpret_cast<int*>(sm + G::F_FLAG);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GTR_PH(a.layer, 0);
  GTR_PH_CLK(a.layer, 6);
  const int Gn = a.bt.hdr[4];
  const int g = blockIdx.x;
  if (g >= Gn) return;
  const int r0 = a.bt.grp_row[g], r1 = a.bt.grp_row[g + 1];
  const int e_lo = a.bt.grp_edge[g], e_hi = a.bt.grp_edge[g + 1];
  const int nrow = r1 - r0;
  const int ne = e_hi - e_lo;
  // fast path: the group's rows, edges and (edge, head) logits fit the LDS carve and
  // every thread's CH-feature chunk lies inside one head
  const bool fast = G::KV && nrow <= RMAX && ne <= G::EMAX && ne * a.H <= G::EH && a.H <= 8 && a.C >= CH;
  const uint32_t ctr = a.rng_ctr ? *a.rng_ctr : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const bool pe_lds = a.first && a.pe_k > 0 && a.pe_k <= KPE;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NCT = (4 * D) / 16;
  const int d0 = lane * VPL;
  const bool act = d0 < D;

  // ---- W fragments of this wave's first column tiles and the gate weights, issued
  //      before anything else so the weight fetch overlaps the staging round trip
  constexpr int PRE = D <= 64 ? (NCT / CONV_WAVES) : 1;
  float4 wpre[PRE][D / 16];
#pragma unroll
  for (int pi = 0; pi < PRE; ++pi) {
    const float* wrow = a.w_all + (size_t)((wave + pi * CONV_WAVES) * 16 + lr) * D + lg * 4;
#pragma unroll
    for (int kb = 0; kb < D / 16; ++kb) wpre[pi][kb] = *reinterpret_cast<const float4*>(wrow + kb * 16);
  }
  // gate weights: the row-parallel fast path holds this thread's CH-feature chunk,
  // the wave-per-row general path VPL features per lane
  const int prow = tid / TPR, pchunk = tid - prow * TPR, f0 = pchunk * CH;
  float w1c[CH], w2c[CH], w3c[CH];
  float w1[VPL], w2[VPL], w3[VPL];
  if (fast) {
#pragma unroll
    for (int c = 0; c < CH; c += 4) {
      const float4 x1 = *reinterpret_cast<const float4*>(a.w_beta + f0 + c);
      const float4 x2 = *reinterpret_cast<const float4*>(a.w_beta + D + f0 + c);
      const float4 x3 = *reinterpret_cast<const float4*>(a.w_beta + 2 * D + f0 + c);
      w1c[c] = x1.x; w1c[c + 1] = x1.y; w1c[c + 2] = x1.z; w1c[c + 3] = x1.w;
      w2c[c] = x2.x; w2c[c + 1] = x2.y; w2c[c + 2] = x2.z; w2c[c + 3] = x2.w;
      w3c[c] = x3.x; w3c[c + 1] = x3.y; w3c[c + 2] = x3.z; w3c[c + 3] = x3.w;
    }
  } else {
    load_vec<VPL>(w1, a.w_beta + d0, act);
    load_vec<VPL>(w2, a.w_beta + D + d0, act);
    load_vec<VPL>(w3, a.w_beta + 2 * D + d0, act);
  }

  // ---- stage: previous BN stats, CSR slice, node items, LapPE projection weight
  if (!a.first) {
    prev_bn_stats<D, CONV_BLOCK>(a.train, a.cred, Gn, a.p_part, a.p_stats, a.p_rmean, a.p_rvar, a.p_nbt, a.bn_eps,
                                 a.bn_mom, s_bn, s_bn + D, XO, LOG);
  }
  if (fast) {
    for (int i = tid; i <= nrow; i += CONV_BLOCK) iptr[i] = a.bt.in_ptr[r0 + i] - e_lo;
    for (int k = tid; k < ne; k += CONV_BLOCK) isrc[k] = a.bt.in_src[e_lo + k] - r0;
    for (int i = tid; i < nrow; i += CONV_BLOCK) {
      const int k1 = a.bt.in_ptr[r0 + i + 1] - e_lo;
      for (int k = a.bt.in_ptr[r0 + i] - e_lo; k < k1; ++k) edst[k] = i;
    }
  }
  if (pe_lds) {
    for (int idx = tid; idx < D * a.pe_k; idx += CONV_BLOCK) {
      const int j = idx / a.pe_k, k = idx - j * a.pe_k;
      PEs[j * KPE + k] = a.wpe[idx];
    }
  }
  if (a.first) {
    for (int i = tid; i < min(RMAX, nrow); i += CONV_BLOCK) items[i] = a.bt.node_item[r0 + i];
  }
  __syncthreads();
  GTR_PH(a.layer, 1);

  // ---- phase P+M: layer input rows -> LDS -> QKVS projection (MFMA f32), chunks of RMAX rows
  const uint32_t st_prev = drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  for (int rc = r0; rc < r1; rc += RMAX) {
    const int m = min(RMAX, r1 - rc);
    if (a.first && rc != r0) {
      for (int i = tid; i < m; i += CONV_BLOCK) items[i] = a.bt.node_item[rc + i];
      __syncthreads();
    }
    if (pe_lds) {
      for (int idx = tid; idx < m * a.pe_k; idx += CONV_BLOCK) {
        const int i = idx / a.pe_k, k = idx - i * a.pe_k;
        const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)(rc + i) * a.pe_k
                                       : a.pe_tab + (size_t)items[i] * a.pe_k;
        PEs[D * KPE + i * KPE + k] = pr[k];
      }
      __syncthreads();
    }
    for (int idx = tid; idx < m * D; idx += CONV_BLOCK) {
      const int i = idx / D, j = idx - i * D;
      const int r = rc + i;
      const size_t o = (size_t)r * D + j;
      float val;
      if (a.first) {
        val = a.table[(size_t)items[i] * D + j];
        if (a.pe_k > 0) {
          float acc = 0.0f;
          if (pe_lds) {
            const float* pr = PEs + D * KPE + i * KPE;
            const float* wr = PEs + j * KPE;
            for (int k = 0; k < a.pe_k; ++k) acc += pr[k] * wr[k];
          } else {
            const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)r * a.pe_k : a.pe_tab + (size_t)items[i] * a.pe_k;
            const float* wr = a.wpe + (size_t)j * a.pe_k;
            for (int k = 0; k < a.pe_k; ++k) acc += pr[k] * wr[k];
          }
          val = val + (acc + a.bpe[j]);
        }
      } else {
        float y = (a.p_out[o] - s_bn[j]) * s_bn[D + j] * a.p_gamma[j] + a.p_beta[j];
        y = y + a.p_xin[o];
        val = y * dr.mul(st_prev, (uint32_t)o);
      }
      a.xin[o] = val;
      XO[i * XS + j] = val;
    }
    __syncthreads();
#pragma unroll
    for (int ti = 0; ti < NCT / CONV_WAVES; ++ti) {
      const int ct = wave + ti * CONV_WAVES;
      float4 wf[D / 16];
      if (ti < PRE) {
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb) wf[kb] = wpre[ti < PRE ? ti : 0][kb];
      } else {
        const float* wrow = a.w_all + (size_t)(ct * 16 + lr) * D + lg * 4;
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb) wf[kb] = *reinterpret_cast<const float4*>(wrow + kb * 16);
      }
      const int col = ct * 16 + lr;
      const float bias = a.b_all[col];
      const int which = col / D, cc = col - which * D;
      // LDS copies on the fast path: 0 = query -> QS[0], 1 = key -> KV[0], 2 = value -> KV[1], 3 = skip -> QS[1]
      float* ldst = nullptr;
      if (fast) ldst = (which == 0 ? QSs : which == 1 ? KVs : which == 2 ? KVs + RMAX * XS : QSs + RMAX * XS) + cc;
      for (int rt = 0; rt * 16 < m; ++rt) {
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        const float* xrow = XO + (rt * 16 + lr) * XS + lg * 4;
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb)
          acc = mfma4(*reinterpret_cast<const float4*>(xrow + kb * 16), wf[kb], acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rt * 16 + lg * 4 + i;
          if (row < m) {
            const float v = acc[i] + bias;
            a.qkvs[(size_t)(rc + row) * (4 * D) + col] = v;
            if (ldst) ldst[row * XS] = v;
          }
        }
      }
    }
    __syncthreads();
  }

  GTR_PH(a.layer, 2);
  // ---- phase A: attention over in-edges + beta gate (wave per destination row)
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  if (fast) {
    const int H = a.H, C = a.C;
    // (L) logits of every (edge, head), the head's C features split over SPL lanes
    const int SPL = C >= 16 ? 4 : 1;
    const int cw = C / SPL;
    const int nit = ne * H * SPL;
    for (int base = 0; base < nit; base += CONV_BLOCK) {
      const int idx = base + tid;
      const int it = idx / SPL;
      float dot = 0.0f;
      if (idx < nit) {
        const int sub = idx - it * SPL;
        const int e = it / H, h = it - e * H;
        const float* q = QSs + edst[e] * XS + h * C + sub * cw;
        const float* k = KVs + isrc[e] * XS + h * C + sub * cw;
        for (int c = 0; c < cw; c += 4) {
          const float4 x = *reinterpret_cast<const float4*>(q + c);
          const float4 y = *reinterpret_cast<const float4*>(k + c);
          dot += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
        }
      }
      if (SPL == 4) {
        dot += __shfl_xor(dot, 1);
        dot += __shfl_xor(dot, 2);
      }
      if (idx < nit && idx == it * SPL) LOG[it] = dot / a.sqrt_c;
    }
    __syncthreads();
    // (S) softmax over each destination's in-edges per head (PyG softmax: exp(l - max) /
    //     (sum + 1e-16)); alpha -> HBM for backward, alpha * dropout mask -> LDS
    for (int idx = tid; idx < nrow * H; idx += CONV_BLOCK) {
      const int i = idx / H, h = idx - i * H;
      const int e0 = iptr[i], e1 = iptr[i + 1];
      float m = -INFINITY;
      for (int e = e0; e < e1; ++e) m = fmaxf(m, LOG[e * H + h]);
      float z = 0.0f;
      for (int e = e0; e < e1; ++e) z += expf(LOG[e * H + h] - m);
      const float zd = z + 1e-16f;
      for (int e = e0; e < e1; ++e) {
        const int eg = (e + e_lo) * H + h;
        const float al = expf(LOG[e * H + h] - m) / zd;
        a.alpha[eg] = al;
        LOG[e * H + h] = al * dr.mul(st_attn, (uint32_t)eg);
      }
    }
    __syncthreads();
    // (G) aggregation + beta gate: TPR lanes per row, CH features each
    float ag[CH], sv[CH];
    float u = 0.0f;
    const bool live = prow < nrow;
    if (live) {
      const int hd = f0 / C;
#pragma unroll
      for (int c = 0; c < CH; ++c) ag[c] = 0.0f;
      const int e1 = iptr[prow + 1];
      for (int e = iptr[prow]; e < e1; ++e) {
        const float ad = LOG[e * H + hd];
        const float* vr = KVs + RMAX * XS + isrc[e] * XS + f0;
#pragma unroll
        for (int c = 0; c < CH; c += 4) {
          const float4 v = *reinterpret_cast<const float4*>(vr + c);
          ag[c] += ad * v.x; ag[c + 1] += ad * v.y; ag[c + 2] += ad * v.z; ag[c + 3] += ad * v.w;
        }
      }
      const float* srow = QSs + RMAX * XS + prow * XS + f0;
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(srow + c);
        sv[c] = v.x; sv[c + 1] = v.y; sv[c + 2] = v.z; sv[c + 3] = v.w;
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) u += w1c[c] * ag[c] + w2c[c] * sv[c] + w3c[c] * (ag[c] - sv[c]);
    }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) u += __shfl_xor(u, o);
    if (live) {
      const float beta = 1.0f / (1.0f + expf(-u));
      const size_t ro = (size_t)(r0 + prow) * D + f0;
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        float4 o4;
        o4.x = beta * sv[c] + (1.0f - beta) * ag[c];
        o4.y = beta * sv[c + 1] + (1.0f - beta) * ag[c + 1];
        o4.z = beta * sv[c + 2] + (1.0f - beta) * ag[c + 2];
        o4.w = beta * sv[c + 3] + (1.0f - beta) * ag[c + 3];
        *reinterpret_cast<float4*>(a.agg + ro + c) = make_float4(ag[c], ag[c + 1], ag[c + 2], ag[c + 3]);
        *reinterpret_cast<float4*>(a.out + ro + c) = o4;
        *reinterpret_cast<float4*>(XO + prow * XS + f0 + c) = o4;
      }
      if (pchunk == 0) a.gate[r0 + prow] = beta;
    }
  } else {
    for (int t = r0 + wave; t < r1; t += CONV_WAVES)
      attn_row<D>(a, t, t, a.qkvs, a.qkvs + 3 * D, a.qkvs + D, a.qkvs + 2 * D, 4 * D, a.bt.in_ptr, a.bt.in_src, 0,
                  lane, dr, st_attn, w1, w2, w3, nullptr);
  }
  if (!a.train) return;

  // ---- phase S: this group's BatchNorm partial (count, mean, M2); slices of rows per thread
  __syncthreads();
  GTR_PH(a.layer, 3);
  constexpr int NS = CONV_BLOCK / D >= 1 ? CONV_BLOCK / D : 1;
  float* red = LOG;  // scratch: the logits are consumed
  float* part = a.bn_part + (size_t)g * (1 + 2 * D);
  {
    const int j = tid % D, sl = tid / D;
    float sum = 0.0f;
    if (sl < NS) {
      if (fast) for (int i = sl; i < nrow; i += NS) sum += XO[i * XS + j];
      else for (int i = sl; i < nrow; i += NS) sum += a.out[(size_t)(r0 + i) * D + j];
    }
    __syncthreads();
    if (sl < NS) red[sl * D + j] = sum;
    __syncthreads();
    if (tid < D) {
      float tot = 0.0f;
      for (int q = 0; q < NS; ++q) tot += red[q * D + tid];
      const float mean = nrow > 0 ? tot / (float)nrow : 0.0f;
      red[NS * D + tid] = mean;
      part[1 + tid] = mean;
    }
    __syncthreads();
    float m2 = 0.0f;
    if (sl < NS) {
      const float mean = red[NS * D + j];
      if (fast) for (int i = sl; i < nrow; i += NS) { const float d = XO[i * XS + j] - mean; m2 += d * d; }
      else for (int i = sl; i < nrow; i += NS) { const float d = a.out[(size_t)(r0 + i) * D + j] - mean; m2 += d * d; }
    }
    __syncthreads();
    if (sl < NS) red[sl * D + j] = m2;
    __syncthreads();
    if (tid < D) {
      float tot = 0.0f;
      for (int q = 0; q < NS; ++q) tot += red[q * D + tid];
      part[1 + D + tid] = tot;
    }
    if (tid == 0) part[0] = (float)nrow;
  }
  GTR_PH(a.layer, 4);
  GTR_PH_CLK(a.layer, 7);
  if (a.cred) return;  // the consuming kernel reduces the partials
  if (!arrive_last(a.cnt, (uint32_t)Gn, s_flag)) return;
  bn_stats_from_parts<D, CONV_BLOCK>(a.bn_part, Gn, a.bn_eps, s_bn, s_bn + D, XO, red);
  for (int j = tid; j < D; j += CONV_BLOCK) {
    a.bn_stats[j] = s_bn[j];
    a.bn_stats[D + j] = s_bn[D + j];
    a.bn_rmean[j] = (1.0f - a.bn_mom) * a.bn_rmean[j] + a.bn_mom * s_bn[j];
    a.bn_rvar[j] = (1.0f - a.bn_mom) * a.bn_rvar[j] + a.bn_mom * XO[j];
  }
  if (tid == 0) {
    reset_counter(a.cnt);
    if (a.bn_nbt) *a.bn_nbt += 1;
  }
}

struct ReadoutK {
  gtr_batch bt;
  int L1, train, flags, loss_kind, cred, fin, pad0, pad1;
  float temperature, dual_alpha, bn_eps, bn_mom, scale;
  uint32_t seed, thresh;
  int drop_on;
  const uint32_t* rng_ctr;
  const float* table;
  const float* out;
  const float* xin;
  float* stats;
  const float* part;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float* se;
  const float* dse_in;
  float* dse_out;
  float* coef_tgt;
  float* coef_neg;
  float* loss_part;
  float* loss_out;
  uint32_t* cnt;
  float* dy;
  float* gpart;
  float* gsum;
};

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_readout(ReadoutK a) {
  constexpr int VPL = D >= 64 ? D / 64 : 1;
  constexpr int NB = 8;   // node rows in flight per wave
  constexpr int NK = 8;   // negative rows in flight per wave
  __shared__ float s_bn[3 * D];
  __shared__ float s_scr[2 * GTR_BLOCK + D];
  __shared__ float s_red[GTR_WAVES][2 * D];
  __shared__ float s_loss[GTR_WAVES][2];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GTR_PH(16, 0);
  const int B = a.bt.hdr[1];
  const int n = a.bt.n_neg;
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const uint32_t ctr = a.rng_ctr ? *a.rng_ctr : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st = drop_stream(1, (uint32_t)a.L1, ctr);
  const bool do_fwd = a.flags & GTR_RO_FWD, do_loss = a.flags & GTR_RO_LOSS, do_bwd = a.flags & GTR_RO_BWD;
  const bool use_lw = a.loss_kind == GTR_LOSS_LISTWISE || a.loss_kind == GTR_LOSS_DUAL;
  const bool use_bpr = a.loss_kind == GTR_LOSS_BPR || a.loss_kind == GTR_LOSS_DUAL;
  const float w_lw = a.loss_kind == GTR_LOSS_DUAL ? a.dual_alpha : 1.0f;
  const float w_bpr = a.loss_kind == GTR_LOSS_DUAL ? 1.0f - a.dual_alpha : 1.0f;
  const float inv_bn = 1.0f / ((float)B * (float)n);  // BPR mean over B*n
  const float inv_b = 1.0f / (float)B;                // listwise mean over B
  const float inv_t = 1.0f / a.temperature;

  if (do_fwd) {
    prev_bn_stats<D, GTR_BLOCK>(a.train, a.cred, a.bt.hdr[4], a.part, a.stats, a.rmean, a.rvar, a.nbt, a.bn_eps,
                                a.bn_mom, s_bn, s_bn + D, s_bn + 2 * D, s_scr);
  } else if (do_bwd) {
    for (int j = tid; j < D; j += GTR_BLOCK) { s_bn[j] = a.stats[j]; s_bn[D + j] = a.stats[D + j]; }
  }
  __syncthreads();
  GTR_PH(16, 1);
  float bm[VPL], br[VPL], bg[VPL], bb[VPL];
  if (do_fwd || do_bwd) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int j = act ? d0 + v : 0;
      bm[v] = s_bn[j]; br[v] = s_bn[D + j]; bg[v] = a.gamma[j]; bb[v] = a.beta[j];
    }
  }

  float gs[VPL], gx[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) { gs[v] = 0.0f; gx[v] = 0.0f; }
  float lw_sum = 0.0f, bpr_sum = 0.0f;

  for (int b = blockIdx.x * GTR_WAVES + wave; b < B; b += gridDim.x * GTR_WAVES) {
    const int n0 = a.bt.node_ptr[b], n1 = a.bt.node_ptr[b + 1];
    const float cnt = (float)(n1 - n0);
    float se[VPL], dse[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) dse[v] = 0.0f;
    if (do_fwd) {
      float acc[VPL];
#pragma unroll
      for (int v = 0; v < VPL; ++v) acc[v] = 0.0f;
      for (int i0 = n0; i0 < n1; i0 += NB) {
        float ov[NB][VPL], xv[NB][VPL];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const bool ok = act && (i0 + q < n1);
          load_vec<VPL>(ov[q], a.out + (size_t)(i0 + q) * D + d0, ok);
          load_vec<VPL>(xv[q], a.xin + (size_t)(i0 + q) * D + d0, ok);
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          if (i0 + q < n1) {
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
              const size_t o = (size_t)(i0 + q) * D + d0 + v;
              float y = (ov[q][v] - bm[v]) * br[v] * bg[v] + bb[v];
              y = y + xv[q][v];
              acc[v] += y * dr.mul(st, (uint32_t)o);
            }
          }
        }
      }
#pragma unroll
      for (int v = 0; v < VPL; ++v) se[v] = acc[v] / cnt;
      store_vec<VPL>(a.se + (size_t)b * D + d0, se, act);
    } else {
      load_vec<VPL>(se, a.se + (size_t)b * D + d0, act);
    }

    if (do_loss) {
      const float* trow = a.table + (size_t)a.bt.target[b] * D;
      const int* negs = a.bt.negatives + (size_t)b * n;
      float tv[VPL];
      load_vec<VPL>(tv, trow + d0, act);
      float pos = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) pos += se[v] * tv[v];
      pos = wave_sum(pos);
      float dpos = 0.0f;
      float m = pos * inv_t, z = 1.0f;
      int nid = 0;
      // pass 1: BPR terms (+ coefficients when BPR only) and online log-sum-exp for listwise
      for (int k0 = 0; k0 < n; k0 += NK) {
        if ((k0 & 63) == 0) nid = (k0 + lane < n) ? negs[k0 + lane] : 0;
        float rv[NK][VPL];
#pragma unroll
        for (int q = 0; q < NK; ++q) {
          const int id = __shfl(nid, (k0 + q) & 63);
          load_vec<VPL>(rv[q], a.table + (size_t)id * D + d0, act && (k0 + q < n));
        }
#pragma unroll
        for (int q = 0; q < NK; ++q) {
          const int k = k0 + q;
          if (k >= n) break;
          float sk = 0.0f;
#pragma unroll
          for (int v = 0; v < VPL; ++v) sk += se[v] * rv[q][v];
          sk = wave_sum(sk);
          float cb = 0.0f;
          if (use_bpr) {
            const float sg = 1.0f / (1.0f + expf(-(pos - sk)));
            bpr_sum += -logf(sg + 1e-8f);
            const float dz = -(sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
            dpos += dz;
            cb = -dz;
          }
          if (use_lw) {
            const float l = sk * inv_t;
            const float mn = fmaxf(m, l);
            z = z * expf(m - mn) + expf(l - mn);
            m = mn;
          } else {
            if (lane == 0) a.coef_neg[(size_t)b * n + k] = cb;
#pragma unroll
            for (int v = 0; v < VPL; ++v) dse[v] += cb * rv[q][v];
          }
        }
      }
      if (use_lw) {
        const float lse = m + logf(z);
        lw_sum += lse - pos * inv_t;
        dpos += (expf(pos * inv_t - lse) - 1.0f) * inv_b * inv_t * w_lw;
        // pass 2: softmax coefficients (+ BPR coefficients for dual)
        for (int k0 = 0; k0 < n; k0 += NK) {
          if ((k0 & 63) == 0) nid = (k0 + lane < n) ? negs[k0 + lane] : 0;
          float rv[NK][VPL];
#pragma unroll
          for (int q = 0; q < NK; ++q) {
            const int id = __shfl(nid, (k0 + q) & 63);
            load_vec<VPL>(rv[q], a.table + (size_t)id * D + d0, act && (k0 + q < n));
          }
#pragma unroll
          for (int q = 0; q < NK; ++q) {
            const int k = k0 + q;
            if (k >= n) break;
            float sk = 0.0f;
#pragma unroll
            for (int v = 0; v < VPL; ++v) sk += se[v] * rv[q][v];
            sk = wave_sum(sk);
            float cb = expf(sk * inv_t - lse) * inv_b * inv_t * w_lw;
            if (use_bpr) {
              const float sg = 1.0f / (1.0f + expf(-(pos - sk)));
              cb += (sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
            }
            if (lane == 0) a.coef_neg[(size_t)b * n + k] = cb;
#pragma unroll
            for (int v = 0; v < VPL; ++v) dse[v] += cb * rv[q][v];
          }
        }
      }
      if (lane == 0) a.coef_tgt[b] = dpos;
#pragma unroll
      for (int v = 0; v < VPL; ++v) dse[v] += dpos * tv[v];
      if (a.dse_out) store_vec<VPL>(a.dse_out + (size_t)b * D + d0, dse, act);
    } else if (do_bwd) {
      load_vec<VPL>(dse, a.dse_in + (size_t)b * D + d0, act);
    }

    if (do_bwd) {
      const float inv_cnt = 1.0f / cnt;
      for (int i0 = n0; i0 < n1; i0 += NB) {
        float ov[NB][VPL];
#pragma unroll
        for (int q = 0; q < NB; ++q) load_vec<VPL>(ov[q], a.out + (size_t)(i0 + q) * D + d0, act && (i0 + q < n1));
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          if (i0 + q < n1) {
            float dyv[VPL];
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
              const size_t o = (size_t)(i0 + q) * D + d0 + v;
              dyv[v] = dse[v] * inv_cnt * dr.mul(st, (uint32_t)o);
              const float xh = (ov[q][v] - bm[v]) * br[v];
              gs[v] += dyv[v];
              gx[v] += dyv[v] * xh;
            }
            store_vec<VPL>(a.dy + (size_t)(i0 + q) * D + d0, dyv, act);
          }
        }
      }
    }
  }

  GTR_PH(16, 2);
  if (!(do_loss || do_bwd)) return;
  // ---- block partials (loss partials pre-scaled by the mean normalisers) in fixed order
  if (lane == 0) { s_loss[wave][0] = lw_sum * (w_lw * inv_b); s_loss[wave][1] = bpr_sum * (w_bpr * inv_bn); }
  if (do_bwd && act) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) { s_red[wave][d0 + v] = gs[v]; s_red[wave][D + d0 + v] = gx[v]; }
  }
  __syncthreads();
  if (do_loss && tid < 2) {
    float acc = 0.0f;
    for (int w = 0; w < GTR_WAVES; ++w) acc += s_loss[w][tid];
    a.loss_part[(size_t)blockIdx.x * 2 + tid] = acc;
  }
  if (do_bwd) {
    for (int j = tid; j < 2 * D; j += GTR_BLOCK) {
      float acc = 0.0f;
      for (int w = 0; w < GTR_WAVES; ++w) acc += s_red[w][j];
      a.gpart[(size_t)blockIdx.x * 2 * D + j] = acc;
    }
  }
  GTR_PH(16, 3);
  if (!a.fin) return;  // loss summed by gtr_step_end, BN sums reduced by the consuming conv_bwd
  if (!arrive_last(a.cnt, gridDim.x, &s_flag)) return;
  if (do_loss && tid == 0) {
    float loss = 0.0f;
    for (int q = 0; q < (int)gridDim.x; ++q) loss += a.loss_part[(size_t)q * 2] + a.loss_part[(size_t)q * 2 + 1];
    a.loss_out[0] = loss;
  }
  if (do_bwd) {
    for (int j = tid; j < 2 * D; j += GTR_BLOCK) {
      float acc = 0.0f;
#pragma unroll 4
      for (int q = 0; q < (int)gridDim.x; ++q) acc += a.gpart[(size_t)q * 2 * D + j];
      a.gsum[j] = acc;
    }
  }
  if (tid == 0) reset_counter(a.cnt);
}

bool check_dims(const gtr_config* c, const char* fn) {
  const int D = c->dim, H = c->heads;
  if (!(D == 32 || D == 64 || D == 128 || D == 256)) {
    set_error("%s: dim %d unsupported (32/64/128/256)", fn, D);
    return false;
  }
  if (H <= 0 || D % H != 0) { set_error("%s: heads %d must divide dim %d", fn, H, D); return false; }
  const int C = D / H, vpl = D >= 64 ? D / 64 : 1;
  if (C < vpl || (C & (C - 1)) != 0) { set_error("%s: head dim %d unsupported", fn, C); return false; }
  if (c->row_group <= 0) { set_error("%s: row_group must be > 0", fn); return false; }
  if (c->pe_k < 0 || c->pe_k > 256) { set_error("%s: pe_k %d out of range", fn, c->pe_k); return false; }
  return true;
}

void drop_params(const gtr_config* c, uint32_t& thresh, float& scale, int& on) {
  on = (c->training && c->dropout > 0.0f) ? 1 : 0;
  double p = c->dropout;
  if (p >= 1.0) p = 0.999999;
  thresh = (uint32_t)(p * 4294967296.0);
  scale = on ? (float)(1.0 / (1.0 - p)) : 1.0f;
}

}  // namespace

GTR_PH_READER(gtr_dbg_fwd_phases)

extern "C" int gtr_conv_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb,
                            const gtr_layer* layers, int l, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_conv_fwd: bad arguments");
    return GTR_E_ARG;
  }
  if (!check_dims(cfg, "gtr_conv_fwd")) return GTR_E_ARG;
  if (!bt->grp_row || !bt->grp_edge) { set_error("gtr_conv_fwd: batch lacks row-group ranges"); return GTR_E_ARG; }
  if (l == 0 && (!emb || !emb->table)) { set_error("gtr_conv_fwd: layer 0 needs the table"); return GTR_E_ARG; }
  if (l == 0 && cfg->pe_k > 0 && (!emb->wpe || !emb->bpe || (!emb->pe_tab && !bt->node_pe))) {
    set_error("gtr_conv_fwd: Laplacian PE not precomputed");
    return GTR_E_ARG;
  }
  const gtr_layer& L = layers[l];
  ConvFwdK k{};
  k.bt = *bt;
  k.H = cfg->heads;
  k.C = cfg->dim / cfg->heads;
  k.first = l == 0;
  k.train = cfg->training;
  k.layer = l;
  k.pe_k = cfg->pe_k;
  k.cred = cfg->consumer_reduce;
  k.sqrt_c = (float)sqrt((double)k.C);
  k.bn_eps = cfg->bn_eps;
  k.bn_mom = cfg->bn_momentum;
  drop_params(cfg, k.thresh, k.scale, k.drop_on);
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  if (l == 0) {
    k.table = emb->table; k.pe_tab = emb->pe_tab; k.wpe = emb->wpe; k.bpe = emb->bpe;
  } else {
    const gtr_layer& P = layers[l - 1];
    k.p_out = P.out; k.p_xin = P.xin; k.p_stats = P.bn_stats; k.p_part = P.bn_part; k.p_gamma = P.bn_gamma;
    k.p_beta = P.bn_beta; k.p_rmean = P.bn_rmean; k.p_rvar = P.bn_rvar; k.p_nbt = P.bn_nbt;
  }
  k.w_all = L.w_all; k.b_all = L.b_all; k.w_beta = L.w_beta;
  k.xin = L.xin; k.qkvs = L.qkvs; k.alpha = L.alpha; k.agg = L.agg; k.gate = L.gate; k.out = L.out;
  k.bn_part = L.bn_part; k.cnt = L.cnt; k.bn_stats = L.bn_stats; k.bn_rmean = L.bn_rmean;
  k.bn_rvar = L.bn_rvar; k.bn_nbt = L.bn_nbt;
  const int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  hipStream_t s = (hipStream_t)stream;
#define GTR_FWD(DD) set_lds_limit<DD>(k_conv_fwd<DD>, (size_t)LayerGeom<DD>::F_WORDS * 4); \
  hipLaunchKernelGGL(k_conv_fwd<DD>, dim3(grid), dim3(CONV_BLOCK), (size_t)LayerGeom<DD>::F_WORDS * 4, s, k)
  switch (cfg->dim) {
    case 32: GTR_FWD(32); break;
    case 64: GTR_FWD(64); break;
    case 128: GTR_FWD(128); break;
    default: GTR_FWD(256); break;
  }
#undef GTR_FWD
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_readout_loss(const gtr_config* cfg, const gtr_batch* bt, const float* table,
                                const gtr_layer* layers, const gtr_head* head, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !head) { set_error("gtr_readout_loss: bad arguments"); return GTR_E_ARG; }
  if (!check_dims(cfg, "gtr_readout_loss")) return GTR_E_ARG;
  if ((head->flags & GTR_RO_LOSS) && (head->loss_kind < GTR_LOSS_BPR || head->loss_kind > GTR_LOSS_DUAL || bt->n_neg <= 0 || !table)) {
    set_error("gtr_readout_loss: bad loss configuration");
    return GTR_E_ARG;
  }
  if ((head->flags & GTR_RO_BWD) && !cfg->training) {
    set_error("gtr_readout_loss: backward requires training mode (batch statistics)");
    return GTR_E_ARG;
  }
  const int L1 = cfg->num_layers - 1;
  const gtr_layer& L = layers[L1];
  ReadoutK k{};
  k.bt = *bt;
  k.L1 = L1;
  k.train = cfg->training;
  k.flags = head->flags;
  k.loss_kind = head->loss_kind;
  k.cred = cfg->consumer_reduce;
  // finalise in-kernel unless a consumer takes over: the BN sums go to conv_bwd and the
  // loss to gtr_step_end in the fused step; a loss-only call always finalises itself.
  k.fin = (!cfg->consumer_reduce || !(head->flags & GTR_RO_BWD)) ? 1 : 0;
  k.temperature = head->temperature;
  k.dual_alpha = head->dual_alpha;
  k.bn_eps = cfg->bn_eps;
  k.bn_mom = cfg->bn_momentum;
  drop_params(cfg, k.thresh, k.scale, k.drop_on);
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.table = table;
  k.out = L.out; k.xin = L.xin; k.stats = L.bn_stats; k.part = L.bn_part; k.gamma = L.bn_gamma; k.beta = L.bn_beta;
  k.rmean = L.bn_rmean; k.rvar = L.bn_rvar; k.nbt = L.bn_nbt;
  k.se = head->se; k.dse_in = head->dse_in; k.dse_out = head->dse_out; k.coef_tgt = head->coef_tgt;
  k.coef_neg = head->coef_neg;
  k.loss_part = head->loss_part; k.loss_out = head->loss_out; k.cnt = head->cnt;
  k.dy = L.dy; k.gpart = L.bn_gpart; k.gsum = L.bn_gsum;
  int grid = (bt->b_cap + GTR_WAVES - 1) / GTR_WAVES;
  if (grid > 256) grid = 256;
  if (grid <= 0) return GTR_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (cfg->dim) {
    case 32: hipLaunchKernelGGL(k_readout<32>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_readout<64>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_readout<128>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_readout<256>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}
