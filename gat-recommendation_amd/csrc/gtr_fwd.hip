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

// The fused forward's projection as QKVS^T tiles (float4 stores; bitwise the same values).
// GTR_CONV_T=0 at build time: the X . W^T form with scalar stores.
#ifndef GTR_CONV_T
#define GTR_CONV_T 1
#endif
#include "gtr_rows.cuh"

#ifndef GTR_WPRE_MAXD
#define GTR_WPRE_MAXD 64  // widths whose projection weights are prefetched whole (per wave); 128 measured slower
#endif

namespace {

using namespace gtr;

GTR_PH_DECL

struct ConvFwdK {
  gtr_batch bt;
  int H, C, first, train, layer, pe_k, cred, split;  // split: split-bf16 projection GEMM
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
  gtr_sweep sw;         // untouched-row AdamW slice run by blocks >= main_grid
  int sw_slot, main_grid;
  int sync, p_nparts;   // SyncBN: previous layer's partials of every rank (p_part_all, p_nparts)
  const float* p_part_all;
  uint32_t ctr_add;     // dropout counter read as *rng_ctr + ctr_add (1 with a fused begin)
  int nbeg;             // fused step begin (layer 0): roles [main_grid, main_grid + nbeg)
  gtr_begin beg;
  int xpack;            // XCD-packed roles (role_block)
  int merge_only;       // split path under SyncBN: the last arriver merges the partials into
                        // bn_part row 0 (count, mean, M2) for the all-gather; no statistics
};

// Block prologue shared by k_conv_fwd (previous layer) and k_readout (last layer):
// BatchNorm mean/rstd of the layer feeding this kernel into s_mean/s_rstd.
//   eval: running stats; train + cred: reduce the producer's partials (block 0 also
//   publishes the stats and updates running_mean/var/num_batches_tracked);
//   train, producer-finalised: read the stats.
template <int D, int BLK>
__device__ __forceinline__ void prev_bn_stats(int train, int cred, int G, const float* part, float* stats,
                                              float* rmean, float* rvar, int64_t* nbt, float eps, float mom,
                                              float* s_mean, float* s_rstd, float* s_uvar, float* scr, bool lead,
                                              bool have_pre, const BnParts<D, BLK>& pre) {
  if (!train) {
    for (int j = threadIdx.x; j < D; j += BLK) {
      s_mean[j] = rmean[j];
      s_rstd[j] = 1.0f / sqrtf(rvar[j] + eps);
    }
  } else if (cred) {
    if (have_pre) bn_stats_from_loaded<D, BLK>(part, G, eps, s_mean, s_rstd, s_uvar, scr, pre);
    else bn_stats_from_parts<D, BLK>(part, G, eps, s_mean, s_rstd, s_uvar, scr);
    if (lead) {
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

// This layer's BatchNorm statistics from the Gn per-workgroup (count, mean, M2) partials
// in bn_part (workgroup g wrote row g): the last arrivers of buckets of GTR_PART_BUCKET
// merge their rows into the bucket's first row, the last bucket merger derives the
// statistics (bn_stats) and updates the running statistics -- or, with merge_only (the
// split path under SyncBN), merges the bucket rows into row 0 for the all-gather.
// red: >= 2 BLK + D floats of LDS scratch; s_bn: 2 D; s_uvar: D.
template <int D, int BLK>
__device__ __forceinline__ void bn_fwd_finalize(const ConvFwdK& a, int g, int Gn, int* s_flag, float* red, float* s_bn,
                                                float* s_uvar) {
  const int tid = threadIdx.x;
  constexpr int PW = 1 + 2 * D;
  const int nbk = (Gn + GTR_PART_BUCKET - 1) / GTR_PART_BUCKET;
  // both levels: the partial rows and the bucket mergers' rows are stored write-through
  // (st_wt) -- no agent-scope release fence anywhere (round 4: the bucket level's fence was
  // part of the ~10 us tail a last arriver added to k_attn_rows)
  if (nbk > 1) {
    constexpr int PB = GTR_PART_BUCKET;
    const int bk = g / PB, b0 = bk * PB;
    if (!arrive_last_wt(a.cnt + 4 + 2 * bk, (uint32_t)min(PB, Gn - b0), s_flag)) return;
    GTR_PH(20 + a.layer, 4);
    float* row0 = a.bn_part + (size_t)b0 * PW;
    bn_merge_parts<D, BLK>(row0, min(PB, Gn - b0), red, PW, row0, true);
    if (tid == 0) reset_counter(a.cnt + 4 + 2 * bk);
    GTR_PH(20 + a.layer, 5);
    // past PB buckets (> 1024 workgroups: C3 / C5 at B = 8192 run ~3.5k) a third level:
    // super-buckets of PB bucket rows, merged by their last arriving bucket merger into the
    // super-bucket's first row, so that no merger walks more than PB rows (a 111-row top
    // merge measured 21 us of the launch's serial tail; one PB-row merge ~5 us).  The
    // super-bucket counters use the odd slots cnt[5 + 2 sb] next to the buckets' even ones;
    // the backward's bucket counters for this layer's sums use the same odd slots in later
    // launches (p_cnt = cnt + 1), and every counter is reset to zero by its last arriver.
    // C3 B = 8192: attention forward 62-68 -> 52 us per layer.
    const int nsb = (nbk + PB - 1) / PB;
    int ntop = nbk;
    size_t top_stride = (size_t)PB * PW;
    if (nsb > 1) {
      const int sb = bk / PB, k0 = sb * PB;
      if (!arrive_last_wt(a.cnt + 5 + 2 * sb, (uint32_t)min(PB, nbk - k0), s_flag)) return;
      float* srow = a.bn_part + (size_t)k0 * PB * PW;  // bucket k0's merged row
      bn_merge_parts<D, BLK>(srow, min(PB, nbk - k0), red, (size_t)PB * PW, srow, true);
      if (tid == 0) reset_counter(a.cnt + 5 + 2 * sb);
      ntop = nsb;
      top_stride = (size_t)PB * PB * PW;
    }
    if (!arrive_last_wt(a.cnt, (uint32_t)ntop, s_flag)) return;
    GTR_PH(20 + a.layer, 6);
    if (a.merge_only) {  // the top rows -> ONE row (row 0, bucket 0's own row: may alias)
      bn_merge_parts<D, BLK>(a.bn_part, ntop, red, top_stride, a.bn_part);
      if (tid == 0) reset_counter(a.cnt);
      return;
    }
    bn_stats_from_parts<D, BLK>(a.bn_part, ntop, a.bn_eps, s_bn, s_bn + D, s_uvar, red, top_stride);
    GTR_PH(20 + a.layer, 7);
  } else {
    if (!arrive_last_wt(a.cnt, (uint32_t)Gn, s_flag)) return;
    if (a.merge_only) {
      bn_merge_parts<D, BLK>(a.bn_part, Gn, red, PW, a.bn_part);
      if (tid == 0) reset_counter(a.cnt);
      return;
    }
    bn_stats_from_parts<D, BLK>(a.bn_part, Gn, a.bn_eps, s_bn, s_bn + D, s_uvar, red);
  }
  for (int j = tid; j < D; j += BLK) {
    a.bn_stats[j] = s_bn[j];
    a.bn_stats[D + j] = s_bn[D + j];
    a.bn_rmean[j] = (1.0f - a.bn_mom) * a.bn_rmean[j] + a.bn_mom * s_bn[j];
    a.bn_rvar[j] = (1.0f - a.bn_mom) * a.bn_rvar[j] + a.bn_mom * s_uvar[j];
  }
  if (tid == 0) {
    reset_counter(a.cnt);
    if (a.bn_nbt) *a.bn_nbt += 1;
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

// gtr_step_begin's work run by extra workgroups of conv_fwd(layer 0) (gtr_begin): each of
// them stages every (row << 13 | slot) composite in LDS and ranks 64 slots, its 8 waves
// counting over slices (the rank sort of k_step_begin with 512 threads); workgroup 0 also
// stamps the touched rows and advances the step counter.  The dropout counter is left
// to the tail: the row groups of this very launch read it (gtr_config.ctr_add).
__device__ __forceinline__ void begin_slice(const gtr_batch& bt, const gtr_begin& g, int blk, uint32_t* ck) {
  int* part = reinterpret_cast<int*>(ck + GTR_BEGIN_MCAP);  // [CONV_WAVES][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int m4 = (m_cap + 3) & ~3;
  const int N = bt.hdr[0], B = bt.hdr[1];
  const bool lead = blk == 0;
  const int32_t tnew = lead ? (int32_t)(*g.step_dev + 1) : 0;
  for (int j = tid; j < m4; j += CONV_BLOCK) {
    uint32_t c = 0xFFFFFFFFu;
    if (j < m_cap) {
      const int key = contrib_key(bt, g.num_items, j, N, B);
      c = ((uint32_t)key << 13) | (uint32_t)j;
      if (lead && g.stamp && key > 0 && key < g.num_items) g.stamp[key] = tnew;
    }
    ck[j] = c;
  }
  __syncthreads();
  const int j = blk * 64 + lane;
  const uint32_t mine = j < m_cap ? ck[j] : 0u;
  const int S = ((m4 / CONV_WAVES) + 4) & ~3;
  const int i0 = wave * S, i1 = min(m4, i0 + S);
  int rank = 0;
  for (int i = i0; i < i1; i += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(ck + i);
    rank += (q.x < mine) + (q.y < mine) + (q.z < mine) + (q.w < mine);
  }
  part[wave * 64 + lane] = rank;
  __syncthreads();
  if (wave == 0 && j < m_cap) {
    int r = 0;
#pragma unroll
    for (int w = 0; w < CONV_WAVES; ++w) r += part[w * 64 + lane];
    g.skeys[r] = (int32_t)(mine >> 13);
    g.svals[r] = (int32_t)(mine & 0x1FFFu);
  }
  if (lead && tid == 0) *g.step_dev = tnew;
}

// Offset of float4 number kb of a lane's W-row fragment: f32 MFMA (k = kb*16 + lg*4 ..)
// or split-bf16 MFMA (k-step kb/2 of 32, lane quad lg's 8 values, half kb&1).
__device__ __forceinline__ int wfrag_off(int kb, int lg, int split) {
  return split ? ((kb >> 1) * 32 + lg * 8 + (kb & 1) * 4) : (kb * 16 + lg * 4);
}

// PROJ = false: the split path's attention kernel (gtr_attn_fwd): xin / qkvs were written
// by gtr_qkvs_fwd (k_proj), so the input build and the projection are left out and the
// group's Q | K | V | S rows are staged from qkvs instead.
template <int D, bool SPLIT, bool PROJ = true>
__device__ __forceinline__ void conv_fwd_body(const ConvFwdK& a, int rb) {
  using G = LayerGeom<D>;
  static_assert(G::F_WORDS >= GTR_BEGIN_MCAP + CONV_WAVES * 64, "LDS carve too small for the fused begin");
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
  __bf16* XH = reinterpret_cast<__bf16*>(sm + G::F_XH);
  __bf16* XL = reinterpret_cast<__bf16*>(sm + G::F_XL);
  float* WB = sm + G::F_WB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GTR_PH(a.layer, 0);
  GTR_PH_CLK(a.layer, 6);
  const int Gn = a.bt.hdr[4];
  const int g = rb;
  if (g >= Gn) {
    if (a.sync && a.train)  // SyncBN: an empty group contributes a zero-count partial
      for (int j = threadIdx.x; j < 1 + 2 * D; j += CONV_BLOCK) a.bn_part[(size_t)g * (1 + 2 * D) + j] = 0.0f;
    return;
  }
  const int r0 = a.bt.grp_row[g], r1 = a.bt.grp_row[g + 1];
  const int e_lo = a.bt.grp_edge[g], e_hi = a.bt.grp_edge[g + 1];
  const int nrow = r1 - r0;
  const int ne = e_hi - e_lo;
  // fast path: the group's rows, edges and (edge, head) logits fit the LDS carve and
  // every thread's CH-feature chunk lies inside one head
  const bool fast = G::KV && nrow <= RMAX && ne <= G::EMAX && ne * a.H <= G::EH && a.H <= 8 && a.C >= CH;
  if (fast) GTR_PH(a.layer, 10);
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const bool pe_lds = a.first && a.pe_k > 0 && a.pe_k <= KPE;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NCT = (4 * D) / 16;
  const int d0 = lane * VPL;
  const bool act = d0 < D;

  // ---- the CSR slice and the node items, requested before the weights: vector loads
  //      retire in order, so the LDS stores of these values below wait only for them and
  //      not for the 16-64 KB weight fetch issued after them (nrow <= RMAX <= 64 and
  //      ne <= EMAX = 2 * CONV_BLOCK on the fast path: at most one / two per thread)
  static_assert(G::EMAX <= 2 * CONV_BLOCK && RMAX < CONV_BLOCK, "one CSR pass per thread");
  int c_ip0 = 0, c_ip1 = 0, c_src0 = 0, c_src1 = 0, c_item = 0;
  if (fast) {
    if (tid <= nrow) c_ip0 = a.bt.in_ptr[r0 + tid];
    if (tid < nrow) c_ip1 = a.bt.in_ptr[r0 + tid + 1];
    if (tid < ne) c_src0 = a.bt.in_src[e_lo + tid];
    if (tid + CONV_BLOCK < ne) c_src1 = a.bt.in_src[e_lo + tid + CONV_BLOCK];
  }
  if (PROJ && a.first && tid < min(RMAX, nrow)) c_item = a.bt.node_item[r0 + tid];
  float4 c_wb = make_float4(0.f, 0.f, 0.f, 0.f);  // gate weights [w1 | w2 | w3] -> LDS (fast path)
  if (fast && tid < (3 * D) / 4) c_wb = *reinterpret_cast<const float4*>(a.w_beta + 4 * tid);
  // layers >= 1, consumer-side BatchNorm: the previous layer's partial rows, also before the
  // weights (the reduction consumes them first)
  const bool pre_bn = PROJ && !a.first && a.train && a.cred;
  const int bn_G = a.sync ? a.p_nparts : Gn;
  const float* bn_part = a.sync ? a.p_part_all : a.p_part;
  BnParts<D, CONV_BLOCK> bnr;
  if (pre_bn) bn_parts_load<D, CONV_BLOCK>(bn_part, bn_G, 1 + 2 * D, bnr);
  if (PROJ && pe_lds) {  // LapPE projection weight, transposed [KPE][D] (k-major, conflict-free
                         // reads), zero-padded past pe_k (stored right away)
    for (int idx = tid; idx < D * KPE; idx += CONV_BLOCK) {
      const int k = idx / D, j = idx - k * D;
      PEs[idx] = k < a.pe_k ? a.wpe[j * a.pe_k + k] : 0.0f;
    }
  }
  GTR_PH(a.layer, 12);

  // ---- W fragments of this wave's first column tiles and the gate weights, issued
  //      early so the weight fetch overlaps the staging round trip
  // every column tile of the wave prefetched up to D = GTR_WPRE_MAXD; beyond, one tile ahead
  // (D = 128 with all 4 tiles held, 128 VGPRs: C3 0.1398 -> 0.1436 ms per step)
  constexpr int PRE = !PROJ ? 1 : D <= GTR_WPRE_MAXD ? (NCT / CONV_WAVES) : 1;
  float4 wpre[PRE][D / 16];
#pragma unroll
  for (int pi = 0; pi < (PROJ ? PRE : 0); ++pi) {
    const float* wrow = a.w_all + (size_t)((wave + pi * CONV_WAVES) * 16 + lr) * D;
#pragma unroll
    for (int kb = 0; kb < D / 16; ++kb)
      wpre[pi][kb] = *reinterpret_cast<const float4*>(wrow + wfrag_off(kb, lg, SPLIT));
  }
  // gate weights: the row-parallel fast path reads its thread's CH-feature chunk from the
  // LDS copy (one 3D-float load per workgroup instead of one per thread); the wave-per-row
  // general path loads VPL features per lane right before its attention loop
  const int prow = tid / TPR, pchunk = tid - prow * TPR, f0 = pchunk * CH;

  GTR_PH(a.layer, 13);
  // ---- layers >= 1: the first chunk's previous-layer rows (out, xin) requested now, so they
  //      arrive while the BatchNorm partials are reduced and the CSR slice is staged
  constexpr int C4 = D / 4;
  constexpr int PRL = (RMAX * C4 + CONV_BLOCK - 1) / CONV_BLOCK;  // float4 per thread and chunk
  constexpr bool PREROWS = D <= 64;  // D = 128 has no registers to spare (spills)
  float4 ppo[PREROWS ? PRL : 1], ppx[PREROWS ? PRL : 1];
  if (PROJ && PREROWS && !a.first) {
    const int m0 = min(RMAX, nrow);
#pragma unroll
    for (int u = 0; u < PRL; ++u) {
      const int idx = tid + u * CONV_BLOCK;
      if (idx < m0 * C4) {
        const int i = idx / C4, j = (idx - i * C4) * 4;
        const size_t o = (size_t)(r0 + i) * D + j;
        if constexpr (PREROWS) {
          ppo[u] = *reinterpret_cast<const float4*>(a.p_out + o);
          ppx[u] = *reinterpret_cast<const float4*>(a.p_xin + o);
        }
      }
    }
  }

  // ---- stage: previous BN stats, CSR slice, node items, LapPE projection weight
  if (PROJ && !a.first) {
    prev_bn_stats<D, CONV_BLOCK>(a.train, a.cred, bn_G, bn_part, a.p_stats, a.p_rmean, a.p_rvar, a.p_nbt,
                                 a.bn_eps, a.bn_mom, s_bn, s_bn + D, XO, LOG, g == 0, pre_bn, bnr);
  }
  GTR_PH(a.layer, 14);
  if (fast) {
    if (tid <= nrow) iptr[tid] = c_ip0 - e_lo;
    if (tid < ne) isrc[tid] = c_src0 - r0;
    if (tid + CONV_BLOCK < ne) isrc[tid + CONV_BLOCK] = c_src1 - r0;
    if (tid < nrow)
      for (int k = c_ip0 - e_lo; k < c_ip1 - e_lo; ++k) edst[k] = tid;
  }
  if (PROJ && a.first && tid < min(RMAX, nrow)) items[tid] = c_item;
  if (fast && tid < (3 * D) / 4) *reinterpret_cast<float4*>(WB + 4 * tid) = c_wb;
  GTR_PH(a.layer, 15);
  __syncthreads();
  GTR_PH(a.layer, 1);

  // ---- phase P+M: layer input rows -> LDS -> QKVS projection (MFMA f32), chunks of RMAX rows
  //      (split path: the group's Q | K | V | S rows of qkvs -> LDS instead)
  const uint32_t st_prev = drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  if constexpr (!PROJ) {
    if (fast) {
      for (int idx = tid; idx < nrow * D; idx += CONV_BLOCK) {  // D float4 per row: Q | K | V | S
        const int i = idx / D, c4 = idx - i * D;
        const int part = c4 / (D / 4), c = (c4 - part * (D / 4)) * 4;
        const float4 v = *reinterpret_cast<const float4*>(a.qkvs + (size_t)(r0 + i) * (4 * D) + part * D + c);
        float* dst = part == 0 ? QSs : part == 1 ? KVs : part == 2 ? KVs + RMAX * XS : QSs + RMAX * XS;
        *reinterpret_cast<float4*>(dst + i * XS + c) = v;
      }
      __syncthreads();
    }
  }
  for (int rc = r0; PROJ && rc < r1; rc += RMAX) {
    const int m = min(RMAX, r1 - rc);
    if (a.first && rc != r0) {
      for (int i = tid; i < m; i += CONV_BLOCK) items[i] = a.bt.node_item[rc + i];
      __syncthreads();
    }
    // layer input rows, float4 per thread: item row + LapPE projection (layer 0) or
    // drop(bn(prev out) + prev in) (layers >= 1); both global gathers of a row in flight together
    constexpr int PRU = PREROWS ? PRL : 1;
#pragma unroll PRU
    for (int u = 0; u < PRL; ++u) {  // m <= RMAX: at most PRL float4 per thread
      const int idx = tid + u * CONV_BLOCK;
      if (idx >= m * C4) break;
      const int i = idx / C4, j = (idx - i * C4) * 4;
      const int r = rc + i;
      const size_t o = (size_t)r * D + j;
      float4 val;
      if (a.first) {
        val = *reinterpret_cast<const float4*>(a.table + (size_t)items[i] * D + j);
        if (a.pe_k > 0) {
          const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)r * a.pe_k : a.pe_tab + (size_t)items[i] * a.pe_k;
          float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (pe_lds && (a.pe_k & 3) == 0) {
            for (int k = 0; k < a.pe_k; k += 4) {
              const float4 p4 = *reinterpret_cast<const float4*>(pr + k);
              pe_fma4(acc, p4, PEs + k * D + j, D);
            }
          } else {
            for (int k = 0; k < a.pe_k; ++k) {
              const float pk = pr[k];
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[q] += pk * a.wpe[(size_t)(j + q) * a.pe_k + k];
            }
          }
          val.x = val.x + (acc[0] + a.bpe[j]);
          val.y = val.y + (acc[1] + a.bpe[j + 1]);
          val.z = val.z + (acc[2] + a.bpe[j + 2]);
          val.w = val.w + (acc[3] + a.bpe[j + 3]);
        }
      } else {
        float4 po, px;
        if constexpr (PREROWS) {
          const bool pre = rc == r0;
          po = pre ? ppo[u] : *reinterpret_cast<const float4*>(a.p_out + o);
          px = pre ? ppx[u] : *reinterpret_cast<const float4*>(a.p_xin + o);
        } else {
          po = *reinterpret_cast<const float4*>(a.p_out + o);
          px = *reinterpret_cast<const float4*>(a.p_xin + o);
        }
        const float4 pg = *reinterpret_cast<const float4*>(a.p_gamma + j);
        const float4 pb = *reinterpret_cast<const float4*>(a.p_beta + j);
        const float4 mu = *reinterpret_cast<const float4*>(s_bn + j);
        const float4 rs = *reinterpret_cast<const float4*>(s_bn + D + j);
        val.x = (((po.x - mu.x) * rs.x * pg.x + pb.x) + px.x) * dr.mul(st_prev, (uint32_t)o);
        val.y = (((po.y - mu.y) * rs.y * pg.y + pb.y) + px.y) * dr.mul(st_prev, (uint32_t)(o + 1));
        val.z = (((po.z - mu.z) * rs.z * pg.z + pb.z) + px.z) * dr.mul(st_prev, (uint32_t)(o + 2));
        val.w = (((po.w - mu.w) * rs.w * pg.w + pb.w) + px.w) * dr.mul(st_prev, (uint32_t)(o + 3));
      }
      *reinterpret_cast<float4*>(a.xin + o) = val;
      *reinterpret_cast<float4*>(XO + i * XS + j) = val;
      if constexpr (SPLIT) {
        bf16x4 h, l;
        split4(val, h, l);
        *reinterpret_cast<bf16x4*>(XH + i * G::XSB + j) = h;
        *reinterpret_cast<bf16x4*>(XL + i * G::XSB + j) = l;
      }
    }
    __syncthreads();
    GTR_PH(a.layer, 11);
    // W fragments of tiles past the prefetched ones are double-buffered: tile ti+1's
    // loads are issued before tile ti's MFMAs and stores (the compiler cannot hoist them
    // over the qkvs stores itself), so only the first such tile waits on L2
    constexpr int NT = NCT / CONV_WAVES;
    constexpr bool DB = NT > PRE && D <= 128;  // D = 256: no registers to spare
    float4 wnext[DB ? D / 16 : 1];
    float bnext = 0.0f;
    if constexpr (DB) {
      const float* wrow = a.w_all + (size_t)((wave + PRE * CONV_WAVES) * 16 + lr) * D;
#pragma unroll
      for (int kb = 0; kb < D / 16; ++kb)
        wnext[kb] = *reinterpret_cast<const float4*>(wrow + wfrag_off(kb, lg, SPLIT));
      bnext = a.b_all[(wave + PRE * CONV_WAVES) * 16 + lr];
    }
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      const int ct = wave + ti * CONV_WAVES;
      float4 wf[D / 16];
      float bias;
      if (ti < PRE) {
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb) wf[kb] = wpre[ti < PRE ? ti : 0][kb];
        bias = a.b_all[ct * 16 + lr];
      } else if constexpr (DB) {
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb) wf[kb] = wnext[kb];
        bias = bnext;
        if (ti + 1 < NT) {
          const float* wrow = a.w_all + (size_t)((ct + CONV_WAVES) * 16 + lr) * D;
#pragma unroll
          for (int kb = 0; kb < D / 16; ++kb)
            wnext[kb] = *reinterpret_cast<const float4*>(wrow + wfrag_off(kb, lg, SPLIT));
          bnext = a.b_all[(ct + CONV_WAVES) * 16 + lr];
        }
      } else {
        const float* wrow = a.w_all + (size_t)(ct * 16 + lr) * D;
#pragma unroll
        for (int kb = 0; kb < D / 16; ++kb)
          wf[kb] = *reinterpret_cast<const float4*>(wrow + wfrag_off(kb, lg, SPLIT));
        bias = a.b_all[ct * 16 + lr];
      }
      const int col = ct * 16 + lr;
      const int which = col / D, cc = col - which * D;
      // LDS copies on the fast path: 0 = query -> QS[0], 1 = key -> KV[0], 2 = value -> KV[1], 3 = skip -> QS[1]
      float* ldst = nullptr;
      if (fast) ldst = (which == 0 ? QSs : which == 1 ? KVs : which == 2 ? KVs + RMAX * XS : QSs + RMAX * XS) + cc;
      bf16x8 bh[D / 32], bl[D / 32];
      if constexpr (SPLIT) {
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) split8(wf[2 * ks], wf[2 * ks + 1], bh[ks], bl[ks]);
      }
      // f32 path (round 5): QKVS^T tiles (the W fragment as the MFMA's A operand; the same
      // products in the same k order, bitwise), so a lane holds four consecutive columns of
      // one row: one float4 store to qkvs and one to LDS instead of four of each
      const int col4 = ct * 16 + lg * 4;
      const int which4 = col4 / D, cc4 = col4 - which4 * D;
      float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
      float* ldst4 = nullptr;
      constexpr bool TT = !SPLIT && GTR_CONV_T;
      if constexpr (TT) {
        bias4 = *reinterpret_cast<const float4*>(a.b_all + col4);
        if (fast) ldst4 = (which4 == 0 ? QSs : which4 == 1 ? KVs : which4 == 2 ? KVs + RMAX * XS : QSs + RMAX * XS) + cc4;
      }
      for (int rt = 0; rt * 16 < m; ++rt) {
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (SPLIT) {
          const __bf16* xh = XH + (rt * 16 + lr) * G::XSB + lg * 8;
          const __bf16* xl = XL + (rt * 16 + lr) * G::XSB + lg * 8;
#pragma unroll
          for (int ks = 0; ks < D / 32; ++ks)
            acc = mfma_split(*reinterpret_cast<const bf16x8*>(xh + ks * 32),
                             *reinterpret_cast<const bf16x8*>(xl + ks * 32), bh[ks], bl[ks], acc);
        } else {
          const float* xrow = XO + (rt * 16 + lr) * XS + lg * 4;
#pragma unroll
          for (int kb = 0; kb < D / 16; ++kb)
            acc = TT ? mfma4(wf[kb], *reinterpret_cast<const float4*>(xrow + kb * 16), acc)
                     : mfma4(*reinterpret_cast<const float4*>(xrow + kb * 16), wf[kb], acc);
        }
        if constexpr (TT) {
          const int row = rt * 16 + lr;
          if (row < m) {
            const float4 v = make_float4(acc[0] + bias4.x, acc[1] + bias4.y, acc[2] + bias4.z, acc[3] + bias4.w);
            *reinterpret_cast<float4*>(a.qkvs + (size_t)(rc + row) * (4 * D) + col4) = v;
            if (ldst4) *reinterpret_cast<float4*>(ldst4 + row * XS) = v;
          }
        } else {
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
        dot = bfly_add<1>(dot);
        dot = bfly_add<2>(dot);
      }
      if (idx < nit && idx == it * SPL) LOG[it] = dot / a.sqrt_c;
    }
    __syncthreads();
    GTR_PH(a.layer, 5);
    // (S) softmax over each destination's in-edges per head (PyG softmax: exp(l - max) /
    //     (sum + 1e-16)); alpha -> HBM for backward, alpha * dropout mask -> LDS.  GL lanes
    //     per (row, head): edges strided over the lanes, max and sum by shuffles (a serial
    //     walk per row made the group's busiest destination the phase's critical path)
    {
      const int pairs = nrow * H;
      const int GL = pair_lanes_deg(pairs, CONV_BLOCK, ne, nrow);
      for (int base = 0; base < pairs; base += CONV_BLOCK / GL) {
        const int pidx = base + tid / GL, gl = tid & (GL - 1);
        int h = 0, e0 = 0, e1 = 0;
        if (pidx < pairs) {
          const int i = pidx / H;
          h = pidx - i * H;
          e0 = iptr[i];
          e1 = iptr[i + 1];
        }
        float m = -INFINITY;
        for (int e = e0 + gl; e < e1; e += GL) m = fmaxf(m, LOG[e * H + h]);
        m = group_max(m, GL);
        float z = 0.0f;
        for (int e = e0 + gl; e < e1; e += GL) z += expf(LOG[e * H + h] - m);
        const float zd = group_sum(z, GL) + 1e-16f;
        for (int e = e0 + gl; e < e1; e += GL) {
          const int eg = (e + e_lo) * H + h;
          const float al = expf(LOG[e * H + h] - m) / zd;
          a.alpha[eg] = al;
          LOG[e * H + h] = al * dr.mul(st_attn, (uint32_t)eg);
        }
      }
    }
    __syncthreads();
    GTR_PH(a.layer, 8);
    // (G) aggregation + beta gate: TPR lanes per row, CH features each (the in-edge walk
    //     can be split ES ways over further lanes, partials summed by shuffles)
    const int ES = 1;  // edge splits measured slower at C2 (1.04 -> 1.32 us): the shuffles cost more than the walk
    const int grow = tid / (TPR * ES), es = (tid / TPR) & (ES - 1);
    float ag[CH], sv[CH];
    float u = 0.0f;
    const bool live = grow < nrow;
#pragma unroll
    for (int c = 0; c < CH; ++c) ag[c] = 0.0f;
    if (live) {
      const int hd = f0 / C;
      const int e1 = iptr[grow + 1];
      for (int e = iptr[grow] + es; e < e1; e += ES) {
        const float ad = LOG[e * H + hd];
        const float* vr = KVs + RMAX * XS + isrc[e] * XS + f0;
#pragma unroll
        for (int c = 0; c < CH; c += 4) {
          const float4 v = *reinterpret_cast<const float4*>(vr + c);
          ag[c] += ad * v.x; ag[c + 1] += ad * v.y; ag[c + 2] += ad * v.z; ag[c + 3] += ad * v.w;
        }
      }
    }
    for (int o = TPR; o < TPR * ES; o <<= 1) {
#pragma unroll
      for (int c = 0; c < CH; ++c) ag[c] += __shfl_xor(ag[c], o);
    }
    if (live) {
      const float* srow = QSs + RMAX * XS + grow * XS + f0;
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(srow + c);
        sv[c] = v.x; sv[c + 1] = v.y; sv[c + 2] = v.z; sv[c + 3] = v.w;
      }
#pragma unroll
      for (int c = 0; c < CH; ++c)
        u += WB[f0 + c] * ag[c] + WB[D + f0 + c] * sv[c] + WB[2 * D + f0 + c] * (ag[c] - sv[c]);
    }
    u = group_sum_c<TPR>(u);
    if (live && es == 0) {
      const float beta = 1.0f / (1.0f + expf(-u));
      const size_t ro = (size_t)(r0 + grow) * D + f0;
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        float4 o4;
        o4.x = beta * sv[c] + (1.0f - beta) * ag[c];
        o4.y = beta * sv[c + 1] + (1.0f - beta) * ag[c + 1];
        o4.z = beta * sv[c + 2] + (1.0f - beta) * ag[c + 2];
        o4.w = beta * sv[c + 3] + (1.0f - beta) * ag[c + 3];
        *reinterpret_cast<float4*>(a.agg + ro + c) = make_float4(ag[c], ag[c + 1], ag[c + 2], ag[c + 3]);
        *reinterpret_cast<float4*>(a.out + ro + c) = o4;
        *reinterpret_cast<float4*>(XO + grow * XS + f0 + c) = o4;
      }
      if (pchunk == 0) a.gate[r0 + grow] = beta;
    }
  } else {
    float w1[VPL], w2[VPL], w3[VPL];
    load_vec<VPL>(w1, a.w_beta + d0, act);
    load_vec<VPL>(w2, a.w_beta + D + d0, act);
    load_vec<VPL>(w3, a.w_beta + 2 * D + d0, act);
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
      st_wt(part + 1 + tid, mean);  // write-through: read by another workgroup in this launch
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
      st_wt(part + 1 + D + tid, tot);
    }
    if (tid == 0) st_wt(part, (float)nrow);
  }
  GTR_PH(a.layer, 4);
  GTR_PH_CLK(a.layer, 7);
  if (a.cred) return;  // the consuming kernel reduces the partials
  bn_fwd_finalize<D, CONV_BLOCK>(a, g, Gn, s_flag, red, s_bn, XO);
}

template <int D, bool SPLIT>
__global__ __launch_bounds__(CONV_BLOCK) void k_conv_fwd(ConvFwdK a) {
  using G = LayerGeom<D>;
  static_assert(G::F_WORDS >= GTR_BEGIN_MCAP + CONV_WAVES * 64, "LDS carve too small for the fused begin");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int rb = role_block(a.main_grid, a.xpack);
  if (rb >= a.main_grid + a.nbeg) {  // extra workgroups: untouched-row AdamW slice
    sweep_slice(a.sw, a.sw_slot, rb - a.main_grid - a.nbeg, gridDim.x - a.main_grid - a.nbeg);
    return;
  }
  if (rb >= a.main_grid) {  // fused step begin (layer 0)
    begin_slice(a.bt, a.beg, rb - a.main_grid, reinterpret_cast<uint32_t*>(sm));
    return;
  }
  conv_fwd_body<D, SPLIT>(a, rb);
}

// Split path (large batches): the attention + gate + BatchNorm partial of one row group
// per workgroup, reading the qkvs rows k_proj wrote (gtr_attn_fwd).
template <int D>
__global__ __launch_bounds__(CONV_BLOCK) void k_attn_fwd(ConvFwdK a) {
  conv_fwd_body<D, false, false>(a, blockIdx.x);
}

// Split path, row-parallel attention (gtr_attn_fwd at large batches): one WAVE per
// destination row instead of one workgroup per row group.  The fused kernels' row-group
// fast path holds ~140 KB of LDS (one group per CU, its phases separated by barriers, no
// overlap between groups); here a workgroup is 4 waves x 2 rows with 20 KB of LDS, so
// several run per CU and one wave's load latency hides behind another's work.  Per row:
// the in-edge source ids one per lane, K rows four edges in flight -> logits (LDS, per
// head) and their maximum; the softmax denominator; V rows four in flight -> alpha,
// dropout, the weighted sum; the beta gate -> agg / out / gate (PyG TransformerConv,
// SURVEY.md Appendix A).  The workgroup's 8 output rows give one BatchNorm partial.
// 8 waves, 16 rows: one BatchNorm partial per 16 rows (half the partials of 4 waves, so
// the bucketed last-arriver merges at the launch's end are half as long): C3 B = 8192
// 0.7676 -> 0.7589 ms per step, C4 B = 1024 (split) 0.3618 -> 0.3586; 16 waves measured
// 0.776 ms at C3 B = 8192.  -DAR_BLOCK=... at build time for A/B.
#ifndef AR_BLOCK
#define AR_BLOCK 512
#endif
#define AR_WAVES (AR_BLOCK / 64)
#define AR_RPW 2                   // rows per wave
#define AR_ROWS (AR_WAVES * AR_RPW)  // rows per workgroup = one BatchNorm partial
#define AR_ECH 64                  // in-edges of a row handled with LDS logits
#define AR_HMAX 8
#ifndef AR_VR
#define AR_VR 8                    // V rows of a row pair held in registers
#endif
#ifndef GTR_AR_WAVES_EU
#define GTR_AR_WAVES_EU 6
#endif

// The BatchNorm partial (count, mean, M2) of a workgroup's nrow output rows (s_out:
// [AR_ROWS][D] in LDS), written through into bn_part row g for the last arrivers.
template <int D>
__device__ __forceinline__ void bn_rows_partial(const ConvFwdK& a, int g, int nrow, const float* s_out, float* s_red) {
  const int tid = threadIdx.x;
  constexpr int NS = AR_BLOCK / D >= 1 ? AR_BLOCK / D : 1;
  float* part = a.bn_part + (size_t)g * (1 + 2 * D);
  {
    const int j = tid % D, sl = tid / D;
    float sum = 0.0f;
    if (sl < NS)
      for (int i = sl; i < nrow; i += NS) sum += s_out[i * D + j];
    s_red[sl * D + j] = sum;
    __syncthreads();
    if (tid < D) {
      float tot = 0.0f;
      for (int q2 = 0; q2 < NS; ++q2) tot += s_red[q2 * D + tid];
      const float mean = tot / (float)nrow;
      s_red[NS * D + tid] = mean;
      st_wt(part + 1 + tid, mean);  // write-through: read by another workgroup in this launch
    }
    __syncthreads();
    float m2 = 0.0f;
    if (sl < NS) {
      const float mean = s_red[NS * D + j];
      for (int i = sl; i < nrow; i += NS) { const float d = s_out[i * D + j] - mean; m2 += d * d; }
    }
    __syncthreads();
    s_red[sl * D + j] = m2;
    __syncthreads();
    if (tid < D) {
      float tot = 0.0f;
      for (int q2 = 0; q2 < NS; ++q2) tot += s_red[q2 * D + tid];
      st_wt(part + 1 + D + tid, tot);
    }
    if (tid == 0) st_wt(part, (float)nrow);
  }
}

template <int D>
__global__ __launch_bounds__(AR_BLOCK) __attribute__((amdgpu_waves_per_eu(GTR_AR_WAVES_EU, 8))) void k_attn_rows(ConvFwdK a) {
  constexpr int VPL = D >= 64 ? D / 64 : 1;
  __shared__ __attribute__((aligned(16))) float s_out[AR_ROWS][D];
  __shared__ float s_lg[AR_WAVES][AR_ECH][AR_HMAX];
  __shared__ float s_red[2 * AR_BLOCK + D];
  __shared__ float s_bn[2 * D];
  __shared__ float s_uv[D];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.bt.hdr[0];
  const int Gn = (N + AR_ROWS - 1) / AR_ROWS;
  const int g = blockIdx.x;
  if (g >= Gn) return;  // block-uniform: only live workgroups write partials and arrive
  const int r0 = g * AR_ROWS, nrow = min(AR_ROWS, N - r0);
  GTR_PH(20 + a.layer, 0);
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int GL = C / VPL;
  const int head = act ? d0 / C : 0;
  const bool leader = act && ((lane & (GL - 1)) == 0);
  float w1[VPL], w2[VPL], w3[VPL];
  load_vec<VPL>(w1, a.w_beta + d0, act);
  load_vec<VPL>(w2, a.w_beta + D + d0, act);
  load_vec<VPL>(w3, a.w_beta + 2 * D + d0, act);
  const float* Q = a.qkvs;
  const float* K = a.qkvs + D;
  const float* V = a.qkvs + 2 * D;
  const float* S = a.qkvs + 3 * D;
  // one row of the wave alone (hub rows, wide heads: the general bodies)
  auto one_row = [&](int i) {
      const int rl = wave * AR_RPW + i;
      const int t = r0 + rl;
      if (t >= N) return;  // wave-uniform
      const int e0 = a.bt.in_ptr[t], e1 = a.bt.in_ptr[t + 1];
      if (e1 - e0 > AR_ECH || H > AR_HMAX) {  // hub rows: the general wave-per-row body
        attn_row<D>(a, t, t, Q, S, K, V, 4 * D, a.bt.in_ptr, a.bt.in_src, 0, lane, dr, st_attn, w1, w2, w3, s_out[rl]);
        return;
      }
      const int ne = e1 - e0;
      const int my_src = lane < ne ? a.bt.in_src[e0 + lane] : 0;
      float q[VPL], sv[VPL], ag[VPL];
      load_vec<VPL>(q, Q + (size_t)t * (4 * D) + d0, act);
      load_vec<VPL>(sv, S + (size_t)t * (4 * D) + d0, act);
      // logits <Q[t], K[src]> / sqrt(C) per head, four K rows in flight
      float m = -INFINITY;
      for (int j = 0; j < ne; j += 4) {
        float kv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(kv[u], K + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float dt = 0.0f;
#pragma unroll
          for (int v = 0; v < VPL; ++v) dt += q[v] * kv[u][v];
          const float l = group_sum(dt, GL) / a.sqrt_c;
          if (j + u < ne) {
            m = fmaxf(m, l);
            if (leader) s_lg[wave][j + u][head] = l;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float z = 0.0f;
      for (int e = 0; e < ne; ++e) z += expf(s_lg[wave][e][head] - m);
      const float zd = z + 1e-16f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) ag[v] = 0.0f;
      // alpha = softmax, attention dropout, aggregate V rows (four in flight)
      for (int j = 0; j < ne; j += 4) {
        float vv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(vv[u], V + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j + u < ne) {
            const int eg = e0 + j + u;
            const float al = expf(s_lg[wave][j + u][head] - m) / zd;
            if (leader) a.alpha[(size_t)eg * H + head] = al;
            const float ad = al * dr.mul(st_attn, (uint32_t)(eg * H + head));
#pragma unroll
            for (int v = 0; v < VPL; ++v) ag[v] += ad * vv[u][v];
          }
        }
      }
      float uu = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) uu += w1[v] * ag[v] + w2[v] * sv[v] + w3[v] * (ag[v] - sv[v]);
      uu = wave_sum(uu);
      const float beta = 1.0f / (1.0f + expf(-uu));
      float o[VPL];
#pragma unroll
      for (int v = 0; v < VPL; ++v) o[v] = beta * sv[v] + (1.0f - beta) * ag[v];
      store_vec<VPL>(a.agg + (size_t)t * D + d0, ag, act);
      store_vec<VPL>(a.out + (size_t)t * D + d0, o, act);
      store_vec<VPL>(s_out[rl] + d0, o, act);
      if (lane == 0) a.gate[t] = beta;
      __builtin_amdgcn_wave_barrier();  // s_lg is reused by the wave's next row
  };
  // The wave's two rows together: their in-edges are contiguous (CSR by destination), so
  // ONE id load covers both rows, and every K row is requested together with its V row
  // (the first AR_VR edges' V rows stay in registers for the aggregation) -- three
  // dependent memory rounds per wave instead of four per row.  Per row the arithmetic is
  // the single-row body's, operation for operation (same edge order for the maximum, the
  // denominator and the weighted sum): bitwise the same outputs.
  const int t0 = r0 + wave * AR_RPW;
  if (t0 < N) {  // wave-uniform
    const bool two = t0 + 1 < N;
    const int e0 = a.bt.in_ptr[t0], em = a.bt.in_ptr[t0 + 1];
    const int e2 = two ? a.bt.in_ptr[t0 + 2] : em;
    const int ne0 = em - e0, ne = e2 - e0;
    static_assert(AR_RPW == 2, "the paired body covers two rows per wave");
    GTR_PH(20 + a.layer, 8);
    if (ne > AR_ECH || H > AR_HMAX) {
      one_row(0);
      one_row(1);
    } else {
      const int my_src = lane < ne ? a.bt.in_src[e0 + lane] : 0;
      float q0[VPL], s0[VPL], q1[VPL], s1[VPL], ag0[VPL], ag1[VPL];
      load_vec<VPL>(q0, Q + (size_t)t0 * (4 * D) + d0, act);
      load_vec<VPL>(s0, S + (size_t)t0 * (4 * D) + d0, act);
      load_vec<VPL>(q1, Q + (size_t)(t0 + 1) * (4 * D) + d0, act && two);
      load_vec<VPL>(s1, S + (size_t)(t0 + 1) * (4 * D) + d0, act && two);
      float m0 = -INFINITY, m1 = -INFINITY;
      float vh[AR_VR][VPL];
      auto logit = [&](int e, const float (&kr)[VPL]) {
        const bool r1 = e >= ne0;  // wave-uniform
        float dt = 0.0f;
#pragma unroll
        for (int v = 0; v < VPL; ++v) dt += (r1 ? q1[v] : q0[v]) * kr[v];
        const float l = group_sum(dt, GL) / a.sqrt_c;
        if (e < ne) {
          if (r1) m1 = fmaxf(m1, l);
          else m0 = fmaxf(m0, l);
          if (leader) s_lg[wave][e][head] = l;
        }
      };
#pragma unroll
      for (int jj = 0; jj < AR_VR; jj += 4) {
        if (jj < ne) {  // wave-uniform
          float kv[4][VPL];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int src = __shfl(my_src, (jj + u) & 63);
            const bool ok = act && jj + u < ne;
            load_vec<VPL>(kv[u], K + (size_t)src * (4 * D) + d0, ok);
            load_vec<VPL>(vh[jj + u], V + (size_t)src * (4 * D) + d0, ok);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) logit(jj + u, kv[u]);
        }
      }
      GTR_PH(20 + a.layer, 9);
      for (int j = AR_VR; j < ne; j += 4) {
        float kv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(kv[u], K + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) logit(j + u, kv[u]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      GTR_PH(20 + a.layer, 10);
      float z0 = 0.0f, z1 = 0.0f;
      for (int e = 0; e < ne0; ++e) z0 += expf(s_lg[wave][e][head] - m0);
      for (int e = ne0; e < ne; ++e) z1 += expf(s_lg[wave][e][head] - m1);
      const float zd0 = z0 + 1e-16f, zd1 = z1 + 1e-16f;
      GTR_PH(20 + a.layer, 11);
#pragma unroll
      for (int v = 0; v < VPL; ++v) { ag0[v] = 0.0f; ag1[v] = 0.0f; }
      auto accum = [&](int e, const float (&vr)[VPL]) {
        const bool r1 = e >= ne0;  // wave-uniform
        const int eg = e0 + e;
        const float al = expf(s_lg[wave][e][head] - (r1 ? m1 : m0)) / (r1 ? zd1 : zd0);
        if (leader) a.alpha[(size_t)eg * H + head] = al;
        const float ad = al * dr.mul(st_attn, (uint32_t)(eg * H + head));
        if (r1) {
#pragma unroll
          for (int v = 0; v < VPL; ++v) ag1[v] = __builtin_fmaf(ad, vr[v], ag1[v]);  // the contracted `ag += ad * v`
        } else {
#pragma unroll
          for (int v = 0; v < VPL; ++v) ag0[v] = __builtin_fmaf(ad, vr[v], ag0[v]);
        }
      };
#pragma unroll
      for (int e = 0; e < AR_VR; ++e)
        if (e < ne) accum(e, vh[e]);
      for (int j = AR_VR; j < ne; j += 4) {
        float vv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(vv[u], V + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (j + u < ne) accum(j + u, vv[u]);
      }
      auto finish = [&](int t, int rl, const float (&ag)[VPL], const float (&sv)[VPL]) {
        float uu = 0.0f;
#pragma unroll
        for (int v = 0; v < VPL; ++v) uu += w1[v] * ag[v] + w2[v] * sv[v] + w3[v] * (ag[v] - sv[v]);
        uu = wave_sum(uu);
        const float beta = 1.0f / (1.0f + expf(-uu));
        float o[VPL];
#pragma unroll
        for (int v = 0; v < VPL; ++v) o[v] = beta * sv[v] + (1.0f - beta) * ag[v];
        store_vec<VPL>(a.agg + (size_t)t * D + d0, ag, act);
        store_vec<VPL>(a.out + (size_t)t * D + d0, o, act);
        store_vec<VPL>(s_out[rl] + d0, o, act);
        if (lane == 0) a.gate[t] = beta;
      };
      GTR_PH(20 + a.layer, 12);
      finish(t0, wave * AR_RPW, ag0, s0);
      if (two) finish(t0 + 1, wave * AR_RPW + 1, ag1, s1);
      GTR_PH(20 + a.layer, 13);
    }
  }
  if (!a.train) return;
  // ---- this workgroup's BatchNorm partial (count, mean, M2) over its rows
  __syncthreads();
  GTR_PH(20 + a.layer, 1);
  bn_rows_partial<D>(a, g, nrow, &s_out[0][0], s_red);
  GTR_PH(20 + a.layer, 2);
  bn_fwd_finalize<D, AR_BLOCK>(a, g, Gn, &s_flag, s_red, s_bn, s_uv);
  GTR_PH(20 + a.layer, 3);
}

// Split path, row-parallel attention with float4 lanes and an online softmax (round 5;
// gtr_attn_fwd for D <= 128, H <= AR_HMAX).  A destination row of D floats is LPR = D/4
// lanes holding one float4 each, so one wave instruction gathers RPI = 64/LPR source
// rows (D = 128: two) -- twice the bytes per instruction of k_attn_rows' VPL = D/64.
// A wave owns two consecutive rows (their in-edges are contiguous: one id load), and its
// RPI sub-groups of LPR lanes walk the pair's edges in rounds of U edges per sub-group:
// every edge's K AND V rows are requested in the same round, the next round's rows are
// requested before this round's arithmetic (the rounds of a hub row overlap), and each
// lane folds its edges into a running (max, sum, weighted-V) per row and head (online
// softmax, no second gather pass).  The sub-groups' states are then combined with xor
// butterflies; alpha = exp(l - m) / (sum + 1e-16) is written in a lane-parallel pass
// over the (edge, head) pairs from the logits kept in LDS (a pair of more than AR_ECH
// edges: in the alpha buffer itself, rewritten in place).  PyG TransformerConv
// (SURVEY.md Appendix A): softmax over in-edges, dropout on alpha, sum alpha*V,
// beta gate.  The weighted sum is (sum_e exp(l_e - m) mask_e V_e) / (sum + 1e-16) with
// the running rescale: the reference's value up to fp32 reordering (oracle tests, 1e-3).
#ifndef AR4_U
#define AR4_U 4
#endif
#ifndef GTR_AR4_WAVES_EU
#define GTR_AR4_WAVES_EU 6
#endif
#ifndef AR4_FOLD      // 1: a round's edges folded with one rescale (U + 1 exps); 0: edge by edge (2 per edge)
#define AR4_FOLD 1
#endif
#ifndef AR4_WBLDS     // 1: the gate's weights staged in LDS per workgroup; 0: loaded per wave after the edges
#define AR4_WBLDS 0
#endif
#ifndef AR4_LANEDROP  // 1: the round's dropout hashes lane-parallel (one per lane) when they fit one wave
#define AR4_LANEDROP 0
#endif

template <int O>
__device__ __forceinline__ float xor_add(float x) {
  if constexpr (O >= 16) return bfly_add<O>(x);
  else return x + __shfl_xor(x, O);
}
template <int O>
__device__ __forceinline__ float xor_max(float x) {
  if constexpr (O >= 16) return bfly_max<O>(x);
  else return fmaxf(x, __shfl_xor(x, O));
}

struct OnlineSm {
  float m, z;
  float4 acc;
};

// fold one edge (logit l, dropout multiplier mk, V row v) into a running state
__device__ __forceinline__ void sm_push(OnlineSm& s, float l, float mk, const float4& v) {
  const float mn = fmaxf(s.m, l);
  const float sc = s.m == -INFINITY ? 0.0f : expf(s.m - mn);
  const float p = expf(l - mn);
  s.z = s.z * sc + p;
  const float w = p * mk;
  s.acc.x = s.acc.x * sc + w * v.x;
  s.acc.y = s.acc.y * sc + w * v.y;
  s.acc.z = s.acc.z * sc + w * v.z;
  s.acc.w = s.acc.w * sc + w * v.w;
  s.m = mn;
}

// combine the states of lanes l and l ^ O (both lanes end with the same state)
template <int O>
__device__ __forceinline__ void sm_combine(OnlineSm& s) {
  const float mn = xor_max<O>(s.m);
  const float f = s.m == -INFINITY ? 0.0f : expf(s.m - mn);
  s.z = xor_add<O>(s.z * f);
  s.acc.x = xor_add<O>(s.acc.x * f);
  s.acc.y = xor_add<O>(s.acc.y * f);
  s.acc.z = xor_add<O>(s.acc.z * f);
  s.acc.w = xor_add<O>(s.acc.w * f);
  s.m = mn;
}

// combine over the xor offsets O, 2 O, ... below END (the lanes of one row's sub-groups)
template <int O, int END>
__device__ __forceinline__ void sm_combine_upto(OnlineSm& s) {
  if constexpr (O < END) {
    sm_combine<O>(s);
    sm_combine_upto<O * 2, END>(s);
  }
}

template <int D>
__global__ __launch_bounds__(AR_BLOCK) __attribute__((amdgpu_waves_per_eu(GTR_AR4_WAVES_EU, 8))) void k_attn_rows4(ConvFwdK a) {
  constexpr int LPR = D / 4, RPI = 64 / LPR, U = AR4_U;
  constexpr int SPR = RPI / 2;   // sub-groups per row of the pair
  constexpr int EPR = U * SPR;   // edges of a row per round
  static_assert(RPI >= 2, "a sub-group per row of the pair");
  __shared__ __attribute__((aligned(16))) float s_out[AR_ROWS][D];
#if AR4_WBLDS
  __shared__ __attribute__((aligned(16))) float s_wb[3 * D];  // the gate's weights
#endif
  __shared__ float s_lg[AR_WAVES][AR_ECH][AR_HMAX];
  __shared__ float s_mz[AR_WAVES][2][AR_HMAX][2];
  __shared__ float s_red[2 * AR_BLOCK + D];
  __shared__ float s_bn[2 * D];
  __shared__ float s_uv[D];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.bt.hdr[0];
  const int Gn = (N + AR_ROWS - 1) / AR_ROWS;
  const int g = blockIdx.x;
  if (g >= Gn) return;  // block-uniform: only live workgroups write partials and arrive
  const int r0 = g * AR_ROWS, nrow = min(AR_ROWS, N - r0);
  GTR_PH(20 + a.layer, 0);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const int t0 = r0 + wave * AR_RPW;
  const bool live = t0 < N;                 // wave-uniform
  const bool two = t0 + 1 < N;
  const int tc = live ? t0 : 0;             // clamped: the loads below are unconditional
  const int e0 = a.bt.in_ptr[tc], em = a.bt.in_ptr[tc + 1];
  const int e2r = a.bt.in_ptr[min(tc + 2, N)];
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  // the gate's weights are staged once per workgroup, their load issued behind the row
  // pointers' (an LDS read after the edges instead of a dependent L2 round trip at the end
  // of every wave)
  static_assert(3 * D / 4 <= AR_BLOCK, "one float4 of the gate weights per thread");
#if AR4_WBLDS
  if (tid < 3 * D / 4)
    *reinterpret_cast<float4*>(&s_wb[4 * tid]) = *reinterpret_cast<const float4*>(a.w_beta + 4 * tid);
  __syncthreads();
#endif
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const int sub = lane / LPR, c4 = lane - sub * LPR, col = 4 * c4;
  const int rr = sub / SPR, si = sub - rr * SPR;  // this lane's row of the pair, its slot in the row
  const int C = a.C, H = a.H;
  const int hsh = __ffs(H) - 1;       // H is a power of two (D and C are)
  const int HL = C >= 4 ? C / 4 : 1;  // lanes of one head inside a sub-group
  const int head = col / C;
  const bool leader = (c4 & (HL - 1)) == 0;
  const float inv_sc = 1.0f / a.sqrt_c;
  // dropout multipliers of a round's (row, slot, head) triples, one per lane, when they fit
  // one wave (EPR * H <= 32): a lane hashes one triple instead of every lane hashing U
  const bool lane_drop = AR4_LANEDROP && dr.on && 2 * EPR * H <= 64;
  if (live) {  // wave-uniform
    const int e2 = two ? e2r : em;
    const int ne0 = em - e0, ne = e2 - e0;
    const bool mine = rr == 0 || two;          // this lane's row exists
    const int eb = rr == 0 ? 0 : ne0;          // the row's first edge (pair-local)
    const int nr = rr == 0 ? ne0 : ne - ne0;   // the row's in-edges
    const int nmax = max(ne0, ne - ne0);
    GTR_PH(20 + a.layer, 8);
    const float* qrow = a.qkvs + (size_t)(t0 + (mine ? rr : 0)) * (4 * D) + col;
    const float4 q = *reinterpret_cast<const float4*>(qrow);
    const float4 sv = *reinterpret_cast<const float4*>(qrow + 3 * D);
    const bool lds_lg = ne <= AR_ECH;
    const float* K = a.qkvs + D + col;
    const float* V = a.qkvs + 2 * D + col;
    OnlineSm st{-INFINITY, 0.0f, z4};
    // the pair's source ids, one per lane (pairs of more than 64 in-edges: per round)
    const bool one_chunk = ne <= 64;
    const int my_src = a.bt.in_src[ne > 0 ? e0 + min(lane, ne - 1) : 0];  // clamped, unconditional
    // this lane's triple for the lane-parallel dropout hash: (row dr_r, slot dr_s, head dr_h)
    const int dr_r = lane >> (hsh + __ffs(EPR) - 1), dr_s = (lane >> hsh) & (EPR - 1), dr_h = lane & (H - 1);
    for (int j = 0; j < nmax; j += EPR) {
      int ids = my_src, ib = eb;
      if (!one_chunk) {  // hub pair: this round's ids -- row 0's edges j.. in lanes 0-31, row 1's in 32-63
        const int k = j + (lane & 31);
        const bool okid = lane < 32 ? k < ne0 : ne0 + k < ne;
        ids = okid ? a.bt.in_src[e0 + (lane < 32 ? k : ne0 + k)] : 0;
        ib = rr * 32 - j;
      }
      float4 kc[U], vc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = j + u * SPR + si;  // edge k of this lane's row
        const int src = __shfl(ids, (ib + k) & 63);
        const size_t off = (mine && k < nr) ? (size_t)src * (4 * D) : 0;  // row 0 of the buffer: in bounds
        kc[u] = *reinterpret_cast<const float4*>(K + off);
        vc[u] = *reinterpret_cast<const float4*>(V + off);
      }
      float mkl = 1.0f;
      if (lane_drop) {
        const int k = j + dr_s;
        const int nrr = dr_r == 0 ? ne0 : ne - ne0;
        const int eg = e0 + (dr_r == 0 ? 0 : ne0) + k;
        mkl = (dr_r < 2 && k < nrr) ? dr.mul(st_attn, (uint32_t)(eg * H + dr_h)) : 0.0f;
      }
#if AR4_FOLD
      float lg[U], mk[U];
      float mx = -INFINITY;
#endif
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = j + u * SPR + si;
        const float dt = q.x * kc[u].x + q.y * kc[u].y + q.z * kc[u].z + q.w * kc[u].w;
        const float l = group_sum(dt, HL) * inv_sc;
        const int e = eb + k;
        float m1 = lane_drop ? __shfl(mkl, (((rr * EPR + u * SPR + si) << hsh) + head) & 63) : 0.0f;
#if AR4_FOLD
        lg[u] = -INFINITY;
#endif
        if (mine && k < nr) {
          if (!lane_drop) m1 = dr.mul(st_attn, (uint32_t)((e0 + e) * H + head));
          if (leader) {
            if (lds_lg) s_lg[wave][e][head] = l;
            else a.alpha[(size_t)(e0 + e) * H + head] = l;
          }
#if AR4_FOLD
          lg[u] = l;
          mx = fmaxf(mx, l);
#else
          sm_push(st, l, m1, vc[u]);
#endif
        }
#if AR4_FOLD
        mk[u] = m1;
#endif
      }
#if AR4_FOLD
      // fold the round's edges: one rescale of the running state, one exp per edge
      if (mx != -INFINITY) {
        const float mn = fmaxf(st.m, mx);
        const float sc = st.m == -INFINITY ? 0.0f : expf(st.m - mn);
        st.z *= sc;
        st.acc.x *= sc; st.acc.y *= sc; st.acc.z *= sc; st.acc.w *= sc;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (lg[u] != -INFINITY) {
            const float p = expf(lg[u] - mn);
            st.z += p;
            const float w = p * mk[u];
            st.acc.x += w * vc[u].x;
            st.acc.y += w * vc[u].y;
            st.acc.z += w * vc[u].z;
            st.acc.w += w * vc[u].w;
          }
        }
        st.m = mn;
      }
#endif
    }
    GTR_PH(20 + a.layer, 9);
    sm_combine_upto<LPR, LPR * SPR>(st);  // the row's SPR sub-groups
    const float zd = st.z + 1e-16f;
    const float rz = 1.0f / zd;
    if (si == 0 && leader) {
      s_mz[wave][rr][head][0] = st.m;
      s_mz[wave][rr][head][1] = rz;
    }
    if (!lds_lg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // raw logits in alpha
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    GTR_PH(20 + a.layer, 10);
    // alpha of every (edge, head) pair of the row pair, lane-parallel (contiguous stores)
    if (lds_lg) {
      for (int idx = lane; idx < ne * H; idx += 64) {
        const int e = idx >> hsh, h = idx & (H - 1);
        const int r = e >= ne0 ? 1 : 0;
        a.alpha[(size_t)(e0 + e) * H + h] = expf(s_lg[wave][e][h] - s_mz[wave][r][h][0]) * s_mz[wave][r][h][1];
      }
    } else {
      for (int idx = lane; idx < ne * H; idx += 64) {
        const int e = idx >> hsh, h = idx & (H - 1);
        const int r = e >= ne0 ? 1 : 0;
        const size_t at = (size_t)(e0 + e) * H + h;
        a.alpha[at] = expf(a.alpha[at] - s_mz[wave][r][h][0]) * s_mz[wave][r][h][1];
      }
    }
    GTR_PH(20 + a.layer, 11);
    // aggregate, beta gate, outputs (slot 0 of each row's sub-groups stores the row)
#if AR4_WBLDS
    const float4 w1 = *reinterpret_cast<const float4*>(&s_wb[col]);
    const float4 w2 = *reinterpret_cast<const float4*>(&s_wb[D + col]);
    const float4 w3 = *reinterpret_cast<const float4*>(&s_wb[2 * D + col]);
#else
    const float4 w1 = *reinterpret_cast<const float4*>(a.w_beta + col);  // late: registers
    const float4 w2 = *reinterpret_cast<const float4*>(a.w_beta + D + col);
    const float4 w3 = *reinterpret_cast<const float4*>(a.w_beta + 2 * D + col);
#endif
    const float4 ag = make_float4(st.acc.x * rz, st.acc.y * rz, st.acc.z * rz, st.acc.w * rz);
    float uu = w1.x * ag.x + w2.x * sv.x + w3.x * (ag.x - sv.x);
    uu += w1.y * ag.y + w2.y * sv.y + w3.y * (ag.y - sv.y);
    uu += w1.z * ag.z + w2.z * sv.z + w3.z * (ag.z - sv.z);
    uu += w1.w * ag.w + w2.w * sv.w + w3.w * (ag.w - sv.w);
    uu = group_sum_c<LPR>(uu);
    const float beta = 1.0f / (1.0f + expf(-uu));
    const float4 o = make_float4(beta * sv.x + (1.0f - beta) * ag.x, beta * sv.y + (1.0f - beta) * ag.y,
                                 beta * sv.z + (1.0f - beta) * ag.z, beta * sv.w + (1.0f - beta) * ag.w);
    if (si == 0 && mine) {
      const int t = t0 + rr;
      *reinterpret_cast<float4*>(a.agg + (size_t)t * D + col) = ag;
      *reinterpret_cast<float4*>(a.out + (size_t)t * D + col) = o;
      *reinterpret_cast<float4*>(&s_out[wave * AR_RPW + rr][col]) = o;
      if (c4 == 0) a.gate[t] = beta;
    }
    GTR_PH(20 + a.layer, 12);
    GTR_PH(20 + a.layer, 13);
  }
  if (!a.train) return;
  __syncthreads();
  GTR_PH(20 + a.layer, 1);
  bn_rows_partial<D>(a, g, nrow, &s_out[0][0], s_red);
  GTR_PH(20 + a.layer, 2);
  bn_fwd_finalize<D, AR_BLOCK>(a, g, Gn, &s_flag, s_red, s_bn, s_uv);
  GTR_PH(20 + a.layer, 3);
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
  gtr_sweep sw;         // untouched-row AdamW slice run by blocks >= main_grid
  int sw_slot, main_grid;
  int sync, nparts;     // SyncBN: the last layer's partials of every rank (part_all, nparts)
  const float* part_all;
  uint32_t ctr_add;
  int xpack;            // XCD-packed roles (role_block)
  float loss_b;         // > 0: the loss means' session count (gtr_config.loss_batch)
};

// Block per session (grid-strided): RO_WAVES waves split the session's node rows and
// its scoring rows.  The target / negative rows are requested before the session
// embedding exists (they depend only on the batch), held in registers (KR rows per
// wave) and reused by the coefficient pass; chunks beyond RO_WAVES*KR rows reload.
#define RO_BLOCK 512
#define RO_WAVES (RO_BLOCK / 64)

template <int D>
__device__ __forceinline__ void readout_body(const ReadoutK& a, int rb) {
  constexpr int VPL = D >= 64 ? D / 64 : 1;
  constexpr int KR = 32 / VPL;       // scoring rows per wave held in registers
  constexpr int CHN = RO_WAVES * KR; // negatives per chunk
  __shared__ float s_bn[3 * D];
  __shared__ float s_scr[2 * RO_BLOCK + D];
  __shared__ __attribute__((aligned(16))) float s_vec[RO_WAVES][D];
  __shared__ float s_w[RO_WAVES][4];
  __shared__ float s_red[RO_WAVES][2 * D];
  __shared__ float s_loss[RO_WAVES][2];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GTR_PH(16, 0);
  const int B = a.bt.hdr[1];
  const int n = a.bt.n_neg;
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st = drop_stream(1, (uint32_t)a.L1, ctr);
  const bool do_fwd = a.flags & GTR_RO_FWD, do_loss = a.flags & GTR_RO_LOSS, do_bwd = a.flags & GTR_RO_BWD;
  const bool use_lw = a.loss_kind == GTR_LOSS_LISTWISE || a.loss_kind == GTR_LOSS_DUAL;
  const bool use_bpr = a.loss_kind == GTR_LOSS_BPR || a.loss_kind == GTR_LOSS_DUAL;
  const float w_lw = a.loss_kind == GTR_LOSS_DUAL ? a.dual_alpha : 1.0f;
  const float w_bpr = a.loss_kind == GTR_LOSS_DUAL ? 1.0f - a.dual_alpha : 1.0f;
  const float Bm = a.loss_b > 0.0f ? a.loss_b : (float)B;  // gtr_config.loss_batch
  const float inv_bn = 1.0f / (Bm * (float)n);  // BPR mean over B*n
  const float inv_b = 1.0f / Bm;                // listwise mean over B
  const float inv_t = 1.0f / a.temperature;
  const int nchunk = do_loss ? (n + CHN - 1) / CHN : 0;

  // scoring rows of the block's next session (chunk 0: target + first CHN negatives),
  // requested before anything that waits: they depend only on the batch, so the first
  // session's gathers overlap the prologue's BatchNorm reduction
  float tv[VPL], rv[KR][VPL], sk[KR];
  float pov[VPL], pxv[VPL];  // the wave's first node row of the session (out, xin), consumed first
  auto issue = [&](int b) {
    if (b >= B) return;
    if (do_fwd) {
      const int i = a.bt.node_ptr[b] + wave;
      if (i < a.bt.node_ptr[b + 1]) {
        load_vec<VPL>(pov, a.out + (size_t)i * D + d0, act);
        load_vec<VPL>(pxv, a.xin + (size_t)i * D + d0, act);
      }
    }
    if (!do_loss) return;
    const int* ng = a.bt.negatives + (size_t)b * n;
    load_vec<VPL>(tv, a.table + (size_t)a.bt.target[b] * D + d0, act);
    const int kq = wave + lane * RO_WAVES;
    const int nid = (lane < KR && kq < n) ? ng[kq] : 0;
#pragma unroll
    for (int q = 0; q < KR; ++q) {
      const int id = __shfl(nid, q);
      if (wave + q * RO_WAVES < n) load_vec<VPL>(rv[q], a.table + (size_t)id * D + d0, act);
    }
  };
  // consumer-side BatchNorm partials first (consumed first: vector loads retire in order)
  const bool pre_bn = do_fwd && a.train && a.cred;
  const int bn_G = a.sync ? a.nparts : a.bt.hdr[4];
  const float* bn_part = a.sync ? a.part_all : a.part;
  BnParts<D, RO_BLOCK> bnr;
  if (pre_bn) bn_parts_load<D, RO_BLOCK>(bn_part, bn_G, 1 + 2 * D, bnr);
  issue(rb);
  if (do_fwd) {
    prev_bn_stats<D, RO_BLOCK>(a.train, a.cred, bn_G, bn_part,
                               a.stats, a.rmean, a.rvar, a.nbt, a.bn_eps,
                               a.bn_mom, s_bn, s_bn + D, s_bn + 2 * D, s_scr, rb == 0, pre_bn, bnr);
  } else if (do_bwd) {
    for (int j = tid; j < D; j += RO_BLOCK) { s_bn[j] = a.stats[j]; s_bn[D + j] = a.stats[D + j]; }
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

  for (int b = rb; b < B; b += a.main_grid) {
    const int n0 = a.bt.node_ptr[b], n1 = a.bt.node_ptr[b + 1];
    const float cnt = (float)(n1 - n0);
    const int* negs = a.bt.negatives + (size_t)b * n;
    // ---- (1) scoring rows of chunk 0: requested by issue() before this iteration
    // ---- (2) session embedding: mean over node rows of drop(bn(out) + xin)
    float se[VPL];
    constexpr int NBR = 2;  // node rows per wave whose conv output stays in registers for (5)
    float oc[NBR][VPL];
    if (do_fwd) {
      float acc[VPL];
#pragma unroll
      for (int v = 0; v < VPL; ++v) acc[v] = 0.0f;
      for (int i = n0 + wave, q = 0; i < n1; i += RO_WAVES, ++q) {
        float ov[VPL], xv[VPL];
        if (q == 0) {  // requested by issue()
#pragma unroll
          for (int v = 0; v < VPL; ++v) { ov[v] = pov[v]; xv[v] = pxv[v]; }
        } else {
          load_vec<VPL>(ov, a.out + (size_t)i * D + d0, act);
          load_vec<VPL>(xv, a.xin + (size_t)i * D + d0, act);
        }
#pragma unroll
        for (int c = 0; c < NBR; ++c)
          if (q == c) {
#pragma unroll
            for (int v = 0; v < VPL; ++v) oc[c][v] = ov[v];
          }
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          const size_t o = (size_t)i * D + d0 + v;
          float y = (ov[v] - bm[v]) * br[v] * bg[v] + bb[v];
          y = y + xv[v];
          acc[v] += y * dr.mul(st, (uint32_t)o);
        }
      }
      if (act) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) s_vec[wave][d0 + v] = acc[v];
      }
      __syncthreads();
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < RO_WAVES; ++w) t += act ? s_vec[w][d0 + v] : 0.0f;
        se[v] = t / cnt;
      }
      if (wave == 0) store_vec<VPL>(a.se + (size_t)b * D + d0, se, act);
      __syncthreads();
    } else {
      load_vec<VPL>(se, a.se + (size_t)b * D + d0, act);
    }

    float dse[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) dse[v] = 0.0f;
    if (do_loss) {
      float pos = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) pos += se[v] * tv[v];
      pos = wave_sum(pos);
      float dpos = 0.0f;
      float m = wave == 0 ? pos * inv_t : -INFINITY, z = wave == 0 ? 1.0f : 0.0f;
      // ---- (3) pass 1: scores, BPR terms, per-wave online log-sum-exp
      for (int c = 0; c < nchunk; ++c) {
        const int kb = c * CHN;
        if (c > 0) {
          const int kq = kb + wave + lane * RO_WAVES;
          const int nid = (lane < KR && kq < n) ? negs[kq] : 0;
#pragma unroll
          for (int q = 0; q < KR; ++q) {
            const int id = __shfl(nid, q);
            if (kb + wave + q * RO_WAVES < n) load_vec<VPL>(rv[q], a.table + (size_t)id * D + d0, act);
          }
        }
#pragma unroll
        for (int q = 0; q < KR; ++q) {
          const int k = kb + wave + q * RO_WAVES;
          if (k < n) {
          float d = 0.0f;
#pragma unroll
          for (int v = 0; v < VPL; ++v) d += se[v] * rv[q][v];
          d = wave_sum(d);
          sk[q] = d;
          {
            if (use_bpr) {
              const float sg = 1.0f / (1.0f + expf(-(pos - d)));
              bpr_sum += -logf(sg + 1e-8f);
              const float dz = -(sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
              dpos += dz;
              if (!use_lw) {
                if (lane == 0) a.coef_neg[(size_t)b * n + k] = -dz;
#pragma unroll
                for (int v = 0; v < VPL; ++v) dse[v] += -dz * rv[q][v];
              }
            }
            if (use_lw) {
              const float l = d * inv_t;
              const float mn = fmaxf(m, l);
              z = z * expf(m - mn) + expf(l - mn);
              m = mn;
            }
          }
          }
        }
      }
      if (use_lw) {
        if (lane == 0) { s_w[wave][0] = m; s_w[wave][1] = z; }
        __syncthreads();
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < RO_WAVES; ++w) M = fmaxf(M, s_w[w][0]);
        float Z = 0.0f;
#pragma unroll
        for (int w = 0; w < RO_WAVES; ++w) Z += s_w[w][1] * expf(s_w[w][0] - M);
        const float lse = M + logf(Z);
        if (wave == 0) {
          lw_sum += lse - pos * inv_t;
          dpos += (expf(pos * inv_t - lse) - 1.0f) * inv_b * inv_t * w_lw;
        }
        // ---- pass 2: softmax (+ BPR) coefficients; rows still in registers for one chunk
        for (int c = 0; c < nchunk; ++c) {
          const int kb = c * CHN;
          if (nchunk > 1) {
            const int kq = kb + wave + lane * RO_WAVES;
            const int nid = (lane < KR && kq < n) ? negs[kq] : 0;
#pragma unroll
            for (int q = 0; q < KR; ++q) {
              const int id = __shfl(nid, q);
              if (kb + wave + q * RO_WAVES < n) load_vec<VPL>(rv[q], a.table + (size_t)id * D + d0, act);
            }
#pragma unroll
            for (int q = 0; q < KR; ++q) {
              if (kb + wave + q * RO_WAVES < n) {
                float d = 0.0f;
#pragma unroll
                for (int v = 0; v < VPL; ++v) d += se[v] * rv[q][v];
                sk[q] = wave_sum(d);
              }
            }
          }
#pragma unroll
          for (int q = 0; q < KR; ++q) {
            const int k = kb + wave + q * RO_WAVES;
            if (k < n) {
              float cb = expf(sk[q] * inv_t - lse) * inv_b * inv_t * w_lw;
              if (use_bpr) {
                const float sg = 1.0f / (1.0f + expf(-(pos - sk[q])));
                cb += (sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
              }
              if (lane == 0) a.coef_neg[(size_t)b * n + k] = cb;
#pragma unroll
              for (int v = 0; v < VPL; ++v) dse[v] += cb * rv[q][v];
            }
          }
        }
      }
      // ---- (4) dse = sum of the waves' partials + dpos * target row
      if (act) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) s_vec[wave][d0 + v] = dse[v];
      }
      if (lane == 0) s_w[wave][2] = dpos;
      __syncthreads();
      float dp = 0.0f;
#pragma unroll
      for (int w = 0; w < RO_WAVES; ++w) dp += s_w[w][2];
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < RO_WAVES; ++w) t += act ? s_vec[w][d0 + v] : 0.0f;
        dse[v] = t + dp * tv[v];
      }
      if (tid == 0) a.coef_tgt[b] = dp;
      if (wave == 0 && a.dse_out) store_vec<VPL>(a.dse_out + (size_t)b * D + d0, dse, act);
      __syncthreads();
    } else if (do_bwd) {
      load_vec<VPL>(dse, a.dse_in + (size_t)b * D + d0, act);
    }

    // ---- (5) readout backward into the node rows + the last BatchNorm's backward sums
    if (do_bwd) {
      const float inv_cnt = 1.0f / cnt;
      for (int i = n0 + wave, q = 0; i < n1; i += RO_WAVES, ++q) {
        float ov[VPL], dyv[VPL];
        if (do_fwd && q < NBR) {
#pragma unroll
          for (int c = 0; c < NBR; ++c)
            if (q == c) {
#pragma unroll
              for (int v = 0; v < VPL; ++v) ov[v] = oc[c][v];
            }
        } else {
          load_vec<VPL>(ov, a.out + (size_t)i * D + d0, act);
        }
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          const size_t o = (size_t)i * D + d0 + v;
          dyv[v] = dse[v] * inv_cnt * dr.mul(st, (uint32_t)o);
          const float xh = (ov[v] - bm[v]) * br[v];
          gs[v] += dyv[v];
          gx[v] += dyv[v] * xh;
        }
        store_vec<VPL>(a.dy + (size_t)i * D + d0, dyv, act);
      }
    }
    issue(b + a.main_grid);  // the next session's rows (rv / tv are free from here)
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
    for (int w = 0; w < RO_WAVES; ++w) acc += s_loss[w][tid];
    st_wt(a.loss_part + (size_t)rb * 2 + tid, acc);
  }
  if (do_bwd) {
    for (int j = tid; j < 2 * D; j += RO_BLOCK) {
      float acc = 0.0f;
      for (int w = 0; w < RO_WAVES; ++w) acc += s_red[w][j];
      st_wt(a.gpart + (size_t)rb * 2 * D + j, acc);
    }
  }
  GTR_PH(16, 3);
  if (!a.fin) return;  // loss summed by the step tail, BN sums reduced by the consuming conv_bwd
  if (!arrive_last_wt(a.cnt, (uint32_t)a.main_grid, &s_flag)) return;
  if (do_loss) {
    __shared__ float s_pair[2];
    block_sum_rows<RO_BLOCK>(a.loss_part, a.main_grid, 2, 2, s_pair, &s_red[0][0]);
    if (tid == 0) a.loss_out[0] = s_pair[0] + s_pair[1];
  }
  if (do_bwd) block_sum_rows<RO_BLOCK>(a.gpart, a.main_grid, 2 * D, (size_t)2 * D, a.gsum, &s_red[0][0]);
  if (tid == 0) reset_counter(a.cnt);
}

template <int D>
__global__ __launch_bounds__(RO_BLOCK) void k_readout(ReadoutK a) {
  const int rb = role_block(a.main_grid, a.xpack);
  if (rb >= a.main_grid) {  // extra workgroups: untouched-row AdamW slice
    sweep_slice(a.sw, a.sw_slot, rb - a.main_grid, gridDim.x - a.main_grid);
    return;
  }
  readout_body<D>(a, rb);
}

// Large-batch readout (b_cap >= ro_wave_min_b(), D <= 128): wave per session, grid-strided;
// RwGeom::RL lanes per row so one wave instruction moves NRG rows (node and scoring rows);
// the scoring rows are streamed in rounds of NRG*KQ and the listwise softmax is
// accumulated online (running max / sum / sum of exp-weighted rows per row group), so
// every table row is read once.  Semantics and outputs identical to k_readout.
#define RW_BLOCK 512
#define RW_WAVES (RW_BLOCK / 64)
#define RW_NMAX 256  // negatives per session whose raw scores stay in LDS

template <int EPL>
__device__ __forceinline__ void ld_row(float (&x)[EPL], const float* p, bool act) {
  if constexpr (EPL == 2) {
    const float2 t = act ? *reinterpret_cast<const float2*>(p) : make_float2(0.f, 0.f);
    x[0] = t.x; x[1] = t.y;
  } else {
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c) {
      const float4 t = act ? reinterpret_cast<const float4*>(p)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
      x[4 * c] = t.x; x[4 * c + 1] = t.y; x[4 * c + 2] = t.z; x[4 * c + 3] = t.w;
    }
  }
}

template <int EPL>
__device__ __forceinline__ void st_row(float* p, const float (&x)[EPL]) {
  if constexpr (EPL == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
  } else {
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c)
      reinterpret_cast<float4*>(p)[c] = make_float4(x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]);
  }
}

// Row-group geometry of the wave readout: NRG row groups of RL = 64 / NRG lanes per wave;
// a lane holds EPL = D / RL features of a row, one load instruction moves NRG rows.
// D = 128 keeps 4 groups of 16 lanes (EPL 8) by measurement: 2 groups of 32 lanes halve
// the row registers (more waves per SIMD) but each round then moves half the rows per
// instruction -- head 87.6 -> 102.4 us at C3 B = 8192, 97.9 -> 118.7 us at C5 B = 8192
// (round-4 A/B, `GTR_RW_NRG128=2`); more waves per EU by launch bounds lost too.
#ifndef GTR_RW_NRG128
#define GTR_RW_NRG128 4
#endif
#ifndef GTR_RW_FOLD
#define GTR_RW_FOLD 1
#endif
template <int D>
struct RwGeom {
  static constexpr int NRG = D >= 128 ? GTR_RW_NRG128 : 4;
  static constexpr int RL = 64 / NRG;
  static constexpr int EPL = D / RL;
};

// sum over the NRG row groups (lanes l, l^RL, ...)
template <int NRG>
__device__ __forceinline__ float sum_groups(float x) {
  if constexpr (NRG == 4) x = bfly_add<16>(x);
  x = bfly_add<32>(x);
  return x;
}

template <int NRG>
__device__ __forceinline__ float max_groups(float x) {
  if constexpr (NRG == 4) x = bfly_max<16>(x);
  return bfly_max<32>(x);
}

// Round r of a session's scoring rows: slot q of row group rg loads negative
// k = r*NRG*KQ + q*NRG + rg (ids fetched by the first NRG*KQ lanes, then shuffled).
template <int D, int KQ>
__device__ __forceinline__ void issue_round(float (&rv)[KQ][RwGeom<D>::EPL], const float* table, const int* negs,
                                            int n, int r, int lane, int rg, int c0) {
  constexpr int NRG = RwGeom<D>::NRG, RND = NRG * KQ;
  const int kl = r * RND + lane;
  const int nid = (lane < RND && kl < n) ? negs[kl] : 0;
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int id = __shfl(nid, q * NRG + rg);
    ld_row<RwGeom<D>::EPL>(rv[q], table + (size_t)id * D + c0, r * RND + q * NRG + rg < n);
  }
}

// The same round from the session's negative ids preloaded into registers (nid[i] holds id
// i * 64 + lane; n <= 256): a round is RND consecutive ids, all in one register (RND divides
// 64), so the round's row loads need no id load of their own (round 4: every round used to
// wait for its ids before its rows -- one memory latency per round on the wave's serial path).
template <int D, int KQ>
__device__ __forceinline__ void issue_round_pre(float (&rv)[KQ][RwGeom<D>::EPL], const float* table,
                                                const int (&nid)[4], int n, int r, int rg, int c0) {
  constexpr int NRG = RwGeom<D>::NRG, RND = NRG * KQ;
  static_assert(64 % RND == 0, "a round never straddles two id registers");
  const int blk = (r * RND) >> 6;  // wave-uniform
  const int src = blk == 0 ? nid[0] : blk == 1 ? nid[1] : blk == 2 ? nid[2] : nid[3];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int id = __shfl(src, ((r * RND) & 63) + q * NRG + rg);
    ld_row<RwGeom<D>::EPL>(rv[q], table + (size_t)id * D + c0, r * RND + q * NRG + rg < n);
  }
}

// Per-session scoring accumulators of one wave (row group rg's share until combined).
template <int EPL>
struct ScoreAcc {
  float dse[EPL];   // BPR part of d loss / d se (sum of -dz * row)
  float accl[EPL];  // listwise: sum of exp(l - mg) * row (online rescaled)
  float mg, zg, dpos, bpr_sum;
};

// Scores of one round's rows (slot q of row group rg = negative k) -> BPR terms and the
// online listwise softmax; raw listwise scores go to sc (LDS, or coef_neg when sc null).
template <int D, int KQ>
__device__ __forceinline__ void consume_round(ScoreAcc<RwGeom<D>::EPL>& A, const float (&rv)[KQ][RwGeom<D>::EPL],
                                              const float (&se)[RwGeom<D>::EPL], float pos, int r, int n, int rg,
                                              bool lead, bool use_bpr, bool use_lw, float inv_bn, float w_bpr,
                                              float inv_t, float* sc, float* coef_row) {
  constexpr int EPL = RwGeom<D>::EPL, NRG = RwGeom<D>::NRG, RND = NRG * KQ;
#if GTR_RW_FOLD
  float lq[KQ];  // the round's listwise logits (-inf past n), folded below with ONE rescale
#endif
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = r * RND + q * NRG + rg;
    float d = 0.0f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) d += se[e] * rv[q][e];
    d = group_sum(d, RwGeom<D>::RL);
#if GTR_RW_FOLD
    lq[q] = k < n ? d * inv_t : -INFINITY;
#endif
    if (k < n) {
      if (use_bpr) {
        const float sg = 1.0f / (1.0f + expf(-(pos - d)));
        if (lead) A.bpr_sum += -logf(sg + 1e-8f);
        const float dz = -(sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
        A.dpos += dz;
#pragma unroll
        for (int e = 0; e < EPL; ++e) A.dse[e] += -dz * rv[q][e];
        if (!use_lw && lead) coef_row[k] = -dz;
      }
      if (use_lw) {
#if !GTR_RW_FOLD
        const float l = d * inv_t;
        const float mn = fmaxf(A.mg, l);
        const float c = expf(A.mg - mn), p = expf(l - mn);
        A.zg = A.zg * c + p;
#pragma unroll
        for (int e = 0; e < EPL; ++e) A.accl[e] = A.accl[e] * c + p * rv[q][e];
        A.mg = mn;
#endif
        if (lead) {
          if (sc) sc[k] = d; else coef_row[k] = d;  // raw score; coefficient once lse is known
        }
      }
    }
  }
#if GTR_RW_FOLD
  // the round's KQ rows into the online softmax with one max and one rescale (KQ + 1 expf
  // instead of 2 KQ, EPL rescale multiplies instead of KQ * EPL); a round with no live row
  // (past n) leaves the state as it is
  if (use_lw) {
    float mn = A.mg;
#pragma unroll
    for (int q = 0; q < KQ; ++q) mn = fmaxf(mn, lq[q]);
    if (mn != -INFINITY) {
      const float c = expf(A.mg - mn);
      float pq[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) pq[q] = expf(lq[q] - mn);
      float z = A.zg * c;
#pragma unroll
      for (int q = 0; q < KQ; ++q) z += pq[q];
      A.zg = z;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        float acc = A.accl[e] * c;
#pragma unroll
        for (int q = 0; q < KQ; ++q) acc = __builtin_fmaf(pq[q], rv[q][e], acc);
        A.accl[e] = acc;
      }
      A.mg = mn;
    }
  }
#endif
}

template <int D>
#ifndef GTR_RW_WAVES_EU
#define GTR_RW_WAVES_EU 1
#endif
__global__ __launch_bounds__(RW_BLOCK) __attribute__((amdgpu_waves_per_eu(GTR_RW_WAVES_EU))) void k_readout_wave(ReadoutK a) {
  using RG = RwGeom<D>;
  constexpr int EPL = RG::EPL;             // features per lane (RL lanes per row)
  constexpr int NRG = RG::NRG;             // row groups per wave
  constexpr int KQ = 4;                    // row slots per lane per round
  constexpr int RND = NRG * KQ;            // scoring rows per wave round
  __shared__ float s_bn[3 * D];            // mean | rstd | unbiased var (prologue)
  __shared__ float s_gb[2 * D];            // gamma | beta
  __shared__ float s_scr[2 * RW_BLOCK + D];
  __shared__ float s_red[RW_WAVES][2 * D];
  __shared__ float s_loss[RW_WAVES][2];
  __shared__ float s_sc[RW_WAVES][RW_NMAX];  // raw listwise scores of the wave's session
  __shared__ int s_flag;
  const int rb = role_block(a.main_grid, a.xpack);
  if (rb >= a.main_grid) {  // extra workgroups: untouched-row AdamW slice
    sweep_slice(a.sw, a.sw_slot, rb - a.main_grid, gridDim.x - a.main_grid);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rg = lane / RG::RL, c0 = (lane & (RG::RL - 1)) * EPL;
  const bool lead = (lane & (RG::RL - 1)) == 0;
  const int B = a.bt.hdr[1];
  const int n = a.bt.n_neg;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st = drop_stream(1, (uint32_t)a.L1, ctr);
  const bool do_fwd = a.flags & GTR_RO_FWD, do_loss = a.flags & GTR_RO_LOSS, do_bwd = a.flags & GTR_RO_BWD;
  const bool use_lw = a.loss_kind == GTR_LOSS_LISTWISE || a.loss_kind == GTR_LOSS_DUAL;
  const bool use_bpr = a.loss_kind == GTR_LOSS_BPR || a.loss_kind == GTR_LOSS_DUAL;
  const float w_lw = a.loss_kind == GTR_LOSS_DUAL ? a.dual_alpha : 1.0f;
  const float w_bpr = a.loss_kind == GTR_LOSS_DUAL ? 1.0f - a.dual_alpha : 1.0f;
  const float Bm = a.loss_b > 0.0f ? a.loss_b : (float)B;  // gtr_config.loss_batch
  const float inv_bn = 1.0f / (Bm * (float)n);
  const float inv_b = 1.0f / Bm;
  const float inv_t = 1.0f / a.temperature;
  GTR_PH(26, 0);

  if (do_fwd) {
    prev_bn_stats<D, RW_BLOCK>(a.train, a.cred, a.sync ? a.nparts : a.bt.hdr[4], a.sync ? a.part_all : a.part,
                               a.stats, a.rmean, a.rvar, a.nbt, a.bn_eps,
                               a.bn_mom, s_bn, s_bn + D, s_bn + 2 * D, s_scr, rb == 0, false, BnParts<D, RW_BLOCK>{});
  } else if (do_bwd) {
    for (int j = tid; j < D; j += RW_BLOCK) { s_bn[j] = a.stats[j]; s_bn[D + j] = a.stats[D + j]; }
  }
  if (do_fwd || do_bwd)
    for (int j = tid; j < D; j += RW_BLOCK) { s_gb[j] = a.gamma[j]; s_gb[D + j] = a.beta[j]; }
  for (int j = lane; j < 2 * D; j += 64) s_red[wave][j] = 0.0f;  // this wave's BN-backward sums
  __syncthreads();
  GTR_PH(26, 1);

  float lw_sum = 0.0f, bpr_sum = 0.0f;

  // sessions interleaved over the workgroups first (b = wave * grid + rb): at B below
  // grid * RW_WAVES every CU gets B / grid busy waves instead of half the CUs getting 8
#pragma unroll 1
  for (int b = wave * a.main_grid + rb; b < B; b += a.main_grid * RW_WAVES) {
    const int n0 = a.bt.node_ptr[b], n1 = a.bt.node_ptr[b + 1];
    const float cnt = (float)(n1 - n0);
    const int* negs = a.bt.negatives + (size_t)b * n;
    float tv[EPL], rv[KQ][EPL], rv2[KQ][EPL];
    const bool pre = n <= RW_NMAX;  // all of the session's negative ids in registers
    int nid[4] = {0, 0, 0, 0};
    if (do_loss) {
      if (pre) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i * 64 < n) nid[i] = i * 64 + lane < n ? negs[i * 64 + lane] : 0;
      }
      ld_row<EPL>(tv, a.table + (size_t)a.bt.target[b] * D + c0, true);
      if (pre) issue_round_pre<D, KQ>(rv, a.table, nid, n, 0, rg, c0);
      else issue_round<D, KQ>(rv, a.table, negs, n, 0, lane, rg, c0);
    }
    // ---- session embedding: mean over node rows of drop(bn(out) + xin)
    float se[EPL];
    if (do_fwd) {
      float acc[EPL];
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] = 0.0f;
#pragma unroll 1
      for (int i = n0 + rg; i < n1; i += NRG) {
        float ov[EPL], xv[EPL];
        ld_row<EPL>(ov, a.out + (size_t)i * D + c0, true);
        ld_row<EPL>(xv, a.xin + (size_t)i * D + c0, true);
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int j = c0 + e;
          float y = (ov[e] - s_bn[j]) * s_bn[D + j] * s_gb[j] + s_gb[D + j];
          y = y + xv[e];
          acc[e] += y * dr.mul(st, (uint32_t)((size_t)i * D + j));
        }
      }
#pragma unroll
      for (int e = 0; e < EPL; ++e) se[e] = sum_groups<NRG>(acc[e]) / cnt;
      if (rg == 0) st_row<EPL>(a.se + (size_t)b * D + c0, se);
      if (b == rb) GTR_PH(26, 6);
    } else {
      ld_row<EPL>(se, a.se + (size_t)b * D + c0, true);
    }

    float dse[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) dse[e] = 0.0f;
    if (do_loss) {
      float pos = 0.0f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) pos += se[e] * tv[e];
      pos = group_sum(pos, RG::RL);
      ScoreAcc<EPL> A;
#pragma unroll
      for (int e = 0; e < EPL; ++e) { A.dse[e] = 0.0f; A.accl[e] = 0.0f; }
      A.mg = rg == 0 ? pos * inv_t : -INFINITY;
      A.zg = rg == 0 ? 1.0f : 0.0f;
      A.dpos = 0.0f;
      A.bpr_sum = 0.0f;
      float* coef_row = a.coef_neg + (size_t)b * n;
      float* sc = n <= RW_NMAX ? s_sc[wave] : nullptr;
      const int nr = (n + RND - 1) / RND;
      // double-buffered rounds: round r+1's rows are in flight while round r is scored
#pragma unroll 1
      for (int r = 0; r < nr; r += 2) {
        if (r + 1 < nr) {
          if (pre) issue_round_pre<D, KQ>(rv2, a.table, nid, n, r + 1, rg, c0);
          else issue_round<D, KQ>(rv2, a.table, negs, n, r + 1, lane, rg, c0);
        }
        consume_round<D, KQ>(A, rv, se, pos, r, n, rg, lead, use_bpr, use_lw, inv_bn, w_bpr, inv_t, sc, coef_row);
        if (r + 1 < nr) {
          if (r + 2 < nr) {
            if (pre) issue_round_pre<D, KQ>(rv, a.table, nid, n, r + 2, rg, c0);
            else issue_round<D, KQ>(rv, a.table, negs, n, r + 2, lane, rg, c0);
          }
          consume_round<D, KQ>(A, rv2, se, pos, r + 1, n, rg, lead, use_bpr, use_lw, inv_bn, w_bpr, inv_t, sc,
                               coef_row);
        }
      }
      if (b == rb) GTR_PH(26, 7);
      bpr_sum += A.bpr_sum;
      float dpos = sum_groups<NRG>(A.dpos);
#pragma unroll
      for (int e = 0; e < EPL; ++e) dse[e] = sum_groups<NRG>(A.dse[e]);
      if (use_lw) {
        const float M = max_groups<NRG>(A.mg);
        const float f = A.zg > 0.0f ? expf(A.mg - M) : 0.0f;
        const float Z = sum_groups<NRG>(A.zg * f);
        const float lse = M + logf(Z);
        if (lane == 0) lw_sum += lse - pos * inv_t;
        dpos += (expf(pos * inv_t - lse) - 1.0f) * inv_b * inv_t * w_lw;
        const float cf = inv_b * inv_t * w_lw / Z;
#pragma unroll
        for (int e = 0; e < EPL; ++e) dse[e] += sum_groups<NRG>(A.accl[e] * f) * cf;
        if (sc) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
          for (int k = lane; k < n; k += 64) {
            const float d = sc[k];
            float cb = expf(d * inv_t - lse) * inv_b * inv_t * w_lw;
            if (use_bpr) {
              const float sg = 1.0f / (1.0f + expf(-(pos - d)));
              cb += (sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
            }
            coef_row[k] = cb;
          }
          __builtin_amdgcn_wave_barrier();  // sc is reused by the wave's next session
        } else if (lead) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's raw-score stores
#pragma unroll 1
          for (int k = rg; k < n; k += NRG) {
            const float d = coef_row[k];
            float cb = expf(d * inv_t - lse) * inv_b * inv_t * w_lw;
            if (use_bpr) {
              const float sg = 1.0f / (1.0f + expf(-(pos - d)));
              cb += (sg * (1.0f - sg)) / (sg + 1e-8f) * inv_bn * w_bpr;
            }
            coef_row[k] = cb;
          }
        }
      }
#pragma unroll
      for (int e = 0; e < EPL; ++e) dse[e] += dpos * tv[e];
      if (lane == 0) a.coef_tgt[b] = dpos;
      if (rg == 0 && a.dse_out) st_row<EPL>(a.dse_out + (size_t)b * D + c0, dse);
      if (b == rb) GTR_PH(26, 8);
    } else if (do_bwd) {
      ld_row<EPL>(dse, a.dse_in + (size_t)b * D + c0, true);
    }

    // ---- readout backward into the node rows + the last BatchNorm's backward sums
    if (do_bwd) {
      const float inv_cnt = 1.0f / cnt;
      float gs[EPL], gx[EPL];
#pragma unroll
      for (int e = 0; e < EPL; ++e) { gs[e] = 0.0f; gx[e] = 0.0f; }
#pragma unroll 1
      for (int i = n0 + rg; i < n1; i += NRG) {
        float ov[EPL], dyv[EPL];
        ld_row<EPL>(ov, a.out + (size_t)i * D + c0, true);
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int j = c0 + e;
          dyv[e] = dse[e] * inv_cnt * dr.mul(st, (uint32_t)((size_t)i * D + j));
          const float xh = (ov[e] - s_bn[j]) * s_bn[D + j];
          gs[e] += dyv[e];
          gx[e] += dyv[e] * xh;
        }
        st_row<EPL>(a.dy + (size_t)i * D + c0, dyv);
      }
      // fold into the wave's running sums (sessions in order, row groups by xor tree)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const float g1 = sum_groups<NRG>(gs[e]), g2 = sum_groups<NRG>(gx[e]);
        if (rg == 0) { s_red[wave][c0 + e] += g1; s_red[wave][D + c0 + e] += g2; }
      }
      if (b == rb) GTR_PH(26, 9);
    }
  }

  GTR_PH(26, 2);
  if (!(do_loss || do_bwd)) return;
  // ---- block partials in fixed order (waves)
  const float bsum = wave_sum(bpr_sum);
  if (lane == 0) { s_loss[wave][0] = lw_sum * (w_lw * inv_b); s_loss[wave][1] = bsum * (w_bpr * inv_bn); }
  __syncthreads();
  if (do_loss && tid < 2) {
    float acc = 0.0f;
    for (int w = 0; w < RW_WAVES; ++w) acc += s_loss[w][tid];
    st_wt(a.loss_part + (size_t)rb * 2 + tid, acc);
  }
  if (do_bwd) {
    for (int j = tid; j < 2 * D; j += RW_BLOCK) {
      float acc = 0.0f;
      for (int w = 0; w < RW_WAVES; ++w) acc += s_red[w][j];
      st_wt(a.gpart + (size_t)rb * 2 * D + j, acc);
    }
  }
  GTR_PH(26, 3);
  if (!a.fin) return;
  if (!arrive_last_wt(a.cnt, (uint32_t)a.main_grid, &s_flag)) return;
  GTR_PH(26, 4);
  if (do_loss) {
    __shared__ float s_pair[2];
    block_sum_rows<RW_BLOCK>(a.loss_part, a.main_grid, 2, 2, s_pair, s_scr);
    if (tid == 0) a.loss_out[0] = s_pair[0] + s_pair[1];
  }
  if (do_bwd) block_sum_rows<RW_BLOCK>(a.gpart, a.main_grid, 2 * D, (size_t)2 * D, a.gsum, s_scr);
  if (tid == 0) reset_counter(a.cnt);
  GTR_PH(26, 5);
}



// Sessions per batch from which the wave-per-session readout runs (env GTR_RO_WAVE_MIN_B
// overrides, for tests); below it the block-per-session kernel has the lower latency.
// (C5 at B = 1024: 57 us block per session, 35 us wave per session.)
int ro_wave_min_b() {
  const char* e = getenv("GTR_RO_WAVE_MIN_B");
  return e ? atoi(e) : 1024;
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

// Arguments of conv_fwd_body for layer l (launch geometry left to the caller).
int make_fwd_args(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb, const gtr_layer* layers,
                  int l, ConvFwdK& k, bool attn_only = false) {
  if (!check_dims(cfg, "gtr_conv_fwd")) return GTR_E_ARG;
  if (!bt->grp_row || !bt->grp_edge) { set_error("gtr_conv_fwd: batch lacks row-group ranges"); return GTR_E_ARG; }
  if (!attn_only && l == 0 && (!emb || !emb->table)) { set_error("gtr_conv_fwd: layer 0 needs the table"); return GTR_E_ARG; }
  if (!attn_only && l == 0 && cfg->pe_k > 0 && (!emb->wpe || !emb->bpe || (!emb->pe_tab && !bt->node_pe))) {
    set_error("gtr_conv_fwd: Laplacian PE not precomputed");
    return GTR_E_ARG;
  }
  const gtr_layer& L = layers[l];
  k = ConvFwdK{};
  k.bt = *bt;
  k.H = cfg->heads;
  k.C = cfg->dim / cfg->heads;
  k.first = l == 0;
  k.train = cfg->training;
  k.layer = l;
  k.pe_k = cfg->pe_k;
  k.cred = cfg->consumer_reduce;
  k.split = gemm_split(cfg->dim);
  k.sqrt_c = (float)sqrt((double)k.C);
  k.bn_eps = cfg->bn_eps;
  k.bn_mom = cfg->bn_momentum;
  drop_params(cfg, k.thresh, k.scale, k.drop_on);
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.ctr_add = (uint32_t)cfg->ctr_add;
  k.sync = cfg->sync_bn;
  if (cfg->sync_bn && !cfg->consumer_reduce) { set_error("gtr_conv_fwd: sync_bn needs consumer_reduce"); return GTR_E_ARG; }
  if (l == 0) {
    if (emb) { k.table = emb->table; k.pe_tab = emb->pe_tab; k.wpe = emb->wpe; k.bpe = emb->bpe; }
  } else {
    const gtr_layer& P = layers[l - 1];
    k.p_part_all = P.bn_part_all;
    k.p_nparts = P.nparts_fwd;
    if (cfg->sync_bn && cfg->training && (!P.bn_part_all || P.nparts_fwd <= 0)) {
      set_error("gtr_conv_fwd: sync_bn needs the gathered partials of layer %d", l - 1);
      return GTR_E_ARG;
    }
    k.p_out = P.out; k.p_xin = P.xin; k.p_stats = P.bn_stats; k.p_part = P.bn_part; k.p_gamma = P.bn_gamma;
    k.p_beta = P.bn_beta; k.p_rmean = P.bn_rmean; k.p_rvar = P.bn_rvar; k.p_nbt = P.bn_nbt;
  }
  k.w_all = L.w_all; k.b_all = L.b_all; k.w_beta = L.w_beta;
  k.xin = L.xin; k.qkvs = L.qkvs; k.alpha = L.alpha; k.agg = L.agg; k.gate = L.gate; k.out = L.out;
  k.bn_part = L.bn_part; k.cnt = L.cnt; k.bn_stats = L.bn_stats; k.bn_rmean = L.bn_rmean;
  k.bn_rvar = L.bn_rvar; k.bn_nbt = L.bn_nbt;
  return GTR_OK;
}

// Arguments of readout_body (launch geometry left to the caller).
int make_readout_args(const gtr_config* cfg, const gtr_batch* bt, const float* table, const gtr_layer* layers,
                      const gtr_head* head, ReadoutK& k) {
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
  k = ReadoutK{};
  k.bt = *bt;
  k.L1 = L1;
  k.train = cfg->training;
  k.flags = head->flags;
  k.loss_kind = head->loss_kind;
  k.cred = cfg->consumer_reduce;
  // finalise in-kernel unless a consumer takes over: the BN sums go to conv_bwd and the
  // loss to gtr_step_end in the fused step; a loss-only call always finalises itself.
  k.fin = (!cfg->consumer_reduce || !(head->flags & GTR_RO_BWD) || cfg->split_sync) ? 1 : 0;
  k.temperature = head->temperature;
  k.dual_alpha = head->dual_alpha;
  k.bn_eps = cfg->bn_eps;
  k.bn_mom = cfg->bn_momentum;
  drop_params(cfg, k.thresh, k.scale, k.drop_on);
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.ctr_add = (uint32_t)cfg->ctr_add;
  k.table = table;
  k.out = L.out; k.xin = L.xin; k.stats = L.bn_stats; k.part = L.bn_part; k.gamma = L.bn_gamma; k.beta = L.bn_beta;
  k.rmean = L.bn_rmean; k.rvar = L.bn_rvar; k.nbt = L.bn_nbt;
  k.se = head->se; k.dse_in = head->dse_in; k.dse_out = head->dse_out; k.coef_tgt = head->coef_tgt;
  k.coef_neg = head->coef_neg;
  k.loss_part = head->loss_part; k.loss_out = head->loss_out; k.cnt = head->cnt;
  k.dy = L.dy; k.gpart = L.bn_gpart; k.gsum = L.bn_gsum;
  k.sync = cfg->sync_bn;
  k.part_all = L.bn_part_all;
  k.nparts = L.nparts_fwd;
  k.loss_b = cfg->loss_batch;
  if (cfg->sync_bn && ((head->flags & GTR_RO_FWD) && cfg->training) && (!L.bn_part_all || L.nparts_fwd <= 0 || !cfg->consumer_reduce)) {
    set_error("gtr_readout_loss: sync_bn needs consumer_reduce and the gathered partials of the last layer");
    return GTR_E_ARG;
  }
  return GTR_OK;
}

}  // namespace

GTR_PH_READER(gtr_dbg_fwd_phases)

extern "C" int gtr_conv_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb,
                            const gtr_layer* layers, int l, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_conv_fwd: bad arguments");
    return GTR_E_ARG;
  }
  if (layers[l].ffn || (l > 0 && layers[l - 1].ffn)) {
    set_error("gtr_conv_fwd: a feed-forward block runs on the split layer path (gtr_qkvs_* / gtr_attn_* / gtr_ffn_*)");
    return GTR_E_ARG;
  }
  ConvFwdK k;
  if (const int rc = make_fwd_args(cfg, bt, emb, layers, l, k)) return rc;
  int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
  if (l == 0 && cfg->begin) {
    const gtr_begin& g = *cfg->begin;
    const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
    if (!g.skeys || !g.svals || !g.step_dev || g.num_items <= 0 || g.num_items >= GTR_BEGIN_KEY_LIMIT ||
        m_cap > GTR_BEGIN_MCAP || bt->n_neg <= 0) {
      set_error("gtr_conv_fwd: fused begin needs skeys/svals/step_dev, m_cap <= %d and T < 2^19", GTR_BEGIN_MCAP);
      return GTR_E_ARG;
    }
    if (cfg->sweep && cfg->sweep->bounds[1] > cfg->sweep->bounds[0]) {
      set_error("gtr_conv_fwd: a fused begin stamps the rows the layer-0 sweep slice would read: slot 0 must be empty");
      return GTR_E_ARG;
    }
    k.beg = g;
    k.nbeg = (m_cap + 63) / 64;
    grid += k.nbeg;
  }
  if (cfg->sweep && l < GTR_SWEEP_SLOTS && cfg->sweep->bounds[l + 1] > cfg->sweep->bounds[l]) {
    k.sw = *cfg->sweep;
    k.sw_slot = l;
    grid += sweep_blocks(cfg->sweep, grid);
  }
  k.xpack = xcd_pack(k.main_grid, grid);
  hipStream_t s = (hipStream_t)stream;
#define GTR_FWD(DD, SP) set_lds_limit<DD>(k_conv_fwd<DD, SP>, (size_t)LayerGeom<DD>::F_WORDS * 4); \
  hipLaunchKernelGGL((k_conv_fwd<DD, SP>), dim3(grid), dim3(CONV_BLOCK), (size_t)LayerGeom<DD>::F_WORDS * 4, s, k)
  switch (cfg->dim * 2 + k.split) {
    case 64: GTR_FWD(32, false); break;
    case 65: GTR_FWD(32, true); break;
    case 128: GTR_FWD(64, false); break;
    case 129: GTR_FWD(64, true); break;
    case 256: GTR_FWD(128, false); break;
    case 257: GTR_FWD(128, true); break;
    default: GTR_FWD(256, false); break;  // D = 256: f32 MFMA (no registers for the split fragments)
  }
#undef GTR_FWD
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_attn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_attn_fwd: bad arguments");
    return GTR_E_ARG;
  }
  if (cfg->training && (cfg->sync_bn ? !cfg->split_sync : cfg->consumer_reduce)) {
    set_error("gtr_attn_fwd: the split path needs producer-finalized BatchNorm statistics (consumer_reduce 0) "
              "or, under sync_bn, split_sync");
    return GTR_E_ARG;
  }
  ConvFwdK k;
  if (const int rc = make_fwd_args(cfg, bt, nullptr, layers, l, k, true)) return rc;
  if (cfg->sync_bn && cfg->training) {  // one merged row per rank for the all-gather
    k.cred = 0;
    k.merge_only = 1;
    k.sync = 0;  // no zero rows for empty groups: only live groups arrive
  }
  hipStream_t s = (hipStream_t)stream;
  const char* am = getenv("GTR_ATTN");  // "group": the fused kernels' row-group body (A/B)
  if (cfg->dim <= 128 && !(am && am[0] == 'g')) {
    // row-parallel: one BatchNorm partial per AR_ROWS rows (gtr_layer.bn_part holds
    // max(n_cap / row_group, n_cap / 8) rows, gtr.h)
    static_assert(AR_ROWS >= 8 && AR_ROWS % 8 == 0, "gtr.h sizes bn_part for (at most) 8-row partials");
    const int grid = (bt->n_cap + AR_ROWS - 1) / AR_ROWS;
    // float4 lanes + online softmax (k_attn_rows4) unless GTR_ATTN=rows (the round-4 body,
    // also the path for more than AR_HMAX heads)
    const bool v4 = cfg->heads <= AR_HMAX && !(am && am[0] == 'r');
    switch (cfg->dim * 2 + (v4 ? 1 : 0)) {
      case 64: hipLaunchKernelGGL(k_attn_rows<32>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
      case 65: hipLaunchKernelGGL(k_attn_rows4<32>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
      case 128: hipLaunchKernelGGL(k_attn_rows<64>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
      case 129: hipLaunchKernelGGL(k_attn_rows4<64>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
      case 256: hipLaunchKernelGGL(k_attn_rows<128>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
      default: hipLaunchKernelGGL(k_attn_rows4<128>, dim3(grid), dim3(AR_BLOCK), 0, s, k); break;
    }
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  const int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
#define GTR_ATT(DD) set_lds_limit<DD>(k_attn_fwd<DD>, (size_t)LayerGeom<DD>::F_WORDS * 4); \
  hipLaunchKernelGGL((k_attn_fwd<DD>), dim3(grid), dim3(CONV_BLOCK), (size_t)LayerGeom<DD>::F_WORDS * 4, s, k)
  switch (cfg->dim) {
    case 32: GTR_ATT(32); break;
    case 64: GTR_ATT(64); break;
    case 128: GTR_ATT(128); break;
    default: GTR_ATT(256); break;
  }
#undef GTR_ATT
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_readout_loss(const gtr_config* cfg, const gtr_batch* bt, const float* table,
                                const gtr_layer* layers, const gtr_head* head, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !head) { set_error("gtr_readout_loss: bad arguments"); return GTR_E_ARG; }
  ReadoutK k;
  if (const int rc = make_readout_args(cfg, bt, table, layers, head, k)) return rc;
  int grid = gtr_readout_grid(bt->b_cap);
  k.main_grid = grid;
  if (cfg->sweep && cfg->num_layers < GTR_SWEEP_SLOTS &&
      cfg->sweep->bounds[cfg->num_layers + 1] > cfg->sweep->bounds[cfg->num_layers]) {
    k.sw = *cfg->sweep;
    k.sw_slot = cfg->num_layers;
    grid += sweep_blocks(cfg->sweep, grid);
  }
  k.xpack = xcd_pack(k.main_grid, grid);
  hipStream_t s = (hipStream_t)stream;
  if (bt->b_cap >= ro_wave_min_b() && cfg->dim <= 128) {
    switch (cfg->dim) {
      case 32: hipLaunchKernelGGL(k_readout_wave<32>, dim3(grid), dim3(RW_BLOCK), 0, s, k); break;
      case 64: hipLaunchKernelGGL(k_readout_wave<64>, dim3(grid), dim3(RW_BLOCK), 0, s, k); break;
      default: hipLaunchKernelGGL(k_readout_wave<128>, dim3(grid), dim3(RW_BLOCK), 0, s, k); break;
    }
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  switch (cfg->dim) {
    case 32: hipLaunchKernelGGL(k_readout<32>, dim3(grid), dim3(RO_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_readout<64>, dim3(grid), dim3(RO_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_readout<128>, dim3(grid), dim3(RO_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_readout<256>, dim3(grid), dim3(RO_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

