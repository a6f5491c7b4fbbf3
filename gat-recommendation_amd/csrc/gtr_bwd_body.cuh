// gtr_bwd_body.cuh — the TransformerConv layer backward (k_conv_bwd) as a device body over
// one row group plus its argument builder, so that other translation units can compose it
// with the forward bodies (a single-launch step middle was built on these and measured
// slower than the launches).  Included inside an anonymous namespace
// after GTR_PH_DECL; see gtr_bwd.hip for the algorithm.
#pragma once

struct ConvBwdK {
  gtr_batch bt;
  int H, C, layer, has_prev, cred, gpart_n;  // gpart_n: partials feeding gsum (-1: hdr G)
  float sqrt_c, scale;
  uint32_t seed, thresh;
  int drop_on, pad1;
  const uint32_t* rng_ctr;
  const float* dy;
  const float* out;
  const float* stats;
  float* gsum;
  const float* gpart;
  const float* gamma;
  const float* qkvs;
  const float* alpha;
  const float* agg;
  const float* gate;
  const float* w_all;
  const float* w_beta;
  float* dqkvs;
  float* du;
  float* dlogit;
  float* dagg;
  const float* p_out;
  const float* p_stats;
  float* p_dy;
  float* p_gpart;
  float* p_gsum;
  uint32_t* p_cnt;
  float* dx0;
  gtr_sweep sw;         // untouched-row AdamW slice run by blocks >= main_grid
  int sw_slot, main_grid;
  int sync, nparts_bwd, nparts_fwd, pad_s;  // SyncBN: every rank's partials (this layer)
  const float* gpart_all;
  const float* part_all;
  uint32_t ctr_add;
  int xpack;            // XCD-packed roles (role_block)
  float* wslab;         // gtr_layer.wfold: this layer's per-row-group weight-gradient partials
  int64_t wstride;      //   (null: the weight gradients run in gtr_wgrad)
  const float* xin;     //   the layer input rows (dW_all = dQKVS^T . X)
};

// Destination-row backward: BatchNorm backward, beta gate, softmax backward, dQ, dS.
// KB/VB (stride KST), AL/DL (edge-indexed, H per edge) are LDS on the fast path.
template <int D>
__device__ __forceinline__ void bwd_dst_row(const ConvBwdK& a, int t, int tl, const float* KB, const float* VB,
                                            int KST, const int* EP, const int* ES, const float* AL, float* DL,
                                            int eoff, int lane, const Drop& dr, uint32_t st_attn,
                                            const float (&k_g)[LayerGeom<D>::VPL],
                                            const float (&k_mean)[LayerGeom<D>::VPL],
                                            const float (&k_rstd)[LayerGeom<D>::VPL],
                                            const float (&k_s1)[LayerGeom<D>::VPL],
                                            const float (&k_s2)[LayerGeom<D>::VPL]) {
  constexpr int VPL = LayerGeom<D>::VPL;
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int GL = C / VPL;
  const int head = act ? d0 / C : 0;
  const bool leader = act && ((lane & (GL - 1)) == 0);
  const size_t ro = (size_t)t * D + d0;
  float dyv[VPL], ov[VPL], ag[VPL], sv[VPL];
  load_vec<VPL>(dyv, a.dy + ro, act);
  load_vec<VPL>(ov, a.out + ro, act);
  load_vec<VPL>(ag, a.agg + ro, act);
  load_vec<VPL>(sv, a.qkvs + (size_t)t * (4 * D) + 3 * D + d0, act);
  const float beta = a.gate[t];
  float gv[VPL];
  float dbeta = 0.0f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const float xh = (ov[v] - k_mean[v]) * k_rstd[v];
    gv[v] = act ? (dyv[v] - k_s1[v] - xh * k_s2[v]) * k_rstd[v] * k_g[v] : 0.0f;
    dbeta += gv[v] * (sv[v] - ag[v]);
  }
  dbeta = wave_sum(dbeta);
  const float du = dbeta * beta * (1.0f - beta);
  if (lane == 0) a.du[t] = du;
  float dag[VPL], ds[VPL], dq[VPL];
  {
    float w1[VPL], w2[VPL], w3[VPL];
    load_vec<VPL>(w1, a.w_beta + d0, act);
    load_vec<VPL>(w2, a.w_beta + D + d0, act);
    load_vec<VPL>(w3, a.w_beta + 2 * D + d0, act);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      dag[v] = gv[v] * (1.0f - beta) + du * (w1[v] + w3[v]);
      ds[v] = gv[v] * beta + du * (w2[v] - w3[v]);
      dq[v] = 0.0f;
    }
  }
  store_vec<VPL>(a.dqkvs + (size_t)t * (4 * D) + 3 * D + d0, ds, act);
  store_vec<VPL>(a.dagg + ro, dag, act);
  const int e0 = EP[tl], e1 = EP[tl + 1];
  float sdot = 0.0f;
  for (int e = e0; e < e1; ++e) {
    float vv[VPL];
    load_vec<VPL>(vv, VB + (size_t)ES[e] * KST + d0, act);
    float d = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) d += dag[v] * vv[v];
    d = group_sum(d, GL);
    const float al = AL[(size_t)e * H + head];
    sdot += al * (d * dr.mul(st_attn, (uint32_t)((e + eoff) * H + head)));
  }
  for (int e = e0; e < e1; ++e) {
    const int src = ES[e];
    float vv[VPL], kv[VPL];
    load_vec<VPL>(vv, VB + (size_t)src * KST + d0, act);
    load_vec<VPL>(kv, KB + (size_t)src * KST + d0, act);
    float d = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) d += dag[v] * vv[v];
    d = group_sum(d, GL);
    const float al = AL[(size_t)e * H + head];
    const float da = d * dr.mul(st_attn, (uint32_t)((e + eoff) * H + head));
    const float dl = al * (da - sdot);
    if (leader) DL[(size_t)e * H + head] = dl;
    const float c = dl / a.sqrt_c;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dq[v] += c * kv[v];
  }
  store_vec<VPL>(a.dqkvs + (size_t)t * (4 * D) + d0, dq, act);
}

// Source-row backward: dK, dV gathered over out-edges (no atomics).
template <int D>
__device__ __forceinline__ void bwd_src_row(const ConvBwdK& a, int s, int sl, const float* QB, int QST,
                                            const float* GB, int GST, const int* OP, const int* OE, const int* OD,
                                            const float* AL, const float* DL, int eoff, int lane, const Drop& dr,
                                            uint32_t st_attn) {
  constexpr int VPL = LayerGeom<D>::VPL;
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int head = act ? d0 / C : 0;
  float dk[VPL], dv[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) { dk[v] = 0.0f; dv[v] = 0.0f; }
  const int i0 = OP[sl], i1 = OP[sl + 1];
  for (int i = i0; i < i1; ++i) {
    const int p = OE[i];
    const int t = OD[i];
    const float dl = DL[(size_t)p * H + head] / a.sqrt_c;
    const float ad = AL[(size_t)p * H + head] * dr.mul(st_attn, (uint32_t)((p + eoff) * H + head));
    float qv[VPL], gv[VPL];
    load_vec<VPL>(qv, QB + (size_t)t * QST + d0, act);
    load_vec<VPL>(gv, GB + (size_t)t * GST + d0, act);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      dk[v] += dl * qv[v];
      dv[v] += ad * gv[v];
    }
  }
  store_vec<VPL>(a.dqkvs + (size_t)s * (4 * D) + D + d0, dk, act);
  store_vec<VPL>(a.dqkvs + (size_t)s * (4 * D) + 2 * D + d0, dv, act);
}
// DX = false: the split path's attention backward (gtr_attn_bwd): stops once dqkvs, du and
// dlogit are written; dX and the previous layer's BatchNorm sums run in k_dx (gtr_gemm.hip).
template <int D, bool SPLIT, bool DX = true>
__device__ __forceinline__ void conv_bwd_body(const ConvBwdK& a, int rb) {
  using G = LayerGeom<D>;
  constexpr int VPL = G::VPL, RMAX = G::RMAX, XS = G::XS, TPR = G::TPR, CH = G::CH;
  constexpr int NCT = D / 16;                                   // dX column tiles
  constexpr int CPW = NCT > CONV_WAVES ? NCT / CONV_WAVES : 1;  // column tiles per wave
  constexpr int WPC = NCT >= CONV_WAVES ? 1 : CONV_WAVES / NCT; // waves sharing a column tile
  constexpr int ASB = 4 * D + 8;                                // LDS split dQKVS row stride (bf16)
  constexpr int AS32 = 4 * D + 4;                               // LDS fp32 dQKVS row stride
  constexpr int RTW = (RMAX / 16 + WPC - 1) / WPC;              // row tiles per wave
  static_assert(!G::KV || RMAX * ASB <= G::B_RN, "split dQKVS rows must fit the K|V|Q|dA region");
  static_assert(!G::KV || RMAX * AS32 <= G::B_RN, "fp32 dQKVS rows must fit the K|V|Q|dA region");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ks = sm + G::B_R;
  float* Vs = Ks + RMAX * XS;
  float* Qs = Vs + RMAX * XS;
  float* DAs = Qs + RMAX * XS;
  float* AL = sm + G::B_AL;
  float* DL = sm + G::B_DL;
  int* iptr = reinterpret_cast<int*>(sm + G::B_IPTR);
  int* isrc = reinterpret_cast<int*>(sm + G::B_ISRC);
  int* edst = reinterpret_cast<int*>(sm + G::B_EDST);
  int* optr = reinterpret_cast<int*>(sm + G::B_OPTR);
  int* oedge = reinterpret_cast<int*>(sm + G::B_OEDGE);
  int* odst = reinterpret_cast<int*>(sm + G::B_ODST);
  float* s_gs = sm + G::B_GS;
  float* s_bnp = sm + G::B_BNP;
  int* s_flag = reinterpret_cast<int*>(sm + G::B_FLAG);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GTR_PH(a.layer, 0);
  const int Gn = a.bt.hdr[4];
  int N = a.bt.hdr[0];
  const int g = rb;
  if (g >= Gn) {
    if (a.sync && a.has_prev)  // SyncBN: an empty group's backward partial is zero
      for (int j = threadIdx.x; j < 2 * D; j += CONV_BLOCK) a.p_gpart[(size_t)g * 2 * D + j] = 0.0f;
    return;
  }
  if (a.sync) {  // BatchNorm over every rank's nodes: N = the sum of all partial counts
    float n = 0.0f;
    for (int q = 0; q < a.nparts_fwd; ++q) n += a.part_all[(size_t)q * (1 + 2 * D)];
    N = (int)(n + 0.5f);
  }
  const int r0 = a.bt.grp_row[g], r1 = a.bt.grp_row[g + 1];
  // groups hold whole sessions, so the group's out-edges (CSR by source) start at the
  // same offset as its in-edges: edges with src < r0 are exactly those with dst < r0
  const int e_lo = a.bt.grp_edge[g], e_hi = a.bt.grp_edge[g + 1];
  const int o_lo = e_lo;
  const int nrow = r1 - r0;
  const int H = a.H, C = a.C;
  const int ne = e_hi - e_lo;
  const bool fast = G::KV && nrow <= RMAX && ne <= G::EMAX && ne * H <= G::EH && H <= 8 && C >= CH;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const float invN = 1.0f / (float)N;
  const int prow = tid / TPR, pchunk = tid - prow * TPR, f0 = pchunk * CH;
  constexpr bool PREB = DX && !SPLIT && CPW == 1 && D <= 128;
  float4 wb[PREB ? D / 4 : 1];

  // ---- this layer's BatchNorm backward sums: reduce the producer's partials (cred).
  //      D <= 64: the first GPR partial rows are requested into registers here and summed
  //      after the staging loads below have been issued, so the two round trips overlap
  //      (same order of the sum: rows ascending)
  constexpr int GPR = (D <= 64 && 2 * D <= CONV_BLOCK) ? 32 : 0;
  const int np = a.sync ? a.nparts_bwd : (a.gpart_n >= 0 ? a.gpart_n : Gn);
  const float* gp = a.sync ? a.gpart_all : a.gpart;
  float gpr[GPR > 0 ? GPR : 1];
  if constexpr (GPR > 0) {
    if (a.cred && tid < 2 * D) {
#pragma unroll
      for (int q = 0; q < GPR; ++q) gpr[q] = q < np ? gp[(size_t)q * 2 * D + tid] : 0.0f;
    }
  }
  // ---- phase W operands (folded weight gradients), requested now so that their latency
  //      hides behind the attention phases: the group's first 8 X rows (MFMA B operands of
  //      k-steps 0 and 1) and this thread's gate-slice rows of agg and S
  //      (compiled for D <= 64 only: at D = 128 the extra registers spill).  Issued once
  //      the staging loads have been consumed (vector loads retire in order), so they wait
  //      behind nothing and arrive during the attention phases.
  constexpr bool WF = DX && D <= 64;
  constexpr int WTK = WF ? D / 16 : 1;                              // dW_all k-tiles (X columns)
  constexpr int NGT = 3 * D / 16;                                   // gate-weight column tiles
  constexpr int GPW = WF ? (NGT + CONV_WAVES - 1) / CONV_WAVES : 1; // per wave (waves 0 .. NGT/GPW-1)
  float wx[2][WTK], wga[2][GPW], wgs[2][GPW];
  float* s_du = sm + G::B_DU;
  auto wprefetch = [&]() {
    if (!(WF && a.wslab)) return;
    const int wlr = lane & 15, wlg = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int rr = ks * 4 + wlg;
#pragma unroll
      for (int t = 0; t < WTK; ++t) wx[ks][t] = rr < nrow ? a.xin[(size_t)(r0 + rr) * D + t * 16 + wlr] : 0.0f;
#pragma unroll
      for (int q = 0; q < GPW; ++q) {
        const int gt = wave * GPW + q, c = (gt * 16 + wlr) % D;
        const bool ok = rr < nrow && gt < NGT;
        wga[ks][q] = ok ? a.agg[(size_t)(r0 + rr) * D + c] : 0.0f;
        wgs[ks][q] = ok ? a.qkvs[(size_t)(r0 + rr) * (4 * D) + 3 * D + c] : 0.0f;
      }
    }
  };
  auto reduce_gsum = [&]() {
    if (!a.cred) return;
    if constexpr (GPR > 0) {
      if (tid < 2 * D) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < GPR; ++q)
          if (q < np) acc += gpr[q];
        for (int q = GPR; q < np; ++q) acc += gp[(size_t)q * 2 * D + tid];
        s_gs[tid] = acc;
        if (g == 0) a.gsum[tid] = acc;
      }
    } else {
      for (int j = tid; j < 2 * D; j += CONV_BLOCK) {
        float acc = 0.0f;
#pragma unroll 8
        for (int q = 0; q < np; ++q) acc += gp[(size_t)q * 2 * D + j];
        s_gs[j] = acc;
        if (g == 0) a.gsum[j] = acc;
      }
    }
  };
  if (!fast) reduce_gsum();

  if (fast) {
    // ---- stage: CSR slices (by destination and by source), alpha, K | V | Q rows.  Each
    //      thread's first element of every array is loaded into registers before any LDS
    //      store (a store waits for its load and vector loads retire in order: one round
    //      trip for the stage instead of one per array); elements past CONV_BLOCK (groups
    //      with > 512 edges, (edge, head) pairs or row float4s) follow in plain loops.
    int s_ip = 0, s_ip1 = 0, s_op = 0, s_is = 0, s_oe = 0, s_od = 0;
    float s_al = 0.0f;
    float4 s_k = make_float4(0.f, 0.f, 0.f, 0.f), s_v = s_k, s_q = s_k;
    constexpr int C4 = D / 4;
    const int i0 = tid / C4, c0 = (tid - i0 * C4) * 4;
    if (tid <= nrow) {
      s_ip = a.bt.in_ptr[r0 + tid];
      s_op = a.bt.out_ptr[r0 + tid];
    }
    if (tid < nrow) s_ip1 = a.bt.in_ptr[r0 + tid + 1];
    if (tid < ne) {
      s_is = a.bt.in_src[e_lo + tid];
      s_oe = a.bt.out_edge[o_lo + tid];
      s_od = a.bt.out_dst[o_lo + tid];
    }
    if (tid < ne * H) s_al = a.alpha[(size_t)e_lo * H + tid];
    if (tid < nrow * C4) {
      const float* src = a.qkvs + (size_t)(r0 + i0) * (4 * D);
      s_k = *reinterpret_cast<const float4*>(src + D + c0);
      s_v = *reinterpret_cast<const float4*>(src + 2 * D + c0);
      s_q = *reinterpret_cast<const float4*>(src + c0);
    }
    // (D1)'s own inputs of this thread's row (dy, out, agg, S, gate, BatchNorm mean / rstd,
    // gamma) requested with the staging loads instead of after its barrier (D <= 64: the
    // registers are free here)
    constexpr bool PRED1 = D <= 64;
    float4 d1_dy[PRED1 ? CH / 4 : 1], d1_o[PRED1 ? CH / 4 : 1], d1_ag[PRED1 ? CH / 4 : 1], d1_s[PRED1 ? CH / 4 : 1];
    float d1_mean[PRED1 ? CH : 1], d1_rstd[PRED1 ? CH : 1], d1_gam[PRED1 ? CH : 1], d1_beta = 0.0f;
    if (PRED1 && prow < nrow) {
      const int t1 = r0 + prow;
      const size_t ro1 = (size_t)t1 * D + f0;
      d1_beta = a.gate[t1];
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        if constexpr (PRED1) {
          d1_dy[c / 4] = *reinterpret_cast<const float4*>(a.dy + ro1 + c);
          d1_o[c / 4] = *reinterpret_cast<const float4*>(a.out + ro1 + c);
          d1_ag[c / 4] = *reinterpret_cast<const float4*>(a.agg + ro1 + c);
          d1_s[c / 4] = *reinterpret_cast<const float4*>(a.qkvs + (size_t)t1 * (4 * D) + 3 * D + f0 + c);
        }
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (PRED1) {
          d1_mean[c] = a.stats[f0 + c];
          d1_rstd[c] = a.stats[D + f0 + c];
          d1_gam[c] = a.gamma[f0 + c];
        }
      }
    }
    if (tid <= nrow) {
      iptr[tid] = s_ip - e_lo;
      optr[tid] = s_op - o_lo;
    }
    if (tid < nrow)
      for (int k = s_ip - e_lo; k < s_ip1 - e_lo; ++k) edst[k] = tid;
    if (tid < ne) {
      isrc[tid] = s_is - r0;
      oedge[tid] = s_oe - e_lo;
      odst[tid] = s_od - r0;
    }
    if (tid < ne * H) AL[tid] = s_al;
    if (tid < nrow * C4) {
      *reinterpret_cast<float4*>(Ks + i0 * XS + c0) = s_k;
      *reinterpret_cast<float4*>(Vs + i0 * XS + c0) = s_v;
      *reinterpret_cast<float4*>(Qs + i0 * XS + c0) = s_q;
    }
    for (int k = tid + CONV_BLOCK; k < ne; k += CONV_BLOCK) {
      isrc[k] = a.bt.in_src[e_lo + k] - r0;
      oedge[k] = a.bt.out_edge[o_lo + k] - e_lo;
      odst[k] = a.bt.out_dst[o_lo + k] - r0;
    }
    for (int k = tid + CONV_BLOCK; k < ne * H; k += CONV_BLOCK) AL[k] = a.alpha[(size_t)e_lo * H + k];
    for (int idx = tid + CONV_BLOCK; idx < nrow * C4; idx += CONV_BLOCK) {
      const int i = idx / C4, c = (idx - i * C4) * 4;
      const float* src = a.qkvs + (size_t)(r0 + i) * (4 * D);
      *reinterpret_cast<float4*>(Ks + i * XS + c) = *reinterpret_cast<const float4*>(src + D + c);
      *reinterpret_cast<float4*>(Vs + i * XS + c) = *reinterpret_cast<const float4*>(src + 2 * D + c);
      *reinterpret_cast<float4*>(Qs + i * XS + c) = *reinterpret_cast<const float4*>(src + c);
    }
  // W_all fragments of this wave's dX column tile, requested once the staging loads are
  // out (vector loads retire in order: issued first they would hold up the staging) so
  // they arrive during the attention phases instead of inside the dX MFMA chain
  if constexpr (PREB) {
    const int ct0 = WPC > 1 ? wave % NCT : wave;
    const float* bcol = a.w_all + (size_t)((lane >> 4) * 4) * D + ct0 * 16 + (lane & 15);
#pragma unroll
    for (int kb = 0; kb < D / 4; ++kb) {
      const float* bp = bcol + (size_t)(kb * 16) * D;
      wb[kb] = make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]);
    }
  }
    reduce_gsum();
    __syncthreads();
    GTR_PH(a.layer, 1);
    wprefetch();

    // ---- (D1) BatchNorm backward, beta gate: TPR lanes per destination row, CH features each
    const bool live = prow < nrow;
    const int t = r0 + prow;
    float gv[CH], sv[CH], agv[CH], dsv[CH];
    float dbeta = 0.0f, beta = 0.0f;
    if (live) {
      const size_t ro = (size_t)t * D + f0;
      const float* gs = a.cred ? s_gs : a.gsum;
      beta = PRED1 ? d1_beta : a.gate[t];
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        float4 dy4, o4, ag4, s4;
        if constexpr (PRED1) {
          dy4 = d1_dy[c / 4]; o4 = d1_o[c / 4]; ag4 = d1_ag[c / 4]; s4 = d1_s[c / 4];
        } else {
          dy4 = *reinterpret_cast<const float4*>(a.dy + ro + c);
          o4 = *reinterpret_cast<const float4*>(a.out + ro + c);
          ag4 = *reinterpret_cast<const float4*>(a.agg + ro + c);
          s4 = *reinterpret_cast<const float4*>(a.qkvs + (size_t)t * (4 * D) + 3 * D + f0 + c);
        }
        const float dyv[4] = {dy4.x, dy4.y, dy4.z, dy4.w}, ov[4] = {o4.x, o4.y, o4.z, o4.w};
        const float agl[4] = {ag4.x, ag4.y, ag4.z, ag4.w}, svl[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = f0 + c + q;
          const float mean = PRED1 ? d1_mean[(c + q) % CH] : a.stats[j];
          const float rstd = PRED1 ? d1_rstd[(c + q) % CH] : a.stats[D + j];
          const float gam = PRED1 ? d1_gam[(c + q) % CH] : a.gamma[j];
          const float xh = (ov[q] - mean) * rstd;
          const float s1 = gs[j] * invN, s2 = gs[D + j] * invN;
          gv[c + q] = (dyv[q] - s1 - xh * s2) * rstd * gam;
          sv[c + q] = svl[q];
          agv[c + q] = agl[q];
          dbeta += gv[c + q] * (svl[q] - agl[q]);
        }
      }
    }
    dbeta = group_sum_c<TPR>(dbeta);
    if (live) {
      const float du = dbeta * beta * (1.0f - beta);
      if (pchunk == 0) {
        a.du[t] = du;
        if (WF) s_du[prow] = du;  // the folded gate-weight gradient (phase W)
      }
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        float dag[4], ds[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = f0 + c + q;
          const float w1 = a.w_beta[j], w2 = a.w_beta[D + j], w3 = a.w_beta[2 * D + j];
          dag[q] = gv[c + q] * (1.0f - beta) + du * (w1 + w3);
          ds[q] = gv[c + q] * beta + du * (w2 - w3);
          dsv[c + q] = ds[q];
        }
        *reinterpret_cast<float4*>(a.dqkvs + (size_t)t * (4 * D) + 3 * D + f0 + c) =
            make_float4(ds[0], ds[1], ds[2], ds[3]);
        *reinterpret_cast<float4*>(DAs + prow * XS + f0 + c) = make_float4(dag[0], dag[1], dag[2], dag[3]);
      }
    }
    (void)sv; (void)agv;
    __syncthreads();

    // ---- (D2) da of every (edge, head): <dA[dst], V[src]> * dropout mask, SPL lanes per item
    {
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
          const float* x = DAs + edst[e] * XS + h * C + sub * cw;
          const float* y = Vs + isrc[e] * XS + h * C + sub * cw;
          for (int c = 0; c < cw; c += 4) {
            const float4 p = *reinterpret_cast<const float4*>(x + c);
            const float4 q = *reinterpret_cast<const float4*>(y + c);
            dot += p.x * q.x + p.y * q.y + p.z * q.z + p.w * q.w;
          }
        }
        if (SPL == 4) {
          dot = bfly_add<1>(dot);
          dot = bfly_add<2>(dot);
        }
        if (idx < nit && idx == it * SPL) DL[it] = dot * dr.mul(st_attn, (uint32_t)(e_lo * H + it));
      }
    }
    __syncthreads();

    // ---- (D3) softmax backward per (destination, head): dlogit = alpha * (da - sum alpha*da)
    //      GL lanes per (row, head), edges strided over the lanes, sum by shuffles
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
        float sdot = 0.0f;
        for (int e = e0 + gl; e < e1; e += GL) sdot += AL[e * H + h] * DL[e * H + h];
        sdot = group_sum(sdot, GL);
        for (int e = e0 + gl; e < e1; e += GL) {
          const int k = e * H + h;
          const float al = AL[k];
          DL[k] = al * (DL[k] - sdot);
          AL[k] = al * dr.mul(st_attn, (uint32_t)((e + e_lo) * H + h));
        }
      }
    }
    __syncthreads();
    GTR_PH(a.layer, 2);

    // ---- (D4) dQ over in-edges, (D5) dK, dV over out-edges: TPR lanes per row
    float dq[CH], dk[CH], dv[CH];
    if (live) {
      const int hd = f0 / C;
      const float isc = 1.0f / a.sqrt_c;
#pragma unroll
      for (int c = 0; c < CH; ++c) { dq[c] = 0.0f; dk[c] = 0.0f; dv[c] = 0.0f; }
      const int e1 = iptr[prow + 1];
      for (int e = iptr[prow]; e < e1; ++e) {
        const float cdl = DL[e * H + hd] * isc;
        const float* kr = Ks + isrc[e] * XS + f0;
#pragma unroll
        for (int c = 0; c < CH; c += 4) {
          const float4 k4 = *reinterpret_cast<const float4*>(kr + c);
          dq[c] += cdl * k4.x; dq[c + 1] += cdl * k4.y; dq[c + 2] += cdl * k4.z; dq[c + 3] += cdl * k4.w;
        }
      }
      const int i1 = optr[prow + 1];
      for (int i = optr[prow]; i < i1; ++i) {
        const int p = oedge[i], dd = odst[i];
        const float cdl = DL[p * H + hd] * isc;
        const float am = AL[p * H + hd];
        const float* qr = Qs + dd * XS + f0;
        const float* gr = DAs + dd * XS + f0;
#pragma unroll
        for (int c = 0; c < CH; c += 4) {
          const float4 q4 = *reinterpret_cast<const float4*>(qr + c);
          const float4 g4 = *reinterpret_cast<const float4*>(gr + c);
          dk[c] += cdl * q4.x; dk[c + 1] += cdl * q4.y; dk[c + 2] += cdl * q4.z; dk[c + 3] += cdl * q4.w;
          dv[c] += am * g4.x; dv[c + 1] += am * g4.y; dv[c + 2] += am * g4.z; dv[c + 3] += am * g4.w;
        }
      }
      float* drow = a.dqkvs + (size_t)t * (4 * D) + f0;
#pragma unroll
      for (int c = 0; c < CH; c += 4) {
        *reinterpret_cast<float4*>(drow + c) = make_float4(dq[c], dq[c + 1], dq[c + 2], dq[c + 3]);
        *reinterpret_cast<float4*>(drow + D + c) = make_float4(dk[c], dk[c + 1], dk[c + 2], dk[c + 3]);
        *reinterpret_cast<float4*>(drow + 2 * D + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
      }
    }
    if constexpr (!DX) return;
    if constexpr (!SPLIT) {
      // the group's dQKVS rows (fp32, row stride AS32) over the K | V | Q | dA rows (dead from
      // here on): the A operand of phase X from LDS instead of L2
      __syncthreads();
      if (live) {
        float* ar = sm + G::B_R + prow * AS32 + f0;
        const float* parts[4] = {dq, dk, dv, dsv};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
          for (int c = 0; c < CH; c += 4)
            *reinterpret_cast<float4*>(ar + p * D + c) =
                make_float4(parts[p][c], parts[p][c + 1], parts[p][c + 2], parts[p][c + 3]);
        }
      }
    }
    if constexpr (SPLIT) {
      // the group's dQKVS rows, split into bf16 hi | lo, over the K | V | Q | dA rows (dead
      // from here on): the A operand of phase X, read from LDS by every wave
      __syncthreads();
      if (live) {
        __bf16* ah = reinterpret_cast<__bf16*>(sm + G::B_R) + prow * ASB + f0;
        __bf16* al = ah + RMAX * ASB;
        const float* parts[4] = {dq, dk, dv, dsv};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
          for (int c = 0; c < CH; c += 4) {
            bf16x4 h, l;
            split4(make_float4(parts[p][c], parts[p][c + 1], parts[p][c + 2], parts[p][c + 3]), h, l);
            *reinterpret_cast<bf16x4*>(ah + p * D + c) = h;
            *reinterpret_cast<bf16x4*>(al + p * D + c) = l;
          }
        }
      }
    }
  } else {
  // W_all fragments of this wave's dX column tile, requested once the staging loads are
  // out (vector loads retire in order: issued first they would hold up the staging) so
  // they arrive during the attention phases instead of inside the dX MFMA chain
  if constexpr (PREB) {
    const int ct0 = WPC > 1 ? wave % NCT : wave;
    const float* bcol = a.w_all + (size_t)((lane >> 4) * 4) * D + ct0 * 16 + (lane & 15);
#pragma unroll
    for (int kb = 0; kb < D / 4; ++kb) {
      const float* bp = bcol + (size_t)(kb * 16) * D;
      wb[kb] = make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]);
    }
  }
    __syncthreads();
    GTR_PH(a.layer, 1);
    wprefetch();
    // ---- general path: wave per row against global memory (any group size / dim)
    const int d0 = lane * VPL;
    const bool act = d0 < D;
    float k_g[VPL], k_mean[VPL], k_rstd[VPL], k_s1[VPL], k_s2[VPL];
    {
      const int j = act ? d0 : 0;
      load_vec<VPL>(k_g, a.gamma + j, true);
      load_vec<VPL>(k_mean, a.stats + j, true);
      load_vec<VPL>(k_rstd, a.stats + D + j, true);
      const float* gs = a.cred ? s_gs : a.gsum;
      load_vec<VPL>(k_s1, gs + j, true);
      load_vec<VPL>(k_s2, gs + D + j, true);
#pragma unroll
      for (int v = 0; v < VPL; ++v) { k_s1[v] *= invN; k_s2[v] *= invN; }
    }
    for (int t = r0 + wave; t < r1; t += CONV_WAVES)
      bwd_dst_row<D>(a, t, t, a.qkvs + D, a.qkvs + 2 * D, 4 * D, a.bt.in_ptr, a.bt.in_src, a.alpha, a.dlogit, 0,
                     lane, dr, st_attn, k_g, k_mean, k_rstd, k_s1, k_s2);
    __syncthreads();
    GTR_PH(a.layer, 2);
    for (int s = r0 + wave; s < r1; s += CONV_WAVES)
      bwd_src_row<D>(a, s, s, a.qkvs, 4 * D, a.dagg, D, a.bt.out_ptr, a.bt.out_edge, a.bt.out_dst, a.alpha,
                     a.dlogit, 0, lane, dr, st_attn);
    if constexpr (!DX) return;
  }
  __syncthreads();
  GTR_PH(a.layer, 3);

  // ---- phase X: dX = dQKVS . W_all (MFMA f32, operands straight from L2), + residual;
  //      previous layer's dropout mask; that BatchNorm's backward sums in the epilogue.
  //      Wave w owns column tile(s) ct = w % NCT (+ CONV_WAVES for CPW = 2) and the row
  //      tiles rt = rs, rs + WPC, ... with rs = w / NCT.
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t st_prev = drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  const int rs = WPC > 1 ? wave / NCT : 0;
  float s1[CPW], s2[CPW], pm[CPW], pr[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    s1[c] = 0.0f; s2[c] = 0.0f; pm[c] = 0.0f; pr[c] = 0.0f;
    const int ct = (WPC > 1 ? wave % NCT : wave) + c * CONV_WAVES;
    if (a.has_prev) { pm[c] = a.p_stats[ct * 16 + lr]; pr[c] = a.p_stats[D + ct * 16 + lr]; }
  }
  if constexpr (SPLIT) {
    if (fast) {
      // split-bf16 MFMA: A (dQKVS rows) hi | lo from LDS; each B fragment (8 K-values of
      // one W_all column) is loaded and split once per wave and used for every row tile
      const __bf16* AH = reinterpret_cast<const __bf16*>(sm + G::B_R);
      const __bf16* AL = AH + RMAX * ASB;
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        const int ct = (WPC > 1 ? wave % NCT : wave) + c * CONV_WAVES;
        f32x4 acc[RTW];
#pragma unroll
        for (int r = 0; r < RTW; ++r) acc[r] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const float* bcol = a.w_all + (size_t)(lg * 8) * D + ct * 16 + lr;
#pragma unroll 2
        for (int ks = 0; ks < D / 8; ++ks) {
          const float* bp = bcol + (size_t)(ks * 32) * D;
          bf16x8 bh, bl;
          split8(make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]), make_float4(bp[4 * D], bp[5 * D], bp[6 * D], bp[7 * D]),
                 bh, bl);
#pragma unroll
          for (int r = 0; r < RTW; ++r) {
            const int tile = rs + r * WPC;
            if (tile * 16 < nrow) {  // wave-uniform
              const int off = (tile * 16 + lr) * ASB + ks * 32 + lg * 8;
              acc[r] = mfma_split(*reinterpret_cast<const bf16x8*>(AH + off), *reinterpret_cast<const bf16x8*>(AL + off),
                                  bh, bl, acc[r]);
            }
          }
        }
        const int col = ct * 16 + lr;
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = r0 + (rs + r * WPC) * 16 + lg * 4 + i;
            if (row < r1) {
              const size_t o = (size_t)row * D + col;
              const float dx = a.dy[o] + acc[r][i];
              if (a.has_prev) {
                const float d = dx * dr.mul(st_prev, (uint32_t)o);
                a.p_dy[o] = d;
                s1[c] += d;
                s2[c] += d * ((a.p_out[o] - pm[c]) * pr[c]);
              } else {
                a.dx0[o] = dx;
              }
            }
          }
        }
      }
    }
  }
  if constexpr (!SPLIT && G::KV) {
    if (fast) {
      // f32 MFMA, A rows from LDS, B from the prefetched fragments; the wave's live row
      // tiles advance together (every output element still sums its k terms in the order
      // of the one-tile-at-a-time loop below, so the results are bitwise those of it)
      const float* A = sm + G::B_R;
      auto tiles = [&](auto nr_c) {
        constexpr int NR = decltype(nr_c)::value;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
          const int ct = (WPC > 1 ? wave % NCT : wave) + c * CONV_WAVES;
          const float* bcol = a.w_all + (size_t)(lg * 4) * D + ct * 16 + lr;
          f32x4 acc[NR];
#pragma unroll
          for (int r = 0; r < NR; ++r) acc[r] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll  // whole: wb[] stays in registers only with constant indices
          for (int kb = 0; kb < D / 4; ++kb) {
            float4 bv;
            if constexpr (PREB) {
              bv = wb[kb];
            } else {
              const float* bp = bcol + (size_t)(kb * 16) * D;
              bv = make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r)
              acc[r] = mfma4(*reinterpret_cast<const float4*>(A + ((rs + r * WPC) * 16 + lr) * AS32 + kb * 16 + lg * 4),
                             bv, acc[r]);
          }
          const int col = ct * 16 + lr;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int row = r0 + (rs + r * WPC) * 16 + lg * 4 + i;
              if (row < r1) {
                const size_t o = (size_t)row * D + col;
                const float dx = a.dy[o] + acc[r][i];
                if (a.has_prev) {
                  const float d = dx * dr.mul(st_prev, (uint32_t)o);
                  a.p_dy[o] = d;
                  s1[c] += d;
                  s2[c] += d * ((a.p_out[o] - pm[c]) * pr[c]);
                } else {
                  a.dx0[o] = dx;
                }
              }
            }
          }
        }
      };
      // live row tiles of this wave: rs, rs + WPC, ... below the group's row count
      const int nlive = rs * 16 < nrow ? min(RTW, ((nrow + 15) / 16 - rs + WPC - 1) / WPC) : 0;
      if (nlive == 1) tiles(std::integral_constant<int, 1>{});
      if constexpr (RTW >= 2) if (nlive == 2) tiles(std::integral_constant<int, 2>{});
      if constexpr (RTW >= 3) if (nlive == 3) tiles(std::integral_constant<int, 3>{});
      if constexpr (RTW >= 4) if (nlive == 4) tiles(std::integral_constant<int, 4>{});
      static_assert(RTW <= 4, "row tiles per wave");
    }
  }
  for (int rt = r0 + rs * 16; !fast && rt < r1; rt += 16 * WPC) {
    const int ar = min(rt + lr, r1 - 1);  // clamp: rows past the group are computed, never stored
    const float* arow = a.dqkvs + (size_t)ar * (4 * D) + lg * 4;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ct = (WPC > 1 ? wave % NCT : wave) + c * CONV_WAVES;
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      const float* bcol = a.w_all + (size_t)(lg * 4) * D + ct * 16 + lr;
#pragma unroll 4
      for (int kb = 0; kb < D / 4; ++kb) {
        const float4 av = *reinterpret_cast<const float4*>(arow + kb * 16);
        const float* bp = bcol + (size_t)(kb * 16) * D;
        acc = mfma4(av, make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]), acc);
      }
      const int col = ct * 16 + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rt + lg * 4 + i;
        if (row < r1) {
          const size_t o = (size_t)row * D + col;
          const float dx = a.dy[o] + acc[i];
          if (a.has_prev) {
            const float d = dx * dr.mul(st_prev, (uint32_t)o);
            a.p_dy[o] = d;
            s1[c] += d;
            s2[c] += d * ((a.p_out[o] - pm[c]) * pr[c]);
          } else {
            a.dx0[o] = dx;
          }
        }
      }
    }
  }

  // ---- phase W (gtr_config.wfold_stride): this group's split-K partial of the layer's
  //      weight gradients -- the gtr_wgrad jobs of the layer over the group's rows, at the
  //      gtr_wgrad slab offsets (w_all [4D][D] | b_all [4D] | w_beta [3D]); the optimizer
  //      tail sums the live groups' partials (gtr_segment.live_groups) in group order.
  //      dW_all = dQKVS^T . X on f32 MFMA 16x16x4 (A: a dQKVS row's 16 output units, B: an X
  //      row's 16 input columns; 4 rows per step); wave w owns j-tiles [w*TJW, (w+1)*TJW) x
  //      every k-tile, JB j-tiles (16 accumulator tiles) at a time.
  GTR_PH(a.layer, 9);
  if (WF && a.wslab) {
    // Everything on f32 MFMA 16x16x4 over the group's rows (4 per step), each sum complete
    // in one accumulator (no cross-wave reduction):
    //   dW_all[j][k] = sum_r dQKVS[r][j] X[r][k]   A: a dQKVS row's 16 output units,
    //                                              B: an X row's 16 input columns;
    //   b_all[j]     = sum_r dQKVS[r][j]           one more B tile: a ones column;
    //   w_beta[c]    = sum_r du[r] G[r][c]         A: du in unit 0, B: [agg | S | agg - S].
    // Wave w owns dW j-tiles [w*TJW, (w+1)*TJW) x every k-tile (+ the ones tile), JB j-tiles
    // at a time, and gate tiles [w*GPW, (w+1)*GPW).
    constexpr int TJ = 4 * D / 16, TK = D / 16;
    constexpr int TJW = TJ / CONV_WAVES > 0 ? TJ / CONV_WAVES : 1;
    constexpr int JB = (16 / (TK + 1)) < 1 ? 1 : ((16 / (TK + 1)) < TJW ? 16 / (TK + 1) : TJW);
    static_assert(TJ % CONV_WAVES == 0 && TJW % JB == 0, "phase W tiling");
    float* slab = a.wslab + (size_t)g * a.wstride;
    float* bias = slab + (size_t)4 * D * D;
    float* gw = bias + 4 * D;
    const float* Xb = a.xin + (size_t)r0 * D;
    const int nks = (nrow + 3) / 4;
    // Ab: the group's dQKVS rows (stride astr), dU its du values -- LDS on the fast path,
    // global rows otherwise.  One body per memory kind (called in two branches, never
    // through one pointer that could be either): a generic (flat) load would make its
    // waits wait for every outstanding global store of the dX phase as well.
    auto body = [&](const float* Ab, int astr, const float* dU, bool lds) {
      auto arow = [&](int rr, int col) {  // LDS rows up to RMAX exist: no branch needed
        if (lds) { const float t = Ab[(size_t)rr * astr + col]; return rr < nrow ? t : 0.0f; }
        return rr < nrow ? Ab[(size_t)rr * astr + col] : 0.0f;
      };
      for (int jb = 0; jb < TJW; jb += JB) {
        const int j0 = (wave * TJW + jb) * 16;
        f32x4 acc[JB][TK + 1];
#pragma unroll
        for (int u = 0; u < JB; ++u)
#pragma unroll
          for (int t = 0; t <= TK; ++t) acc[u][t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (int ks = 0; ks < nks; ++ks) {
          const int rr = ks * 4 + lg;
          const bool live = rr < nrow;
          float bv[TK + 1], av[JB];
          if (ks < 2) {  // prefetched after the staging
#pragma unroll
            for (int t = 0; t < TK; ++t) bv[t] = ks == 0 ? wx[0][t] : wx[1][t];
          } else {
#pragma unroll
            for (int t = 0; t < TK; ++t) bv[t] = live ? Xb[(size_t)rr * D + t * 16 + lr] : 0.0f;
          }
          bv[TK] = (live && lr == 0) ? 1.0f : 0.0f;
#pragma unroll
          for (int u = 0; u < JB; ++u) av[u] = arow(rr, j0 + u * 16 + lr);
#pragma unroll
          for (int u = 0; u < JB; ++u)
#pragma unroll
            for (int t = 0; t <= TK; ++t)
              acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[t], acc[u][t], 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < JB; ++u) {
#pragma unroll
          for (int t = 0; t < TK; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) slab[(size_t)(j0 + u * 16 + lg * 4 + i) * D + t * 16 + lr] = acc[u][t][i];
          if (lr == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) bias[j0 + u * 16 + lg * 4 + i] = acc[u][TK][i];
          }
        }
      }
      if (wave * GPW < NGT) {  // wave-uniform
        f32x4 gacc[GPW];
#pragma unroll
        for (int q = 0; q < GPW; ++q) gacc[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (int ks = 0; ks < nks; ++ks) {
          const int rr = ks * 4 + lg;
          const bool live = rr < nrow;
          float du = 0.0f;
          if (lr == 0 && live) du = dU[rr];
#pragma unroll
          for (int q = 0; q < GPW; ++q) {
            const int gt = wave * GPW + q, c = gt * 16 + lr, sel = c / D, col = c % D;
            float x, y;
            if (ks < 2) {
              x = ks == 0 ? wga[0][q] : wga[1][q];
              y = ks == 0 ? wgs[0][q] : wgs[1][q];
            } else {
              const bool ok = live && gt < NGT;
              x = ok ? a.agg[(size_t)(r0 + rr) * D + col] : 0.0f;
              y = ok ? a.qkvs[(size_t)(r0 + rr) * (4 * D) + 3 * D + col] : 0.0f;
            }
            const float bvg = sel == 0 ? x : (sel == 1 ? y : x - y);
            gacc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(du, bvg, gacc[q], 0, 0, 0);
          }
        }
#pragma unroll
        for (int q = 0; q < GPW; ++q) {
          const int gt = wave * GPW + q;
          if (lg == 0 && gt < NGT) gw[gt * 16 + lr] = gacc[q][0];  // row 0 of the tile: unit du
        }
      }
    };
    if (fast && !SPLIT) body(sm + G::B_R, AS32, s_du, true);  // fp32 dQKVS rows and du in LDS
    else body(a.dqkvs + (size_t)r0 * (4 * D), 4 * D, a.du + r0, false);
  }
  GTR_PH(a.layer, 4);
  if (!a.has_prev) return;
  // ---- previous layer's BatchNorm backward partials: reduce the 4 row quads of each
  //      column, then the WPC waves sharing a column tile (fixed order)
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const int ct = (WPC > 1 ? wave % NCT : wave) + c * CONV_WAVES;
    float x1 = s1[c], x2 = s2[c];
    x1 = bfly_add<32>(bfly_add<16>(x1));
    x2 = bfly_add<32>(bfly_add<16>(x2));
    if (lg == 0) {
      s_bnp[rs * 2 * D + ct * 16 + lr] = x1;
      s_bnp[rs * 2 * D + D + ct * 16 + lr] = x2;
    }
  }
  __syncthreads();
  float* part = a.p_gpart + (size_t)g * 2 * D;
  for (int j = tid; j < 2 * D; j += CONV_BLOCK) {
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < WPC; ++q) acc += s_bnp[q * 2 * D + j];
    if (a.cred) part[j] = acc;
    else st_wt(part + j, acc);  // write-through: read by the last arriver of this launch
  }
  if (a.cred) return;  // the next conv_bwd reduces the partials
  const int nbk = (Gn + GTR_PART_BUCKET - 1) / GTR_PART_BUCKET;  // LDS is dead by now: scratch
  if (nbk > 1) {  // bucketed: merge 32 partial rows into the bucket's first, then the buckets
    const int bk = g / GTR_PART_BUCKET, b0 = bk * GTR_PART_BUCKET;
    if (!arrive_last_wt(a.p_cnt + 4 + 2 * bk, (uint32_t)min(GTR_PART_BUCKET, Gn - b0), s_flag)) return;
    float* row0 = a.p_gpart + (size_t)b0 * 2 * D;
    block_sum_rows<CONV_BLOCK>(row0, min(GTR_PART_BUCKET, Gn - b0), 2 * D, (size_t)2 * D, row0, sm, true);
    if (tid == 0) reset_counter(a.p_cnt + 4 + 2 * bk);
    if (!arrive_last_wt(a.p_cnt, (uint32_t)nbk, s_flag)) return;
    block_sum_rows<CONV_BLOCK>(a.p_gpart, nbk, 2 * D, (size_t)GTR_PART_BUCKET * 2 * D, a.p_gsum, sm);
  } else {
    if (!arrive_last_wt(a.p_cnt, (uint32_t)Gn, s_flag)) return;
    block_sum_rows<CONV_BLOCK>(a.p_gpart, Gn, 2 * D, (size_t)2 * D, a.p_gsum, sm);
  }
  if (tid == 0) reset_counter(a.p_cnt);
}

// Arguments of conv_bwd_body for layer l (the launch geometry -- main_grid, sweep, xpack --
// is left to the caller).  0 or a GTR_E_* status with gtr_last_error() set.
inline int make_bwd_args(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                         float* dx0, ConvBwdK& k) {
  const int D = cfg->dim;
  if (!(D == 32 || D == 64 || D == 128 || D == 256) || cfg->heads <= 0 || D % cfg->heads) {
    set_error("gtr_conv_bwd: unsupported dims");
    return GTR_E_ARG;
  }
  if (!cfg->training) { set_error("gtr_conv_bwd: backward requires training mode"); return GTR_E_ARG; }
  if (l == 0 && !dx0) { set_error("gtr_conv_bwd: layer 0 needs dx0"); return GTR_E_ARG; }
  if (!bt->grp_row || !bt->grp_edge) { set_error("gtr_conv_bwd: batch lacks row-group ranges"); return GTR_E_ARG; }
  const gtr_layer& L = layers[l];
  k = ConvBwdK{};
  k.bt = *bt;
  k.H = cfg->heads;
  k.C = D / cfg->heads;
  k.layer = l;
  k.cred = cfg->consumer_reduce;
  // partials feeding this layer's sums: the readout grid for the last layer, else the conv groups
  k.gpart_n = -1;
  if (l == cfg->num_layers - 1) {
    k.gpart_n = gtr_readout_grid(bt->b_cap);
  }
  k.has_prev = l > 0;
  k.sqrt_c = (float)sqrt((double)k.C);
  k.drop_on = (cfg->dropout > 0.0f) ? 1 : 0;
  double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
  k.thresh = (uint32_t)(p * 4294967296.0);
  k.scale = k.drop_on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.ctr_add = (uint32_t)cfg->ctr_add;
  k.dy = L.dy; k.out = L.out; k.stats = L.bn_stats; k.gsum = L.bn_gsum; k.gpart = L.bn_gpart; k.gamma = L.bn_gamma;
  k.qkvs = L.qkvs; k.alpha = L.alpha; k.agg = L.agg; k.gate = L.gate; k.w_all = L.w_all; k.w_beta = L.w_beta;
  k.dqkvs = L.dqkvs; k.du = L.du; k.dlogit = L.dlogit; k.dagg = L.dagg;
  if (l > 0) {
    const gtr_layer& P = layers[l - 1];
    k.p_out = P.out; k.p_stats = P.bn_stats; k.p_dy = P.dy; k.p_gpart = P.bn_gpart;
    k.p_gsum = P.bn_gsum; k.p_cnt = P.cnt + 1;
  }
  k.dx0 = dx0;
  k.sync = cfg->sync_bn;
  k.gpart_all = L.bn_gpart_all;
  k.nparts_bwd = L.nparts_bwd;
  k.part_all = L.bn_part_all;
  k.nparts_fwd = L.nparts_fwd;
  if (cfg->wfold_stride > 0 && L.wfold) {  // weight gradients folded into the row groups
    if (D > 64) {
      set_error("gtr_conv_bwd: folded weight gradients cover D <= 64 (gtr_wgrad otherwise)");
      return GTR_E_ARG;
    }
    if ((reinterpret_cast<uintptr_t>(L.wfold) & 15) || cfg->wfold_stride < (int64_t)4 * D * D + 7 * D) {
      set_error("gtr_conv_bwd: wfold slab misaligned or its stride below 4D^2 + 7D");
      return GTR_E_ARG;
    }
    k.wslab = L.wfold;
    k.wstride = cfg->wfold_stride;
    k.xin = L.xin;
  }
  if (cfg->sync_bn && (!cfg->consumer_reduce || !L.bn_gpart_all || !L.bn_part_all || L.nparts_bwd <= 0 ||
                       L.nparts_fwd <= 0)) {
    set_error("gtr_conv_bwd: sync_bn needs consumer_reduce and the gathered partials of layer %d", l);
    return GTR_E_ARG;
  }
  return GTR_OK;
}
