// gtr_bwd.hip — backward kernels of the GraphTransformer hot path (gfx950).
//
// k_conv_bwd<D>: autograd of graph_transformer.py:171-177 for one layer
//   (BatchNorm backward from finalized batch sums, beta-gate backward, attention
//   softmax backward, dK/dV gathered over out-edges (CSR by source — no float
//   atomics, deterministic), dX = dQKVS . W_all on MFMA, residual add, previous
//   layer's dropout mask and BatchNorm backward sums).  Same row groups as the
//   forward: every edge of a processed destination stays inside the workgroup.
// k_wgrad: lin_{query,key,value,skip} weight/bias, lin_beta and LapPE projection
//   gradients as deterministic per-chunk partial slabs (summed by the optimizer).

#include "gtr_common.cuh"

namespace {

using namespace gtr;

struct ConvBwdK {
  gtr_batch bt;
  int H, C, R, layer, has_prev, pad0;
  float sqrt_c, scale;
  uint32_t seed, thresh;
  int drop_on, pad1;
  const uint32_t* rng_ctr;
  const float* dy;
  const float* out;
  const float* stats;
  const float* gsum;
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
};

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_conv_bwd(ConvBwdK a) {
  constexpr int VPL = D >= 64 ? D / 64 : 1;
  constexpr int AS = 4 * D + 4;
  extern __shared__ __attribute__((aligned(16))) float As[];  // [16][AS] + flag word
  int& s_flag = *reinterpret_cast<int*>(As + 16 * AS);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.bt.hdr[0], B = a.bt.hdr[1];
  const int G = (N + a.R - 1) / a.R;
  const int g = blockIdx.x;
  if (g >= G) return;
  int r0, r1;
  group_rows(a.bt.node_ptr, B, a.R, g, r0, r1);
  const uint32_t ctr = a.rng_ctr ? *a.rng_ctr : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int GL = C / VPL;
  const int head = act ? d0 / C : 0;
  const bool leader = act && ((lane & (GL - 1)) == 0);
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const float invN = 1.0f / (float)N;

  // per-lane BatchNorm backward constants
  float k_g[VPL], k_mean[VPL], k_rstd[VPL], k_s1[VPL], k_s2[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int j = act ? d0 + v : 0;
    k_g[v] = a.gamma[j];
    k_mean[v] = a.stats[j];
    k_rstd[v] = a.stats[D + j];
    k_s1[v] = a.gsum[j] * invN;
    k_s2[v] = a.gsum[D + j] * invN;
  }

  // ---- phase 1: per destination row: BN backward, gate backward, softmax backward, dQ, dS
  for (int t = r0 + wave; t < r1; t += GTR_WAVES) {
    const float* qt = a.qkvs + (size_t)t * (4 * D);
    float gv[VPL], ag[VPL], sv[VPL];
    const float beta = a.gate[t];
    float dbeta = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      if (act) {
        const size_t o = (size_t)t * D + d0 + v;
        const float xh = (a.out[o] - k_mean[v]) * k_rstd[v];
        gv[v] = (a.dy[o] - k_s1[v] - xh * k_s2[v]) * k_rstd[v] * k_g[v];
        ag[v] = a.agg[o];
        sv[v] = qt[3 * D + d0 + v];
        dbeta += gv[v] * (sv[v] - ag[v]);
      } else {
        gv[v] = ag[v] = sv[v] = 0.0f;
      }
    }
    dbeta = wave_sum(dbeta);
    const float du = dbeta * beta * (1.0f - beta);
    if (lane == 0) a.du[t] = du;
    float dag[VPL], dq[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      dq[v] = 0.0f;
      dag[v] = 0.0f;
      if (act) {
        const int j = d0 + v;
        const float w1 = a.w_beta[j], w2 = a.w_beta[D + j], w3 = a.w_beta[2 * D + j];
        dag[v] = gv[v] * (1.0f - beta) + du * (w1 + w3);
        const float ds = gv[v] * beta + du * (w2 - w3);
        a.dqkvs[(size_t)t * (4 * D) + 3 * D + j] = ds;
        a.dagg[(size_t)t * D + j] = dag[v];
      }
    }
    const int e0 = a.bt.in_ptr[t], e1 = a.bt.in_ptr[t + 1];
    float sdot = 0.0f;
    for (int e = e0; e < e1; ++e) {
      const float* vt = a.qkvs + (size_t)a.bt.in_src[e] * (4 * D) + 2 * D;
      float d = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) d += act ? dag[v] * vt[d0 + v] : 0.0f;
      d = group_sum(d, GL);
      const float al = a.alpha[(size_t)e * H + head];
      const float da = d * dr.mul(st_attn, (uint32_t)(e * H + head));
      sdot += al * da;
    }
    for (int e = e0; e < e1; ++e) {
      const float* kv = a.qkvs + (size_t)a.bt.in_src[e] * (4 * D);
      float d = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) d += act ? dag[v] * kv[2 * D + d0 + v] : 0.0f;
      d = group_sum(d, GL);
      const float al = a.alpha[(size_t)e * H + head];
      const float da = d * dr.mul(st_attn, (uint32_t)(e * H + head));
      const float dl = al * (da - sdot);
      if (leader) a.dlogit[(size_t)e * H + head] = dl;
      const float c = dl / a.sqrt_c;
#pragma unroll
      for (int v = 0; v < VPL; ++v) dq[v] += act ? c * kv[D + d0 + v] : 0.0f;
    }
    if (act) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) a.dqkvs[(size_t)t * (4 * D) + d0 + v] = dq[v];
    }
  }
  __syncthreads();

  // ---- phase 2: per source row: dK, dV over out-edges (CSR by source)
  for (int s = r0 + wave; s < r1; s += GTR_WAVES) {
    float dk[VPL], dv[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) { dk[v] = 0.0f; dv[v] = 0.0f; }
    const int i0 = a.bt.out_ptr[s], i1 = a.bt.out_ptr[s + 1];
    for (int i = i0; i < i1; ++i) {
      const int p = a.bt.out_edge[i];
      const int t = a.bt.out_dst[i];
      const float dl = a.dlogit[(size_t)p * H + head] / a.sqrt_c;
      const float ad = a.alpha[(size_t)p * H + head] * dr.mul(st_attn, (uint32_t)(p * H + head));
      const float* qt = a.qkvs + (size_t)t * (4 * D);
      const float* dgt = a.dagg + (size_t)t * D;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        if (act) {
          dk[v] += dl * qt[d0 + v];
          dv[v] += ad * dgt[d0 + v];
        }
      }
    }
    if (act) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        a.dqkvs[(size_t)s * (4 * D) + D + d0 + v] = dk[v];
        a.dqkvs[(size_t)s * (4 * D) + 2 * D + d0 + v] = dv[v];
      }
    }
  }
  __syncthreads();

  // ---- phase 3: dX = dQKVS . W_all (MFMA f32), + residual; prev-layer dropout mask
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t st_prev = drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  for (int rt = r0; rt < r1; rt += 16) {
    for (int idx = tid; idx < 16 * 4 * D; idx += GTR_BLOCK) {
      const int i = idx / (4 * D), j = idx - i * (4 * D);
      const int r = rt + i;
      As[i * AS + j] = r < r1 ? a.dqkvs[(size_t)r * (4 * D) + j] : 0.0f;
    }
    __syncthreads();
    for (int ct = wave; ct < D / 16; ct += GTR_WAVES) {
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      const float* arow = As + lr * AS + lg * 4;
      const float* bcol = a.w_all + (size_t)(lg * 4) * D + ct * 16 + lr;
#pragma unroll 4
      for (int kb = 0; kb < D / 4; ++kb) {
        const float4 av = *reinterpret_cast<const float4*>(arow + kb * 16);
        const float* bp = bcol + (size_t)(kb * 16) * D;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bp[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bp[D], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bp[2 * D], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bp[3 * D], acc, 0, 0, 0);
      }
      const int col = ct * 16 + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rt + lg * 4 + i;
        if (row < r1) {
          const size_t o = (size_t)row * D + col;
          const float dx = a.dy[o] + acc[i];
          if (a.has_prev) a.p_dy[o] = dx * dr.mul(st_prev, (uint32_t)o);
          else a.dx0[o] = dx;
        }
      }
    }
    __syncthreads();
  }

  if (!a.has_prev) return;
  // ---- phase 4: previous layer's BatchNorm backward sums: sum(dy), sum(dy * xhat)
  float* part = a.p_gpart + (size_t)g * 2 * D;
  for (int j = tid; j < D; j += GTR_BLOCK) {
    const float mean = a.p_stats[j], rstd = a.p_stats[D + j];
    float s1 = 0.0f, s2 = 0.0f;
    for (int r = r0; r < r1; ++r) {
      const size_t o = (size_t)r * D + j;
      const float d = a.p_dy[o];
      s1 += d;
      s2 += d * ((a.p_out[o] - mean) * rstd);
    }
    part[j] = s1;
    part[D + j] = s2;
  }
  if (!arrive_last(a.p_cnt, (uint32_t)G, &s_flag)) return;
  for (int j = tid; j < 2 * D; j += GTR_BLOCK) {
    float acc = 0.0f;
    for (int q = 0; q < G; ++q) acc += a.p_gpart[(size_t)q * 2 * D + j];
    a.p_gsum[j] = acc;
  }
  if (tid == 0) reset_counter(a.p_cnt);
}

// ------------------------------------------------------------------------------------
// weight gradients
// ------------------------------------------------------------------------------------

enum { WJ_MM = 0, WJ_GATE = 1 };

struct WJob {
  int type, M1, M2, lda, ldb, tn, nt, blk0;
  const float* A;
  const float* B;
  const int32_t* bidx;
  const float* agg;
  const float* s;   // skip rows (qkvs + 3D), row stride lda
  float* outW;
  float* outB;
};

#define GTR_MAX_WJOBS 16

struct WgradK {
  const int32_t* hdr;
  int P, njobs, D, pad0;
  int64_t stride;
  WJob jobs[GTR_MAX_WJOBS];
};

__global__ __launch_bounds__(GTR_BLOCK) void k_wgrad(WgradK a) {
  __shared__ __attribute__((aligned(16))) float As[16][64];
  __shared__ __attribute__((aligned(16))) float Bs[16][64];
  const int tid = threadIdx.x;
  const int blk = blockIdx.x;
  int jid = 0;
  while (jid + 1 < a.njobs && blk >= a.jobs[jid + 1].blk0) ++jid;
  const WJob& J = a.jobs[jid];
  const int local = blk - J.blk0;
  const int tile = local / a.P, p = local - tile * a.P;
  const int N = a.hdr[0];
  const int per = (N + a.P - 1) / a.P;
  const int t0 = p * per;
  const int t1 = min(N, t0 + per);
  const int64_t so = (int64_t)p * a.stride;

  if (J.type == WJ_GATE) {
    const int D = a.D;
    const int j = tile * GTR_BLOCK + tid;
    if (j >= 3 * D) return;
    float acc = 0.0f;
    for (int t = t0; t < t1; ++t) {
      const float u = J.A[t];
      float f;
      if (j < D) f = J.agg[(size_t)t * D + j];
      else if (j < 2 * D) f = J.s[(size_t)t * J.lda + (j - D)];
      else f = J.agg[(size_t)t * D + (j - 2 * D)] - J.s[(size_t)t * J.lda + (j - 2 * D)];
      acc += u * f;
    }
    J.outW[so + j] = acc;
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
  for (int tb = t0; tb < t1; tb += 16) {
    for (int idx = tid; idx < 16 * 64; idx += GTR_BLOCK) {
      const int i = idx >> 6, c = idx & 63;
      const int t = tb + i;
      float av = 0.0f, bv = 0.0f;
      if (t < t1) {
        if (m0 + c < J.M1) av = J.A[(size_t)t * J.lda + m0 + c];
        const int col = n0 + c;
        if (col < J.M2) {
          const float* brow = J.bidx ? J.B + (size_t)J.bidx[t] * J.ldb : J.B + (size_t)t * J.ldb;
          bv = brow[col];
        } else if (col == J.M2) {
          bv = 1.0f;
        }
      }
      As[i][c] = av;
      Bs[i][c] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float4 a4 = *reinterpret_cast<const float4*>(&As[k][ty * 4]);
      const float4 b4 = *reinterpret_cast<const float4*>(&Bs[k][tx * 4]);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
      const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] += av[i] * bv[q];
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
      if (nn < J.M2) J.outW[so + (int64_t)m * J.M2 + nn] = acc[i][q];
      else if (nn == J.M2) J.outB[so + m] = acc[i][q];
    }
  }
}

}  // namespace

extern "C" int gtr_conv_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            float* dx0, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_conv_bwd: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim;
  if (!(D == 32 || D == 64 || D == 128 || D == 256) || cfg->heads <= 0 || D % cfg->heads) {
    set_error("gtr_conv_bwd: unsupported dims");
    return GTR_E_ARG;
  }
  if (!cfg->training) { set_error("gtr_conv_bwd: backward requires training mode"); return GTR_E_ARG; }
  if (l == 0 && !dx0) { set_error("gtr_conv_bwd: layer 0 needs dx0"); return GTR_E_ARG; }
  const gtr_layer& L = layers[l];
  ConvBwdK k{};
  k.bt = *bt;
  k.H = cfg->heads;
  k.C = D / cfg->heads;
  k.R = cfg->row_group;
  k.layer = l;
  k.has_prev = l > 0;
  k.sqrt_c = (float)sqrt((double)k.C);
  k.drop_on = (cfg->dropout > 0.0f) ? 1 : 0;
  double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
  k.thresh = (uint32_t)(p * 4294967296.0);
  k.scale = k.drop_on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.dy = L.dy; k.out = L.out; k.stats = L.bn_stats; k.gsum = L.bn_gsum; k.gamma = L.bn_gamma;
  k.qkvs = L.qkvs; k.alpha = L.alpha; k.agg = L.agg; k.gate = L.gate; k.w_all = L.w_all; k.w_beta = L.w_beta;
  k.dqkvs = L.dqkvs; k.du = L.du; k.dlogit = L.dlogit; k.dagg = L.dagg;
  if (l > 0) {
    const gtr_layer& P = layers[l - 1];
    k.p_out = P.out; k.p_stats = P.bn_stats; k.p_dy = P.dy; k.p_gpart = P.bn_gpart;
    k.p_gsum = P.bn_gsum; k.p_cnt = P.cnt + 1;
  }
  k.dx0 = dx0;
  const int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  const size_t lds = (size_t)16 * (4 * D + 4) * sizeof(float) + 16;
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 32: hipLaunchKernelGGL(k_conv_bwd<32>, dim3(grid), dim3(GTR_BLOCK), lds, s, k); break;
    case 64: hipLaunchKernelGGL(k_conv_bwd<64>, dim3(grid), dim3(GTR_BLOCK), lds, s, k); break;
    case 128: hipLaunchKernelGGL(k_conv_bwd<128>, dim3(grid), dim3(GTR_BLOCK), lds, s, k); break;
    default: hipLaunchKernelGGL(k_conv_bwd<256>, dim3(grid), dim3(GTR_BLOCK), lds, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers,
                         const float* dx0, const float* pe_tab, float* const* layer_slab, float* pe_slab,
                         int n_chunks, int64_t slab_stride, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !layer_slab || n_chunks <= 0) {
    set_error("gtr_wgrad: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim, Lc = cfg->num_layers;
  if (2 * Lc + 1 > GTR_MAX_WJOBS) { set_error("gtr_wgrad: too many layers"); return GTR_E_ARG; }
  WgradK k{};
  k.hdr = bt->hdr;
  k.P = n_chunks;
  k.D = D;
  k.stride = slab_stride;
  int nj = 0, blocks = 0;
  for (int l = 0; l < Lc; ++l) {
    const gtr_layer& L = layers[l];
    float* base = layer_slab[l];
    WJob& w = k.jobs[nj++];
    w.type = WJ_MM; w.M1 = 4 * D; w.M2 = D; w.lda = 4 * D; w.ldb = D;
    w.tn = (D + 1 + 63) / 64; w.nt = ((4 * D + 63) / 64) * w.tn; w.blk0 = blocks;
    w.A = L.dqkvs; w.B = L.xin; w.bidx = nullptr;
    w.outW = base; w.outB = base + (size_t)4 * D * D;
    blocks += w.nt * n_chunks;
    WJob& q = k.jobs[nj++];
    q.type = WJ_GATE; q.M1 = 1; q.M2 = 3 * D; q.lda = 4 * D; q.tn = 1; q.nt = (3 * D + GTR_BLOCK - 1) / GTR_BLOCK;
    q.blk0 = blocks; q.A = L.du; q.agg = L.agg; q.s = L.qkvs + 3 * D;
    q.outW = base + (size_t)4 * D * D + 4 * D;
    blocks += q.nt * n_chunks;
  }
  if (cfg->pe_k > 0 && pe_slab) {
    if (!dx0 || (!pe_tab && !bt->node_pe)) { set_error("gtr_wgrad: PE gradient needs dx0 and PE rows"); return GTR_E_ARG; }
    const int K = cfg->pe_k;
    WJob& w = k.jobs[nj++];
    w.type = WJ_MM; w.M1 = D; w.M2 = K; w.lda = D; w.ldb = K;
    w.tn = (K + 1 + 63) / 64; w.nt = ((D + 63) / 64) * w.tn; w.blk0 = blocks;
    w.A = dx0;
    if (bt->node_pe) { w.B = bt->node_pe; w.bidx = nullptr; }
    else { w.B = pe_tab; w.bidx = bt->node_item; }
    w.outW = pe_slab; w.outB = pe_slab + (size_t)D * K;
    blocks += w.nt * n_chunks;
  }
  k.njobs = nj;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_wgrad, dim3(blocks), dim3(GTR_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}
