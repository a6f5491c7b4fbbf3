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

#include <string.h>

#include "gtr_layer.cuh"
#include "gtr_wgrad.cuh"

namespace {

using namespace gtr;

GTR_PH_DECL

#include "gtr_bwd_body.cuh"

template <int D, bool SPLIT>
__global__ __launch_bounds__(CONV_BLOCK) void k_conv_bwd(ConvBwdK a) {
  const int rb = role_block(a.main_grid, a.xpack);
  if (rb >= a.main_grid) {  // extra workgroups: untouched-row AdamW slice
    sweep_slice(a.sw, a.sw_slot, rb - a.main_grid, gridDim.x - a.main_grid);
    return;
  }
  conv_bwd_body<D, SPLIT>(a, rb);
}

// Split path (large batches): the attention backward of one row group per workgroup
// (gtr_attn_bwd); dX runs in k_dx (gtr_qkvs_bwd).
template <int D>
__global__ __launch_bounds__(CONV_BLOCK) void k_attn_bwd(ConvBwdK a) {
  conv_bwd_body<D, false, false>(a, blockIdx.x);
}

// Split path, row-parallel attention backward (gtr_attn_bwd at large batches): two
// launches, one wave per row -- (1) per DESTINATION row: BatchNorm backward from the
// finalized sums, beta-gate backward, softmax backward -> dS, dQ, dlogit, dagg; (2) per
// SOURCE row: dK, dV gathered over its out-edges (CSR by source; no atomics) from (1)'s
// dlogit / dagg.  Small LDS, several workgroups per CU (see k_attn_rows); in-edge /
// out-edge rows are fetched four at a time.
#define BR_BLOCK 256
#define BR_WAVES (BR_BLOCK / 64)
#define BR_RPW 2
#define BR_ECH 64
#define BR_HMAX 8
#define BR_VR 8   // K rows of a row pair held in registers

// This layer's BatchNorm constants per lane: gamma, mean, rstd and the backward sums / N
// (sync: every rank's gathered sums, N from the gathered counts).
template <int D>
__device__ __forceinline__ void bwd_row_consts(const ConvBwdK& a, float* s_gs, int& N, float (&k_g)[LayerGeom<D>::VPL],
                                               float (&k_mean)[LayerGeom<D>::VPL], float (&k_rstd)[LayerGeom<D>::VPL],
                                               float (&k_s1)[LayerGeom<D>::VPL], float (&k_s2)[LayerGeom<D>::VPL]) {
  constexpr int VPL = LayerGeom<D>::VPL;
  const int tid = threadIdx.x, lane = tid & 63;
  N = a.bt.hdr[0];
  const float* gs = a.gsum;
  if (a.sync) {
    float n = 0.0f;
    for (int q = 0; q < a.nparts_fwd; ++q) n += a.part_all[(size_t)q * (1 + 2 * D)];
    N = (int)(n + 0.5f);
    for (int j = tid; j < 2 * D; j += blockDim.x) {
      float acc = 0.0f;
      for (int q = 0; q < a.nparts_bwd; ++q) acc += a.gpart_all[(size_t)q * 2 * D + j];
      s_gs[j] = acc;
    }
    __syncthreads();
    gs = s_gs;
  }
  const float invN = 1.0f / (float)N;
  const int d0 = lane * VPL;
  const int j = d0 < D ? d0 : 0;
  load_vec<VPL>(k_g, a.gamma + j, true);
  load_vec<VPL>(k_mean, a.stats + j, true);
  load_vec<VPL>(k_rstd, a.stats + D + j, true);
  load_vec<VPL>(k_s1, gs + j, true);
  load_vec<VPL>(k_s2, gs + D + j, true);
#pragma unroll
  for (int v = 0; v < VPL; ++v) { k_s1[v] *= invN; k_s2[v] *= invN; }
}

template <int D>
__global__ __launch_bounds__(BR_BLOCK) void k_attn_rows_bwd_dst(ConvBwdK a) {
  constexpr int VPL = LayerGeom<D>::VPL;
  __shared__ float s_gs[2 * D];
  __shared__ float s_da[BR_WAVES][BR_ECH][BR_HMAX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int N;
  float k_g[VPL], k_mean[VPL], k_rstd[VPL], k_s1[VPL], k_s2[VPL];
  bwd_row_consts<D>(a, s_gs, N, k_g, k_mean, k_rstd, k_s1, k_s2);
  const int Nl = a.bt.hdr[0];
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
  const float* K = a.qkvs + D;
  const float* V = a.qkvs + 2 * D;
  // one row of the wave alone (hub rows, wide heads: the general bodies)
  auto one_row = [&](int i) {
      const int t = (blockIdx.x * BR_WAVES + wave) * BR_RPW + i;
      if (t >= Nl) return;  // wave-uniform
      const int e0 = a.bt.in_ptr[t], e1 = a.bt.in_ptr[t + 1];
      if (e1 - e0 > BR_ECH || H > BR_HMAX) {  // hub rows: the general wave-per-row body
        bwd_dst_row<D>(a, t, t, K, V, 4 * D, a.bt.in_ptr, a.bt.in_src, a.alpha, a.dlogit, 0, lane, dr, st_attn, k_g,
                       k_mean, k_rstd, k_s1, k_s2);
        return;
      }
      const int ne = e1 - e0;
      const int my_src = lane < ne ? a.bt.in_src[e0 + lane] : 0;
      const size_t ro = (size_t)t * D + d0;
      float dyv[VPL], ov[VPL], agv[VPL], sv[VPL];
      load_vec<VPL>(dyv, a.dy + ro, act);
      load_vec<VPL>(ov, a.out + ro, act);
      load_vec<VPL>(agv, a.agg + ro, act);
      load_vec<VPL>(sv, a.qkvs + (size_t)t * (4 * D) + 3 * D + d0, act);
      const float beta = a.gate[t];
      // BatchNorm backward, then the beta gate (as bwd_dst_row)
      float gv[VPL];
      float dbeta = 0.0f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        const float xh = (ov[v] - k_mean[v]) * k_rstd[v];
        gv[v] = act ? (dyv[v] - k_s1[v] - xh * k_s2[v]) * k_rstd[v] * k_g[v] : 0.0f;
        dbeta += gv[v] * (sv[v] - agv[v]);
      }
      dbeta = wave_sum(dbeta);
      const float du = dbeta * beta * (1.0f - beta);
      if (lane == 0) a.du[t] = du;
      float dag[VPL], ds[VPL], dq[VPL];
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        dag[v] = gv[v] * (1.0f - beta) + du * (w1[v] + w3[v]);
        ds[v] = gv[v] * beta + du * (w2[v] - w3[v]);
        dq[v] = 0.0f;
      }
      store_vec<VPL>(a.dqkvs + (size_t)t * (4 * D) + 3 * D + d0, ds, act);
      store_vec<VPL>(a.dagg + ro, dag, act);
      // da = <dA[t], V[src]> * mask per edge (LDS), sdot = sum alpha * da (four V rows in flight)
      float sdot = 0.0f;
      for (int j = 0; j < ne; j += 4) {
        float vv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(vv[u], V + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float d = 0.0f;
#pragma unroll
          for (int v = 0; v < VPL; ++v) d += dag[v] * vv[u][v];
          d = group_sum(d, GL);
          if (j + u < ne) {
            const int eg = e0 + j + u;
            const float da = d * dr.mul(st_attn, (uint32_t)(eg * H + head));
            sdot += a.alpha[(size_t)eg * H + head] * da;
            if (leader) s_da[wave][j + u][head] = da;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // dlogit = alpha * (da - sdot); dQ += dlogit / sqrt(C) * K[src] (four K rows in flight)
      for (int j = 0; j < ne; j += 4) {
        float kv[4][VPL];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = __shfl(my_src, (j + u) & 63);
          load_vec<VPL>(kv[u], K + (size_t)src * (4 * D) + d0, act && j + u < ne);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j + u < ne) {
            const int eg = e0 + j + u;
            const float al = a.alpha[(size_t)eg * H + head];
            const float dl = al * (s_da[wave][j + u][head] - sdot);
            if (leader) a.dlogit[(size_t)eg * H + head] = dl;
            const float c = dl / a.sqrt_c;
#pragma unroll
            for (int v = 0; v < VPL; ++v) dq[v] += c * kv[u][v];
          }
        }
      }
      store_vec<VPL>(a.dqkvs + (size_t)t * (4 * D) + d0, dq, act);
      __builtin_amdgcn_wave_barrier();  // s_da is reused by the wave's next row
  };
  // The wave's two rows together (as k_attn_rows): one id load for both rows' contiguous
  // in-edges, every V row requested with its K row (the first BR_VR edges' K rows stay in
  // registers for dQ).  Per row the arithmetic is the single-row body's, in the same edge
  // order: bitwise the same outputs.
  const int t0 = (blockIdx.x * BR_WAVES + wave) * BR_RPW;
  if (t0 >= Nl) return;  // wave-uniform
  const bool two = t0 + 1 < Nl;
  const int e0 = a.bt.in_ptr[t0], em = a.bt.in_ptr[t0 + 1];
  const int e2 = two ? a.bt.in_ptr[t0 + 2] : em;
  const int ne0 = em - e0, ne = e2 - e0;
  static_assert(BR_RPW == 2, "the paired body covers two rows per wave");
  if (ne > BR_ECH || H > BR_HMAX) {
    one_row(0);
    one_row(1);
    return;
  }
  const int my_src = lane < ne ? a.bt.in_src[e0 + lane] : 0;
  // BatchNorm backward, then the beta gate, of one row (as bwd_dst_row) -> dA of the row
  auto head_of = [&](int t, float (&dag)[VPL]) {
    const size_t ro = (size_t)t * D + d0;
    float dyv[VPL], ov[VPL], agv[VPL], sv[VPL];
    load_vec<VPL>(dyv, a.dy + ro, act);
    load_vec<VPL>(ov, a.out + ro, act);
    load_vec<VPL>(agv, a.agg + ro, act);
    load_vec<VPL>(sv, a.qkvs + (size_t)t * (4 * D) + 3 * D + d0, act);
    const float beta = a.gate[t];
    float gv[VPL];
    float dbeta = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const float xh = (ov[v] - k_mean[v]) * k_rstd[v];
      gv[v] = act ? (dyv[v] - k_s1[v] - xh * k_s2[v]) * k_rstd[v] * k_g[v] : 0.0f;
      dbeta += gv[v] * (sv[v] - agv[v]);
    }
    dbeta = wave_sum(dbeta);
    const float du = dbeta * beta * (1.0f - beta);
    if (lane == 0) a.du[t] = du;
    float ds[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      dag[v] = gv[v] * (1.0f - beta) + du * (w1[v] + w3[v]);
      ds[v] = gv[v] * beta + du * (w2[v] - w3[v]);
    }
    store_vec<VPL>(a.dqkvs + (size_t)t * (4 * D) + 3 * D + d0, ds, act);
    store_vec<VPL>(a.dagg + ro, dag, act);
  };
  float dag0[VPL], dag1[VPL], dq0[VPL], dq1[VPL];
  head_of(t0, dag0);
  if (two) head_of(t0 + 1, dag1);
  else {
#pragma unroll
    for (int v = 0; v < VPL; ++v) dag1[v] = 0.0f;
  }
#pragma unroll
  for (int v = 0; v < VPL; ++v) { dq0[v] = 0.0f; dq1[v] = 0.0f; }
  // da = <dA[t], V[src]> * mask per edge (LDS), sdot = sum alpha * da
  float sdot0 = 0.0f, sdot1 = 0.0f;
  auto dot_v = [&](int e, const float (&vr)[VPL]) {
    const bool r1 = e >= ne0;  // wave-uniform
    float d = 0.0f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) d += (r1 ? dag1[v] : dag0[v]) * vr[v];
    d = group_sum(d, GL);
    if (e < ne) {
      const int eg = e0 + e;
      const float da = d * dr.mul(st_attn, (uint32_t)(eg * H + head));
      // explicit fma: the single-row body's contracted `sdot += alpha * da` (the two
      // accumulators' branches must not share one rounded product)
      const float al = a.alpha[(size_t)eg * H + head];
      if (r1) sdot1 = __builtin_fmaf(al, da, sdot1);
      else sdot0 = __builtin_fmaf(al, da, sdot0);
      if (leader) s_da[wave][e][head] = da;
    }
  };
  float kh[BR_VR][VPL];
#pragma unroll
  for (int jj = 0; jj < BR_VR; jj += 4) {
    if (jj < ne) {  // wave-uniform
      float vv[4][VPL];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int src = __shfl(my_src, (jj + u) & 63);
        const bool ok = act && jj + u < ne;
        load_vec<VPL>(vv[u], V + (size_t)src * (4 * D) + d0, ok);
        load_vec<VPL>(kh[jj + u], K + (size_t)src * (4 * D) + d0, ok);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) dot_v(jj + u, vv[u]);
    }
  }
  for (int j = BR_VR; j < ne; j += 4) {
    float vv[4][VPL];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int src = __shfl(my_src, (j + u) & 63);
      load_vec<VPL>(vv[u], V + (size_t)src * (4 * D) + d0, act && j + u < ne);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) dot_v(j + u, vv[u]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // dlogit = alpha * (da - sdot); dQ += dlogit / sqrt(C) * K[src]
  auto acc_q = [&](int e, const float (&kr)[VPL]) {
    const bool r1 = e >= ne0;  // wave-uniform
    const int eg = e0 + e;
    const float al = a.alpha[(size_t)eg * H + head];
    const float dl = al * (s_da[wave][e][head] - (r1 ? sdot1 : sdot0));
    if (leader) a.dlogit[(size_t)eg * H + head] = dl;
    const float c = dl / a.sqrt_c;
    if (r1) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) dq1[v] = __builtin_fmaf(c, kr[v], dq1[v]);
    } else {
#pragma unroll
      for (int v = 0; v < VPL; ++v) dq0[v] = __builtin_fmaf(c, kr[v], dq0[v]);
    }
  };
#pragma unroll
  for (int e = 0; e < BR_VR; ++e)
    if (e < ne) acc_q(e, kh[e]);
  for (int j = BR_VR; j < ne; j += 4) {
    float kv[4][VPL];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int src = __shfl(my_src, (j + u) & 63);
      load_vec<VPL>(kv[u], K + (size_t)src * (4 * D) + d0, act && j + u < ne);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (j + u < ne) acc_q(j + u, kv[u]);
  }
  store_vec<VPL>(a.dqkvs + (size_t)t0 * (4 * D) + d0, dq0, act);
  if (two) store_vec<VPL>(a.dqkvs + (size_t)(t0 + 1) * (4 * D) + d0, dq1, act);
}

// Destination-row backward with float4 lanes (round 5; the layout of k_attn_rows4): a
// wave owns two consecutive rows, each row's SPR sub-groups of LPR = D/4 lanes walk its
// in-edges U at a time with the edge's V row, K row and alpha requested in the same round.
// Per row: BatchNorm backward and the beta-gate backward (-> dS, dA, du); per edge
// da = <dA, V> * mask and the row's sdot = sum alpha * da; dlogit = alpha (da - sdot)
// (written for the source-row launch) and dQ = sum dlogit / sqrt(C) * K.  A row of at most
// U * SPR in-edges keeps its K rows in registers (one gather round); longer rows take a
// second round of K loads.  Same arithmetic as k_attn_rows_bwd_dst up to fp32 reordering.
#ifndef BR4_U
#define BR4_U 4
#endif

template <int O>
__device__ __forceinline__ float xor_add_b(float x) {
  if constexpr (O >= 16) return bfly_add<O>(x);
  else return x + __shfl_xor(x, O);
}
template <int O, int END>
__device__ __forceinline__ float xor_sum_upto(float x) {
  if constexpr (O < END) return xor_sum_upto<O * 2, END>(xor_add_b<O>(x));
  else return x;
}

template <int D>
__global__ __launch_bounds__(BR_BLOCK) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_attn_rows_bwd_dst4(ConvBwdK a) {
  constexpr int LPR = D / 4, RPI = 64 / LPR, U = BR4_U;
  constexpr int SPR = RPI / 2, EPR = U * SPR;
  static_assert(RPI >= 2, "a sub-group per row of the pair");
  __shared__ float s_gs[2 * D];
  __shared__ float s_da[BR_WAVES][BR_ECH][BR_HMAX];
  __shared__ float s_sd[BR_WAVES][2][BR_HMAX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // BatchNorm constants of this lane's four columns (bwd_row_consts at float4 width)
  int Nstat = a.bt.hdr[0];
  const float* gs = a.gsum;
  if (a.sync) {
    float n = 0.0f;
    for (int q = 0; q < a.nparts_fwd; ++q) n += a.part_all[(size_t)q * (1 + 2 * D)];
    Nstat = (int)(n + 0.5f);
    for (int j = tid; j < 2 * D; j += BR_BLOCK) {
      float acc = 0.0f;
      for (int q = 0; q < a.nparts_bwd; ++q) acc += a.gpart_all[(size_t)q * 2 * D + j];
      s_gs[j] = acc;
    }
    __syncthreads();
    gs = s_gs;
  }
  const int Nl = a.bt.hdr[0];
  const int t0 = (blockIdx.x * BR_WAVES + wave) * BR_RPW;
  if (t0 >= Nl) return;  // wave-uniform
  const int sub = lane / LPR, c4 = lane - sub * LPR, col = 4 * c4;
  const int rr = sub / SPR, si = sub - rr * SPR;
  const int C = a.C, H = a.H;
  const int HL = C >= 4 ? C / 4 : 1;
  const int head = col / C;
  const bool leader = (c4 & (HL - 1)) == 0;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool two = t0 + 1 < Nl;
  const int e0 = a.bt.in_ptr[t0], em = a.bt.in_ptr[t0 + 1];
  const int e2 = two ? a.bt.in_ptr[t0 + 2] : em;
  const int ne0 = em - e0, ne = e2 - e0;
  const bool mine = rr == 0 || two;
  const int eb = rr == 0 ? 0 : ne0;
  const int nr = rr == 0 ? ne0 : ne - ne0;
  const int nmax = max(ne0, ne - ne0);
  const int t = t0 + rr;
  const bool lds_da = ne <= BR_ECH;
  const int my_src = lane < ne ? a.bt.in_src[e0 + lane] : 0;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const size_t ro = (size_t)(mine ? t : t0) * D + col;
  const float4 dyv = *reinterpret_cast<const float4*>(a.dy + ro);
  const float4 ov = *reinterpret_cast<const float4*>(a.out + ro);
  const float4 agv = *reinterpret_cast<const float4*>(a.agg + ro);
  const float4 sv = *reinterpret_cast<const float4*>(a.qkvs + (size_t)(mine ? t : t0) * (4 * D) + 3 * D + col);
  const float beta = a.gate[mine ? t : t0];
  // ---- BatchNorm backward, then the beta gate (as bwd_dst_row, per float4)
  float4 dag, ds;
  {
    const float invN = 1.0f / (float)Nstat;
    const float4 g4 = *reinterpret_cast<const float4*>(a.gamma + col);
    const float4 mu = *reinterpret_cast<const float4*>(a.stats + col);
    const float4 rs = *reinterpret_cast<const float4*>(a.stats + D + col);
    const float4 s1 = *reinterpret_cast<const float4*>(gs + col);
    const float4 s2 = *reinterpret_cast<const float4*>(gs + D + col);
    const float4 w1 = *reinterpret_cast<const float4*>(a.w_beta + col);
    const float4 w2 = *reinterpret_cast<const float4*>(a.w_beta + D + col);
    const float4 w3 = *reinterpret_cast<const float4*>(a.w_beta + 2 * D + col);
    float gv[4], dbeta = 0.0f;
    const float dyc[4] = {dyv.x, dyv.y, dyv.z, dyv.w}, oc[4] = {ov.x, ov.y, ov.z, ov.w};
    const float agc[4] = {agv.x, agv.y, agv.z, agv.w}, sc[4] = {sv.x, sv.y, sv.z, sv.w};
    const float gc[4] = {g4.x, g4.y, g4.z, g4.w}, muc[4] = {mu.x, mu.y, mu.z, mu.w};
    const float rsc[4] = {rs.x, rs.y, rs.z, rs.w}, s1c[4] = {s1.x, s1.y, s1.z, s1.w};
    const float s2c[4] = {s2.x, s2.y, s2.z, s2.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float xh = (oc[v] - muc[v]) * rsc[v];
      gv[v] = (dyc[v] - s1c[v] * invN - xh * (s2c[v] * invN)) * rsc[v] * gc[v];
      dbeta += gv[v] * (sc[v] - agc[v]);
    }
    dbeta = group_sum_c<LPR>(dbeta);
    const float du = dbeta * beta * (1.0f - beta);
    if (mine && si == 0 && c4 == 0) a.du[t] = du;
    const float w1c[4] = {w1.x, w1.y, w1.z, w1.w}, w2c[4] = {w2.x, w2.y, w2.z, w2.w}, w3c[4] = {w3.x, w3.y, w3.z, w3.w};
    float dgc[4], dsc[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      dgc[v] = gv[v] * (1.0f - beta) + du * (w1c[v] + w3c[v]);
      dsc[v] = gv[v] * beta + du * (w2c[v] - w3c[v]);
    }
    dag = make_float4(dgc[0], dgc[1], dgc[2], dgc[3]);
    ds = make_float4(dsc[0], dsc[1], dsc[2], dsc[3]);
    if (mine && si == 0) {
      *reinterpret_cast<float4*>(a.dqkvs + (size_t)t * (4 * D) + 3 * D + col) = ds;
      *reinterpret_cast<float4*>(a.dagg + (size_t)t * D + col) = dag;
    }
  }
  const float* K = a.qkvs + D + col;
  const float* V = a.qkvs + 2 * D + col;
  const float isc = 1.0f / a.sqrt_c;
  // ---- pass 1: da per edge (LDS, or the dlogit buffer for a hub pair) and sdot
  float4 kh[U];      // single-round rows: the K rows, kept for dQ
  float dah[U], alh[U];
  float sdot = 0.0f;
  auto ids_of = [&](int j, int& ids, int& ib) {
    ids = my_src;
    ib = eb;
    if (ne > 64) {  // hub pair: this round's ids -- row 0's edges j.. in lanes 0-31, row 1's in 32-63
      const int k = j + (lane & 31);
      const bool okid = lane < 32 ? k < ne0 : ne0 + k < ne;
      ids = okid ? a.bt.in_src[e0 + (lane < 32 ? k : ne0 + k)] : 0;
      ib = rr * 32 - j;
    }
  };
  for (int j = 0; j < nmax; j += EPR) {
    int ids, ib;
    ids_of(j, ids, ib);
    float4 vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = j + u * SPR + si;
      const bool ok = mine && k < nr;
      const int src = __shfl(ids, (ib + k) & 63);
      const size_t off = ok ? (size_t)src * (4 * D) : 0;
      vc[u] = *reinterpret_cast<const float4*>(V + off);
      kh[u] = *reinterpret_cast<const float4*>(K + off);
      alh[u] = ok ? a.alpha[(size_t)(e0 + eb + k) * H + head] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = j + u * SPR + si;
      float d = dag.x * vc[u].x + dag.y * vc[u].y + dag.z * vc[u].z + dag.w * vc[u].w;
      d = group_sum(d, HL);
      dah[u] = 0.0f;
      if (mine && k < nr) {
        const int e = eb + k, eg = e0 + e;
        const float da = d * dr.mul(st_attn, (uint32_t)(eg * H + head));
        dah[u] = da;
        sdot = __builtin_fmaf(alh[u], da, sdot);
        if (leader) {
          if (lds_da) s_da[wave][e][head] = da;
          else a.dlogit[(size_t)eg * H + head] = da;  // parked; rewritten as dlogit below
        }
      }
    }
  }
  sdot = xor_sum_upto<LPR, LPR * SPR>(sdot);  // the row's sub-groups
  // ---- pass 2: dlogit = alpha (da - sdot), dQ
  float4 dq = z4;
  if (nmax <= EPR) {  // every row of the pair in one round: K rows, alpha and da in registers
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = u * SPR + si;
      if (mine && k < nr) {
        const int eg = e0 + eb + k;
        const float dl = alh[u] * (dah[u] - sdot);
        if (leader) a.dlogit[(size_t)eg * H + head] = dl;
        const float c = dl * isc;
        dq.x = __builtin_fmaf(c, kh[u].x, dq.x);
        dq.y = __builtin_fmaf(c, kh[u].y, dq.y);
        dq.z = __builtin_fmaf(c, kh[u].z, dq.z);
        dq.w = __builtin_fmaf(c, kh[u].w, dq.w);
      }
    }
  } else {
    if (!lds_da) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // parked da in dlogit
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int j = 0; j < nmax; j += EPR) {
      int ids, ib;
      ids_of(j, ids, ib);
      float4 kc[U];
      float al[U], dv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = j + u * SPR + si;
        const bool ok = mine && k < nr;
        const int src = __shfl(ids, (ib + k) & 63);
        kc[u] = *reinterpret_cast<const float4*>(K + (ok ? (size_t)src * (4 * D) : 0));
        const size_t at = (size_t)(e0 + eb + k) * H + head;
        al[u] = ok ? a.alpha[at] : 0.0f;
        dv[u] = ok ? (lds_da ? s_da[wave][eb + k][head] : a.dlogit[at]) : 0.0f;
      }
      // every lane of a head group has its parked da before its leader overwrites it
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = j + u * SPR + si;
        if (mine && k < nr) {
          const float dl = al[u] * (dv[u] - sdot);
          if (leader) a.dlogit[(size_t)(e0 + eb + k) * H + head] = dl;
          const float c = dl * isc;
          dq.x = __builtin_fmaf(c, kc[u].x, dq.x);
          dq.y = __builtin_fmaf(c, kc[u].y, dq.y);
          dq.z = __builtin_fmaf(c, kc[u].z, dq.z);
          dq.w = __builtin_fmaf(c, kc[u].w, dq.w);
        }
      }
    }
  }
  dq.x = xor_sum_upto<LPR, LPR * SPR>(dq.x);
  dq.y = xor_sum_upto<LPR, LPR * SPR>(dq.y);
  dq.z = xor_sum_upto<LPR, LPR * SPR>(dq.z);
  dq.w = xor_sum_upto<LPR, LPR * SPR>(dq.w);
  if (mine && si == 0) *reinterpret_cast<float4*>(a.dqkvs + (size_t)t * (4 * D) + col) = dq;
  (void)s_sd;
}

template <int D>
__global__ __launch_bounds__(BR_BLOCK) void k_attn_rows_bwd_src(ConvBwdK a) {
  constexpr int VPL = LayerGeom<D>::VPL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // source rows: the batch rows, plus the ghost rows of a halo batch (hdr[6], gtr.h)
  const int Nl = max(a.bt.hdr[0], a.bt.hdr[6]);
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const int d0 = lane * VPL;
  const bool act = d0 < D;
  const int C = a.C, H = a.H;
  const int head = act ? d0 / C : 0;
  const float isc = 1.0f / a.sqrt_c;
  auto one_row = [&](int i) {
    const int s = (blockIdx.x * BR_WAVES + wave) * BR_RPW + i;
    if (s >= Nl) return;
    const int i0 = a.bt.out_ptr[s], i1 = a.bt.out_ptr[s + 1];
    float dk[VPL], dv[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) { dk[v] = 0.0f; dv[v] = 0.0f; }
    for (int cb = i0; cb < i1; cb += 64) {
      const int cnt = min(64, i1 - cb);
      const int my_p = lane < cnt ? a.bt.out_edge[cb + lane] : 0;
      const int my_t = lane < cnt ? a.bt.out_dst[cb + lane] : 0;
      for (int j = 0; j < cnt; j += 4) {
        float qv[4][VPL], gv[4][VPL];
        int p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          p[u] = __shfl(my_p, (j + u) & 63);
          const int t = __shfl(my_t, (j + u) & 63);
          load_vec<VPL>(qv[u], a.qkvs + (size_t)t * (4 * D) + d0, act && j + u < cnt);
          load_vec<VPL>(gv[u], a.dagg + (size_t)t * D + d0, act && j + u < cnt);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j + u < cnt) {
            const float dl = a.dlogit[(size_t)p[u] * H + head] * isc;
            const float ad = a.alpha[(size_t)p[u] * H + head] * dr.mul(st_attn, (uint32_t)(p[u] * H + head));
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
              dk[v] = __builtin_fmaf(dl, qv[u][v], dk[v]);
              dv[v] = __builtin_fmaf(ad, gv[u][v], dv[v]);
            }
          }
        }
      }
    }
    store_vec<VPL>(a.dqkvs + (size_t)s * (4 * D) + D + d0, dk, act);
    store_vec<VPL>(a.dqkvs + (size_t)s * (4 * D) + 2 * D + d0, dv, act);
  };
  // The wave's two source rows together: their out-edges are contiguous (CSR by source),
  // so one id load covers both and every edge's Q / dA rows are requested in one round;
  // per row the same edge order and arithmetic as one_row (bitwise the same dK / dV).
  const int s0 = (blockIdx.x * BR_WAVES + wave) * BR_RPW;
  if (s0 >= Nl) return;  // wave-uniform
  const bool two = s0 + 1 < Nl;
  const int i0 = a.bt.out_ptr[s0], im = a.bt.out_ptr[s0 + 1];
  const int i2 = two ? a.bt.out_ptr[s0 + 2] : im;
  const int n0 = im - i0, n = i2 - i0;
  if (n > 64) {
    one_row(0);
    one_row(1);
    return;
  }
  const int my_p = lane < n ? a.bt.out_edge[i0 + lane] : 0;
  const int my_t = lane < n ? a.bt.out_dst[i0 + lane] : 0;
  float dk0[VPL], dv0[VPL], dk1[VPL], dv1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) { dk0[v] = 0.0f; dv0[v] = 0.0f; dk1[v] = 0.0f; dv1[v] = 0.0f; }
  for (int j = 0; j < n; j += 4) {
    float qv[4][VPL], gv[4][VPL];
    int p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      p[u] = __shfl(my_p, (j + u) & 63);
      const int t = __shfl(my_t, (j + u) & 63);
      load_vec<VPL>(qv[u], a.qkvs + (size_t)t * (4 * D) + d0, act && j + u < n);
      load_vec<VPL>(gv[u], a.dagg + (size_t)t * D + d0, act && j + u < n);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u < n) {  // wave-uniform
        const float dl = a.dlogit[(size_t)p[u] * H + head] * isc;
        const float ad = a.alpha[(size_t)p[u] * H + head] * dr.mul(st_attn, (uint32_t)(p[u] * H + head));
        if (j + u >= n0) {
#pragma unroll
          for (int v = 0; v < VPL; ++v) {
            dk1[v] = __builtin_fmaf(dl, qv[u][v], dk1[v]);
            dv1[v] = __builtin_fmaf(ad, gv[u][v], dv1[v]);
          }
        } else {
#pragma unroll
          for (int v = 0; v < VPL; ++v) {
            dk0[v] = __builtin_fmaf(dl, qv[u][v], dk0[v]);
            dv0[v] = __builtin_fmaf(ad, gv[u][v], dv0[v]);
          }
        }
      }
    }
  }
  store_vec<VPL>(a.dqkvs + (size_t)s0 * (4 * D) + D + d0, dk0, act);
  store_vec<VPL>(a.dqkvs + (size_t)s0 * (4 * D) + 2 * D + d0, dv0, act);
  if (two) {
    store_vec<VPL>(a.dqkvs + (size_t)(s0 + 1) * (4 * D) + D + d0, dk1, act);
    store_vec<VPL>(a.dqkvs + (size_t)(s0 + 1) * (4 * D) + 2 * D + d0, dv1, act);
  }
}

// Source-row backward with float4 lanes (round 5; the layout of k_attn_rows_bwd_dst4): a
// wave owns two consecutive SOURCE rows (their out-edges are contiguous in the CSR by
// source), each row's SPR sub-groups walk its out-edges U at a time, gathering the
// destination's Q row and dA row per edge: dK = sum dlogit / sqrt(C) * Q[dst],
// dV = sum alpha * mask * dA[dst].  The sub-groups' partial sums are combined by xor
// butterflies (same sums as k_attn_rows_bwd_src up to fp32 reordering).
template <int D>
__global__ __launch_bounds__(BR_BLOCK) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_attn_rows_bwd_src4(ConvBwdK a) {
  constexpr int LPR = D / 4, RPI = 64 / LPR, U = BR4_U;
  constexpr int SPR = RPI / 2, EPR = U * SPR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // source rows: the batch rows, plus the ghost rows of a halo batch (hdr[6], gtr.h)
  const int Nl = max(a.bt.hdr[0], a.bt.hdr[6]);
  const int s0 = (blockIdx.x * BR_WAVES + wave) * BR_RPW;
  if (s0 >= Nl) return;  // wave-uniform
  const int sub = lane / LPR, c4 = lane - sub * LPR, col = 4 * c4;
  const int rr = sub / SPR, si = sub - rr * SPR;
  const int C = a.C, H = a.H;
  const int head = col / C;
  const bool two = s0 + 1 < Nl;
  const int i0 = a.bt.out_ptr[s0], im = a.bt.out_ptr[s0 + 1];
  const int i2 = two ? a.bt.out_ptr[s0 + 2] : im;
  const int n0 = im - i0, n = i2 - i0;
  const bool mine = rr == 0 || two;
  const int eb = rr == 0 ? 0 : n0;
  const int nr = rr == 0 ? n0 : n - n0;
  const int nmax = max(n0, n - n0);
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_attn = drop_stream(0, (uint32_t)a.layer, ctr);
  const float isc = 1.0f / a.sqrt_c;
  const int my_p = lane < n ? a.bt.out_edge[i0 + lane] : 0;
  const int my_t = lane < n ? a.bt.out_dst[i0 + lane] : 0;
  float4 dk = make_float4(0.f, 0.f, 0.f, 0.f), dv = dk;
  for (int j = 0; j < nmax; j += EPR) {
    int ps = my_p, ts = my_t, ib = eb;
    if (n > 64) {  // hub pair: this round's out-edges -- row 0's in lanes 0-31, row 1's in 32-63
      const int k = j + (lane & 31);
      const bool ok = lane < 32 ? k < n0 : n0 + k < n;
      const int at = i0 + (lane < 32 ? k : n0 + k);
      ps = ok ? a.bt.out_edge[at] : 0;
      ts = ok ? a.bt.out_dst[at] : 0;
      ib = rr * 32 - j;
    }
    float4 qv[U], gv[U];
    float dl[U], ad[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = j + u * SPR + si;
      const bool ok = mine && k < nr;
      // every lane joins both shuffles (a lane a shuffle skips reads as 0 to the others)
      const int p = __shfl(ps, (ib + k) & 63);
      const int tt = __shfl(ts, (ib + k) & 63);
      const int t = ok ? tt : 0;
      qv[u] = *reinterpret_cast<const float4*>(a.qkvs + (size_t)t * (4 * D) + col);
      gv[u] = *reinterpret_cast<const float4*>(a.dagg + (size_t)t * D + col);
      const size_t at = (size_t)p * H + head;
      dl[u] = ok ? a.dlogit[at] * isc : 0.0f;
      ad[u] = ok ? a.alpha[at] * dr.mul(st_attn, (uint32_t)(p * H + head)) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dk.x = __builtin_fmaf(dl[u], qv[u].x, dk.x);
      dk.y = __builtin_fmaf(dl[u], qv[u].y, dk.y);
      dk.z = __builtin_fmaf(dl[u], qv[u].z, dk.z);
      dk.w = __builtin_fmaf(dl[u], qv[u].w, dk.w);
      dv.x = __builtin_fmaf(ad[u], gv[u].x, dv.x);
      dv.y = __builtin_fmaf(ad[u], gv[u].y, dv.y);
      dv.z = __builtin_fmaf(ad[u], gv[u].z, dv.z);
      dv.w = __builtin_fmaf(ad[u], gv[u].w, dv.w);
    }
  }
  dk.x = xor_sum_upto<LPR, LPR * SPR>(dk.x);
  dk.y = xor_sum_upto<LPR, LPR * SPR>(dk.y);
  dk.z = xor_sum_upto<LPR, LPR * SPR>(dk.z);
  dk.w = xor_sum_upto<LPR, LPR * SPR>(dk.w);
  dv.x = xor_sum_upto<LPR, LPR * SPR>(dv.x);
  dv.y = xor_sum_upto<LPR, LPR * SPR>(dv.y);
  dv.z = xor_sum_upto<LPR, LPR * SPR>(dv.z);
  dv.w = xor_sum_upto<LPR, LPR * SPR>(dv.w);
  if (mine && si == 0) {
    float* row = a.dqkvs + (size_t)(s0 + rr) * (4 * D);
    *reinterpret_cast<float4*>(row + D + col) = dk;
    *reinterpret_cast<float4*>(row + 2 * D + col) = dv;
  }
}

// ------------------------------------------------------------------------------------
// weight gradients
// ------------------------------------------------------------------------------------


__global__ __launch_bounds__(GTR_BLOCK) void k_wgrad(WgradK a) {
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
  auto emit = [&](int which, int64_t idx, float v) {
    if (which == 0) J.outW[so + idx] = v;
    else J.outB[so + idx] = v;
  };
  auto emit4 = [&](int64_t idx, float4 v) { *reinterpret_cast<float4*>(J.outW + so + idx) = v; };
  if (J.mfma == 1) wgrad_tile_mfma<false>(J, tile, t0, t1, emit, emit4);
  else if (J.mfma == 2) wgrad_tile_mfma<true>(J, tile, t0, t1, emit, emit4);
  else wgrad_tile(J, tile, t0, t1, a.D, emit);
}

}  // namespace

GTR_PH_READER(gtr_dbg_bwd_phases)

extern "C" int gtr_conv_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            float* dx0, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_conv_bwd: bad arguments");
    return GTR_E_ARG;
  }
  if (layers[l].ffn || (l > 0 && layers[l - 1].ffn)) {
    set_error("gtr_conv_bwd: a feed-forward block runs on the split layer path (gtr_qkvs_* / gtr_attn_* / gtr_ffn_*)");
    return GTR_E_ARG;
  }
  const int D = cfg->dim;
  ConvBwdK k;
  if (const int rc = make_bwd_args(cfg, bt, layers, l, dx0, k)) return rc;
  int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
  {
    const int slot = 2 * cfg->num_layers - l;  // after the forward slots and the readout's
    if (cfg->sweep && slot < GTR_SWEEP_SLOTS && cfg->sweep->bounds[slot + 1] > cfg->sweep->bounds[slot]) {
      k.sw = *cfg->sweep;
      k.sw_slot = slot;
      grid += sweep_blocks(cfg->sweep, grid);
    }
  }
  k.xpack = xcd_pack(k.main_grid, grid);
  hipStream_t s = (hipStream_t)stream;
#define GTR_BWD(DD, SP) set_lds_limit<DD>(k_conv_bwd<DD, SP>, (size_t)LayerGeom<DD>::B_WORDS * 4); \
  hipLaunchKernelGGL((k_conv_bwd<DD, SP>), dim3(grid), dim3(CONV_BLOCK), \
                                       (size_t)LayerGeom<DD>::B_WORDS * 4, s, k)
  const bool sp = gemm_split(D) != 0;
  switch (D) {
    case 32: if (sp) { GTR_BWD(32, true); } else { GTR_BWD(32, false); } break;
    case 64: if (sp) { GTR_BWD(64, true); } else { GTR_BWD(64, false); } break;
    case 128: if (sp) { GTR_BWD(128, true); } else { GTR_BWD(128, false); } break;
    default: GTR_BWD(256, false); break;  // no LDS-staged rows at D = 256: f32 MFMA from L2
  }
#undef GTR_BWD
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_attn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_attn_bwd: bad arguments");
    return GTR_E_ARG;
  }
  if (cfg->sync_bn ? !cfg->split_sync : cfg->consumer_reduce) {
    set_error("gtr_attn_bwd: the split path reads producer-finalized BatchNorm sums (consumer_reduce 0) or, "
              "under sync_bn, the gathered per-rank sums (split_sync)");
    return GTR_E_ARG;
  }
  ConvBwdK k;
  float dummy = 0.0f;  // dx0 is written by gtr_qkvs_bwd, not here
  if (const int rc = make_bwd_args(cfg, bt, layers, l, &dummy, k)) return rc;
  k.dx0 = nullptr;
  hipStream_t s = (hipStream_t)stream;
  const char* am = getenv("GTR_ATTN");  // "group": the fused kernels' row-group body (A/B)
  if (cfg->dim <= 128 && !(am && am[0] == 'g')) {
    const int grid = (bt->n_cap + BR_WAVES * BR_RPW - 1) / (BR_WAVES * BR_RPW);
    // float4 lanes (k_attn_rows_bwd_dst4) unless GTR_ATTN=rows or more than BR_HMAX heads
    const bool v4 = cfg->heads <= BR_HMAX && !(am && am[0] == 'r');
    if (v4) {
      switch (cfg->dim) {
        case 32: hipLaunchKernelGGL(k_attn_rows_bwd_dst4<32>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
        case 64: hipLaunchKernelGGL(k_attn_rows_bwd_dst4<64>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
        default: hipLaunchKernelGGL(k_attn_rows_bwd_dst4<128>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
      }
      switch (cfg->dim) {
        case 32: hipLaunchKernelGGL(k_attn_rows_bwd_src4<32>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
        case 64: hipLaunchKernelGGL(k_attn_rows_bwd_src4<64>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
        default: hipLaunchKernelGGL(k_attn_rows_bwd_src4<128>, dim3(grid), dim3(BR_BLOCK), 0, s, k); break;
      }
      GTR_HIP_CHECK_LAUNCH();
      return GTR_OK;
    }
    switch (cfg->dim) {
      case 32:
        hipLaunchKernelGGL(k_attn_rows_bwd_dst<32>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        hipLaunchKernelGGL(k_attn_rows_bwd_src<32>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        break;
      case 64:
        hipLaunchKernelGGL(k_attn_rows_bwd_dst<64>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        hipLaunchKernelGGL(k_attn_rows_bwd_src<64>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        break;
      default:
        hipLaunchKernelGGL(k_attn_rows_bwd_dst<128>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        hipLaunchKernelGGL(k_attn_rows_bwd_src<128>, dim3(grid), dim3(BR_BLOCK), 0, s, k);
        break;
    }
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  const int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
#define GTR_ABW(DD) set_lds_limit<DD>(k_attn_bwd<DD>, (size_t)LayerGeom<DD>::B_WORDS * 4); \
  hipLaunchKernelGGL((k_attn_bwd<DD>), dim3(grid), dim3(CONV_BLOCK), (size_t)LayerGeom<DD>::B_WORDS * 4, s, k)
  switch (cfg->dim) {
    case 32: GTR_ABW(32); break;
    case 64: GTR_ABW(64); break;
    case 128: GTR_ABW(128); break;
    default: GTR_ABW(256); break;
  }
#undef GTR_ABW
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers,
                         const float* dx0, const float* pe_tab, float* const* layer_slab, float* pe_slab,
                         int n_chunks, int64_t slab_stride, int l_begin, int l_end, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !layer_slab || n_chunks <= 0) {
    set_error("gtr_wgrad: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim, Lc = cfg->num_layers;
  if (3 * Lc + 1 > GTR_MAX_WJOBS) { set_error("gtr_wgrad: too many layers"); return GTR_E_ARG; }
  WgradK k{};
  k.hdr = bt->hdr;
  k.P = n_chunks;
  k.D = D;
  k.stride = slab_stride;
  if (l_begin < 0 || l_end > Lc || l_begin > l_end) { set_error("gtr_wgrad: bad layer range"); return GTR_E_ARG; }
  int nj = 0, blocks = 0;
  // MFMA tiles for the QKVS weight once a chunk holds enough rows to amortize them
  // (GTR_WGRAD=mfma|valu overrides; the float4 slab stores need 16 B aligned slabs)
  const char* wm = getenv("GTR_WGRAD");
  const int rows_per_chunk = (bt->n_cap + n_chunks - 1) / n_chunks;
  bool mfma = rows_per_chunk >= GTR_WGRAD_MFMA_ROWS;
  if (wm && !strcmp(wm, "mfma")) mfma = true;
  if (wm && !strcmp(wm, "valu")) mfma = false;
  if (slab_stride % 4) mfma = false;
  for (int l = l_begin; l < l_end; ++l)
    if (reinterpret_cast<uintptr_t>(layer_slab[l]) % 16) mfma = false;
  const int rc = build_wjobs(cfg, bt, layers, dx0, pe_tab, layer_slab, pe_slab, nullptr, nullptr, n_chunks, l_begin,
                             l_end, k.jobs, nj, blocks, mfma);
  if (rc) return rc;
  if (const char* jm = getenv("GTR_WGRAD_JOBS")) {  // diagnostics (timing only): keep job types in the mask
    const int mask = atoi(jm);
    int kept = 0;
    blocks = 0;
    for (int i = 0; i < nj; ++i) {
      const bool pe = k.jobs[i].type == WJ_MM && k.jobs[i].M1 == D;
      const int bit = pe ? 8 : 1 << k.jobs[i].type;
      if (!(mask & bit)) continue;
      WJob j = k.jobs[i];
      j.blk0 = blocks;
      blocks += j.nt * n_chunks;
      k.jobs[kept++] = j;
    }
    nj = kept;
  }
  k.njobs = nj;
  if (nj == 0 || blocks == 0) return GTR_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_wgrad, dim3(blocks), dim3(GTR_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}
