// gtr_gemm.hip — the dense GEMMs of the TransformerConv layer as persistent f32-MFMA
// kernels, for the large-batch ("split") layer path (gtr_qkvs_fwd / gtr_qkvs_bwd).
//
// At large batches the fused layer kernels (k_conv_fwd / k_conv_bwd) spend most of their
// time in the per-row-group projection: every 16-row group re-fetches the layer's whole
// W_all (256 KB at D = 128) for 16 rows of reuse and pads its 16-20 rows to two 16-row
// MFMA tiles.  Here the GEMMs run over ALL node rows instead:
//
//   k_proj<D>  X = [layer 0: item row + LapPE projection | layer >= 1: dropout(BN(prev out)
//              + prev in)] (graph_transformer.py:140-152,175-177) -> xin, and
//              qkvs = X . W_all^T + b_all (the four PyG TransformerConv Linears,
//              SURVEY.md Appendix A);
//   k_dx<D>    dX = dQKVS . W_all + dy (the residual), the previous layer's dropout mask,
//              -> that layer's dy (or dx0 at layer 0), and its BatchNorm backward sums.
//
// The feed-forward block of the use_ffn=True variant (graph_transformer.py:88-100,160-170)
// runs on the same two kernels, by mode:
//   k_proj<PJ_FOLD>     y = dropout(BN(out) + x) -> ffn.y, a = y W1^T + b1 -> ffn.a (W1 is
//                       [4D, D] like W_all: the conv projection with other pointers);
//   k_dx<DX_FFN_DOWN>   z = y + dropout(dropout(GELU(a)) W2^T + b2) -> ffn.z (K = 4D);
//   k_proj<PJ_FFN_DH>   g2 = dz * mask -> ffn.g2, da = (g2 W2) * mask * GELU'(a) -> ffn.da;
//   k_dx<DX_CONV>       dy = (dz + da W1) * the layer's output mask -> layers[l].dy + sums;
//   k_proj<PJ_READY>    the next layer's X = ffn.z as it is (no BatchNorm fold);
// and k_ffn_wgrad reduces dW1 / db1 / dW2 / db2 over row chunks on f32 MFMA.
//
// One workgroup per CU, 8 waves, persistent over 16- (D = 128) or 32-row (D = 64) tiles.
// Each wave keeps ITS column tiles of W_all in registers for the whole launch (128 VGPRs
// at D = 128: loaded once per CU instead of once per row group), the row tile is staged
// in LDS (double-buffered; the next tile's rows are fetched while the MFMAs run), and the
// MFMAs run exactly the k order of the fused kernels' mfma4 chains (k = kb*16 + lg*4 + j),
// so qkvs / dX are BITWISE those of k_conv_fwd / k_conv_bwd (tests/test_gpu_split.py).
// The attention phases then run in gtr_attn_fwd / gtr_attn_bwd (the fused kernels' row
// group bodies with the projection / dX phase left out).

#include "gtr_layer.cuh"

#include <type_traits>

namespace gtr {  // gtr_gemm_gen.hip: the LDS-staged GEMMs for D = 256 and FFN expansions != 4
int gen_qkvs_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb, const gtr_layer* layers, int l,
                 hipStream_t s);
int gen_qkvs_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, float* dx0,
                 hipStream_t s);
int gen_ffn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, hipStream_t s);
int gen_ffn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, hipStream_t s);
int gen_ffn_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, float* slab,
                  int n_chunks, int64_t slab_stride, hipStream_t s);
}  // namespace gtr

namespace {

using namespace gtr;

GTR_PH_DECL

#define GM_BLOCK 512
#define GM_WAVES (GM_BLOCK / 64)

#define GM_MFMA4(a, b, c) mfma4(a, b, c)

// k_proj computes QKVS^T tiles (W fragment as the MFMA's A operand, the X rows as B): a
// lane's four accumulators are then four CONSECUTIVE output columns of one row, stored as
// one float4, instead of one column of four rows (four scalar stores).  The products and
// the k order per instruction are the same.  GTR_PROJ_T=0 at build time: the X . W^T form.
#ifndef GTR_PROJ_T
#define GTR_PROJ_T 1
#endif
// k_dx likewise (dX^T = W^T-fragment x dQKVS rows): float4 residual loads, stores and
// BatchNorm-sum columns per lane.  GTR_DX_T=0 at build time: the dQKVS . W form.
#ifndef GTR_DX_T
#define GTR_DX_T 1
#endif

// k_proj modes: layer 0 (item row + LapPE), layer >= 1 (BatchNorm fold of the previous
// layer), rows taken as they are (after a feed-forward block), FFN hidden-gradient GEMM
enum { PJ_FIRST = 0, PJ_FOLD = 1, PJ_READY = 2, PJ_FFN_DH = 3 };
// k_dx modes: the conv dX GEMM (+ previous layer's mask and BatchNorm sums), FFN down-projection
enum { DX_CONV = 0, DX_FFN_DOWN = 1 };

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  return cdf + x * (0.39894228040143268f * expf(-0.5f * x * x));
}

template <int D>
struct ProjGeom {
  static constexpr int NCT = 4 * D / 16;          // output column tiles of qkvs
  static constexpr int CT = NCT / GM_WAVES;       // per wave (D = 64: 2, D = 128: 4)
  static constexpr int RT = D <= 64 ? 2 : 1;      // 16-row MFMA tiles per block tile
  static constexpr int BM = 16 * RT;
  static constexpr int XS = D + 4;                // padded LDS row
  static constexpr int C4 = D / 4;
  static constexpr int KPE = 16;                  // LapPE width staged in LDS
  static_assert(BM * C4 == GM_BLOCK, "one float4 of X per thread and tile");
};

struct ProjK {
  gtr_batch bt;
  int first, train, pe_k, layer;
  float bn_eps, scale;
  uint32_t seed, thresh;
  int drop_on;
  uint32_t ctr_add;
  const uint32_t* rng_ctr;
  const float* table;
  const float* pe_tab;
  const float* wpe;
  const float* bpe;
  const float* p_out;
  const float* p_xin;
  float* p_stats;
  float* p_rmean;
  float* p_rvar;
  int64_t* p_nbt;
  const float* p_gamma;
  const float* p_beta;
  const float* w_all;
  const float* b_all;
  float* xin;
  float* qkvs;
  int sync, p_nparts;        // split_sync: fold the ranks' merged rows of the previous layer
  const float* p_part_all;   // [p_nparts][1 + 2D] (count, mean, M2)
  float bn_mom;
  const float* fa;           // PJ_FFN_DH: the saved pre-activation a [n, 4D]
};

// Inputs of one thread's float4 of X for one tile: layer 0 the item row (+ its LapPE row),
// layers >= 1 the previous layer's out and in rows.
template <int NPE>
struct ProjIn {
  float4 u, v;
  float4 pe[NPE > 0 ? NPE : 1];  // D = 64 (4 waves per SIMD, 128 VGPRs): no PE prefetch
  int item;  // layer 0: the tile row's item id (the LapPE fallback path reads by it)
};

// CS > 1 (round 5, small batches): the output columns are split over CS workgroups per
// row-tile stream (workgroup b: column slice b % CS of stream b / CS), each holding 1/CS of
// W_all in registers: at a few thousand rows (one or two tiles per CU) the launch is its
// W prologue plus one tile's MFMA chain, both CS times shorter per workgroup; the X tile
// is built by every slice (its xin store by slice 0 only).  Same products, same k order.
template <int D, int MODE, int CS = 1>
__global__ __launch_bounds__(GM_BLOCK) __attribute__((amdgpu_waves_per_eu(D == 64 || CS > 1 ? 4 : 2))) void k_proj(ProjK a) {
  constexpr bool FIRST = MODE == PJ_FIRST, FOLD = MODE == PJ_FOLD, DH = MODE == PJ_FFN_DH;
  using G = ProjGeom<D>;
  static_assert(G::CT % CS == 0, "column slices of whole tiles per wave");
  constexpr int CT = G::CT / CS, RT = G::RT, BM = G::BM, XS = G::XS, C4 = G::C4, KPE = G::KPE;
  constexpr int NPE = FIRST && D >= 128 ? 4 : 0;  // LapPE float4s prefetched per thread
  using ProjIn = ::ProjIn<NPE>;
  __shared__ __attribute__((aligned(16))) float Xs[2][BM * XS];
  __shared__ __attribute__((aligned(16))) float s_pw[KPE * D];  // W_pe^T [KPE][D] (layer 0)
  __shared__ __attribute__((aligned(16))) float s_c[4 * D];     // bpe | mean | rstd | gamma | beta
  __shared__ __attribute__((aligned(16))) float s_bias[4 * D];  // b_all (GTR_PROJ_T epilogue)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int N = a.bt.hdr[0];
  const int ntile = (N + BM - 1) / BM;
  const int cg = (int)blockIdx.x % CS;  // this workgroup's column slice
  if ((int)blockIdx.x / CS >= ntile) return;  // block-uniform
  GTR_PH(10 + a.layer, 0);
  // Round 5: the waves' column tiles rotate with the workgroup's position on its XCD
  // (blocks b and b + 8 share an XCD), so that the 32 CUs of an XCD, loading W_all at
  // the same moment, do not all request the same W rows (the same L2 channels) at once;
  // only which wave computes which columns changes, not the arithmetic.
  const int wsw = (wave + ((int)blockIdx.x >> 3)) & (GM_WAVES - 1);
  // ---- W fragments of this wave's column tiles (ct = wave + c * GM_WAVES, the fused
  //      kernel's assignment) and biases, held in registers for every tile of the block
  float4 wf[CT][D / 16];
  float bias[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int ct = wsw + (cg * CT + c) * GM_WAVES;
    if (DH) {  // B[k][col] = W2[k][col], W2 = [D, 4D] row-major
      const float* wcol = a.w_all + (size_t)(lg * 4) * (4 * D) + ct * 16 + lr;
#pragma unroll
      for (int kb = 0; kb < D / 16; ++kb) {
        const float* wp = wcol + (size_t)(kb * 16) * (4 * D);
        wf[c][kb] = make_float4(wp[0], wp[4 * D], wp[8 * D], wp[12 * D]);
      }
      bias[c] = 0.0f;
    } else {
      const float* wrow = a.w_all + (size_t)(ct * 16 + lr) * D;
#pragma unroll
      for (int kb = 0; kb < D / 16; ++kb) wf[c][kb] = *reinterpret_cast<const float4*>(wrow + kb * 16 + lg * 4);
      bias[c] = a.b_all[ct * 16 + lr];
    }
  }
  if (GTR_PROJ_T)
    for (int j = tid; j < 4 * D; j += GM_BLOCK) s_bias[j] = DH ? 0.0f : a.b_all[j];
  const bool pe_lds = FIRST && a.pe_k > 0 && a.pe_k <= KPE;
  if (FIRST) {
    // transposed (k-major): a thread's four output columns of one k are one float4, and a
    // wave's reads of one k are consecutive (no LDS bank conflicts)
    if (pe_lds)
      for (int idx = tid; idx < D * KPE; idx += GM_BLOCK) {
        const int k = idx / D, j = idx - k * D;
        s_pw[idx] = k < a.pe_k ? a.wpe[j * a.pe_k + k] : 0.0f;
      }
    if (a.pe_k > 0)
      for (int j = tid; j < D; j += GM_BLOCK) s_c[j] = a.bpe[j];
  } else if (!FOLD) {
    // PJ_READY / PJ_FFN_DH: no BatchNorm of a previous layer
  } else if (a.sync && a.train) {
    // SyncBN (split_sync): every rank's merged (count, mean, M2) row of the previous layer,
    // folded in rank order; workgroup 0 publishes the statistics (read by the backward) and
    // updates the running statistics -- prev_bn_stats of k_conv_fwd with P rows
    float* s_uvar = Xs[1];
    bn_stats_from_parts<D, GM_BLOCK>(a.p_part_all, a.p_nparts, a.bn_eps, s_c + D, s_c + 2 * D, s_uvar, Xs[0]);
    for (int j = tid; j < D; j += GM_BLOCK) {
      s_c[3 * D + j] = a.p_gamma[j];
      if (blockIdx.x == 0) {
        a.p_stats[j] = s_c[D + j];
        a.p_stats[D + j] = s_c[2 * D + j];
        a.p_rmean[j] = (1.0f - a.bn_mom) * a.p_rmean[j] + a.bn_mom * s_c[D + j];
        a.p_rvar[j] = (1.0f - a.bn_mom) * a.p_rvar[j] + a.bn_mom * s_uvar[j];
      }
    }
    if (blockIdx.x == 0 && tid == 0 && a.p_nbt) *a.p_nbt += 1;
  } else {
    for (int j = tid; j < D; j += GM_BLOCK) {
      // the previous layer's BatchNorm: batch statistics (finalized by its producer) or,
      // in eval mode, the running statistics -- as prev_bn_stats of k_conv_fwd
      s_c[D + j] = a.train ? a.p_stats[j] : a.p_rmean[j];
      s_c[2 * D + j] = a.train ? a.p_stats[D + j] : 1.0f / sqrtf(a.p_rvar[j] + a.bn_eps);
      s_c[3 * D + j] = a.p_gamma[j];
    }
  }
  __syncthreads();
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  // FOLD: the previous layer's output mask; FFN_DH: this layer's FFN output mask (kind 3)
  const uint32_t st_prev = DH ? drop_stream(3, (uint32_t)a.layer, ctr) : drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  const uint32_t st_h = drop_stream(2, (uint32_t)a.layer, ctr);  // FFN_DH: the hidden mask
  const int xi = tid / C4, xj = (tid - (tid / C4) * C4) * 4;  // this thread's row / column of X
  float4 pg = make_float4(0.f, 0.f, 0.f, 0.f), pb = pg, mu = pg, rs = pg;
  if (FOLD) {
    mu = *reinterpret_cast<const float4*>(s_c + D + xj);
    rs = *reinterpret_cast<const float4*>(s_c + 2 * D + xj);
    pg = *reinterpret_cast<const float4*>(s_c + 3 * D + xj);
    pb = *reinterpret_cast<const float4*>(a.p_beta + xj);
  }

  // Round 5: every load of the tile pipeline issues unconditionally (rows past N and
  // tiles past the last read row N - 1, whose values produce() then discards) and the
  // stores go through bounds-checked buffers, so no memory op sits under an exec-skipping
  // branch and the compiler counts them: the wait for a set's rows no longer drains the
  // other set's rows and the previous tile's stores (vmcnt(0)).
  const Buf xin_buf(a.xin, cg == 0 ? (uint64_t)N * D * 4 : 0), qkvs_buf(a.qkvs, (uint64_t)N * 4 * D * 4);
  auto item_of = [&](int t) -> int {
    return FIRST ? a.bt.node_item[min(t * BM + xi, N - 1)] : 0;
  };
  auto fetch = [&](int t, int item, ProjIn& in) {
    const int r = min(t * BM + xi, N - 1);
    in.item = item;
    in.v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (FIRST) {
      in.u = *reinterpret_cast<const float4*>(a.table + (size_t)item * D + xj);
      if (NPE > 0 && pe_lds && (a.pe_k & 3) == 0) {
        const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)r * a.pe_k : a.pe_tab + (size_t)item * a.pe_k;
        // float4 q past pe_k re-reads float4 0 (unused: produce() stops at pe_k)
#pragma unroll
        for (int q = 0; q < NPE; ++q) in.pe[q] = *reinterpret_cast<const float4*>(pr + (4 * q < a.pe_k ? 4 * q : 0));
      }
    } else {
      const size_t o = (size_t)r * D + xj;
      in.u = *reinterpret_cast<const float4*>(a.p_out + o);
      if (FOLD) in.v = *reinterpret_cast<const float4*>(a.p_xin + o);
    }
  };
  // X of one tile -> LDS (rows past N: zero) and xin; the arithmetic of k_conv_fwd's
  // input build, expression for expression (bitwise the same rows)
  auto produce = [&](int t, int item, const ProjIn& in, float* X) {
    const int r = t * BM + xi;
    float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
    {
      const size_t o = (size_t)r * D + xj;
      if (FIRST) {
        val = in.u;
        if (a.pe_k > 0) {
          float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (NPE > 0 && pe_lds && (a.pe_k & 3) == 0) {
#pragma unroll
            for (int kq = 0; kq < (NPE > 0 ? NPE : 1); ++kq) {  // k = 0, 4, .. < pe_k: the fused loop's order
              if (4 * kq >= a.pe_k) break;
              const int k = 4 * kq;
              pe_fma4(acc, in.pe[kq < NPE ? kq : 0], s_pw + k * D + xj, D);
            }
          } else {
            const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)min(r, N - 1) * a.pe_k : a.pe_tab + (size_t)item * a.pe_k;
            for (int k = 0; k < a.pe_k; ++k) {
              const float pk = pr[k];
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[q] += pk * a.wpe[(size_t)(xj + q) * a.pe_k + k];
            }
          }
          val.x = val.x + (acc[0] + s_c[xj]);
          val.y = val.y + (acc[1] + s_c[xj + 1]);
          val.z = val.z + (acc[2] + s_c[xj + 2]);
          val.w = val.w + (acc[3] + s_c[xj + 3]);
        }
      } else if (MODE == PJ_READY) {
        val = in.u;
      } else if (DH) {
        val.x = in.u.x * dr.mul(st_prev, (uint32_t)o);
        val.y = in.u.y * dr.mul(st_prev, (uint32_t)(o + 1));
        val.z = in.u.z * dr.mul(st_prev, (uint32_t)(o + 2));
        val.w = in.u.w * dr.mul(st_prev, (uint32_t)(o + 3));
      } else {
        const float4 po = in.u, px = in.v;
        val.x = (((po.x - mu.x) * rs.x * pg.x + pb.x) + px.x) * dr.mul(st_prev, (uint32_t)o);
        val.y = (((po.y - mu.y) * rs.y * pg.y + pb.y) + px.y) * dr.mul(st_prev, (uint32_t)(o + 1));
        val.z = (((po.z - mu.z) * rs.z * pg.z + pb.z) + px.z) * dr.mul(st_prev, (uint32_t)(o + 2));
        val.w = (((po.w - mu.w) * rs.w * pg.w + pb.w) + px.w) * dr.mul(st_prev, (uint32_t)(o + 3));
      }
      if (r >= N) val = make_float4(0.f, 0.f, 0.f, 0.f);
      xin_buf.st4((uint32_t)(o * 4), val);  // rows past N: dropped
    }
    *reinterpret_cast<float4*>(X + xi * XS + xj) = val;
  };

  // Pipeline (round 5).  Phase k multiplies tile T_k = t0 + k GS out of LDS buffer k % 2;
  // in the middle of its MFMA chain the waves build tile T_{k+1} into the other buffer
  // from register set S[(k+1) % 2] (its rows requested two phases earlier), then request
  // the rows of T_{k+3} into that same set, and the item ids of T_{k+5}; one barrier per
  // phase.  Two explicit register sets (the loop is unrolled by two, so no set is ever
  // COPIED: a copy of an in-flight load is a use, whose wait -- vector loads retire in
  // order -- drained every load behind it at each tile boundary).
  const int GS = gridDim.x / CS;
  const int t0 = blockIdx.x / CS;
  ProjIn S0, S1;
  {
    const int i0 = item_of(t0), i1 = item_of(t0 + GS);
    fetch(t0, i0, S0);
    fetch(t0 + GS, i1, S1);
  }
  int I0 = item_of(t0 + 2 * GS), I1 = item_of(t0 + 3 * GS);
  produce(t0, S0.item, S0, Xs[0]);
  fetch(t0 + 2 * GS, I0, S0);
  I0 = item_of(t0 + 4 * GS);
  __syncthreads();
  GTR_PH(10 + a.layer, 2);
  constexpr int KB_STAGE = D / 32;  // the k block after which the next tile is built
  auto phase = [&](auto P, int t) {
    constexpr int p = decltype(P)::value;
    ProjIn& Sn = p ? S0 : S1;  // the set of tile t + GS (then refilled with t + 3 GS)
    int& In = p ? I0 : I1;     // the item ids of tile t + 3 GS (then of t + 5 GS)
    const float* X = Xs[p];
    const bool more = t + GS < ntile;  // block-uniform
    // ---- QKVS = X . W_all^T (f32 MFMA, k order of the fused kernel)
    f32x4 acc[RT][CT];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int kb = 0; kb < D / 16; ++kb) {
      float4 av[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) av[r] = *reinterpret_cast<const float4*>(X + (r * 16 + lr) * XS + kb * 16 + lg * 4);
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c)
          acc[r][c] = GTR_PROJ_T ? GM_MFMA4(wf[c][kb], av[r], acc[r][c]) : GM_MFMA4(av[r], wf[c][kb], acc[r][c]);
      if (kb == KB_STAGE) {
        if (more) produce(t + GS, Sn.item, Sn, Xs[p ^ 1]);
        fetch(t + 3 * GS, In, Sn);  // past the last tile: zeros, nothing loaded
        In = item_of(t + 5 * GS);
      }
    }
    if (t == t0) GTR_PH(10 + a.layer, 3);
    if (GTR_PROJ_T) {  // lane (lr, lg): row lr of the 16-row tile, columns 4 lg .. 4 lg + 3
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int row = t * BM + r * 16 + lr;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int col = (wsw + (cg * CT + c) * GM_WAVES) * 16 + lg * 4;
          const size_t o = (size_t)row * (4 * D) + col;
          float4 v;
          if (DH) {
            const float4 f = *reinterpret_cast<const float4*>(a.fa + (size_t)min(row, N - 1) * (4 * D) + col);
            v.x = acc[r][c][0] * dr.mul(st_h, (uint32_t)o) * gelu_erf_grad(f.x);
            v.y = acc[r][c][1] * dr.mul(st_h, (uint32_t)(o + 1)) * gelu_erf_grad(f.y);
            v.z = acc[r][c][2] * dr.mul(st_h, (uint32_t)(o + 2)) * gelu_erf_grad(f.z);
            v.w = acc[r][c][3] * dr.mul(st_h, (uint32_t)(o + 3)) * gelu_erf_grad(f.w);
          } else {
            const float4 b = *reinterpret_cast<const float4*>(s_bias + col);
            v = make_float4(acc[r][c][0] + b.x, acc[r][c][1] + b.y, acc[r][c][2] + b.z, acc[r][c][3] + b.w);
          }
          qkvs_buf.st4((uint32_t)(o * 4), v);  // rows past N: dropped
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int col = (wsw + (cg * CT + c) * GM_WAVES) * 16 + lr;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = t * BM + r * 16 + lg * 4 + i;
            if (row < N) {
              const size_t o = (size_t)row * (4 * D) + col;
              if (DH) a.qkvs[o] = acc[r][c][i] * dr.mul(st_h, (uint32_t)o) * gelu_erf_grad(a.fa[o]);
              else a.qkvs[o] = acc[r][c][i] + bias[c];
            }
          }
        }
    }
    if (t == t0) GTR_PH(10 + a.layer, 4);
    __syncthreads();  // the next tile's X is built; this tile's buffer is free
    if (t == t0) GTR_PH(10 + a.layer, 5);
  };
  for (int t = t0; t < ntile; t += 2 * GS) {
    phase(std::integral_constant<int, 0>{}, t);
    if (t + GS >= ntile) break;  // block-uniform
    phase(std::integral_constant<int, 1>{}, t + GS);
  }
  GTR_PH(10 + a.layer, 1);
}

template <int D>
struct DxGeom {
  static constexpr int NCT = D / 16;                 // output column tiles of dX
  static constexpr int WPC = GM_WAVES / NCT;         // waves per column tile (D = 64: 2, D = 128: 1)
  static constexpr int BM = 16 * WPC;                // rows per block tile: one 16-row tile per wave
  static constexpr int K = 4 * D;
  static constexpr int AS = K + 4;                   // padded LDS row
  static constexpr int PER = BM * K / 4 / GM_BLOCK;  // float4 of dQKVS per thread and tile
  static_assert(NCT * WPC == GM_WAVES, "waves cover the column tiles");
  static_assert(PER * 4 * GM_BLOCK == BM * K, "whole float4 per thread");
};

struct DxK {
  gtr_batch bt;
  int has_prev, layer;
  float scale;
  uint32_t seed, thresh;
  int drop_on;
  uint32_t ctr_add;
  const uint32_t* rng_ctr;
  const float* dqkvs;
  const float* w_all;
  const float* dy;
  const float* p_out;
  const float* p_stats;
  float* p_dy;
  float* p_gpart;
  float* p_gsum;
  uint32_t* p_cnt;
  float* dx0;
  const float* b2;  // DX_FFN_DOWN: the second Linear's bias
};

template <int D, int MODE>
__global__ __launch_bounds__(GM_BLOCK) void k_dx(DxK a) {
  constexpr bool DOWN = MODE == DX_FFN_DOWN;
  using G = DxGeom<D>;
  constexpr int NCT = G::NCT, BM = G::BM, K = G::K, AS = G::AS, PER = G::PER;
  __shared__ __attribute__((aligned(16))) float As[2][BM * AS];
  __shared__ __attribute__((aligned(16))) float s_bnp[GM_WAVES / NCT][2 * D];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int N = a.bt.hdr[0];
  const int ntile = (N + BM - 1) / BM;
  // this wave's column tile and 16-row slice; the column tiles rotate with the workgroup's
  // position on its XCD (see k_proj: the XCD's CUs fetch different W columns at once)
  const int ct = (wave + ((int)blockIdx.x >> 3)) % NCT, rs = wave / NCT;
  const int col = ct * 16 + lr;
  // ---- W_all column fragments (B[k][col] = W_all[k][col], k = kb*16 + lg*4 + j): the
  //      fused kernel's bv, held in registers for every tile
  float4 wb[K / 16];
  if (DOWN) {  // B[k][col] = W2[col][k], W2 = [D, 4D] row-major: contiguous in k
    const float* brow = a.w_all + (size_t)col * K + lg * 4;
#pragma unroll
    for (int kb = 0; kb < K / 16; ++kb) wb[kb] = *reinterpret_cast<const float4*>(brow + kb * 16);
  } else {
    const float* bcol = a.w_all + (size_t)(lg * 4) * D + col;
#pragma unroll
    for (int kb = 0; kb < K / 16; ++kb) {
      const float* bp = bcol + (size_t)(kb * 16) * D;
      wb[kb] = make_float4(bp[0], bp[D], bp[2 * D], bp[3 * D]);
    }
  }
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_prev = drop_stream(1, (uint32_t)(a.layer - 1), ctr);
  // DX_FFN_DOWN: the hidden mask (kind 2) and the block-output mask (kind 3) of layer a.layer
  const uint32_t st_h = drop_stream(2, (uint32_t)a.layer, ctr), st_o = drop_stream(3, (uint32_t)a.layer, ctr);
  const float b2c = DOWN ? a.b2[col] : 0.0f;
  float pm = 0.0f, pr = 0.0f;
  if (a.has_prev) { pm = a.p_stats[col]; pr = a.p_stats[D + col]; }
  float s1 = 0.0f, s2 = 0.0f;
  // GTR_DX_T: this lane's four columns col4 .. col4 + 3 of row rs*16 + lr
  const int col4 = ct * 16 + lg * 4;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 b24 = z4, pm4 = z4, pr4 = z4, s14 = z4, s24 = z4;
  if (GTR_DX_T) {
    if (DOWN) b24 = *reinterpret_cast<const float4*>(a.b2 + col4);
    if (a.has_prev) {
      pm4 = *reinterpret_cast<const float4*>(a.p_stats + col4);
      pr4 = *reinterpret_cast<const float4*>(a.p_stats + D + col4);
    }
  }
  // this thread's float4s of a tile's dQKVS rows: row i = idx / (K/4), column (idx % (K/4))*4.
  // Round 5 (as k_proj): the loads issue unconditionally -- rows past N and tiles past the
  // last read row N - 1, zeroed by stage() -- and the epilogue stores go through
  // bounds-checked buffers, so the compiler counts every memory op of the pipeline and
  // the wait for a register set does not drain the other set and the tile's stores.
  const Buf dx0_buf(a.dx0, (uint64_t)N * D * 4), pdy_buf(a.p_dy, (uint64_t)N * D * 4);
  auto fetch = [&](int t, float4 (&v)[PER]) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * GM_BLOCK;
      const int i = idx / (K / 4), c = (idx - i * (K / 4)) * 4;
      const int r = min(t * BM + i, N - 1);
      v[u] = *reinterpret_cast<const float4*>(a.dqkvs + (size_t)r * K + c);
    }
  };
  // a tile's dQKVS rows (h = dropout(GELU(a)) for DX_FFN_DOWN) -> LDS; rows past N zero
  auto stage = [&](int tt, const float4 (&src)[PER], float* A) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * GM_BLOCK;
      const int i = idx / (K / 4), c = (idx - i * (K / 4)) * 4;
      float4 v = src[u];
      if (tt * BM + i >= N) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (DOWN) {  // h = dropout(GELU(a)) (rows past N are zero: GELU(0) = 0)
        const uint32_t e = (uint32_t)((size_t)(tt * BM + i) * K + c);
        v.x = gelu_erf(v.x) * dr.mul(st_h, e);
        v.y = gelu_erf(v.y) * dr.mul(st_h, e + 1);
        v.z = gelu_erf(v.z) * dr.mul(st_h, e + 2);
        v.w = gelu_erf(v.w) * dr.mul(st_h, e + 3);
      }
      *reinterpret_cast<float4*>(A + i * AS + c) = v;
    }
  };
  // Pipeline (round 5, as k_proj): phase k multiplies tile T_k out of LDS buffer k % 2,
  // stages T_{k+1} from register set S[(k+1) % 2] into the other buffer in the middle of
  // its MFMA chain and refills that set with T_{k+3}; two explicit sets, never copied.
  const int GD = gridDim.x;
  const int t0 = blockIdx.x;
  float4 S0[PER], S1[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) S0[u] = S1[u] = z4;
  if (N > 0) {  // (an empty batch: no row to clamp to; stage() zeroes every row)
    fetch(t0, S0);
    fetch(t0 + GD, S1);
  }
  stage(t0, S0, As[0]);
  if (N > 0) fetch(t0 + 2 * GD, S0);
  __syncthreads();
  constexpr int KB_STAGE = K / 32;
  auto phase = [&](auto P, int t) {
    constexpr int p = decltype(P)::value;
    float4 (&Sn)[PER] = p ? S0 : S1;
    const float* A = As[p];
    const bool more = t + GD < ntile;  // block-uniform
    // the epilogue's residual / previous-output values requested before the MFMA chain, so
    // that the tile's stores do not wait one memory round after it
    float ydv[4], pov[4];
    float4 ydv4 = z4, pov4 = z4;
    const int rowT = t * BM + rs * 16 + lr;
    if (GTR_DX_T) {
      const size_t o = (size_t)min(rowT, N - 1) * D + col4;  // (row N - 1's values: unused)
      ydv4 = *reinterpret_cast<const float4*>(a.dy + o);
      if (!DOWN && a.has_prev) pov4 = *reinterpret_cast<const float4*>(a.p_out + o);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = t * BM + rs * 16 + lg * 4 + i;
        const size_t o = (size_t)row * D + col;
        ydv[i] = row < N ? a.dy[o] : 0.0f;
        pov[i] = (!DOWN && a.has_prev && row < N) ? a.p_out[o] : 0.0f;
      }
    }
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const float* arow = A + (rs * 16 + lr) * AS + lg * 4;
#pragma unroll
    for (int kb = 0; kb < K / 16; ++kb) {
      acc = GTR_DX_T ? GM_MFMA4(wb[kb], *reinterpret_cast<const float4*>(arow + kb * 16), acc)
                     : GM_MFMA4(*reinterpret_cast<const float4*>(arow + kb * 16), wb[kb], acc);
      if (kb == KB_STAGE) {
        if (more) stage(t + GD, Sn, As[p ^ 1]);
        fetch(t + 3 * GD, Sn);  // past the last tile: zeros, nothing loaded
      }
    }
    if (GTR_DX_T) {
      const bool live = rowT < N;
      {
        const size_t o = (size_t)rowT * D + col4;
        const uint32_t ob = (uint32_t)(o * 4);  // rows past N: the buffer drops the store
        float4 v;
        if (DOWN) {  // z = y + dropout(h W2^T + b2)
          v.x = ydv4.x + (acc[0] + b24.x) * dr.mul(st_o, (uint32_t)o);
          v.y = ydv4.y + (acc[1] + b24.y) * dr.mul(st_o, (uint32_t)(o + 1));
          v.z = ydv4.z + (acc[2] + b24.z) * dr.mul(st_o, (uint32_t)(o + 2));
          v.w = ydv4.w + (acc[3] + b24.w) * dr.mul(st_o, (uint32_t)(o + 3));
          dx0_buf.st4(ob, v);
        } else {
          v = make_float4(ydv4.x + acc[0], ydv4.y + acc[1], ydv4.z + acc[2], ydv4.w + acc[3]);
          if (a.has_prev) {
            v.x *= dr.mul(st_prev, (uint32_t)o);
            v.y *= dr.mul(st_prev, (uint32_t)(o + 1));
            v.z *= dr.mul(st_prev, (uint32_t)(o + 2));
            v.w *= dr.mul(st_prev, (uint32_t)(o + 3));
            pdy_buf.st4(ob, v);
            // live rows only (a select, not a branch: the same sums as skipping the rest)
            const float4 t1 = make_float4(s14.x + v.x, s14.y + v.y, s14.z + v.z, s14.w + v.w);
            const float4 t2 = make_float4(s24.x + v.x * ((pov4.x - pm4.x) * pr4.x),
                                          s24.y + v.y * ((pov4.y - pm4.y) * pr4.y),
                                          s24.z + v.z * ((pov4.z - pm4.z) * pr4.z),
                                          s24.w + v.w * ((pov4.w - pm4.w) * pr4.w));
            if (live) { s14 = t1; s24 = t2; }
          } else {
            dx0_buf.st4(ob, v);
          }
        }
      }
      __syncthreads();  // the next tile is staged; this tile's buffer is free
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = t * BM + rs * 16 + lg * 4 + i;
      if (row < N) {
        const size_t o = (size_t)row * D + col;
        if (DOWN) {  // z = y + dropout(h W2^T + b2)
          a.dx0[o] = ydv[i] + (acc[i] + b2c) * dr.mul(st_o, (uint32_t)o);
          continue;
        }
        const float dx = ydv[i] + acc[i];
        if (a.has_prev) {
          const float d = dx * dr.mul(st_prev, (uint32_t)o);
          a.p_dy[o] = d;
          s1 += d;
          s2 += d * ((pov[i] - pm) * pr);
        } else {
          a.dx0[o] = dx;
        }
      }
    }
    __syncthreads();  // the next tile is staged; this tile's buffer is free
  };
  for (int t = t0; t < ntile; t += 2 * GD) {
    phase(std::integral_constant<int, 0>{}, t);
    if (t + GD >= ntile) break;  // block-uniform
    phase(std::integral_constant<int, 1>{}, t + GD);
  }
  if (DOWN || !a.has_prev) return;
  // ---- the previous layer's BatchNorm backward sums: one partial row per workgroup (its
  //      tiles in order), reduced by the bucketed last arrivers (fixed order: deterministic)
  if (GTR_DX_T) {  // a column's rows sit in the 16 lanes of one lane group: xor 1 .. 8
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s14.x += __shfl_xor(s14.x, o); s14.y += __shfl_xor(s14.y, o);
      s14.z += __shfl_xor(s14.z, o); s14.w += __shfl_xor(s14.w, o);
      s24.x += __shfl_xor(s24.x, o); s24.y += __shfl_xor(s24.y, o);
      s24.z += __shfl_xor(s24.z, o); s24.w += __shfl_xor(s24.w, o);
    }
    if (lr == 0) {
      *reinterpret_cast<float4*>(&s_bnp[rs][col4]) = s14;
      *reinterpret_cast<float4*>(&s_bnp[rs][D + col4]) = s24;
    }
  } else {
    s1 = bfly_add<32>(bfly_add<16>(s1));
    s2 = bfly_add<32>(bfly_add<16>(s2));
    if (lg == 0) {
      s_bnp[rs][col] = s1;
      s_bnp[rs][D + col] = s2;
    }
  }
  __syncthreads();
  float* part = a.p_gpart + (size_t)blockIdx.x * 2 * D;
  for (int j = tid; j < 2 * D; j += GM_BLOCK) {
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < GM_WAVES / NCT; ++q) acc += s_bnp[q][j];
    st_wt(part + j, acc);  // write-through: read by the last arriver of this launch
  }
  const int Gn = gridDim.x;
  const int nbk = (Gn + GTR_PART_BUCKET - 1) / GTR_PART_BUCKET;
  float* scr = As[0];
  if (nbk > 1) {
    const int bk = blockIdx.x / GTR_PART_BUCKET, b0 = bk * GTR_PART_BUCKET;
    if (!arrive_last_wt(a.p_cnt + 4 + 2 * bk, (uint32_t)min(GTR_PART_BUCKET, Gn - b0), &s_flag)) return;
    float* row0 = a.p_gpart + (size_t)b0 * 2 * D;
    block_sum_rows<GM_BLOCK>(row0, min(GTR_PART_BUCKET, Gn - b0), 2 * D, (size_t)2 * D, row0, scr, true);
    if (tid == 0) reset_counter(a.p_cnt + 4 + 2 * bk);
    if (!arrive_last_wt(a.p_cnt, (uint32_t)nbk, &s_flag)) return;
    block_sum_rows<GM_BLOCK>(a.p_gpart, nbk, 2 * D, (size_t)GTR_PART_BUCKET * 2 * D, a.p_gsum, scr);
  } else {
    if (!arrive_last_wt(a.p_cnt, (uint32_t)Gn, &s_flag)) return;
    block_sum_rows<GM_BLOCK>(a.p_gpart, Gn, 2 * D, (size_t)2 * D, a.p_gsum, scr);
  }
  if (tid == 0) reset_counter(a.p_cnt);
}

// ---- FFN weight gradients: workgroup (p, prod) reduces row chunk p of
//   prod 0: dW1[f][d] = sum_n da[n][f] y[n][d]   and db1[f] = sum_n da[n][f]
//   prod 1: dW2[d][f] = sum_n g2[n][d] h[n][f]   and db2[d] = sum_n g2[n][d],  h = dropout(GELU(a))
// into its slab (adamw_small sums the chunks).  16-row blocks of both operands are staged in
// LDS (h recomputed from a); each wave owns a contiguous run of the 16x16 output tiles and
// accumulates them on f32 MFMA with k = the node rows.
struct FfnWK {
  gtr_batch bt;
  int layer, n_chunks;
  float scale;
  uint32_t seed, thresh;
  int drop_on;
  uint32_t ctr_add;
  const uint32_t* rng_ctr;
  const float* y;
  const float* fa;
  const float* g2;
  const float* da;
  float* slab;
  int64_t stride;
};

template <int D>
__global__ __launch_bounds__(GM_BLOCK) void k_ffn_wgrad(FfnWK a) {
  constexpr int F = 4 * D, WA = F + 4, WB = F + 4;  // padded LDS rows (bank-conflict free)
  constexpr int TILES = (F / 16) * (D / 16), TW = TILES / GM_WAVES;
  static_assert(TW * GM_WAVES == TILES, "tiles split evenly over the waves");
  __shared__ __attribute__((aligned(16))) float As[16 * WA];
  __shared__ __attribute__((aligned(16))) float Bs[16 * WB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int prod = blockIdx.y;
  const int N = a.bt.hdr[0];
  const int per = (((N + a.n_chunks - 1) / a.n_chunks) + 15) & ~15;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  // prod 0: A = da [16][F] (M = F), B = y [16][D] (N' = D); prod 1: A = g2 [16][D], B = h [16][F]
  const int MA = prod == 0 ? F : D, NB = prod == 0 ? D : F;
  const int NT = NB / 16;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_h = drop_stream(2, (uint32_t)a.layer, ctr);
  f32x4 acc[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) acc[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum = 0.0f;  // bias gradient of column tid (tid < MA)
  for (int rb = r0; rb < r1; rb += 16) {
    __syncthreads();
    // stage A (16 x MA) and B (16 x NB); rows past r1 are zero
    for (int idx = tid; idx < 16 * (MA / 4); idx += GM_BLOCK) {
      const int i = idx / (MA / 4), c = (idx - i * (MA / 4)) * 4, r = rb + i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < r1) v = *reinterpret_cast<const float4*>((prod == 0 ? a.da : a.g2) + (size_t)r * MA + c);
      *reinterpret_cast<float4*>(As + i * WA + c) = v;
    }
    for (int idx = tid; idx < 16 * (NB / 4); idx += GM_BLOCK) {
      const int i = idx / (NB / 4), c = (idx - i * (NB / 4)) * 4, r = rb + i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < r1) {
        if (prod == 0) {
          v = *reinterpret_cast<const float4*>(a.y + (size_t)r * D + c);
        } else {
          const size_t e = (size_t)r * F + c;
          v = *reinterpret_cast<const float4*>(a.fa + e);
          v.x = gelu_erf(v.x) * dr.mul(st_h, (uint32_t)e);
          v.y = gelu_erf(v.y) * dr.mul(st_h, (uint32_t)(e + 1));
          v.z = gelu_erf(v.z) * dr.mul(st_h, (uint32_t)(e + 2));
          v.w = gelu_erf(v.w) * dr.mul(st_h, (uint32_t)(e + 3));
        }
      }
      *reinterpret_cast<float4*>(Bs + i * WB + c) = v;
    }
    __syncthreads();
    if (tid < MA) {
#pragma unroll
      for (int i = 0; i < 16; ++i) bsum += As[i * WA + tid];
    }
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const int tile = wave * TW + q, m0 = (tile / NT) * 16, n0 = (tile - (tile / NT) * NT) * 16;
      const float* ap = As + (lg * 4) * WA + m0 + lr;
      const float* bp = Bs + (lg * 4) * WB + n0 + lr;
      const float4 av = make_float4(ap[0], ap[WA], ap[2 * WA], ap[3 * WA]);
      const float4 bv = make_float4(bp[0], bp[WB], bp[2 * WB], bp[3 * WB]);
      acc[q] = mfma4(av, bv, acc[q]);
    }
  }
  // slab: [dW1 F*D | db1 F | dW2 D*F | db2 D]
  float* out = a.slab + (size_t)blockIdx.x * a.stride + (prod == 0 ? 0 : (size_t)F * D + F);
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    const int tile = wave * TW + q, m0 = (tile / NT) * 16, n0 = (tile - (tile / NT) * NT) * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(size_t)(m0 + lg * 4 + i) * NB + n0 + lr] = acc[q][i];
  }
  if (tid < MA) out[(size_t)F * D + tid] = bsum;
}

// Persistent grid: `per_cu` workgroups per CU (the register / LDS budget: 2 at D = 64,
// 1 at D = 128), never more than the tiles.
int gemm_cus() {
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

int gemm_grid(int tiles, int per_cu) {
  const int cus = gemm_cus();
  const char* e = getenv("GTR_GEMM_GRID");  // tuning / tests
  const int cap = e ? atoi(e) : cus * per_cu;
  return tiles < cap ? (tiles > 0 ? tiles : 1) : (cap > 0 ? cap : 1);
}

// The epilogues store through raw buffers (Buf) addressed by 32-bit byte offsets: the
// widest array, n_cap rows of 4D floats, must fit in 4 GB.
int check_buf_rows(const gtr_batch* bt, int D, const char* who) {
  if ((uint64_t)bt->n_cap * 4 * D * 4 >= (1ull << 32)) {
    set_error("%s: n_cap %d rows of 4 x %d floats exceed the 4 GB reach of a buffer offset", who, bt->n_cap, D);
    return GTR_E_ARG;
  }
  return GTR_OK;
}

}  // namespace

GTR_PH_READER(gtr_dbg_gemm_phases)

extern "C" int gtr_qkvs_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb,
                            const gtr_layer* layers, int l, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_qkvs_fwd: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim;
  if (const int rc = check_buf_rows(bt, D, "gtr_qkvs_fwd")) return rc;
  if (D != 64 && D != 128 && D != 256) {
    set_error("gtr_qkvs_fwd: dim %d (the split layer path covers 64 / 128 / 256)", D);
    return GTR_E_ARG;
  }
  if (l == 0 && (!emb || !emb->table)) { set_error("gtr_qkvs_fwd: layer 0 needs the table"); return GTR_E_ARG; }
  if (l == 0 && cfg->pe_k > 0 && (!emb->wpe || !emb->bpe || (!emb->pe_tab && !bt->node_pe))) {
    set_error("gtr_qkvs_fwd: Laplacian PE not precomputed");
    return GTR_E_ARG;
  }
  if (cfg->pe_k < 0 || cfg->pe_k > 256) { set_error("gtr_qkvs_fwd: pe_k out of range"); return GTR_E_ARG; }
  const bool ready = l > 0 && layers[l - 1].ffn;  // input rows = the previous layer's FFN output
  if (l > 0 && !ready && cfg->training && (cfg->sync_bn ? !cfg->split_sync : cfg->consumer_reduce)) {
    set_error("gtr_qkvs_fwd: the split path reads producer-finalized BatchNorm statistics (consumer_reduce 0) "
              "or, under sync_bn, the ranks' merged rows (split_sync)");
    return GTR_E_ARG;
  }
  const char* gg = getenv("GTR_GEMM_GEN");  // A/B: the LDS-staged GEMMs at D = 64 / 128 too
  if (D == 256 || (gg && gg[0] == '1' && !(cfg->sync_bn && cfg->training))) {  // LDS-staged GEMM (gtr_gemm_gen.hip): no SyncBN merged-row mode there
    if (cfg->sync_bn && cfg->training) { set_error("gtr_qkvs_fwd: dim 256 on the split path has no SyncBN"); return GTR_E_ARG; }
    if (l == 0 && cfg->pe_k > 0 && (!emb->wpe || !emb->bpe)) { set_error("gtr_qkvs_fwd: Laplacian PE not precomputed"); return GTR_E_ARG; }
    return gen_qkvs_fwd(cfg, bt, emb, layers, l, (hipStream_t)stream);
  }
  const gtr_layer& L = layers[l];
  ProjK k{};
  k.bt = *bt;
  k.first = l == 0;
  k.train = cfg->training;
  k.pe_k = cfg->pe_k;
  k.layer = l;
  k.bn_eps = cfg->bn_eps;
  k.drop_on = (cfg->training && cfg->dropout > 0.0f) ? 1 : 0;
  {
    double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
    k.thresh = (uint32_t)(p * 4294967296.0);
    k.scale = k.drop_on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  }
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.ctr_add = (uint32_t)cfg->ctr_add;
  if (l == 0) {
    k.table = emb->table; k.pe_tab = emb->pe_tab; k.wpe = emb->wpe; k.bpe = emb->bpe;
  } else if (ready) {
    if (!layers[l - 1].ffn->z) { set_error("gtr_qkvs_fwd: layer %d's FFN has no output rows", l - 1); return GTR_E_ARG; }
    k.p_out = layers[l - 1].ffn->z;
  } else {
    const gtr_layer& P = layers[l - 1];
    k.p_out = P.out; k.p_xin = P.xin; k.p_stats = P.bn_stats; k.p_rmean = P.bn_rmean; k.p_rvar = P.bn_rvar;
    k.p_nbt = P.bn_nbt; k.p_gamma = P.bn_gamma; k.p_beta = P.bn_beta;
    k.bn_mom = cfg->bn_momentum;
    if (cfg->sync_bn && cfg->training) {
      if (!P.bn_part_all || P.nparts_fwd <= 0) {
        set_error("gtr_qkvs_fwd: sync_bn needs the gathered merged rows of layer %d", l - 1);
        return GTR_E_ARG;
      }
      k.sync = 1;
      k.p_part_all = P.bn_part_all;
      k.p_nparts = P.nparts_fwd;
    }
  }
  k.w_all = L.w_all; k.b_all = L.b_all; k.xin = L.xin; k.qkvs = L.qkvs;
  const int bm = D == 64 ? ProjGeom<64>::BM : ProjGeom<128>::BM;
  const int tiles = (bt->n_cap + bm - 1) / bm;
  hipStream_t s = (hipStream_t)stream;
  // Column slices at D = 128 when the row tiles number at most one per CU (a few thousand
  // rows: C4 / C5 at B = 1024, 225 tiles): one workgroup per CU, i.e. CUs / 4 streams of
  // ~4 pipelined tiles each.  Per-launch (C4 B = 1024, layer 0 / 1): 19.2 / 17.8 us whole
  // rows, 15.7 / 13.8 us in slices at 4 tiles per stream (24.4 / 19.2 at 1, 18.2 / 15.2 at 2,
  // 20.5 / 17.3 at 3, 18.6 / 16.1 at 6).  GTR_PROJ_CS=1|4 and GTR_PROJ_CS_TPB override.
  // (Half-width slices at C3 B = 8192, four waves per SIMD: 49.5 / 46.5 -> 79 / 53 us.)
  const char* pcs = getenv("GTR_PROJ_CS");
  const int cs = D != 128 ? 1 : pcs ? (atoi(pcs) == 4 ? 4 : 1) : (tiles <= gemm_cus() ? 4 : 1);
  if (cs == 4) {
    const char* tpb = getenv("GTR_PROJ_CS_TPB");
    const int nst = gemm_cus() / 4 > 0 ? gemm_cus() / 4 : 1;
    const int tp = tpb && atoi(tpb) > 0 ? atoi(tpb) : (tiles + nst - 1) / nst;
    const int grid = 4 * gemm_grid((tiles + tp - 1) / tp, 2);  // streams of row tiles, four column slices each
    if (l == 0) hipLaunchKernelGGL((k_proj<128, PJ_FIRST, 4>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else if (ready) hipLaunchKernelGGL((k_proj<128, PJ_READY, 4>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else hipLaunchKernelGGL((k_proj<128, PJ_FOLD, 4>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  const int grid = gemm_grid(tiles, D == 64 ? 2 : 1);
  if (D == 64) {
    if (l == 0) hipLaunchKernelGGL((k_proj<64, PJ_FIRST>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else if (ready) hipLaunchKernelGGL((k_proj<64, PJ_READY>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else hipLaunchKernelGGL((k_proj<64, PJ_FOLD>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  } else {
    if (l == 0) hipLaunchKernelGGL((k_proj<128, PJ_FIRST>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else if (ready) hipLaunchKernelGGL((k_proj<128, PJ_READY>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
    else hipLaunchKernelGGL((k_proj<128, PJ_FOLD>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_qkvs_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, float* dx0,
                            gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers || (l == 0 && !dx0)) {
    set_error("gtr_qkvs_bwd: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim;
  if (const int rc = check_buf_rows(bt, D, "gtr_qkvs_bwd")) return rc;
  if (D != 64 && D != 128 && D != 256) {
    set_error("gtr_qkvs_bwd: dim %d (the split layer path covers 64 / 128 / 256)", D);
    return GTR_E_ARG;
  }
  if (!cfg->training) { set_error("gtr_qkvs_bwd: backward requires training mode"); return GTR_E_ARG; }
  if (cfg->sync_bn && !cfg->split_sync) { set_error("gtr_qkvs_bwd: sync_bn needs split_sync"); return GTR_E_ARG; }
  const char* gg = getenv("GTR_GEMM_GEN");
  if (D == 256 || (gg && gg[0] == '1' && !cfg->sync_bn)) {
    if (cfg->sync_bn) { set_error("gtr_qkvs_bwd: dim 256 on the split path has no SyncBN"); return GTR_E_ARG; }
    if (l > 0 && layers[l - 1].ffn && !layers[l - 1].ffn->dz) { set_error("gtr_qkvs_bwd: layer %d's FFN has no dz rows", l - 1); return GTR_E_ARG; }
    return gen_qkvs_bwd(cfg, bt, layers, l, dx0, (hipStream_t)stream);
  }
  const gtr_layer& L = layers[l];
  const bool ffn_prev = l > 0 && layers[l - 1].ffn;  // dX is d/dz of the previous layer's FFN
  if (ffn_prev && !layers[l - 1].ffn->dz) { set_error("gtr_qkvs_bwd: layer %d's FFN has no dz rows", l - 1); return GTR_E_ARG; }
  DxK k{};
  k.bt = *bt;
  k.has_prev = l > 0 && !ffn_prev;
  k.layer = l;
  k.drop_on = (cfg->dropout > 0.0f) ? 1 : 0;
  {
    double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
    k.thresh = (uint32_t)(p * 4294967296.0);
    k.scale = k.drop_on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  }
  k.seed = cfg->seed;
  k.rng_ctr = cfg->rng_ctr;
  k.ctr_add = (uint32_t)cfg->ctr_add;
  k.dqkvs = L.dqkvs; k.w_all = L.w_all; k.dy = L.dy; k.dx0 = ffn_prev ? layers[l - 1].ffn->dz : dx0;
  if (k.has_prev) {
    const gtr_layer& P = layers[l - 1];
    k.p_out = P.out; k.p_stats = P.bn_stats; k.p_dy = P.dy; k.p_gpart = P.bn_gpart; k.p_gsum = P.bn_gsum;
    k.p_cnt = P.cnt + 1;
  }
  const int bm = D == 64 ? DxGeom<64>::BM : DxGeom<128>::BM;
  const int grid = gemm_grid((bt->n_cap + bm - 1) / bm, 1);
  if (grid > 256) { set_error("gtr_qkvs_bwd: more than 256 partial rows"); return GTR_E_ARG; }
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) hipLaunchKernelGGL((k_dx<64, DX_CONV>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  else hipLaunchKernelGGL((k_dx<128, DX_CONV>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

namespace {

// Shared argument checks of the FFN entry points; fills the dropout parameters.
bool ffn_generic(const gtr_config* cfg, const gtr_ffn& f);

int ffn_check(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, const char* fn,
              bool need_train, uint32_t& thresh, float& scale, int& drop_on) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers || !layers[l].ffn) {
    set_error("%s: bad arguments (layer %d needs gtr_layer.ffn)", fn, l);
    return GTR_E_ARG;
  }
  const gtr_ffn& f = *layers[l].ffn;
  if (cfg->dim != 64 && cfg->dim != 128 && cfg->dim != 256) {
    set_error("%s: dim %d (the FFN GEMMs cover 64 / 128 / 256)", fn, cfg->dim);
    return GTR_E_ARG;
  }
  if (f.expansion != 1 && f.expansion != 2 && f.expansion != 4) {
    set_error("%s: ffn_expansion %d (1 / 2 / 4 supported)", fn, f.expansion);
    return GTR_E_ARG;
  }
  if (!f.w1 || !f.b1 || !f.w2 || !f.b2 || !f.y || !f.a || !f.z) { set_error("%s: missing FFN buffers", fn); return GTR_E_ARG; }
  if (need_train && !cfg->training) { set_error("%s: backward requires training mode", fn); return GTR_E_ARG; }
  // BatchNorm statistics: producer-finalized, or (SyncBN, split_sync) folded by the FFN's
  // first GEMM from every rank's merged row like the next layer's projection does
  if (cfg->training && (cfg->sync_bn || cfg->consumer_reduce) &&
      !(cfg->sync_bn && cfg->split_sync && !ffn_generic(cfg, f))) {
    set_error("%s: the FFN variant takes producer-finalized BatchNorm statistics, or SyncBN's merged rows "
              "(split_sync) at dim 64 / 128 with expansion 4", fn);
    return GTR_E_ARG;
  }
  drop_on = (cfg->training && cfg->dropout > 0.0f) ? 1 : 0;
  const double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
  thresh = (uint32_t)(p * 4294967296.0);
  scale = drop_on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  return GTR_OK;
}

// The register-resident kernels above cover D = 64 / 128 with F = 4 D; every other FFN
// shape runs on the LDS-staged GEMMs of gtr_gemm_gen.hip.
bool ffn_generic(const gtr_config* cfg, const gtr_ffn& f) {
  return !((cfg->dim == 64 || cfg->dim == 128) && f.expansion == 4);
}

}  // namespace

extern "C" int gtr_ffn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                           gtr_stream_t stream) {
  uint32_t thresh;
  float scale;
  int drop_on;
  if (const int rc = ffn_check(cfg, bt, layers, l, "gtr_ffn_fwd", false, thresh, scale, drop_on)) return rc;
  if (ffn_generic(cfg, *layers[l].ffn)) return gen_ffn_fwd(cfg, bt, layers, l, (hipStream_t)stream);
  const int D = cfg->dim;
  if (const int rc = check_buf_rows(bt, D, "gtr_ffn_fwd")) return rc;
  const gtr_layer& L = layers[l];
  const gtr_ffn& f = *L.ffn;
  hipStream_t s = (hipStream_t)stream;
  // y = dropout(BN(out) + xin) and a = y W1^T + b1: the conv projection of a "layer l + 1"
  ProjK k{};
  k.bt = *bt;
  k.first = 0;
  k.train = cfg->training;
  k.layer = l + 1;
  k.bn_eps = cfg->bn_eps;
  k.drop_on = drop_on; k.thresh = thresh; k.scale = scale;
  k.seed = cfg->seed; k.rng_ctr = cfg->rng_ctr; k.ctr_add = (uint32_t)cfg->ctr_add;
  k.p_out = L.out; k.p_xin = L.xin; k.p_stats = L.bn_stats; k.p_rmean = L.bn_rmean; k.p_rvar = L.bn_rvar;
  k.p_nbt = L.bn_nbt; k.p_gamma = L.bn_gamma; k.p_beta = L.bn_beta; k.bn_mom = cfg->bn_momentum;
  k.w_all = f.w1; k.b_all = f.b1; k.xin = f.y; k.qkvs = f.a;
  if (cfg->sync_bn && cfg->training) {  // SyncBN: the ranks' merged rows of this layer (gtr_qkvs_fwd's fold)
    if (!L.bn_part_all || L.nparts_fwd <= 0) {
      set_error("gtr_ffn_fwd: sync_bn needs the gathered merged rows of layer %d", l);
      return GTR_E_ARG;
    }
    k.sync = 1;
    k.p_part_all = L.bn_part_all;
    k.p_nparts = L.nparts_fwd;
  }
  const int bm = D == 64 ? ProjGeom<64>::BM : ProjGeom<128>::BM;
  const int grid = gemm_grid((bt->n_cap + bm - 1) / bm, D == 64 ? 2 : 1);
  if (D == 64) hipLaunchKernelGGL((k_proj<64, PJ_FOLD>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  else hipLaunchKernelGGL((k_proj<128, PJ_FOLD>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  // z = y + dropout(dropout(GELU(a)) W2^T + b2)
  DxK d{};
  d.bt = *bt;
  d.has_prev = 0;
  d.layer = l;
  d.drop_on = drop_on; d.thresh = thresh; d.scale = scale;
  d.seed = cfg->seed; d.rng_ctr = cfg->rng_ctr; d.ctr_add = (uint32_t)cfg->ctr_add;
  d.dqkvs = f.a; d.w_all = f.w2; d.dy = f.y; d.dx0 = f.z; d.b2 = f.b2;
  const int bmd = D == 64 ? DxGeom<64>::BM : DxGeom<128>::BM;
  const int gd = gemm_grid((bt->n_cap + bmd - 1) / bmd, 1);
  if (D == 64) hipLaunchKernelGGL((k_dx<64, DX_FFN_DOWN>), dim3(gd), dim3(GM_BLOCK), 0, s, d);
  else hipLaunchKernelGGL((k_dx<128, DX_FFN_DOWN>), dim3(gd), dim3(GM_BLOCK), 0, s, d);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_ffn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                           gtr_stream_t stream) {
  uint32_t thresh;
  float scale;
  int drop_on;
  if (const int rc = ffn_check(cfg, bt, layers, l, "gtr_ffn_bwd", true, thresh, scale, drop_on)) return rc;
  const int D = cfg->dim;
  if (const int rc = check_buf_rows(bt, D, "gtr_ffn_bwd")) return rc;
  const gtr_layer& L = layers[l];
  const gtr_ffn& f = *L.ffn;
  if (!f.dz || !f.g2 || !f.da) { set_error("gtr_ffn_bwd: missing FFN gradient buffers"); return GTR_E_ARG; }
  if (ffn_generic(cfg, f)) return gen_ffn_bwd(cfg, bt, layers, l, (hipStream_t)stream);
  hipStream_t s = (hipStream_t)stream;
  // g2 = dz * mask3 -> ffn.g2; da = (g2 W2) * mask2 * GELU'(a) -> ffn.da
  ProjK k{};
  k.bt = *bt;
  k.train = 1;
  k.layer = l;
  k.drop_on = drop_on; k.thresh = thresh; k.scale = scale;
  k.seed = cfg->seed; k.rng_ctr = cfg->rng_ctr; k.ctr_add = (uint32_t)cfg->ctr_add;
  k.p_out = f.dz; k.w_all = f.w2; k.xin = f.g2; k.qkvs = f.da; k.fa = f.a;
  const int bm = D == 64 ? ProjGeom<64>::BM : ProjGeom<128>::BM;
  const int grid = gemm_grid((bt->n_cap + bm - 1) / bm, D == 64 ? 2 : 1);
  if (D == 64) hipLaunchKernelGGL((k_proj<64, PJ_FFN_DH>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  else hipLaunchKernelGGL((k_proj<128, PJ_FFN_DH>), dim3(grid), dim3(GM_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  // dy = (dz + da W1) * the layer's output mask -> layers[l].dy, + its BatchNorm backward sums
  DxK d{};
  d.bt = *bt;
  d.has_prev = 1;
  d.layer = l + 1;
  d.drop_on = drop_on; d.thresh = thresh; d.scale = scale;
  d.seed = cfg->seed; d.rng_ctr = cfg->rng_ctr; d.ctr_add = (uint32_t)cfg->ctr_add;
  d.dqkvs = f.da; d.w_all = f.w1; d.dy = f.dz;
  d.p_out = L.out; d.p_stats = L.bn_stats; d.p_dy = L.dy; d.p_gpart = L.bn_gpart; d.p_gsum = L.bn_gsum;
  d.p_cnt = L.cnt + 1;
  const int bmd = D == 64 ? DxGeom<64>::BM : DxGeom<128>::BM;
  const int gd = gemm_grid((bt->n_cap + bmd - 1) / bmd, 1);
  if (gd > 256) { set_error("gtr_ffn_bwd: more than 256 partial rows"); return GTR_E_ARG; }
  if (D == 64) hipLaunchKernelGGL((k_dx<64, DX_CONV>), dim3(gd), dim3(GM_BLOCK), 0, s, d);
  else hipLaunchKernelGGL((k_dx<128, DX_CONV>), dim3(gd), dim3(GM_BLOCK), 0, s, d);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_ffn_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                             float* slab, int n_chunks, int64_t slab_stride, gtr_stream_t stream) {
  uint32_t thresh;
  float scale;
  int drop_on;
  if (const int rc = ffn_check(cfg, bt, layers, l, "gtr_ffn_wgrad", true, thresh, scale, drop_on)) return rc;
  const int D = cfg->dim;
  const gtr_ffn& f = *layers[l].ffn;
  const int64_t F = (int64_t)f.expansion * D;
  if (!slab || n_chunks <= 0 || slab_stride < 2 * F * D + F + D || !f.g2 || !f.da) {
    set_error("gtr_ffn_wgrad: bad slab / chunks");
    return GTR_E_ARG;
  }
  if (ffn_generic(cfg, f)) return gen_ffn_wgrad(cfg, bt, layers, l, slab, n_chunks, slab_stride, (hipStream_t)stream);
  FfnWK k{};
  k.bt = *bt;
  k.layer = l;
  k.n_chunks = n_chunks;
  k.drop_on = drop_on; k.thresh = thresh; k.scale = scale;
  k.seed = cfg->seed; k.rng_ctr = cfg->rng_ctr; k.ctr_add = (uint32_t)cfg->ctr_add;
  k.y = f.y; k.fa = f.a; k.g2 = f.g2; k.da = f.da; k.slab = slab; k.stride = slab_stride;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) hipLaunchKernelGGL(k_ffn_wgrad<64>, dim3(n_chunks, 2), dim3(GM_BLOCK), 0, s, k);
  else hipLaunchKernelGGL(k_ffn_wgrad<128>, dim3(n_chunks, 2), dim3(GM_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}
