// gtr_gemm_gen.hip — the layer and feed-forward GEMMs of the split layer path for the
// shapes the register-resident kernels of gtr_gemm.hip do not cover: hidden width 256 and
// feed-forward expansions other than 4 (the reference's create_graph_transformer defaults,
// d = 256 with FFN x 4 -- graph_transformer.py:109-124,185-197 -- and the optimized
// factory's ffn_expansion = 2, :231-280).
//
// At D = 256 the projection's W_all alone is 1 MB: no longer a per-wave register tile.
// These kernels stage BOTH operands through LDS instead, in K chunks of 32:
//
//   k_gen_gemm   C[M, N] tile of 32 x 64 per workgroup (4 waves, 16 x 32 each, two
//                16x16 f32-MFMA accumulators per wave); A row-major [M][K] or transposed
//                [K][M] (weight gradients: K = node rows), B as [N][K] (X W^T) or [K][N];
//                optional GELU x dropout transform of an operand on load; epilogues: bias,
//                the FFN down-projection residual, the FFN hidden gradient, dX with the
//                previous layer's dropout mask and per-tile BatchNorm backward column sums;
//                split-K over row chunks (grid.z) into the weight-gradient slabs.
//   k_gen_rows   the elementwise row builds the register kernels fuse into their GEMM
//                prologue: layer 0's item row + LapPE projection, the previous layer's
//                BatchNorm fold + residual + dropout, the FFN output-mask gradient.
//   k_gen_colsum fixed-order column sums of per-tile partial rows (BatchNorm backward sums,
//                the FFN bias gradients per row chunk).
//
// Exact f32 (v_mfma_f32_16x16x4f32): the sums run in another order than the register
// kernels', so these results equal the CPU oracle at the 1e-3 bar, not those kernels bit
// for bit (no configuration runs both).

#include "gtr_layer.cuh"

namespace {

using namespace gtr;

#define GG_BLOCK 256
#define GG_BM 32
#define GG_BN 64
#define GG_BK 32
#define GG_AS (GG_BK + 4)  // padded LDS rows (k contiguous): float4 reads without bank conflicts

__device__ __forceinline__ float gelu_erf_g(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad_g(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  return cdf + x * (0.39894228040143268f * expf(-0.5f * x * x));
}

enum { GA_MK = 0, GA_KM = 1 };            // A[m][k] row-major | A[k][m] (transposed)
enum { GB_NK = 0, GB_KN = 1 };            // B[k][n] = W[n][k] | W[k][n]
enum { GT_NONE = 0, GT_GELU_MASK = 1 };   // operand transform on load: dropout(GELU(x)) (kind 2)
enum { GE_STORE = 0, GE_BIAS = 1, GE_FFN_DOWN = 2, GE_FFN_DH = 3, GE_DX = 4 };

struct GenK {
  const float* A;
  const float* B;
  float* C;
  int M, N, K;            // C is M x N; K the reduction length (rows per chunk for split-K)
  int lda, ldb, ldc;
  const int32_t* m_live;  // rows >= *m_live are zero (the batch's live node count), or null
  int k_live_from_hdr;    // split-K over node rows: K = *m_live rows cut into gridDim.z chunks
  int64_t c_chunk_stride; // split-K: output slab stride per chunk
  // epilogue / transform operands
  const float* bias;
  const float* res;       // GE_FFN_DOWN: y; GE_DX: dy
  const float* fa;        // GE_FFN_DH: pre-activation a [M, N]
  float* p_dy;            // GE_DX with a previous layer: its dy
  const float* p_out;     // GE_DX: the previous layer's conv output (x-hat for the sums)
  const float* p_stats;   // GE_DX: its mean | rstd
  float* gpart;           // GE_DX: [row tiles][2 N] partial BatchNorm backward sums
  int has_prev, layer;
  uint32_t seed, thresh;
  float scale;
  int drop_on;
  uint32_t ctr_add;
  const uint32_t* rng_ctr;
  int tr_ld;              // GT_GELU_MASK: row stride of the transformed operand's element index
};

template <int AL, int BL, int AT, int BT, int EP>
__global__ __launch_bounds__(GG_BLOCK) void k_gen_gemm(GenK a) {
  __shared__ __attribute__((aligned(16))) float As[GG_BM * GG_AS];  // [m][k]
  __shared__ __attribute__((aligned(16))) float Bs[GG_BN * GG_AS];  // [n][k]
  __shared__ float s_sum[2][2][GG_BN];                              // GE_DX: [row wave][s1|s2][col]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * GG_BM, n0 = blockIdx.y * GG_BN;
  int M = a.M;
  if (a.m_live && !a.k_live_from_hdr) M = min(M, *a.m_live);
  if (m0 >= M && EP != GE_STORE) return;  // block-uniform (split-K slabs are written whole)
  // split-K over node rows (weight gradients): this chunk's [k0, k1)
  int kb0 = 0, kb1 = a.K;
  float* C = a.C;
  if (a.k_live_from_hdr) {
    const int rows = *a.m_live;
    const int per = (((rows + (int)gridDim.z - 1) / (int)gridDim.z) + GG_BK - 1) / GG_BK * GG_BK;
    kb0 = min(rows, (int)blockIdx.z * per);
    kb1 = min(rows, kb0 + per);
    C += (int64_t)blockIdx.z * a.c_chunk_stride;
  }
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  const uint32_t st_h = drop_stream(2, (uint32_t)a.layer, ctr);
  auto tr = [&](float v, int r, int c) -> float {  // dropout(GELU(x)) of element (r, c)
    return gelu_erf_g(v) * dr.mul(st_h, (uint32_t)((size_t)r * a.tr_ld + c));
  };
  const int wr = (wave >> 1) * 16, wc = (wave & 1) * 32;  // this wave's 16 x 32 of the tile
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb0; k0 < kb1; k0 += GG_BK) {
    // ---- stage A (32 x 32: one float4 per thread) and B (64 x 32: two per thread)
    if (AL == GA_MK) {
      const int i = tid >> 3, c = (tid & 7) * 4, r = m0 + i, k = k0 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < M && k < kb1) {
        v = *reinterpret_cast<const float4*>(a.A + (size_t)r * a.lda + k);
        if (AT == GT_GELU_MASK) { v.x = tr(v.x, r, k); v.y = tr(v.y, r, k + 1); v.z = tr(v.z, r, k + 2); v.w = tr(v.w, r, k + 3); }
      }
      *reinterpret_cast<float4*>(As + i * GG_AS + c) = v;
    } else {  // A[k][m]: a float4 along m, scattered into the k-contiguous LDS rows
      const int kk = tid >> 3, c = (tid & 7) * 4, k = k0 + kk, m = m0 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < kb1 && m < M) v = *reinterpret_cast<const float4*>(a.A + (size_t)k * a.lda + m);
      As[(c + 0) * GG_AS + kk] = v.x; As[(c + 1) * GG_AS + kk] = v.y;
      As[(c + 2) * GG_AS + kk] = v.z; As[(c + 3) * GG_AS + kk] = v.w;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + u * GG_BLOCK;
      if (BL == GB_NK) {  // W[n][k]: float4 along k
        const int j = idx >> 3, c = (idx & 7) * 4, n = n0 + j, k = k0 + c;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n < a.N && k < kb1) v = *reinterpret_cast<const float4*>(a.B + (size_t)n * a.ldb + k);
        *reinterpret_cast<float4*>(Bs + j * GG_AS + c) = v;
      } else {  // W[k][n]: float4 along n, scattered into the k-contiguous LDS rows
        const int kk = idx >> 4, c = (idx & 15) * 4, k = k0 + kk, n = n0 + c;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kb1 && n < a.N) {
          v = *reinterpret_cast<const float4*>(a.B + (size_t)k * a.ldb + n);
          if (BT == GT_GELU_MASK) { v.x = tr(v.x, k, n); v.y = tr(v.y, k, n + 1); v.z = tr(v.z, k, n + 2); v.w = tr(v.w, k, n + 3); }
        }
        Bs[(c + 0) * GG_AS + kk] = v.x; Bs[(c + 1) * GG_AS + kk] = v.y;
        Bs[(c + 2) * GG_AS + kk] = v.z; Bs[(c + 3) * GG_AS + kk] = v.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < GG_BK / 16; ++kb) {
      const float4 av = *reinterpret_cast<const float4*>(As + (wr + lr) * GG_AS + kb * 16 + lg * 4);
      const float4 b0 = *reinterpret_cast<const float4*>(Bs + (wc + lr) * GG_AS + kb * 16 + lg * 4);
      const float4 b1 = *reinterpret_cast<const float4*>(Bs + (wc + 16 + lr) * GG_AS + kb * 16 + lg * 4);
      acc0 = mfma4(av, b0, acc0);
      acc1 = mfma4(av, b1, acc1);
    }
    __syncthreads();
  }
  // ---- epilogue: lane (lr, lg) holds C[wr + lg*4 + i][wc + lr] (acc0) and [.. + 16] (acc1)
  const uint32_t pm = drop_stream(1, (uint32_t)(a.layer - 1), ctr), po = drop_stream(3, (uint32_t)a.layer, ctr);
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int col = n0 + wc + h * 16 + lr;
    const f32x4& acc = h == 0 ? acc0 : acc1;
    float mean = 0.f, rstd = 0.f, bb = 0.f;
    if (EP == GE_BIAS || EP == GE_FFN_DOWN) bb = col < a.N ? a.bias[col] : 0.f;
    if (EP == GE_DX && a.has_prev && col < a.N) { mean = a.p_stats[col]; rstd = a.p_stats[a.N + col]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wr + lg * 4 + i;
      if (row >= M || col >= a.N) continue;
      const size_t o = (size_t)row * a.ldc + col;
      const float v = acc[i];
      if (EP == GE_STORE) {
        C[o] = v;
      } else if (EP == GE_BIAS) {
        C[o] = v + bb;
      } else if (EP == GE_FFN_DOWN) {  // z = y + dropout(h W2^T + b2)
        C[o] = a.res[o] + (v + bb) * dr.mul(po, (uint32_t)o);
      } else if (EP == GE_FFN_DH) {  // da = (g2 W2) * mask2 * GELU'(a)
        C[o] = v * dr.mul(st_h, (uint32_t)o) * gelu_erf_grad_g(a.fa[o]);
      } else {  // GE_DX: dx = dy + dQKVS W_all (+ the previous layer's mask, BatchNorm sums)
        const float dx = a.res[o] + v;
        if (a.has_prev) {
          const float d = dx * dr.mul(pm, (uint32_t)o);
          a.p_dy[o] = d;
          s1[h] += d;
          s2[h] += d * ((a.p_out[o] - mean) * rstd);
        } else {
          C[o] = dx;
        }
      }
    }
  }
  if (EP != GE_DX || !a.has_prev) return;
  // per-tile column partials of the previous layer's BatchNorm backward sums (fixed order:
  // lane groups by butterfly, the two row waves through LDS), reduced by k_gen_colsum
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    s1[h] = bfly_add<32>(bfly_add<16>(s1[h]));
    s2[h] = bfly_add<32>(bfly_add<16>(s2[h]));
    if (lg == 0) {
      s_sum[wave >> 1][0][wc + h * 16 + lr] = s1[h];
      s_sum[wave >> 1][1][wc + h * 16 + lr] = s2[h];
    }
  }
  __syncthreads();
  if (tid < 2 * GG_BN) {
    const int which = tid / GG_BN, j = tid % GG_BN, col = n0 + j;
    if (col < a.N)
      a.gpart[(size_t)blockIdx.x * 2 * a.N + which * a.N + col] = s_sum[0][which][j] + s_sum[1][which][j];
  }
}

// Column sums out[c] = sum over rows r < rows of p[r * stride + c] (c < W), rows in order.
// split (grid.y > 1): row chunk y of `per` rows -> out + y * out_stride (weight-gradient
// slabs); rows from *rows_live when given.
__global__ __launch_bounds__(256) void k_gen_colsum(const float* p, int rows, const int32_t* rows_live, int W,
                                                    int64_t stride, float* out, int64_t out_stride, int chunks,
                                                    int row_div) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= W) return;
  int R = rows_live ? (*rows_live + row_div - 1) / row_div : rows;
  int r0 = 0, r1 = R;
  if (chunks > 1) {
    const int per = (((R + chunks - 1) / chunks) + GG_BK - 1) / GG_BK * GG_BK;
    r0 = min(R, (int)blockIdx.y * per);
    r1 = min(R, r0 + per);
  }
  float acc = 0.0f;
#pragma unroll 16
  for (int r = r0; r < r1; ++r) acc += p[(size_t)r * stride + c];
  out[(int64_t)blockIdx.y * out_stride + c] = acc;
}

// Row builds (one float4 per thread) of the split path's GEMM inputs:
//   RB_FIRST  layer 0: item row + LapPE projection (+ bias)            -> dst (xin)
//   RB_FOLD   dropout(BN(out) + xin) with the layer's finalized stats   -> dst (xin of the
//             next layer, or the FFN input y); eval: running statistics
//   RB_READY  the previous FFN's z as it is                             -> dst (xin)
//   RB_G2     dz * the FFN output mask (kind 3)                         -> dst (g2)
enum { RB_FIRST = 0, RB_FOLD = 1, RB_READY = 2, RB_G2 = 3 };

struct RowsK {
  gtr_batch bt;
  int D, pe_k, train, layer;
  float bn_eps;
  const float* table;
  const float* pe_tab;
  const float* wpe;
  const float* bpe;
  const float* src;    // FOLD: out; READY: z; G2: dz
  const float* src2;   // FOLD: xin
  const float* stats;  // FOLD (train): mean | rstd
  const float* rmean;  // FOLD (eval)
  const float* rvar;
  const float* gamma;
  const float* beta;
  float* dst;
  uint32_t seed, thresh;
  float scale;
  int drop_on;
  uint32_t ctr_add;
  const uint32_t* rng_ctr;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_gen_rows(RowsK a) {
  const int N = a.bt.hdr[0];
  const int C4 = a.D / 4;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(gid / C4), j = (int)(gid - (int64_t)r * C4) * 4;
  if (r >= N) return;
  const size_t o = (size_t)r * a.D + j;
  const uint32_t ctr = a.rng_ctr ? load_step_ctr(a.rng_ctr) + a.ctr_add : 0u;
  const Drop dr{a.seed, a.thresh, a.scale, a.drop_on != 0};
  float4 v;
  if (MODE == RB_FIRST) {
    const int item = a.bt.node_item[r];
    v = *reinterpret_cast<const float4*>(a.table + (size_t)item * a.D + j);
    if (a.pe_k > 0) {
      const float* pr = a.bt.node_pe ? a.bt.node_pe + (size_t)r * a.pe_k : a.pe_tab + (size_t)item * a.pe_k;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < a.pe_k; ++k) {
        const float pk = pr[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = __builtin_fmaf(pk, a.wpe[(size_t)(j + q) * a.pe_k + k], acc[q]);
      }
      v.x = v.x + (acc[0] + a.bpe[j]);
      v.y = v.y + (acc[1] + a.bpe[j + 1]);
      v.z = v.z + (acc[2] + a.bpe[j + 2]);
      v.w = v.w + (acc[3] + a.bpe[j + 3]);
    }
  } else if (MODE == RB_READY) {
    v = *reinterpret_cast<const float4*>(a.src + o);
  } else if (MODE == RB_G2) {
    const uint32_t st = drop_stream(3, (uint32_t)a.layer, ctr);
    v = *reinterpret_cast<const float4*>(a.src + o);
    v.x *= dr.mul(st, (uint32_t)o); v.y *= dr.mul(st, (uint32_t)(o + 1));
    v.z *= dr.mul(st, (uint32_t)(o + 2)); v.w *= dr.mul(st, (uint32_t)(o + 3));
  } else {  // RB_FOLD with layer a.layer's BatchNorm and its output dropout (kind 1)
    const uint32_t st = drop_stream(1, (uint32_t)a.layer, ctr);
    const float4 po = *reinterpret_cast<const float4*>(a.src + o);
    const float4 px = *reinterpret_cast<const float4*>(a.src2 + o);
    float mu[4], rs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      mu[q] = a.train ? a.stats[j + q] : a.rmean[j + q];
      rs[q] = a.train ? a.stats[a.D + j + q] : 1.0f / sqrtf(a.rvar[j + q] + a.bn_eps);
    }
    v.x = (((po.x - mu[0]) * rs[0] * a.gamma[j] + a.beta[j]) + px.x) * dr.mul(st, (uint32_t)o);
    v.y = (((po.y - mu[1]) * rs[1] * a.gamma[j + 1] + a.beta[j + 1]) + px.y) * dr.mul(st, (uint32_t)(o + 1));
    v.z = (((po.z - mu[2]) * rs[2] * a.gamma[j + 2] + a.beta[j + 2]) + px.z) * dr.mul(st, (uint32_t)(o + 2));
    v.w = (((po.w - mu[3]) * rs[3] * a.gamma[j + 3] + a.beta[j + 3]) + px.w) * dr.mul(st, (uint32_t)(o + 3));
  }
  *reinterpret_cast<float4*>(a.dst + o) = v;
}

void fill_drop(const gtr_config* cfg, bool train_only, uint32_t& seed, uint32_t& thresh, float& scale, int& on,
               uint32_t& ctr_add, const uint32_t*& rng) {
  on = ((!train_only || cfg->training) && cfg->dropout > 0.0f) ? 1 : 0;
  const double p = cfg->dropout >= 1.0f ? 0.999999 : cfg->dropout;
  thresh = (uint32_t)(p * 4294967296.0);
  scale = on ? (float)(1.0 / (1.0 - p)) : 1.0f;
  seed = cfg->seed;
  ctr_add = (uint32_t)cfg->ctr_add;
  rng = cfg->rng_ctr;
}

template <int AL, int BL, int AT, int BT, int EP>
void launch_gemm(const GenK& k, int M_cap, int N, int chunks, hipStream_t s) {
  const dim3 grid((unsigned)((M_cap + GG_BM - 1) / GG_BM), (unsigned)((N + GG_BN - 1) / GG_BN), (unsigned)chunks);
  hipLaunchKernelGGL((k_gen_gemm<AL, BL, AT, BT, EP>), grid, dim3(GG_BLOCK), 0, s, k);
}

void launch_rows(int mode, const RowsK& k, int n_cap, hipStream_t s) {
  const dim3 grid((unsigned)(((int64_t)n_cap * (k.D / 4) + 255) / 256));
  switch (mode) {
    case RB_FIRST: hipLaunchKernelGGL(k_gen_rows<RB_FIRST>, grid, dim3(256), 0, s, k); break;
    case RB_FOLD: hipLaunchKernelGGL(k_gen_rows<RB_FOLD>, grid, dim3(256), 0, s, k); break;
    case RB_READY: hipLaunchKernelGGL(k_gen_rows<RB_READY>, grid, dim3(256), 0, s, k); break;
    default: hipLaunchKernelGGL(k_gen_rows<RB_G2>, grid, dim3(256), 0, s, k); break;
  }
}

// dX = dQKVS W_all + dy (or dy = (dz + da W1) * mask for the FFN backward): the GEMM with
// the GE_DX epilogue, then the previous layer's BatchNorm backward sums from the tiles'
// partial rows.
int gen_dx(const gtr_config* cfg, const gtr_batch* bt, const float* dq, int K, const float* w, const float* dy,
           float* out, int has_prev, int layer, const gtr_layer* prev, hipStream_t s) {
  const int D = cfg->dim;
  GenK k{};
  k.A = dq; k.B = w; k.C = out; k.M = bt->n_cap; k.N = D; k.K = K; k.lda = K; k.ldb = D; k.ldc = D;
  k.m_live = bt->hdr; k.res = dy; k.has_prev = has_prev; k.layer = layer;
  fill_drop(cfg, false, k.seed, k.thresh, k.scale, k.drop_on, k.ctr_add, k.rng_ctr);
  if (has_prev) {
    k.p_dy = prev->dy; k.p_out = prev->out; k.p_stats = prev->bn_stats; k.gpart = prev->bn_gpart;
  }
  launch_gemm<GA_MK, GB_KN, GT_NONE, GT_NONE, GE_DX>(k, bt->n_cap, D, 1, s);
  GTR_HIP_CHECK_LAUNCH();
  if (has_prev) {
    const int tiles = (bt->n_cap + GG_BM - 1) / GG_BM;
    hipLaunchKernelGGL(k_gen_colsum, dim3((unsigned)((2 * D + 255) / 256), 1), dim3(256), 0, s, prev->bn_gpart, tiles,
                       bt->hdr, 2 * D, (int64_t)2 * D, prev->bn_gsum, (int64_t)0, 1, GG_BM);
    GTR_HIP_CHECK_LAUNCH();
  }
  return GTR_OK;
}

}  // namespace

namespace gtr {

// ---- entry points used by gtr_gemm.hip for the shapes its register kernels do not cover

int gen_qkvs_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb, const gtr_layer* layers, int l,
                 hipStream_t s) {
  const int D = cfg->dim;
  const gtr_layer& L = layers[l];
  const bool ready = l > 0 && layers[l - 1].ffn;
  RowsK r{};
  r.bt = *bt; r.D = D; r.pe_k = cfg->pe_k; r.train = cfg->training; r.layer = l - 1; r.bn_eps = cfg->bn_eps;
  r.dst = L.xin;
  fill_drop(cfg, true, r.seed, r.thresh, r.scale, r.drop_on, r.ctr_add, r.rng_ctr);
  int mode;
  if (l == 0) {
    mode = RB_FIRST;
    r.table = emb->table; r.pe_tab = emb->pe_tab; r.wpe = emb->wpe; r.bpe = emb->bpe;
  } else if (ready) {
    mode = RB_READY;
    r.src = layers[l - 1].ffn->z;
  } else {
    mode = RB_FOLD;
    const gtr_layer& P = layers[l - 1];
    r.src = P.out; r.src2 = P.xin; r.stats = P.bn_stats; r.rmean = P.bn_rmean; r.rvar = P.bn_rvar;
    r.gamma = P.bn_gamma; r.beta = P.bn_beta;
  }
  launch_rows(mode, r, bt->n_cap, s);
  GTR_HIP_CHECK_LAUNCH();
  GenK k{};
  k.A = L.xin; k.B = L.w_all; k.C = L.qkvs; k.M = bt->n_cap; k.N = 4 * D; k.K = D; k.lda = D; k.ldb = D;
  k.ldc = 4 * D; k.m_live = bt->hdr; k.bias = L.b_all;
  launch_gemm<GA_MK, GB_NK, GT_NONE, GT_NONE, GE_BIAS>(k, bt->n_cap, 4 * D, 1, s);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gen_qkvs_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, float* dx0,
                 hipStream_t s) {
  const gtr_layer& L = layers[l];
  const bool ffn_prev = l > 0 && layers[l - 1].ffn;
  const bool has_prev = l > 0 && !ffn_prev;
  float* out = ffn_prev ? layers[l - 1].ffn->dz : dx0;
  return gen_dx(cfg, bt, L.dqkvs, 4 * cfg->dim, L.w_all, L.dy, out, has_prev ? 1 : 0, l,
                has_prev ? &layers[l - 1] : nullptr, s);
}

int gen_ffn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, hipStream_t s) {
  const int D = cfg->dim;
  const gtr_layer& L = layers[l];
  const gtr_ffn& f = *L.ffn;
  const int F = f.expansion * D;
  // y = dropout(BN(out) + xin) with layer l's statistics and output mask
  RowsK r{};
  r.bt = *bt; r.D = D; r.train = cfg->training; r.layer = l; r.bn_eps = cfg->bn_eps;
  r.src = L.out; r.src2 = L.xin; r.stats = L.bn_stats; r.rmean = L.bn_rmean; r.rvar = L.bn_rvar;
  r.gamma = L.bn_gamma; r.beta = L.bn_beta; r.dst = f.y;
  fill_drop(cfg, true, r.seed, r.thresh, r.scale, r.drop_on, r.ctr_add, r.rng_ctr);
  launch_rows(RB_FOLD, r, bt->n_cap, s);
  GTR_HIP_CHECK_LAUNCH();
  // a = y W1^T + b1
  GenK k{};
  k.A = f.y; k.B = f.w1; k.C = f.a; k.M = bt->n_cap; k.N = F; k.K = D; k.lda = D; k.ldb = D; k.ldc = F;
  k.m_live = bt->hdr; k.bias = f.b1;
  launch_gemm<GA_MK, GB_NK, GT_NONE, GT_NONE, GE_BIAS>(k, bt->n_cap, F, 1, s);
  GTR_HIP_CHECK_LAUNCH();
  // z = y + dropout(dropout(GELU(a)) W2^T + b2)
  GenK d{};
  d.A = f.a; d.B = f.w2; d.C = f.z; d.M = bt->n_cap; d.N = D; d.K = F; d.lda = F; d.ldb = F; d.ldc = D;
  d.m_live = bt->hdr; d.bias = f.b2; d.res = f.y; d.layer = l; d.tr_ld = F;
  fill_drop(cfg, true, d.seed, d.thresh, d.scale, d.drop_on, d.ctr_add, d.rng_ctr);
  launch_gemm<GA_MK, GB_NK, GT_GELU_MASK, GT_NONE, GE_FFN_DOWN>(d, bt->n_cap, D, 1, s);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gen_ffn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, hipStream_t s) {
  const int D = cfg->dim;
  const gtr_layer& L = layers[l];
  const gtr_ffn& f = *L.ffn;
  const int F = f.expansion * D;
  // g2 = dz * mask3
  RowsK r{};
  r.bt = *bt; r.D = D; r.layer = l; r.src = f.dz; r.dst = f.g2;
  fill_drop(cfg, false, r.seed, r.thresh, r.scale, r.drop_on, r.ctr_add, r.rng_ctr);
  launch_rows(RB_G2, r, bt->n_cap, s);
  GTR_HIP_CHECK_LAUNCH();
  // da = (g2 W2) * mask2 * GELU'(a): B[k = d][n = f] = W2[d][f]
  GenK k{};
  k.A = f.g2; k.B = f.w2; k.C = f.da; k.M = bt->n_cap; k.N = F; k.K = D; k.lda = D; k.ldb = F; k.ldc = F;
  k.m_live = bt->hdr; k.fa = f.a; k.layer = l;
  fill_drop(cfg, false, k.seed, k.thresh, k.scale, k.drop_on, k.ctr_add, k.rng_ctr);
  launch_gemm<GA_MK, GB_KN, GT_NONE, GT_NONE, GE_FFN_DH>(k, bt->n_cap, F, 1, s);
  GTR_HIP_CHECK_LAUNCH();
  // dy = (dz + da W1) * layer l's output mask -> layers[l].dy + its BatchNorm sums
  return gen_dx(cfg, bt, f.da, F, f.w1, f.dz, nullptr, 1, l + 1, &L, s);
}

// Weight gradients of one FFN block into slab chunk c (split-K over node rows):
// [dW1 F*D | db1 F | dW2 D*F | db2 D].
int gen_ffn_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l, float* slab,
                  int n_chunks, int64_t slab_stride, hipStream_t s) {
  const int D = cfg->dim;
  const gtr_ffn& f = *layers[l].ffn;
  const int F = f.expansion * D;
  // dW1[f][d] = sum_n da[n][f] y[n][d]: A = da^T (KM, lda F), B = y (KN, ldb D)
  GenK k{};
  k.A = f.da; k.B = f.y; k.C = slab; k.M = F; k.N = D; k.K = 0; k.lda = F; k.ldb = D; k.ldc = D;
  k.m_live = bt->hdr; k.k_live_from_hdr = 1; k.c_chunk_stride = slab_stride;
  launch_gemm<GA_KM, GB_KN, GT_NONE, GT_NONE, GE_STORE>(k, F, D, n_chunks, s);
  GTR_HIP_CHECK_LAUNCH();
  // dW2[d][f] = sum_n g2[n][d] h[n][f], h = dropout(GELU(a)): A = g2^T (KM, lda D), B = h (KN)
  GenK w{};
  w.A = f.g2; w.B = f.a; w.C = slab + (size_t)F * D + F; w.M = D; w.N = F; w.K = 0; w.lda = D; w.ldb = F;
  w.ldc = F; w.m_live = bt->hdr; w.k_live_from_hdr = 1; w.c_chunk_stride = slab_stride; w.layer = l; w.tr_ld = F;
  fill_drop(cfg, false, w.seed, w.thresh, w.scale, w.drop_on, w.ctr_add, w.rng_ctr);
  launch_gemm<GA_KM, GB_KN, GT_NONE, GT_GELU_MASK, GE_STORE>(w, D, F, n_chunks, s);
  GTR_HIP_CHECK_LAUNCH();
  // bias gradients per chunk: db1 = column sums of da, db2 of g2
  hipLaunchKernelGGL(k_gen_colsum, dim3((unsigned)((F + 255) / 256), (unsigned)n_chunks), dim3(256), 0, s, f.da,
                     0, bt->hdr, F, (int64_t)F, slab + (size_t)F * D, slab_stride, n_chunks, 1);
  hipLaunchKernelGGL(k_gen_colsum, dim3((unsigned)((D + 255) / 256), (unsigned)n_chunks), dim3(256), 0, s, f.g2,
                     0, bt->hdr, D, (int64_t)D, slab + (size_t)2 * F * D + F, slab_stride, n_chunks, 1);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

}  // namespace gtr
