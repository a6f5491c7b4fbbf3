// gtr_eval.hip — full-catalog scoring + top-k of GraphTransformer.predict
// (base.py:59-78: scores = se @ W^T, torch.topk(scores, k)) for Trainer.evaluate
// (trainer.py:138-173: Recall@K / NDCG@K over the validation sessions).
//
// Two stages, no [B, T] score matrix in HBM:
//   k_topk_chunk: workgroup = (256-row table chunk) x (16*NSW sessions).  Each wave owns 16
//     sessions and computes their scores against the chunk with v_mfma_f32_16x16x4f32
//     (fp32 in, fp32 accumulate: the [B,d]x[d,T] product is a real dense GEMM), the scores
//     stay in registers (lane = one table row of each 16-row tile, 4 sessions per lane),
//     and the chunk's top-k of every session is selected by iterated 16-lane argmax.
//   k_topk_merge: 4096 candidates per workgroup -> top-k (repeated until one group is left).
// Candidates are 64-bit keys (order-preserving score bits << 32 | ~row): the order is
// score descending, then row ascending, so the result is deterministic and ties resolve
// to the lower item id.  A NaN score ranks above +inf, as in torch.topk.

#include "gtr_common.cuh"
#include "gtr_layer.cuh"

namespace {

using namespace gtr;

#define TK_CH 256       // table rows per stage-1 chunk (16 MFMA tiles of 16 rows)
#define TK_MERGE 4096   // candidates per stage-2 workgroup (4 waves x 64 lanes x 16)
#define TK_KMAX 128

__device__ __forceinline__ uint32_t ord_f32(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float f32_ord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

__device__ __forceinline__ uint64_t make_key(float s, int row) {
  return ((uint64_t)ord_f32(s) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)row);
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)x, m), hi = __shfl_xor((uint32_t)(x >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

// Iterated argmax over the NV keys of each lane inside aligned groups of W lanes:
// emit(j, key) is called by every lane with the group's j-th largest key (0 = exhausted).
template <int NV, int W, typename F>
__device__ __forceinline__ void group_topk(uint64_t (&key)[NV], int k, F&& emit) {
  for (int j = 0; j < k; ++j) {
    uint64_t b = key[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) b = key[v] > b ? key[v] : b;
#pragma unroll
    for (int o = 1; o < W; o <<= 1) {
      const uint64_t t = shfl_xor_u64(b, o);
      b = t > b ? t : b;
    }
    emit(j, b);
#pragma unroll
    for (int v = 0; v < NV; ++v) key[v] = key[v] == b ? 0ull : key[v];
  }
}

// Stage 1.  blockIdx.x = chunk (rows [c*TK_CH, +TK_CH)), blockIdx.y = session group.
// out: cand[(b * nchunk + c) * k + j].
// excl_ptr / excl_ids (optional): per-session sorted item ids that may not be returned
// (serving: the session's own items and the padding row, recommender.py:128-129).
template <int D, int NSW>
__global__ __launch_bounds__(64 * NSW) void k_topk_chunk(const float* __restrict__ se, int B,
                                                         const float* __restrict__ table, int T, int k,
                                                         int nchunk, uint64_t* __restrict__ cand,
                                                         const int32_t* __restrict__ excl_ptr,
                                                         const int32_t* __restrict__ excl_ids) {
  constexpr int KC = D / 16;
  constexpr int NT = TK_CH / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int c = blockIdx.x;
  const int s0 = (blockIdx.y * NSW + wave) * 16;
  if (s0 >= B) return;  // whole wave idle (no barriers below)
  const int r0 = c * TK_CH;
  // A operand: session s0 + lr, k values kc*16 + lg*4 .. +3
  float4 af[KC];
  {
    const bool ok = s0 + lr < B;
    const float* p = se + (size_t)(s0 + lr) * D + lg * 4;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      af[kc] = ok ? *reinterpret_cast<const float4*>(p + kc * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // scores: sc[t][i] = score(session s0 + lg*4 + i, row r0 + t*16 + lr)
  f32x4 sc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int row = r0 + t * 16 + lr;
    const bool ok = row < T;
    const float* p = table + (size_t)(ok ? row : 0) * D + lg * 4;
    float4 bf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      bf[kc] = ok ? *reinterpret_cast<const float4*>(p + kc * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) acc = mfma4(af[kc], bf[kc], acc);
    sc[t] = acc;
  }
  // top-k per session: the 16 lanes of group lg hold session s0 + lg*4 + i (16 rows each)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = s0 + lg * 4 + i;
    uint64_t key[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = r0 + t * 16 + lr;
      key[t] = row < T ? make_key(sc[t][i], row) : 0ull;
    }
    if (excl_ptr && s < B) {
      const int e0 = excl_ptr[s], e1 = excl_ptr[s + 1];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int row = r0 + t * 16 + lr;
        int lo = e0, hi = e1;  // sorted ids: binary search
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (excl_ids[mid] < row) lo = mid + 1; else hi = mid;
        }
        if (lo < e1 && excl_ids[lo] == row) key[t] = 0ull;
      }
    }
    uint64_t* out = cand + ((size_t)s * nchunk + c) * k;
    const bool wr = s < B && lr == 0;
    group_topk<NT, 16>(key, k, [&](int j, uint64_t b) {
      if (wr) out[j] = b;
    });
  }
}

// Stage 2.  blockIdx.x = candidate group g (TK_MERGE keys), blockIdx.y = session.
// in: [B][M]; out keys [B][ngrp][k], or (final) out_idx/out_score [B][k].
__global__ __launch_bounds__(256) void k_topk_merge(const uint64_t* __restrict__ in, int M, int k, int ngrp,
                                                    uint64_t* __restrict__ out, int64_t* __restrict__ out_idx,
                                                    float* __restrict__ out_score) {
  __shared__ uint64_t s_k[4][TK_KMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x, b = blockIdx.y;
  const uint64_t* src = in + (size_t)b * M;
  const int base = g * TK_MERGE + wave * (TK_MERGE / 4);
  uint64_t key[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int q = base + v * 64 + lane;
    key[v] = q < M ? src[q] : 0ull;
  }
  group_topk<16, 64>(key, k, [&](int j, uint64_t kb) {
    if (lane == 0) s_k[wave][j] = kb;
  });
  __syncthreads();
  if (wave != 0) return;
  uint64_t k2[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    const int q = v * 64 + lane;  // q = w * k + j over the 4 waves' lists
    k2[v] = q < 4 * k ? s_k[q / k][q % k] : 0ull;
  }
  const bool fin = out == nullptr;
  group_topk<8, 64>(k2, k, [&](int j, uint64_t kb) {
    if (lane != 0) return;
    if (fin) {
      const uint32_t row = 0xFFFFFFFFu - (uint32_t)kb;
      out_idx[(size_t)b * k + j] = kb ? (int64_t)row : (int64_t)-1;
      out_score[(size_t)b * k + j] = kb ? f32_ord((uint32_t)(kb >> 32)) : -INFINITY;
    } else {
      out[((size_t)b * ngrp + g) * k + j] = kb;
    }
  });
}

int nchunks(int T) { return (T + TK_CH - 1) / TK_CH; }

}  // namespace

extern "C" int gtr_topk_workspace_bytes(int B, int num_items, int k, size_t* bytes) {
  if (!bytes || B <= 0 || num_items <= 0 || k <= 0 || k > TK_KMAX || k > num_items) {
    set_error("gtr_topk_workspace_bytes: bad arguments (B=%d T=%d k=%d, k <= %d)", B, num_items, k, TK_KMAX);
    return GTR_E_ARG;
  }
  const size_t m0 = (size_t)nchunks(num_items) * k;
  const size_t m1 = ((m0 + TK_MERGE - 1) / TK_MERGE) * k;
  *bytes = (size_t)B * (m0 + m1) * sizeof(uint64_t);
  return GTR_OK;
}

extern "C" int gtr_score_topk_masked(const float* se, int B, int dim, const float* table, int num_items, int k,
                                     const int32_t* excl_ptr, const int32_t* excl_ids, int64_t* out_idx,
                                     float* out_score, void* ws, size_t ws_bytes, gtr_stream_t stream);

extern "C" int gtr_score_topk(const float* se, int B, int dim, const float* table, int num_items, int k,
                              int64_t* out_idx, float* out_score, void* ws, size_t ws_bytes,
                              gtr_stream_t stream) {
  return gtr_score_topk_masked(se, B, dim, table, num_items, k, nullptr, nullptr, out_idx, out_score, ws,
                               ws_bytes, stream);
}

extern "C" int gtr_score_topk_masked(const float* se, int B, int dim, const float* table, int num_items, int k,
                                     const int32_t* excl_ptr, const int32_t* excl_ids, int64_t* out_idx,
                                     float* out_score, void* ws, size_t ws_bytes, gtr_stream_t stream) {
  if ((excl_ptr == nullptr) != (excl_ids == nullptr)) {
    set_error("gtr_score_topk_masked: excl_ptr and excl_ids go together");
    return GTR_E_ARG;
  }
  size_t need = 0;
  if (int e = gtr_topk_workspace_bytes(B, num_items, k, &need)) return e;
  if (!se || !table || !out_idx || !out_score || !ws || ws_bytes < need) {
    set_error("gtr_score_topk: bad arguments (workspace %zu < %zu bytes?)", ws_bytes, need);
    return GTR_E_ARG;
  }
  if (!(dim == 32 || dim == 64 || dim == 128 || dim == 256)) {
    set_error("gtr_score_topk: dim %d unsupported (32/64/128/256)", dim);
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nc = nchunks(num_items);
  const size_t m0 = (size_t)nc * k;
  uint64_t* buf0 = reinterpret_cast<uint64_t*>(ws);
  uint64_t* buf1 = buf0 + (size_t)B * m0;
  const int nsw = B > 32 ? 4 : (B > 16 ? 2 : 1);
  const dim3 g1(nc, (B + 16 * nsw - 1) / (16 * nsw));
#define TK_LAUNCH(DD, NS) hipLaunchKernelGGL((k_topk_chunk<DD, NS>), g1, dim3(64 * NS), 0, s, se, B, table, \
                                             num_items, k, nc, buf0, excl_ptr, excl_ids)
#define TK_DIM(DD)                                  \
  if (nsw == 4) TK_LAUNCH(DD, 4);                   \
  else if (nsw == 2) TK_LAUNCH(DD, 2);              \
  else TK_LAUNCH(DD, 1);
  switch (dim) {
    case 32: TK_DIM(32) break;
    case 64: TK_DIM(64) break;
    case 128: TK_DIM(128) break;
    default: TK_DIM(256) break;
  }
#undef TK_DIM
#undef TK_LAUNCH
  GTR_HIP_CHECK_LAUNCH();
  // merge passes: [B][M] -> [B][ceil(M / TK_MERGE) * k] until one group remains
  const uint64_t* cur = buf0;
  uint64_t* nxt = buf1;
  size_t M = m0;
  while (true) {
    const int ngrp = (int)((M + TK_MERGE - 1) / TK_MERGE);
    if (ngrp == 1) {
      hipLaunchKernelGGL(k_topk_merge, dim3(1, B), dim3(256), 0, s, cur, (int)M, k, 1, (uint64_t*)nullptr,
                         out_idx, out_score);
      GTR_HIP_CHECK_LAUNCH();
      break;
    }
    hipLaunchKernelGGL(k_topk_merge, dim3(ngrp, B), dim3(256), 0, s, cur, (int)M, k, ngrp, nxt,
                       (int64_t*)nullptr, (float*)nullptr);
    GTR_HIP_CHECK_LAUNCH();
    M = (size_t)ngrp * k;
    const uint64_t* done = cur;
    cur = nxt;
    nxt = const_cast<uint64_t*>(done);
  }
  return GTR_OK;
}
