// gtr_layer.cuh — geometry shared by the layer kernels (forward and backward).
//
// A layer kernel's workgroup owns one row group: every session whose first node lies
// in [g*R, (g+1)*R).  On the fast path (group rows <= RMAX, group edges <= EMAX) the
// group's CSR slices and K/V (forward) or K/V, Q, dA (backward) rows are staged in LDS
// so that the per-edge work of the attention never waits on HBM/L2; otherwise the
// same code runs against global memory (any session size, any dim).
#pragma once

#include "gtr_common.cuh"

#define CONV_BLOCK 512
#define CONV_WAVES (CONV_BLOCK / 64)

namespace gtr {

template <int D>
struct LayerGeom {
  static constexpr int VPL = D >= 64 ? D / 64 : 1;    // features per lane in row loops
  static constexpr int RMAX = D <= 64 ? 64 : (D == 128 ? 32 : 16);
  static constexpr bool KV = D <= 128;                 // K/V rows staged in LDS
  static constexpr int XS = D + 4;                     // padded LDS row (16B aligned)
  static constexpr int EMAX = 1024;                    // edges of a group staged in LDS
  static constexpr int KPE = 16;                       // LapPE width staged in LDS
  static constexpr int EH = 4096;                      // (edge, head) pairs of a group staged in LDS
  static constexpr int TPR = CONV_BLOCK / RMAX;        // threads per row in the row-parallel phases
  static constexpr int CH = D / TPR;                   // features per thread in those phases
  // ---- forward LDS carve (4-byte words); row arrays use the padded stride XS
  static constexpr int F_XO = 0;                              // [RMAX][XS]   X rows, then OUT rows
  static constexpr int F_KV = F_XO + RMAX * XS;               // [2][RMAX][XS] K rows | V rows
  static constexpr int F_QS = F_KV + (KV ? 2 * RMAX * XS : 0);// [2][RMAX][XS] Q rows | S rows
  static constexpr int F_PE = F_QS + (KV ? 2 * RMAX * XS : 0);// [D][KPE] Wpe | [RMAX][KPE] P rows
  static constexpr int F_LOG = F_PE + (D + RMAX) * KPE;       // [EH] logits -> alpha*mask; scratch
  static constexpr int F_BN = F_LOG + EH;                     // [2D] previous BN mean | rstd
  static constexpr int F_ITEMS = F_BN + 2 * D;                // [RMAX] node items
  static constexpr int F_IPTR = F_ITEMS + RMAX;               // [RMAX+1] local in_ptr
  static constexpr int F_ISRC = F_IPTR + RMAX + 4;            // [EMAX] local in_src
  static constexpr int F_EDST = F_ISRC + EMAX;                // [EMAX] local dst of each in-edge
  static constexpr int F_FLAG = F_EDST + EMAX;
  static constexpr int XSB = D + 8;                           // padded bf16 row (16B aligned)
  static constexpr int F_XH = F_FLAG + 4;                     // [RMAX][XSB] bf16 hi part of X rows
  static constexpr int F_XL = F_XH + RMAX * XSB / 2;          // [RMAX][XSB] bf16 lo part (split GEMM)
  static constexpr int F_WB = F_XL + RMAX * XSB / 2;          // [3D] gate weights w_beta (fast path)
  static constexpr int F_WORDS = F_WB + 3 * D;
  // ---- backward LDS carve (4-byte words)
  static constexpr int B_RN = KV ? 4 * RMAX * XS : 0;
  static constexpr int B_R = 0;                               // [4][RMAX][XS] K | V | Q | dA rows
  static constexpr int B_AL = B_R + B_RN;                     // [EH] alpha -> alpha * mask
  static constexpr int B_DL = B_AL + EH;                      // [EH] da -> dlogit
  static constexpr int B_IPTR = B_DL + EH;                    // [RMAX+1] local in_ptr
  static constexpr int B_ISRC = B_IPTR + RMAX + 4;            // [EMAX] local in_src
  static constexpr int B_EDST = B_ISRC + EMAX;                // [EMAX] local dst of each in-edge
  static constexpr int B_OPTR = B_EDST + EMAX;                // [RMAX+1] local out_ptr
  static constexpr int B_OEDGE = B_OPTR + RMAX + 4;           // [EMAX] local dst-order position
  static constexpr int B_ODST = B_OEDGE + EMAX;               // [EMAX] local dst row
  static constexpr int B_GS = B_ODST + EMAX;                  // [2D] reduced BN backward sums
  static constexpr int B_BNP = B_GS + 2 * D;                  // [CONV_WAVES][2D] dX-epilogue BN partials
  static constexpr int B_DU = B_BNP + CONV_WAVES * 2 * D;    // [RMAX] du of the group's rows (fast path)
  static constexpr int B_FLAG = B_DU + RMAX;
  static constexpr int B_WORDS = B_FLAG + 4;
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Split-bf16 GEMM operands: x = hi + lo with hi = bf16(x), lo = bf16(x - hi), so that
// hi*hi' + hi*lo' + lo*hi' (three bf16 MFMAs, fp32 accumulation) carries ~16 bits of
// each product (relative error ~2^-16) at 3/16 of the f32-input MFMA cycles.
__device__ __forceinline__ void split4(const float4 v, bf16x4& h, bf16x4& l) {
  h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
  l[0] = (__bf16)(v.x - (float)h[0]); l[1] = (__bf16)(v.y - (float)h[1]);
  l[2] = (__bf16)(v.z - (float)h[2]); l[3] = (__bf16)(v.w - (float)h[3]);
}
__device__ __forceinline__ void split8(const float4 a, const float4 b, bf16x8& h, bf16x8& l) {
  bf16x4 ha, la, hb, lb;
  split4(a, ha, la);
  split4(b, hb, lb);
  h = __builtin_shufflevector(ha, hb, 0, 1, 2, 3, 4, 5, 6, 7);
  l = __builtin_shufflevector(la, lb, 0, 1, 2, 3, 4, 5, 6, 7);
}
// acc += A*B for one 16x16x32 step from split operands (small terms first).
__device__ __forceinline__ f32x4 mfma_split(const bf16x8 ah, const bf16x8 al, const bf16x8 bh, const bf16x8 bl,
                                            f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// One 16x16 f32 MFMA tile-step over 4 k values held as float4 by each lane.
__device__ __forceinline__ f32x4 mfma4(const float4 a, const float4 b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

// LapPE projection of four pe values k..k+3 into a thread's four output columns j..j+3:
// w points at W_pe^T[k][j] in LDS (k-major, row stride `ld`).  Explicit fmas in k order, so
// every kernel that projects the PE rows (k_conv_fwd, k_proj) rounds identically.
__device__ __forceinline__ void pe_fma4(float (&acc)[4], const float4 p4, const float* w, int ld) {
  const float4 w0 = *reinterpret_cast<const float4*>(w);
  const float4 w1 = *reinterpret_cast<const float4*>(w + ld);
  const float4 w2 = *reinterpret_cast<const float4*>(w + 2 * ld);
  const float4 w3 = *reinterpret_cast<const float4*>(w + 3 * ld);
  const float wq[4][4] = {{w0.x, w1.x, w2.x, w3.x}, {w0.y, w1.y, w2.y, w3.y},
                          {w0.z, w1.z, w2.z, w3.z}, {w0.w, w1.w, w2.w, w3.w}};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc[q] = __builtin_fmaf(p4.x, wq[q][0], acc[q]);
    acc[q] = __builtin_fmaf(p4.y, wq[q][1], acc[q]);
    acc[q] = __builtin_fmaf(p4.z, wq[q][2], acc[q]);
    acc[q] = __builtin_fmaf(p4.w, wq[q][3], acc[q]);
  }
}

template <int VPL>
__device__ __forceinline__ void load_vec(float (&x)[VPL], const float* p, bool act) {
  if constexpr (VPL == 4) {
    float4 t = act ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
    x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
  } else if constexpr (VPL == 2) {
    float2 t = act ? *reinterpret_cast<const float2*>(p) : make_float2(0.f, 0.f);
    x[0] = t.x; x[1] = t.y;
  } else {
    x[0] = act ? p[0] : 0.0f;
  }
}

template <int VPL>
__device__ __forceinline__ void store_vec(float* p, const float (&x)[VPL], bool act) {
  if (!act) return;
  if constexpr (VPL == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  } else if constexpr (VPL == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
  } else {
    p[0] = x[0];
  }
}

// Combine G per-group (count, mean, M2) partials (rows `rstride` floats apart) in
// fixed order (deterministic): BLK/D slices of the groups are folded in parallel (Chan's
// parallel-variance formula), then the slices are combined.  Two uses, one helper each
// below, so that the modes cannot be mixed at a call site:
//   bn_stats_from_parts  -> mean / rstd / unbiased var in LDS (s_mean, s_rstd, s_uvar);
//   bn_merge_parts       -> ONE merged (count, mean, M2) row written to `merged`, which
//                           may alias the first partial row (every read of the partials
//                           completes before the internal __syncthreads that precedes
//                           the write); s_mean / s_rstd / s_uvar are not written.
// After a forward with more than GTR_PART_BUCKET row groups (the last-arriver mode,
// consumer_reduce = 0), gtr_layer.bn_part row b*GTR_PART_BUCKET therefore holds bucket
// b's MERGED row, not group b*GTR_PART_BUCKET's partial: nothing may re-read bn_part
// as per-group partials after such a forward.
// The first QR partial rows of each slice, loaded whole (count, mean, M2) into registers
// by bn_parts_load -- which a caller may issue early, before loads whose wait it must not
// join (vector loads retire in order) -- and kept for both passes of bn_fold_parts_ (same
// summation order as re-reading them).
// QR covers a whole GTR_PART_BUCKET of rows per slice up to 16 rows (3 x 16 VGPRs): a
// bucket merge at 2 slices is then ONE round of loads, and past QR the loops keep 16 in
// flight (the same order of additions either way).
template <int D, int BLK>
struct BnParts {
  static constexpr int NSL = BLK / D >= 1 ? BLK / D : 1;
  static constexpr int QR = (32 + NSL - 1) / NSL < 16 ? (32 + NSL - 1) / NSL : 16;
  float rc[QR], rmu[QR], rm2[QR];
};

template <int D, int BLK>
__device__ __forceinline__ void bn_parts_load(const float* part, int G, size_t rstride, BnParts<D, BLK>& r) {
  constexpr int NSL = BnParts<D, BLK>::NSL, QR = BnParts<D, BLK>::QR;
  const int tid = threadIdx.x;
  const int j = tid % D, sl = tid / D;
  if (sl < NSL) {
#pragma unroll
    for (int u = 0; u < QR; ++u) {
      const int q = sl + u * NSL;
      if (q < G) {
        const float* pp = part + (size_t)q * rstride;
        r.rc[u] = pp[0];
        r.rmu[u] = pp[1 + j];
        r.rm2[u] = pp[1 + D + j];
      }
    }
  }
}

// scr: >= 2*BLK + D floats of LDS.  Call with the whole block, after bn_parts_load.
// Three barriers: each slice thread forms the slice totals itself (same order as one
// thread per feature would), so the mean needs no LDS round of its own; the count of a
// slice is the same for every feature and is kept once per slice.
template <int D, int BLK>
__device__ __forceinline__ void bn_fold_parts_(const float* part, int G, float eps, float* s_mean,
                                               float* s_rstd, float* s_uvar, float* scr, size_t rstride,
                                               float* merged, const BnParts<D, BLK>& r, bool wt = false) {
  constexpr int NSL = BnParts<D, BLK>::NSL, QR = BnParts<D, BLK>::QR;
  const int tid = threadIdx.x;
  const int j = tid % D, sl = tid / D;
  float* s_sum = scr;              // [NSL][D]
  float* s_m2 = scr + NSL * D;     // [NSL][D]
  float* s_n = scr + 2 * NSL * D;  // [NSL] (a slice's count)
  if (sl < NSL) {
    float n = 0.0f, sum = 0.0f;
#pragma unroll
    for (int u = 0; u < QR; ++u)
      if (sl + u * NSL < G) {
        n += r.rc[u];
        sum += r.rc[u] * r.rmu[u];
      }
#pragma unroll 16
    for (int q = sl + QR * NSL; q < G; q += NSL) {
      const float* pp = part + (size_t)q * rstride;
      const float c = pp[0];
      n += c;
      sum += c * pp[1 + j];
    }
    s_sum[sl * D + j] = sum;
    if (j == 0) s_n[sl] = n;
  }
  __syncthreads();
  float n_tot = 0.0f, mean = 0.0f;
  if (sl < NSL) {
    float sum = 0.0f;
    for (int q = 0; q < NSL; ++q) { n_tot += s_n[q]; sum += s_sum[q * D + j]; }
    mean = n_tot > 0.0f ? sum / n_tot : 0.0f;  // a bucket of empty groups merges to (0, 0, 0)
    float m2 = 0.0f;
#pragma unroll
    for (int u = 0; u < QR; ++u)
      if (sl + u * NSL < G) {
        const float d = r.rmu[u] - mean;
        m2 += r.rm2[u] + r.rc[u] * d * d;
      }
#pragma unroll 16
    for (int q = sl + QR * NSL; q < G; q += NSL) {
      const float* pp = part + (size_t)q * rstride;
      const float d = pp[1 + j] - mean;
      m2 += pp[1 + D + j] + pp[0] * d * d;
    }
    s_m2[sl * D + j] = m2;
  }
  __syncthreads();
  if (tid < D) {  // slice 0's threads: tid == j, n_tot and mean already formed
    float m2 = 0.0f;
    for (int q = 0; q < NSL; ++q) m2 += s_m2[q * D + tid];
    if (merged && wt) {  // written through: read on another XCD after arrive_last_wt
      st_wt(merged + 1 + tid, mean);
      st_wt(merged + 1 + D + tid, m2);
      if (tid == 0) st_wt(merged, n_tot);
    } else if (merged) {  // the G partials combined into one (count, mean, M2) row (may alias row 0)
      merged[1 + tid] = mean;
      merged[1 + D + tid] = m2;
      if (tid == 0) merged[0] = n_tot;
    } else {
      const float var = m2 / n_tot;
      s_mean[tid] = mean;
      s_rstd[tid] = 1.0f / sqrtf(var + eps);
      s_uvar[tid] = n_tot > 1.0f ? m2 / (n_tot - 1.0f) : var;
    }
  }
  __syncthreads();
}

template <int D, int BLK>
__device__ __forceinline__ void bn_stats_from_parts(const float* part, int G, float eps, float* s_mean,
                                                    float* s_rstd, float* s_uvar, float* scr,
                                                    size_t rstride = 1 + 2 * D) {
  BnParts<D, BLK> r;
  bn_parts_load<D, BLK>(part, G, rstride, r);
  bn_fold_parts_<D, BLK>(part, G, eps, s_mean, s_rstd, s_uvar, scr, rstride, nullptr, r);
}

// The same with the partial rows already requested by bn_parts_load.
template <int D, int BLK>
__device__ __forceinline__ void bn_stats_from_loaded(const float* part, int G, float eps, float* s_mean,
                                                     float* s_rstd, float* s_uvar, float* scr,
                                                     const BnParts<D, BLK>& r, size_t rstride = 1 + 2 * D) {
  bn_fold_parts_<D, BLK>(part, G, eps, s_mean, s_rstd, s_uvar, scr, rstride, nullptr, r);
}

template <int D, int BLK>
__device__ __forceinline__ void bn_merge_parts(const float* part, int G, float* scr, size_t rstride,
                                               float* merged, bool wt = false) {
  BnParts<D, BLK> r;
  bn_parts_load<D, BLK>(part, G, rstride, r);
  bn_fold_parts_<D, BLK>(part, G, 0.0f, nullptr, nullptr, nullptr, scr, rstride, merged, r, wt);
}

// Row groups whose partials one last-arriving workgroup combines; past that the groups
// are bucketed: each bucket's last arriver merges its partials into the bucket's first
// row, and the last bucket merger combines the bucket rows (two short reductions
// instead of one pass over hundreds of partial rows).
#define GTR_PART_BUCKET 32

// Dynamic LDS above 64 KiB needs the per-kernel limit raised once (gfx950: 160 KiB per CU).
template <int D, typename K>
inline void set_lds_limit(K kernel, size_t bytes) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    done = true;
  }
}

}  // namespace gtr
