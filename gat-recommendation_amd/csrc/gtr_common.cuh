// gtr_common.cuh — shared device helpers for the gfx950 GraphTransformer kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/gtr.h"

#define GTR_BLOCK 256
#define GTR_WAVES (GTR_BLOCK / 64)

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace gtr {

void set_error(const char* fmt, ...);

// A global array as a raw buffer (MUBUF, hardware bounds check): loads past `bytes` return
// zero and stores past it are dropped, with no branch.  Used where a per-lane condition
// would otherwise put a load or store under an exec-skipping branch: the compiler cannot
// count a memory op that may not have issued, so the next wait on a load issued before it
// becomes vmcnt(0) -- which also waits for every later load and store in flight.
struct Buf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Buf(const void* p, uint64_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                            (int)(uint32_t)(bytes < 0xFFFFFFFFull ? bytes : 0xFFFFFFFFull),
                                            0x00020000)) {}
  __device__ __forceinline__ float4 ld4(uint32_t off) const {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  }
  __device__ __forceinline__ int ld_i32(uint32_t off) const {
    return (int)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
  }
  __device__ __forceinline__ void st4(uint32_t off, float4 v) const {
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, (int)off, 0, 0);
  }
};

// Cross-lane butterflies without the LDS crossbar.  Step O of an ASCENDING butterfly
// (offsets 1, 2, 4, ...) combines each lane with its xor-O partner:
//  - O = 1, 2: DPP quad_perm, an exact xor permutation inside a quad;
//  - O = 4, 8: every lane of an aligned O-group already holds the same value, so the
//    mirrors inside 8 / 16 lanes (DPP row_half_mirror / row_mirror) deliver the xor
//    partner's value;
//  - O = 16, 32: gfx950's v_permlane16_swap / v_permlane32_swap exchange the odd rows
//    (upper half) of one copy with the even rows (lower half) of another, so a
//    commutative op over the two swapped copies gives every lane op(x[l], x[l^O]).
// All VALU work, bitwise what the __shfl_xor (ds_bpermute through LDS) butterfly gives.
// The swaps are inline asm: the builtin folds its two outputs into one when both
// operands carry the same value (measured: v_add_f32 vN, vN, vN).  The s_nop pairs
// cover the VALU-write -> permlane-read hazards the compiler cannot see inside asm.
template <int O>
__device__ __forceinline__ float dpp_partner(float x) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8, "DPP butterfly offset");
  constexpr int CTRL = O == 1 ? 0xB1 : O == 2 ? 0x4E : O == 4 ? 0x141 : 0x140;
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

template <int O>
__device__ __forceinline__ void swap_halves(float& a, float& b) {
  static_assert(O == 16 || O == 32, "permlane swap offset");
  if constexpr (O == 16)
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
}

template <int O>
__device__ __forceinline__ float bfly_add(float x) {
  if constexpr (O <= 8) {
    return x + dpp_partner<O>(x);
  } else {
    float a = x, b = x;
    swap_halves<O>(a, b);
    return a + b;
  }
}

template <int O>
__device__ __forceinline__ float bfly_max(float x) {
  if constexpr (O <= 8) {
    return fmaxf(x, dpp_partner<O>(x));
  } else {
    float a = x, b = x;
    swap_halves<O>(a, b);
    return fmaxf(a, b);
  }
}

// Inclusive prefix sum of an integer over the wave's 64 lanes in DPP steps (VALU only, no
// LDS round trip per step): row_shr 1 / 2 / 4 / 8 inside each row of 16 (out-of-row lanes
// read 0), then row_bcast:15 (lane 15 of row r into rows 1 and 3) and row_bcast:31 (lane
// 31 into rows 2 and 3).  Integer sums: exact in any order.
__device__ __forceinline__ int wave_incl_scan_dpp(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Ascending butterfly sum over aligned groups of G lanes (G a compile-time power of two).
template <int G>
__device__ __forceinline__ float group_sum_c(float x) {
  if constexpr (G > 1) x = bfly_add<1>(x);
  if constexpr (G > 2) x = bfly_add<2>(x);
  if constexpr (G > 4) x = bfly_add<4>(x);
  if constexpr (G > 8) x = bfly_add<8>(x);
  if constexpr (G > 16) x = bfly_add<16>(x);
  if constexpr (G > 32) x = bfly_add<32>(x);
  return x;
}

template <int G>
__device__ __forceinline__ float group_max_c(float x) {
  if constexpr (G > 1) x = bfly_max<1>(x);
  if constexpr (G > 2) x = bfly_max<2>(x);
  if constexpr (G > 4) x = bfly_max<4>(x);
  if constexpr (G > 8) x = bfly_max<8>(x);
  if constexpr (G > 16) x = bfly_max<16>(x);
  if constexpr (G > 32) x = bfly_max<32>(x);
  return x;
}

__device__ __forceinline__ float wave_sum(float x) { return group_sum_c<64>(x); }
__device__ __forceinline__ float wave_max(float x) { return group_max_c<64>(x); }

// Sum inside aligned groups of `gl` lanes (gl a power of two <= 64; wave-uniform).
__device__ __forceinline__ float group_sum(float x, int gl) {
  if (gl > 1) x = bfly_add<1>(x);
  if (gl > 2) x = bfly_add<2>(x);
  if (gl > 4) x = bfly_add<4>(x);
  if (gl > 8) x = bfly_add<8>(x);
  if (gl > 16) x = bfly_add<16>(x);
  if (gl > 32) x = bfly_add<32>(x);
  return x;
}

// Max inside aligned groups of `gl` lanes (gl a power of two <= 64; wave-uniform).
__device__ __forceinline__ float group_max(float x, int gl) {
  if (gl > 1) x = bfly_max<1>(x);
  if (gl > 2) x = bfly_max<2>(x);
  if (gl > 4) x = bfly_max<4>(x);
  if (gl > 8) x = bfly_max<8>(x);
  if (gl > 16) x = bfly_max<16>(x);
  if (gl > 32) x = bfly_max<32>(x);
  return x;
}

// Lanes per (destination row, head) pair of a row group's segmented softmax passes: the
// widest power of two <= 64 that keeps every pair of the group in one round of `blk`
// threads (the in-edges of a pair are strided over its lanes, reduced by shuffles).
__device__ __forceinline__ int pair_lanes(int pairs, int blk) {
  int gl = 64;
  while (gl > 1 && gl * pairs > blk) gl >>= 1;
  return gl;
}

// The same, but no wider than the group's mean in-degree rounded up to a power of two:
// every lane beyond a pair's edge count only adds shuffle rounds (each a cross-lane LDS
// permute) to the max / sum, while a hub row's few lanes loop over its edges.
__device__ __forceinline__ int pair_lanes_deg(int pairs, int blk, int edges, int rows) {
  const int deg = rows > 0 ? (edges + rows - 1) / rows : 1;
  int gl = 1;
  while (gl < deg && gl < 64) gl <<= 1;
  const int cap = pair_lanes(pairs, blk);
  return gl < cap ? gl : cap;
}

// Counter-based dropout stream: one 32-bit hash per (seed, stream, element).
__device__ __forceinline__ uint32_t mix3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u;
  h ^= b + 0x7F4A7C15u + (h << 6) + (h >> 2);
  h *= 0x85EBCA77u;
  h ^= c * 0xC2B2AE3Du;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

// kind 0: attention-probability dropout of layer l; kind 1: layer-output dropout.
__device__ __forceinline__ uint32_t drop_stream(uint32_t kind, uint32_t layer, uint32_t ctr) {
  return (kind << 28) ^ (layer << 20) ^ (ctr * 0x632BE5ABu);
}

// The step's dropout counter, read through the scalar (constant) path: it is written only
// by the step tail / counter kernels, never during the kernels that read it, and a scalar
// load waits on its own counter (lgkmcnt) instead of joining the in-order vector-load queue
// ahead of the staging loads.
__device__ __forceinline__ uint32_t load_step_ctr(const uint32_t* p) {
  return *(const __attribute__((address_space(4))) uint32_t*)p;
}

struct Drop {
  uint32_t seed, thresh;
  float scale;
  bool on;
  __device__ __forceinline__ float mul(uint32_t stream, uint32_t idx) const {
    if (!on) return 1.0f;
    return mix3(seed, stream, idx) >= thresh ? scale : 0.0f;
  }
};

__device__ __forceinline__ int lower_bound_i32(const int32_t* a, int n, int v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// First s in [0, B) with a[s] >= v (B if none), a non-decreasing; wave-cooperative
// 64-ary search: one round of 64 parallel loads per 64x narrowing (1 round for B <= 64).
__device__ __forceinline__ int wave_lower_bound(const int32_t* a, int B, int v) {
  const int lane = threadIdx.x & 63;
  int lo = 0, hi = B;
  while (hi - lo > 64) {
    const int step = (hi - lo + 63) >> 6;
    const int idx = lo + lane * step;
    const int val = idx < hi ? a[idx] : 0x7FFFFFFF;
    const int c = __popcll(__ballot(val < v));
    const int nlo = c > 0 ? lo + (c - 1) * step + 1 : lo;
    const int nhi = min(hi, lo + c * step);
    lo = nlo;
    hi = nhi;
  }
  const int idx = lo + lane;
  const int val = idx < hi ? a[idx] : 0x7FFFFFFF;
  return lo + __popcll(__ballot(val < v));
}

// Rows [r0, r1) of row-group g: all sessions whose first node lies in [g*R, (g+1)*R).
// Must be called by every lane of a wave (ballot); every wave gets the same answer.
__device__ __forceinline__ void group_rows(const int32_t* node_ptr, int B, int R, int g, int& r0, int& r1) {
  const int s0 = wave_lower_bound(node_ptr, B, g * R);
  const int s1 = wave_lower_bound(node_ptr, B, (g + 1) * R);
  r0 = node_ptr[s0];
  r1 = node_ptr[s1];
}

// XCD-packed block roles (speed only, never correctness): hardware blocks b and b + 8
// share an XCD under the round-robin dispatch, so with `pack` the launch's M main
// workgroups (row groups / readout sessions) run on blocks 0, 8, 16, ...: they then share
// one XCD's L2 for the layer's weights (fetched once, not once per XCD) and for the rows
// they exchange; the extra workgroups (sweep slices, fused begin) take the other blocks.
// Returns the ROLE index: [0, M) main, [M, gridDim.x) extra.  Host: pack only when
// 8 * (M - 1) < gridDim.x (gtr::xcd_pack).
__device__ __forceinline__ int role_block(int M, int pack) {
  const int b = blockIdx.x;
  if (!pack) return b;
  if ((b & 7) == 0 && (b >> 3) < M) return b >> 3;
  return M + b - min(M, (b + 7) >> 3);
}

// Last-arriver election across the workgroups of one launch (placement independent:
// plain stores -> every wave drains -> barrier -> lane-0 agent release -> counter;
// the last arriver does an agent acquire before reading the other groups' partials).
__device__ __forceinline__ bool arrive_last(uint32_t* cnt, uint32_t total, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = (prev == total - 1) ? 1 : 0;
  }
  __syncthreads();
  if (*s_flag == 0) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return true;
}

// Write-through (sc1) store of one float: a relaxed agent-scope atomic store, visible to
// every XCD without a release fence once the storing wave's vmcnt has drained
// (cdna_hip_programming.md Guideline 16, R1).
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)(p), __float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// arrive_last for partials stored write-through (st_wt): every wave drains its stores, then
// ONE relaxed agent-scope ticket per workgroup -- no release fence (an agent-scope release
// writes back the XCD's dirty L2 lines: with ~3.5k row-group workgroups per layer launch
// at B = 8192 those fences cost ~85 us of the launch, measured in round 2 with
// scripts/dbg/kbench.py); the last arriver acquires (one buffer_inv) and reads plainly.
__device__ __forceinline__ bool arrive_last_wt(uint32_t* cnt, uint32_t total, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = (prev == total - 1) ? 1 : 0;
  }
  __syncthreads();
  if (*s_flag == 0) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ void reset_counter(uint32_t* cnt) {
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Column sums of a [G][stride] partial array (columns [0, W)) with the whole block, in a
// fixed order: slice sl of NSL = BLK / W sums rows sl, sl + NSL, ... with 32 loads in
// flight, then the slices are combined through LDS (scr: >= BLK floats).  Used by the
// last-arriving workgroup of a launch, where hundreds of partial rows (large batches)
// summed by one thread per column were a serial chain of L2 round trips: the partial rows
// sit in the Infinity Cache (written through by the producers), ~1 us away, so the launch's
// tail is one such latency per unrolled round (round 4: 8 -> 32 in flight, the readout's
// 256-row sum from 16 rounds to 4; the same order of additions, so the same sums).
// wt: `out` written through (st_wt) -- a bucket's merged row read by the launch's final
// last arriver on another XCD after arrive_last_wt (no agent-scope release fence).
template <int BLK>
__device__ __forceinline__ void block_sum_rows(const float* p, int G, int W, size_t stride, float* out,
                                               float* scr, bool wt = false) {
  const int tid = threadIdx.x;
  if (W >= BLK) {
    for (int j = tid; j < W; j += BLK) {
      float acc = 0.0f;
#pragma unroll 32
      for (int q = 0; q < G; ++q) acc += p[(size_t)q * stride + j];
      if (wt) st_wt(out + j, acc); else out[j] = acc;
    }
    __syncthreads();
    return;
  }
  const int NSL = BLK / W;
  const int j = tid % W, sl = tid / W;
  if (sl < NSL) {
    float acc = 0.0f;
#pragma unroll 32
    for (int q = sl; q < G; q += NSL) acc += p[(size_t)q * stride + j];
    scr[sl * W + j] = acc;
  }
  __syncthreads();
  if (tid < W) {
    float t = 0.0f;
    for (int q = 0; q < NSL; ++q) t += scr[q * W + tid];
    if (wt) st_wt(out + tid, t); else out[tid] = t;
  }
  __syncthreads();
}

// torch.optim.AdamW / Adam single-tensor arithmetic (fp32 element ops; bias
// corrections computed in double like the Python scalars of torch/optim/adamw.py).
struct AdamStep {
  float lr, b1, b2, eps, wd, decay_mul, step_size, inv_bc2;
  int decoupled;
  __device__ __forceinline__ void init(const gtr_adam& o, int64_t t) {
    lr = o.lr; b1 = o.beta1; b2 = o.beta2; eps = o.eps; wd = o.weight_decay;
    decoupled = o.decoupled;
    double bc1 = 1.0 - pow((double)o.beta1, (double)t);
    double bc2 = 1.0 - pow((double)o.beta2, (double)t);
    step_size = (float)((double)o.lr / bc1);
    inv_bc2 = (float)(1.0 / sqrt(bc2));
    decay_mul = (float)(1.0 - (double)o.lr * (double)o.weight_decay);
  }
  // torch AdamW's fp32 update (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_, denom =
  // sqrt(exp_avg_sq) / sqrt(bc2) + eps, param.addcdiv_) with the square root and the two
  // divisions on the hardware v_sqrt_f32 / v_rcp_f32 (1 ulp each) instead of the
  // correctly rounded IEEE sequences: ~12 instead of ~50 VALU instructions per element
  // and step, which bounds the zero-gradient catch-up of the 1M-row table (C5); each
  // update differs from torch's by a few ulp of the update term (tests hold 1e-3 against
  // the oracle).  Every kernel that updates parameters uses this one function, so the
  // single-GPU, data-parallel, sharded, eager and lazy paths stay bitwise equal.
  __device__ __forceinline__ void apply(float& p, float& m, float& v, float g) const {
#pragma clang fp contract(off)
    if (decoupled) p = p * decay_mul;
    else g = g + wd * p;
    m = m + (1.0f - b1) * (g - m);          // exp_avg.lerp_(grad, 1 - beta1)
    v = v * b2 + (1.0f - b2) * g * g;       // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2 + eps;
    p = p + (-step_size) * (m * __builtin_amdgcn_rcpf(denom));  // param.addcdiv_(exp_avg, denom, -step_size)
  }
  // apply(p, m, v, 0.0f) in 11 instead of 15 VALU instructions, BITWISE the same for every
  // input (the standalone sweep and the lazy catch-up kernels; the sweep slices inside the
  // layer kernels keep apply(.., 0): there the shorter form measured C3 0.1268 -> 0.135 ms,
  // the fused kernels' code generation, not the arithmetic):
  //   m + c*(0 - m) == m - c*m: 0 - m is -m exactly for m != 0, c*(-m) == -(c*m), and
  //     x + (-y) is x - y; m = +-0 gives +0 on both sides;
  //   v*b2 + ((1-b2)*0)*0 == v*b2 + (+0) == v*b2, since v >= +0 (exp_avg_sq starts at +0 and
  //     only grows by squares), so v*b2 is never -0.
  // Plain Adam (L2 into the gradient) has g = wd*p != 0: the general update.
  // the moments' part of apply_zero alone (decoupled AdamW: m and v do not depend on p):
  // the lazy table's tail re-derives a lagging row's m / v with it (gtr_rows.cuh)
  __device__ __forceinline__ void apply_zero_mv(float& m, float& v) const {
#pragma clang fp contract(off)
    m = m - (1.0f - b1) * m;
    v = v * b2;
  }
  __device__ __forceinline__ void apply_zero(float& p, float& m, float& v) const {
#pragma clang fp contract(off)
    if (!decoupled) { apply(p, m, v, 0.0f); return; }
    p = p * decay_mul;
    apply_zero_mv(m, v);
    const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2 + eps;
    p = p + (-step_size) * (m * __builtin_amdgcn_rcpf(denom));
  }
};

// Untouched-row AdamW slice of a fused-step launch (see gtr_sweep in gtr.h): workgroup
// blk of nblk streams float4s of rows [bounds[slot], bounds[slot+1]) whose stamp is not
// the current step, SW_U float4 per thread in flight per tensor (one workgroup per CU
// next to the layer kernels' LDS-heavy groups, so each thread keeps several in flight).
// lag = 1: lazy-table stamps; rows behind the previous step are brought to it (one
// zero-gradient update when one step behind, the consts chain otherwise) and stamped.
// A row's float4s are consecutive lanes of one wave (D/4 <= 64 divides the wave), and
// every lane reads the stamp before any lane of the row writes it.
#define SW_U 4
// Streaming (non-temporal) accesses: the sweep's table traffic must not evict the layer
// kernels' working set (weights, CSR, activations) from L2 -- measured +8.5 % (C2) and
// +4.4 % (C3) sessions/s against plain loads/stores.
__device__ __forceinline__ float4 sw_ld(const float4* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void sw_st(float4* p, const float4 x) {
  const f32x4 v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ void sweep_slice(const gtr_sweep& sw, int slot, int blk, int nblk) {
  __shared__ AdamStep s_sw_st;
  __shared__ int32_t s_sw_t;
  const int64_t r0 = sw.bounds[slot], r1 = sw.bounds[slot + 1];
  if (r1 <= r0) return;
  const bool lag = sw.lag != 0;
  if (threadIdx.x == 0) {
    const int64_t t = *sw.opt.step_dev + sw.opt.step_offset - (lag ? 1 : 0);
    if (t >= 1) s_sw_st.init(sw.opt, t);
    s_sw_t = (int32_t)t;
  }
  __syncthreads();
  const AdamStep st = s_sw_st;
  const int32_t tcur = s_sw_t;  // eager: the current step; lag: the step rows are brought to
  if (lag && tcur < 1) return;
  int lg = 0;
  while ((1 << lg) < sw.dim / 4) ++lg;
  const int64_t v0 = r0 << lg, v1 = r1 << lg;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  float4* P = reinterpret_cast<float4*>(sw.table);
  float4* M = reinterpret_cast<float4*>(sw.m);
  float4* V = reinterpret_cast<float4*>(sw.v);
  for (int64_t i = v0 + (int64_t)blk * blockDim.x + threadIdx.x; i < v1; i += SW_U * stride) {
    bool on[SW_U];
    int32_t old[SW_U];
    float4 p[SW_U], m[SW_U], q[SW_U];
#pragma unroll
    for (int u = 0; u < SW_U; ++u) {
      const int64_t j = i + u * stride;
      old[u] = j < v1 ? sw.stamp[j >> lg] : tcur;
      on[u] = j < v1 && (lag ? old[u] < tcur : old[u] != tcur);
    }
#pragma unroll
    for (int u = 0; u < SW_U; ++u) {
      const int64_t j = i + u * stride;
      if (on[u]) { p[u] = sw_ld(P + j); m[u] = sw_ld(M + j); q[u] = sw_ld(V + j); }
    }
#pragma unroll
    for (int u = 0; u < SW_U; ++u) {
      const int64_t j = i + u * stride;
      if (on[u]) {
        if (!lag || old[u] == tcur - 1) {
          st.apply(p[u].x, m[u].x, q[u].x, 0.0f); st.apply(p[u].y, m[u].y, q[u].y, 0.0f);
          st.apply(p[u].z, m[u].z, q[u].z, 0.0f); st.apply(p[u].w, m[u].w, q[u].w, 0.0f);
        } else {  // more than one step behind: each missed step with its own scalars
          AdamStep sc = st;
          for (int tt = old[u] + 1; tt <= tcur; ++tt) {
            const float2 c = reinterpret_cast<const float2*>(sw.consts)[tt];
            sc.step_size = c.x;
            sc.inv_bc2 = c.y;
            sc.apply(p[u].x, m[u].x, q[u].x, 0.0f); sc.apply(p[u].y, m[u].y, q[u].y, 0.0f);
            sc.apply(p[u].z, m[u].z, q[u].z, 0.0f); sc.apply(p[u].w, m[u].w, q[u].w, 0.0f);
          }
        }
        sw_st(P + j, p[u]); sw_st(M + j, m[u]); sw_st(V + j, q[u]);
        if (lag && (j & ((1 << lg) - 1)) == 0) sw.stamp[j >> lg] = tcur;
      }
    }
  }
}

// GEMM arithmetic of the layer kernels (host side): exact f32-input MFMA (default, every
// width) or split-bf16 MFMA (opt-in, GTR_GEMM=split).  Split-bf16 carries ~16 bits of
// each product; after a few AdamW steps that moved a few parameters per million past the
// north star's elementwise 1e-3 bar against the fp32 oracle on the full C3 / C5 tables
// (tests/test_gpu_fullsize.py), so it is not the default at any width.
// Sweep workgroups appended to a launch with `grid_main` other workgroups: gtr_sweep.blocks,
// or (blocks <= 0) enough to fill the chip's CUs exactly -- every workgroup on a CU of its
// own, and the main workgroups packable onto one XCD (xcd_pack) -- at least 64.
inline int sweep_blocks(const gtr_sweep* sw, int grid_main) {
  if (sw->blocks > 0) return sw->blocks;
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus - grid_main > 64 ? cus - grid_main : 64;
}

inline int xcd_pack(int main_blocks, int grid) {
  const char* e = getenv("GTR_XCD_PACK");
  if (e && e[0] == '0') return 0;
  return main_blocks > 0 && 8 * (main_blocks - 1) < grid ? 1 : 0;
}

inline int gemm_split(int dim) {
  (void)dim;
  const char* e = getenv("GTR_GEMM");  // read per launch: tests switch it within a process
  return (e && (e[0] == 's' || e[0] == 'S')) ? 1 : 0;
}

}  // namespace gtr

// Diagnostic build only (make timing): per-workgroup phase stamps of the layer
// kernels, s_memrealtime (100 MHz) taken by thread 0; read back by gtr_dbg_*_phases.
#define GTR_PH_KERNELS 32
#define GTR_PH_GROUPS 4096
#define GTR_PH_SLOTS 16
#ifdef GTR_PHASE_TIMING
#define GTR_PH_DECL static __device__ unsigned long long g_ph[GTR_PH_KERNELS][GTR_PH_GROUPS][GTR_PH_SLOTS];
#define GTR_PH(kid, k)                                                                               \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < GTR_PH_GROUPS) {                                            \
      unsigned long long _t;                                                                         \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                 \
      g_ph[(kid)][blockIdx.x][(k)] = _t;                                                             \
    }                                                                                                \
  } while (0)
#define GTR_PH_CLK(kid, k)                                                                           \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < GTR_PH_GROUPS) {                                            \
      unsigned long long _t;                                                                         \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                     \
      g_ph[(kid)][blockIdx.x][(k)] = _t;                                                             \
    }                                                                                                \
  } while (0)
#define GTR_PH_READER(name)                                                                          \
  extern "C" int name(void* host, size_t bytes) {                                                    \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ph), bytes < sizeof(g_ph) ? bytes : sizeof(g_ph), 0, \
                                    hipMemcpyDeviceToHost);                                          \
  }
#else
#define GTR_PH_DECL
#define GTR_PH(kid, k) do { } while (0)
#define GTR_PH_CLK(kid, k) do { } while (0)
#define GTR_PH_READER(name)
#endif

#define GTR_HIP_CHECK_LAUNCH()                                              \
  do {                                                                      \
    hipError_t _e = hipGetLastError();                                      \
    if (_e != hipSuccess) {                                                 \
      gtr::set_error("%s: launch failed: %s", __func__, hipGetErrorString(_e)); \
      return (int)_e;                                                       \
    }                                                                       \
  } while (0)
