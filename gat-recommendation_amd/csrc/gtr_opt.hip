// gtr_opt.hip — item-table gradient bookkeeping and the fused AdamW/Adam kernels.
//
// The reference materialises a dense [T, D] embedding gradient every step
// (nn.Embedding(sparse=False), base.py:36) and runs torch.optim.AdamW over all
// T*D elements (train_baseline.py:252-256).  Here the table gradient is kept as a
// contribution list (node rows dx0, target/negative rows coef*se) sorted by row
// (stable radix sort => deterministic segmented sums), and the optimizer is split:
//   * gtr_adamw_sweep: rows NOT touched this step — AdamW with g = 0 (identical
//     arithmetic to the dense update), 24 B/element, independent of the backward,
//     so it can run concurrently with the forward/backward chain;
//   * gtr_adamw_rows:  touched rows — segmented sum + AdamW;
//   * gtr_adamw_small: every other parameter (flat buffer, partial slabs summed).

#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdarg>
#include <cstdio>

#include "gtr_rows.cuh"
#include <string.h>

#include "gtr_wgrad.cuh"

namespace gtr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace gtr

namespace {

using namespace gtr;

struct SmallK {
  float* param;
  float* m;
  float* v;
  float* grad_out;
  int64_t total;
  int nseg, pad0;
  gtr_adam opt;
  gtr_segment segs[GTR_SMALL_MAX_SEG];
};

__global__ __launch_bounds__(GTR_BLOCK) void k_adamw_small(SmallK a) {
  __shared__ AdamStep s_st;
  const int64_t e = (int64_t)blockIdx.x * GTR_BLOCK + threadIdx.x;
  if (a.grad_out == nullptr && threadIdx.x == 0) s_st.init(a.opt, *a.opt.step_dev + a.opt.step_offset);
  __syncthreads();
  const AdamStep st = s_st;
  small_body(e, a.segs, a.nseg, nullptr, a.param, a.m, a.v, a.grad_out, st);
}

__global__ __launch_bounds__(GTR_BLOCK) void k_contrib_prep(gtr_batch bt, int T, int32_t* keys, int32_t* vals,
                                                            int32_t* stamp, const int64_t* step_dev) {
  const int j = blockIdx.x * GTR_BLOCK + threadIdx.x;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  if (j >= m_cap) return;
  const int key = contrib_key(bt, T, j, bt.hdr[0], bt.hdr[1]);
  keys[j] = key;
  vals[j] = j;
  if (stamp && key > 0 && key < T) stamp[key] = (int32_t)(*step_dev + 1);
}

// Touched rows: one thread per (segment start, float4 column).  p/m/v of the row are
// fetched up front (they depend only on the key), the segment's contributions are
// summed in sorted (stable) order, then AdamW — or the dense gradient is written.
// wait(): called after every load is issued, before `st` / `lazy_t` are first read.
template <int D, class Wait = NoWait>
__device__ __forceinline__ void rows_body(int gid, const gtr_batch& bt, int T, const int32_t* skeys,
                                          const int32_t* svals, const float* dx0, const float* se,
                                          const float* coef_tgt, const float* coef_neg, float* table, float* m,
                                          float* v, float* grad_dense, const AdamStep& st,
                                          int32_t* lazy_stamp = nullptr, const int32_t& lazy_t = 0,
                                          Wait wait = Wait{}) {
  constexpr int C4 = D / 4;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int i = gid / C4, c = gid - (gid / C4) * C4;
  if (i >= m_cap) return;
  const int key = skeys[i];
  const int prev = i > 0 ? skeys[i - 1] : -1;
  if (key <= 0 || key >= T || prev == key) return;
  const size_t base = (size_t)key * C4 + c;
  float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), mv = pv, vv = pv;
  int32_t sw = 0;
  if (!grad_dense) {
    pv = reinterpret_cast<const float4*>(table)[base];
    mv = reinterpret_cast<const float4*>(m)[base];
    vv = reinterpret_cast<const float4*>(v)[base];
    if (lazy_stamp) sw = lazy_stamp[key];
  }
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = i;
  do {
    const int j = svals[k];
    const float* src;
    float cf;
    if (j < bt.n_cap) {
      src = dx0 + (size_t)j * D;
      cf = 1.0f;
    } else if (j < bt.n_cap + bt.b_cap) {
      const int b = j - bt.n_cap;
      src = se + (size_t)b * D;
      cf = coef_tgt[b];
    } else {
      const int qn = j - bt.n_cap - bt.b_cap;
      src = se + (size_t)(qn / bt.n_neg) * D;
      cf = coef_neg[qn];
    }
    const float4 sv = reinterpret_cast<const float4*>(src)[c];
    g.x += cf * sv.x; g.y += cf * sv.y; g.z += cf * sv.z; g.w += cf * sv.w;
    ++k;
  } while (k < m_cap && skeys[k] == key);
  if (grad_dense) {
    reinterpret_cast<float4*>(grad_dense)[base] = g;
    return;
  }
  wait();
  if (lazy_stamp) lazy_mv_forward(mv, vv, sw, lazy_t, st);
  st.apply(pv.x, mv.x, vv.x, g.x);
  st.apply(pv.y, mv.y, vv.y, g.y);
  st.apply(pv.z, mv.z, vv.z, g.z);
  st.apply(pv.w, mv.w, vv.w, g.w);
  reinterpret_cast<float4*>(table)[base] = pv;
  reinterpret_cast<float4*>(m)[base] = mv;
  reinterpret_cast<float4*>(v)[base] = vv;
  if (lazy_stamp && c == 0) lazy_stamp[key] = lazy_t;  // lazy table: current through this step
}

// Touched rows: one thread per (segment start, float4 column).  p/m/v of the row are
// fetched up front (they depend only on the key), the segment's contributions are
// summed in sorted (stable) order, then AdamW — or the dense gradient is written.
template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_adamw_rows(gtr_batch bt, int T, const int32_t* skeys,
                                                          const int32_t* svals, const float* dx0,
                                                          const float* se, const float* coef_tgt,
                                                          const float* coef_neg, float* table, float* m,
                                                          float* v, float* grad_dense, gtr_adam opt) {
  __shared__ AdamStep s_st;
  if (grad_dense == nullptr && threadIdx.x == 0) s_st.init(opt, *opt.step_dev + opt.step_offset);
  __syncthreads();
  const AdamStep st = s_st;
  rows_body<D>(blockIdx.x * GTR_BLOCK + threadIdx.x, bt, T, skeys, svals, dx0, se, coef_tgt, coef_neg, table, m, v,
               grad_dense, st);
}

// Untouched rows: 16 B per thread per tensor, grid-stride over nblk blocks; rows with
// stamp == t (touched this step) skipped.
__device__ __forceinline__ void sweep_body(int blk, int nblk, int64_t nvec, int vpr_log2, const int32_t* stamp,
                                           int32_t t, float4* table, float4* m, float4* v, const AdamStep& st,
                                           int64_t vbegin = 0) {
  const int64_t stride = (int64_t)nblk * GTR_BLOCK;
  for (int64_t i = vbegin + (int64_t)blk * GTR_BLOCK + threadIdx.x; i < nvec; i += stride) {
    const int64_t row = i >> vpr_log2;
    if (stamp[row] == t) continue;
    float4 p = sw_ld(table + i), mm = sw_ld(m + i), vv = sw_ld(v + i);  // streaming: spare L2
    st.apply_zero(p.x, mm.x, vv.x);
    st.apply_zero(p.y, mm.y, vv.y);
    st.apply_zero(p.z, mm.z, vv.z);
    st.apply_zero(p.w, mm.w, vv.w);
    sw_st(table + i, p);
    sw_st(m + i, mm);
    sw_st(v + i, vv);
  }
}

__global__ __launch_bounds__(GTR_BLOCK) void k_adamw_sweep(int64_t nvec, int vpr_log2, const int32_t* stamp,
                                                           float4* table, float4* m, float4* v, gtr_adam opt) {
  __shared__ AdamStep s_st;
  __shared__ int32_t s_t;
  if (threadIdx.x == 0) {
    const int64_t t = *opt.step_dev + opt.step_offset;
    s_st.init(opt, t);
    s_t = (int32_t)t;
  }
  __syncthreads();
  const AdamStep st = s_st;
  sweep_body(blockIdx.x, gridDim.x, nvec, vpr_log2, stamp, s_t, table, m, v, st);
}


// Claim row `key` for catch-up to step t-1 (first claimer gets the old stamp; later
// claimers of the same row see t-1) and bring it forward with the 16 lanes of a group
// (lanes gl = 0..15 at gbase; they cover the row's float4 columns).  The per-step
// scalars are fetched 16 steps at a time (one per lane) and broadcast by shuffles, so
// the serial chain of updates never waits on memory.
// Zero-gradient catch-up of one row from step old to t-1 by its 16-lane group: every
// lane holds NP float4 columns of p / m / v in registers for the whole chain (one read
// and one write of the row), the steps' scalars come 16 at a time from consts[] and are
// broadcast from the lane that loaded them.
template <int NP>
__device__ __forceinline__ void lazy_catch_up_lanes(float4* P, float4* M, float4* V, int C4, int old, int32_t t,
                                                    int gl, int gbase, const gtr_lazy& lz) {
  const gtr_adam& o = lz.opt;
  AdamStep st;
  st.lr = o.lr; st.b1 = o.beta1; st.b2 = o.beta2; st.eps = o.eps; st.wd = o.weight_decay;
  st.decoupled = o.decoupled;
  st.decay_mul = (float)(1.0 - (double)o.lr * (double)o.weight_decay);
  float4 p[NP], m[NP], v[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int c = gl + 16 * k;
    const bool on = c < C4;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    p[k] = on ? P[c] : z;
    m[k] = on ? M[c] : z;
    v[k] = on ? V[c] : z;
  }
  for (int t0 = old + 1; t0 <= t - 1; t0 += 16) {
    const int cnt = min(16, t - t0);
    const float2 cc = gl < cnt ? reinterpret_cast<const float2*>(lz.consts)[t0 + gl] : make_float2(0.f, 0.f);
    for (int q = 0; q < cnt; ++q) {
      st.step_size = __shfl(cc.x, gbase + q);
      st.inv_bc2 = __shfl(cc.y, gbase + q);
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        st.apply_zero(p[k].x, m[k].x, v[k].x);
        st.apply_zero(p[k].y, m[k].y, v[k].y);
        st.apply_zero(p[k].z, m[k].z, v[k].z);
        st.apply_zero(p[k].w, m[k].w, v[k].w);
      }
    }
  }
  const bool p_only = lazy_p_only(o.decoupled);  // the tail re-derives m / v (gtr_rows.cuh)
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int c = gl + 16 * k;
    if (c < C4) {
      P[c] = p[k];
      if (!p_only) { M[c] = m[k]; V[c] = v[k]; }
    }
  }
}

__device__ __forceinline__ void lazy_claim_row(int key, int T, int D, int32_t t, int gl, int gbase,
                                               int32_t* stamp, const gtr_lazy& lz) {
  int old = 0;
  if (gl == 0 && key > 0 && key < T) {
    old = atomicOr(stamp + key, GTR_LAZY_CLAIM);  // a later claimer of the row sees the bit
    if (old & GTR_LAZY_CLAIM) old = t - 1;
  }
  old = __shfl(old, gbase);
  if (!(key > 0 && key < T) || old >= t - 1) return;
  const int C4 = D / 4;
  float4* P = reinterpret_cast<float4*>(lz.table) + (size_t)key * C4;
  float4* M = reinterpret_cast<float4*>(lz.m) + (size_t)key * C4;
  float4* V = reinterpret_cast<float4*>(lz.v) + (size_t)key * C4;
  if (C4 <= 16) lazy_catch_up_lanes<1>(P, M, V, C4, old, t, gl, gbase, lz);
  else if (C4 <= 32) lazy_catch_up_lanes<2>(P, M, V, C4, old, t, gl, gbase, lz);
  else lazy_catch_up_lanes<4>(P, M, V, C4, old, t, gl, gbase, lz);
}

// ---- fused step: begin (counters, stamps, sorted contribution list) -------------------
#define GTR_BEGIN_BLOCK 1024
#define GTR_BEGIN_WAVES (GTR_BEGIN_BLOCK / 64)

// Rank sort: composite keys (row << 13 | slot) are unique, so the stable order by row
// is the plain order of the composites and slot j goes to rank #{composites < c_j}.
// Every workgroup stages all composites in LDS and ranks 64 slots, its 16 waves each
// counting over one slice of the composites (broadcast LDS reads; no atomics,
// deterministic).  Workgroup 0 also stamps the touched rows and advances the counters.
__global__ __launch_bounds__(GTR_BEGIN_BLOCK) void k_step_begin(gtr_batch bt, int T, int32_t* skeys, int32_t* svals,
                                                               int32_t* stamp, int64_t* step_dev, uint32_t* rng_ctr) {
  __shared__ __attribute__((aligned(16))) uint32_t ck[GTR_BEGIN_MCAP];
  __shared__ int s_part[GTR_BEGIN_WAVES][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int m4 = (m_cap + 3) & ~3;
  const int N = bt.hdr[0], B = bt.hdr[1];
  const bool lead = blockIdx.x == 0;
  const int32_t tnew = lead ? (int32_t)(*step_dev + 1) : 0;
  for (int j = tid; j < m4; j += GTR_BEGIN_BLOCK) {
    uint32_t c = 0xFFFFFFFFu;
    if (j < m_cap) {
      const int key = contrib_key(bt, T, j, N, B);
      c = ((uint32_t)key << 13) | (uint32_t)j;
      if (lead && stamp && key > 0 && key < T) stamp[key] = tnew;
    }
    ck[j] = c;
  }
  __syncthreads();
  const int j = blockIdx.x * 64 + lane;
  const uint32_t mine = j < m_cap ? ck[j] : 0u;
  const int S = ((m4 / GTR_BEGIN_WAVES) + 4) & ~3;
  const int i0 = wave * S, i1 = min(m4, i0 + S);
  int rank = 0;
  for (int i = i0; i < i1; i += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(ck + i);
    rank += (q.x < mine) + (q.y < mine) + (q.z < mine) + (q.w < mine);
  }
  s_part[wave][lane] = rank;
  __syncthreads();
  if (wave == 0 && j < m_cap) {
    int r = 0;
#pragma unroll
    for (int w = 0; w < GTR_BEGIN_WAVES; ++w) r += s_part[w][lane];
    skeys[r] = (int32_t)(mine >> 13);
    svals[r] = (int32_t)(mine & 0x1FFFu);
  }
  if (lead && tid == 0) {
    *step_dev = tnew;
    if (rng_ctr) *rng_ctr += 1;
  }
}

// Lazy variant: the same rank sort; each workgroup also claims and brings forward the
// rows of its 64 slots (16 lanes per slot); the last arriving workgroup writes
// consts[t] and advances the counters (every workgroup read the step first).
__global__ __launch_bounds__(GTR_BEGIN_BLOCK) void k_step_begin_lazy(gtr_batch bt, int T, int D, int32_t* skeys,
                                                                    int32_t* svals, int32_t* stamp,
                                                                    int64_t* step_dev, uint32_t* rng_ctr,
                                                                    gtr_lazy lz) {
  __shared__ __attribute__((aligned(16))) uint32_t ck[GTR_BEGIN_MCAP];
  __shared__ int s_part[GTR_BEGIN_WAVES][64];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int m4 = (m_cap + 3) & ~3;
  const int N = bt.hdr[0], B = bt.hdr[1];
  const int64_t t64 = *step_dev + 1;
  const int32_t t = (int32_t)t64;
  for (int j = tid; j < m4; j += GTR_BEGIN_BLOCK) {
    uint32_t c = 0xFFFFFFFFu;
    if (j < m_cap) c = ((uint32_t)contrib_key(bt, T, j, N, B) << 13) | (uint32_t)j;
    ck[j] = c;
  }
  __syncthreads();
  const int j = blockIdx.x * 64 + lane;
  const uint32_t mine = j < m_cap ? ck[j] : 0u;
  const int S = ((m4 / GTR_BEGIN_WAVES) + 4) & ~3;
  const int i0 = wave * S, i1 = min(m4, i0 + S);
  int rank = 0;
  for (int i = i0; i < i1; i += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(ck + i);
    rank += (q.x < mine) + (q.y < mine) + (q.z < mine) + (q.w < mine);
  }
  s_part[wave][lane] = rank;
  __syncthreads();
  if (wave == 0 && j < m_cap) {
    int r = 0;
#pragma unroll
    for (int w = 0; w < GTR_BEGIN_WAVES; ++w) r += s_part[w][lane];
    skeys[r] = (int32_t)(mine >> 13);
    svals[r] = (int32_t)(mine & 0x1FFFu);
  }
  {  // catch-up of this workgroup's 64 slots: 16 lanes per slot
    const int slot = blockIdx.x * 64 + tid / 16;
    const int key = slot < m_cap ? (int)(ck[slot] >> 13) : T;
    lazy_claim_row(key, T, D, t, tid & 15, lane & ~15, stamp, lz);
  }
  // consts[t] (two f64 pows) depends on t alone: written by the first workgroup's last
  // wave after its catch-up, not on the last arriver's serial path (nothing in this launch
  // reads consts[t]; the catch-up reads steps < t)
  if (blockIdx.x == 0 && tid == GTR_BEGIN_BLOCK - 64) lazy_consts_for(lz.opt, t64, lz.consts);
  // the last arriver only advances the counters: every workgroup has read *step_dev before
  // its ticket (t is consumed above) and nothing it wrote is read here -- a relaxed ticket
  if (!arrive_last_wt(lz.cnt, gridDim.x, &s_flag)) return;
  if (tid == 0) {
    *step_dev = t64;
    if (rng_ctr) *rng_ctr += 1;
    reset_counter(lz.cnt);
  }
}

// Zero-gradient catch-up of a row by a whole wave: lane holds EPL consecutive floats of
// p / m / v (D = 64 * EPL; D = 32: the upper lanes idle).  Every lane of the wave follows
// the same row, so the chain of missed steps is wave-uniform: no lane waits on another
// row's longer gap, and the per-step scalars (64 steps per load, one per lane) reach the
// update through v_readlane into scalar registers instead of LDS shuffles.
template <int EPL>
struct RowRegs {
  float p[EPL], m[EPL], v[EPL];
};

template <int EPL>
__device__ __forceinline__ void row_load(RowRegs<EPL>& r, const gtr_lazy& lz, int key, int D, int lane) {
  const int c = lane * EPL;
  const size_t o = (size_t)key * D + c;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    r.p[k] = c < D ? lz.table[o + k] : 0.0f;
    r.m[k] = c < D ? lz.m[o + k] : 0.0f;
    r.v[k] = c < D ? lz.v[o + k] : 0.0f;
  }
}

// cw: consts[wb + lane] for the last 64 steps (wb = t - 64), loaded once per wave: a row
// whose gap lies inside that window (nearly every row) runs its chain without a load on
// its serial path; older steps are fetched 64 at a time as before.
template <int EPL>
__device__ __forceinline__ void row_catch_up_store(RowRegs<EPL>& r, const gtr_lazy& lz, int key, int D, int old,
                                                   int32_t t, int lane, AdamStep st, float2 cw, int wb) {
  const int wlo = max(old + 1, wb);
  for (int t0 = old + 1; t0 < wlo; t0 += 64) {
    const int cnt = min(64, wlo - t0);
    const float2 cc = lane < cnt ? reinterpret_cast<const float2*>(lz.consts)[t0 + lane] : make_float2(0.f, 0.f);
    for (int q = 0; q < cnt; ++q) {
      st.step_size = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cc.x), q));
      st.inv_bc2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cc.y), q));
#pragma unroll
      for (int k = 0; k < EPL; ++k) st.apply_zero(r.p[k], r.m[k], r.v[k]);
    }
  }
  for (int q = wlo - wb; q < t - wb; ++q) {  // steps wlo .. t-1 from the window
    st.step_size = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cw.x), q));
    st.inv_bc2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cw.y), q));
#pragma unroll
    for (int k = 0; k < EPL; ++k) st.apply_zero(r.p[k], r.m[k], r.v[k]);
  }
  const int c = lane * EPL;
  if (c < D) {
    const size_t o = (size_t)key * D + c;
    const bool p_only = lazy_p_only(st.decoupled);  // the tail re-derives m / v (gtr_rows.cuh)
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      lz.table[o + k] = r.p[k];
      if (!p_only) { lz.m[o + k] = r.m[k]; lz.v[o + k] = r.v[k]; }
    }
  }
}

// Lazy catch-up for the large-batch (radix) path, over the SORTED contribution list.  A
// wave takes `spw` (<= 64) slots at a time (grid-strided); the lane of a row's first slot
// (a segment start) is the row's only claimer: it reads the stamp and writes it back with
// GTR_LAZY_CLAIM -- plain accesses, no atomics, so a popular row's thousands of slots no
// longer serialize on one stamp word.  The wave then brings its claimed rows forward one
// after the other, loading the next claimed row while the current one runs its chain of
// missed steps.  spw trades claim parallelism against the rows a wave walks serially
// (host: ~2 tasks per resident wave).
template <int EPL>
__global__ __launch_bounds__(GTR_BLOCK) void k_lazy_catchup(const int32_t* skeys, int m_cap, int T, int D,
                                                            int32_t* stamp, const int64_t* step_dev, gtr_lazy lz,
                                                            int spw, int adv) {
  const int lane = threadIdx.x & 63;
  const int32_t t = (int32_t)(*step_dev + (adv ? 0 : 1));  // adv: the sort already advanced the step
  const gtr_adam& o = lz.opt;
  AdamStep st;
  st.lr = o.lr; st.b1 = o.beta1; st.b2 = o.beta2; st.eps = o.eps; st.wd = o.weight_decay;
  st.decoupled = o.decoupled;
  st.decay_mul = (float)(1.0 - (double)o.lr * (double)o.weight_decay);
  st.step_size = 0.0f;
  st.inv_bc2 = 0.0f;
  const int nw = gridDim.x * (GTR_BLOCK / 64);
  const int wb = t - 64;  // the last 64 steps' scalars, one per lane (steps >= 1 only are read)
  const float2 cw = wb + lane >= 1 ? reinterpret_cast<const float2*>(lz.consts)[wb + lane] : make_float2(0.f, 0.f);
  for (int base = (blockIdx.x * (GTR_BLOCK / 64) + (threadIdx.x >> 6)) * spw; base < m_cap; base += nw * spw) {
    const int slot = base + lane;
    int key = T;
    if (lane < spw && slot < m_cap) {
      key = skeys[slot];
      if (slot > 0 && skeys[slot - 1] == key) key = T;  // not the row's first slot
    }
    int old = t - 1;
    if (key > 0 && key < T) {
      old = stamp[key];
      stamp[key] = old | GTR_LAZY_CLAIM;  // claimed: the low bits keep the row's step
    }
    uint64_t todo = __ballot(old < t - 1);
    if (!todo) continue;
    int i = __builtin_ctzll(todo);
    int k_cur = __builtin_amdgcn_readlane(key, i);
    RowRegs<EPL> cur, nxt;
    row_load<EPL>(cur, lz, k_cur, D, lane);
    while (true) {
      const int o_cur = __builtin_amdgcn_readlane(old, i);
      todo &= todo - 1;
      int i_n = 0, k_n = 0;
      if (todo) {  // the next claimed row's loads fly during this row's chain
        i_n = __builtin_ctzll(todo);
        k_n = __builtin_amdgcn_readlane(key, i_n);
        row_load<EPL>(nxt, lz, k_n, D, lane);
      }
      row_catch_up_store<EPL>(cur, lz, k_cur, D, o_cur, t, lane, st, cw, wb);
      if (!todo) break;
      cur = nxt;
      i = i_n;
      k_cur = k_n;
    }
  }
}

__global__ void k_counters_lazy(int64_t* step_dev, uint32_t* rng_ctr, gtr_lazy lz) {
  const int64_t t = *step_dev + 1;
  lazy_consts_for(lz.opt, t, lz.consts);
  *step_dev = t;
  if (rng_ctr) *rng_ctr += 1;
}

// Bring every row to step *step_dev.
__global__ __launch_bounds__(GTR_BLOCK) void k_lazy_flush(int T, int D, int32_t* stamp, const int64_t* step_dev,
                                                          gtr_lazy lz) {
  const int C4 = D / 4;
  const int64_t gid = (int64_t)blockIdx.x * GTR_BLOCK + threadIdx.x;
  const int64_t row = gid / C4;
  const int c = (int)(gid - row * C4);
  if (row >= T) return;
  const int32_t t = (int32_t)*step_dev;
  const int old = stamp[row];  // every column lane reads before lane 0 writes (same wave)
  if (old >= t) return;
  const size_t i = (size_t)row * C4 + c;
  float4 p = reinterpret_cast<float4*>(lz.table)[i], m = reinterpret_cast<float4*>(lz.m)[i],
         v = reinterpret_cast<float4*>(lz.v)[i];
  catch_up4(p, m, v, old, t, lz.opt, lz.consts);
  reinterpret_cast<float4*>(lz.table)[i] = p;
  reinterpret_cast<float4*>(lz.m)[i] = m;
  reinterpret_cast<float4*>(lz.v)[i] = v;
  __builtin_amdgcn_wave_barrier();
  if (c == 0) stamp[row] = t;
}

__global__ void k_counters(int64_t* step_dev, uint32_t* rng_ctr) {
  if (step_dev) *step_dev += 1;
  if (rng_ctr) *rng_ctr += 1;
}

// ---- fused step: tail (touched rows | small parameters | untouched rows) ---------------
struct TailK {
  gtr_batch bt;
  gtr_tail tl;
  gtr_adam opt;
  int T, nb_rows, nb_small, nb_sweep;
  int windowed, pad_w;  // 1: rows part = one block per TW-slot window of the sorted list
  int64_t vbegin;       // first float4 of the untouched-row sweep (rows below: swept in the chain)
  int64_t nvec;
  int vpr_log2, nseg;
  gtr_segment segs[GTR_SMALL_MAX_SEG];
};


// ---- large batches: windowed segmented sums (gtr_rows.cuh) ----------------------------
template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_tail_carry(gtr_batch bt, int T, gtr_tail tl) {
  tail_carry_block<D>(bt, T, tl.skeys, tl.svals, tl.dx0, tl.se, tl.coef_tgt, tl.coef_neg, tl.carry);
}

#ifndef GTR_TAIL_QF
#define GTR_TAIL_QF 4  // contribution rows in flight per lane in the tail's segment sums (A/B: 8 -> 4 frees
                       // 20 VGPRs, tail 119 -> 112 us at C3 B = 8192, 391 -> 380 us at C5 B = 8192)
#endif
// Rows part of the tail for window w = blk: every segment starting in the window is
// summed (in-window piece + carries of the following windows) and AdamW-updated.
template <int D>
__device__ __forceinline__ void window_rows(int w, const gtr_batch& bt, int T, const gtr_tail& tl, const AdamStep& st,
                                            int32_t* lazy_stamp, int32_t lazy_t) {
  constexpr int C4 = D / 4, NG = GTR_BLOCK / C4;
  __shared__ int s_bnd[TW + 1];
  const int tid = threadIdx.x;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int w0 = w * TW, w1 = min(w0 + TW, m_cap);
  __shared__ WinSlots s_ws;
  if (GTR_WIN_LDS) window_decode(bt, tl.skeys, tl.svals, tl.coef_tgt, tl.coef_neg, w0, w1, s_ws);
  const int nb = window_bounds<GTR_BLOCK>(tl.skeys, w0, w1, s_bnd);
  const int grp = tid / C4, gl = tid % C4, gb = grp * C4 % 64;
  for (int q = grp; q < nb; q += NG) {
    const int s0 = s_bnd[q];
    const int key = GTR_WIN_LDS ? s_ws.key[s0 - w0] : tl.skeys[s0];
    if (key <= 0 || key >= T) continue;
    const int e = q + 1 < nb ? s_bnd[q + 1] : w1;
    const size_t base = (size_t)key * C4 + gl;
    // p / m / v streamed (non-temporal): every row is touched once, so keeping them out of
    // L2 leaves it to the session rows se[b] that every target / negative contribution reads
    float4 pv = sw_ld(reinterpret_cast<const float4*>(tl.table) + base);
    float4 mv = sw_ld(reinterpret_cast<const float4*>(tl.table_m) + base);
    float4 vv = sw_ld(reinterpret_cast<const float4*>(tl.table_v) + base);
    const int32_t sw = lazy_stamp ? lazy_stamp[key] : 0;
    const float4 g = window_segment_sum<D, GTR_TAIL_QF>(bt, tl.skeys, tl.svals, tl.dx0, tl.se, tl.coef_tgt,
                                                        tl.coef_neg, tl.carry, w, s0, e, w1, m_cap, key, gl, gb, &s_ws);
    if (lazy_stamp) lazy_mv_forward(mv, vv, sw, lazy_t, st);
    st.apply(pv.x, mv.x, vv.x, g.x);
    st.apply(pv.y, mv.y, vv.y, g.y);
    st.apply(pv.z, mv.z, vv.z, g.z);
    st.apply(pv.w, mv.w, vv.w, g.w);
    sw_st(reinterpret_cast<float4*>(tl.table) + base, pv);
    sw_st(reinterpret_cast<float4*>(tl.table_m) + base, mv);
    sw_st(reinterpret_cast<float4*>(tl.table_v) + base, vv);
    if (lazy_stamp && gl == 0) lazy_stamp[key] = lazy_t;
  }
}

// DEFER (small batches): one wave more than the body waves loads the step counter and
// computes the step's AdamW scalars (two f64 pow, ~1.7 us at C2 when every wave waited
// for them) while the body waves issue their loads; they wait on s_ready only right
// before AdamW.  Large batches (windowed rows, HBM-bound) keep four-wave blocks: a fifth
// wave costs them a resident block per CU (C3 B = 8192: 1.195 -> 1.232 ms).
#define GTR_TAIL_BLOCK (GTR_BLOCK + 64)

template <int D, bool DEFER>
#ifndef GTR_TAIL_WAVES_EU
#define GTR_TAIL_WAVES_EU 1
#endif
__global__ __launch_bounds__(DEFER ? GTR_TAIL_BLOCK : GTR_BLOCK) __attribute__((amdgpu_waves_per_eu(DEFER ? 1 : GTR_TAIL_WAVES_EU))) void k_step_tail(TailK a) {
  __shared__ AdamStep s_st;
  __shared__ int32_t s_t;
  __shared__ int s_ready;
  __shared__ float s_acc[GTR_BLOCK];
  const int tid = threadIdx.x;
  if constexpr (DEFER) {
    if (tid == 0) s_ready = 0;
    __syncthreads();
    if (tid >= GTR_BLOCK) {  // the step-scalar wave
      if (tid == GTR_BLOCK) {
        const int64_t t = *a.opt.step_dev + a.opt.step_offset;
        s_st.init(a.opt, t);
        s_t = (int32_t)t;
        __hip_atomic_store(&s_ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return;
    }
  } else {
    if (tid == 0) {
      const int64_t t = *a.opt.step_dev + a.opt.step_offset;
      s_st.init(a.opt, t);
      s_t = (int32_t)t;
      s_ready = 1;
    }
    __syncthreads();
  }
  auto wait = [&]() {
    while (__hip_atomic_load(&s_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
      __builtin_amdgcn_s_sleep(1);
  };
  const int blk = blockIdx.x;
  if (blk == 0 && tid == 0 && a.tl.rng_inc) *a.tl.rng_inc += 1;  // fused begin: the step's dropout counter
  if (blk < a.nb_rows && a.windowed) {
    wait();
    const AdamStep st = s_st;
    window_rows<D>(blk, a.bt, a.T, a.tl, st, a.tl.lazy_consts ? a.tl.stamp : nullptr, s_t);
    return;
  }
  if (blk < a.nb_rows) {
    rows_body<D>(blk * GTR_BLOCK + tid, a.bt, a.T, a.tl.skeys, a.tl.svals, a.tl.dx0, a.tl.se, a.tl.coef_tgt,
                 a.tl.coef_neg, a.tl.table, a.tl.table_m, a.tl.table_v, nullptr, s_st,
                 a.tl.lazy_consts ? a.tl.stamp : nullptr, s_t, wait);
    return;
  }
  if (blk < a.nb_rows + a.nb_small) {
    const int sb = blk - a.nb_rows;
    small_body((int64_t)sb * GTR_BLOCK + tid, a.segs, a.nseg, a.bt.hdr, a.tl.flat, a.tl.flat_m, a.tl.flat_v, nullptr,
               s_st, wait);
    if (sb == 0 && a.tl.loss_part) {  // loss of the step: the readout's partials, fixed order
      float acc = 0.0f;
      for (int q = tid; q < a.tl.loss_nparts; q += GTR_BLOCK)
        acc += a.tl.loss_part[(size_t)q * 2] + a.tl.loss_part[(size_t)q * 2 + 1];
      s_acc[tid] = acc;
      __syncthreads();
      if (tid == 0) {
        float t = 0.0f;
        for (int q = 0; q < GTR_BLOCK; ++q) t += s_acc[q];
        a.tl.loss_out[0] = t;
        if (a.tl.loss_acc) a.tl.loss_acc[0] += (double)t;
      }
    } else if (sb == 0 && a.tl.loss_acc && tid == 0) {  // the readout wrote the loss itself
      a.tl.loss_acc[0] += (double)a.tl.loss_out[0];
    }
    return;
  }
  wait();
  const AdamStep st = s_st;
  sweep_body(blk - a.nb_rows - a.nb_small, a.nb_sweep, a.nvec, a.vpr_log2, a.tl.stamp, s_t,
             reinterpret_cast<float4*>(a.tl.table), reinterpret_cast<float4*>(a.tl.table_m),
             reinterpret_cast<float4*>(a.tl.table_v), st, a.vbegin);
}

// ---- small batches: the weight gradients and the optimizer tail in ONE launch ----------
// Workgroups: [weight-gradient tile chunks | touched rows | BatchNorm gamma / beta + loss].
// Each (tile, row chunk) workgroup computes its split-K partial slab exactly as k_wgrad
// does and records the slab indices it wrote in LDS; the tile's P-th arriving chunk
// (agent-scope last-arriver election) then sums the P partials of each of those indices in
// chunk order -- the sum the tail's small-parameter part takes -- and applies AdamW to the
// flat parameter.  Touched rows and the bn_gsum segments depend only on the backward, so
// they run beside the tiles.  One launch less on the step's chain, bitwise equal to
// gtr_wgrad + gtr_step_tail (trainer.py:123-127: backward + optimizer.step()).
#define GTR_TAILW_SEGS 16
#define GTR_WT_LIST 4352  // slab indices one tile writes: <= 64 x 64 W + 64 bias, or 64 x (K + 1)
struct TailWK {
  gtr_batch bt;
  gtr_tail tl;
  gtr_adam opt;
  int T, nb_rows, nb_wg, nb_small, njobs, D, nseg, P;
  int64_t stride;
  int small_total, pad0;
  uint32_t* cnt;  // one arrival counter per tile (zero between launches)
  gtr_segment segs[GTR_TAILW_SEGS];
  WJob jobs[GTR_MAX_WJOBS];
};

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_step_tail_wgrad(TailWK a) {
  __shared__ AdamStep s_st;
  __shared__ int32_t s_t;
  __shared__ float s_acc[GTR_BLOCK];
  __shared__ uint32_t s_list[GTR_WT_LIST];
  __shared__ int s_n;
  __shared__ int s_flag;
  const int tid = threadIdx.x;
  if (tid == 0) {
    const int64_t t = *a.opt.step_dev + a.opt.step_offset;
    s_st.init(a.opt, t);
    s_t = (int32_t)t;
    s_n = 0;
  }
  __syncthreads();
  const AdamStep st = s_st;
  int blk = blockIdx.x;
  if (blk == 0 && tid == 0 && a.tl.rng_inc) *a.tl.rng_inc += 1;  // fused begin: the step's dropout counter
  if (blk < a.nb_wg) {
    int jid = 0;
    while (jid + 1 < a.njobs && blk >= a.jobs[jid + 1].blk0) ++jid;
    const WJob& J = a.jobs[jid];
    const int local = blk - J.blk0;
    const int tile = local / a.P, p = local - tile * a.P;
    const int N = a.bt.hdr[0];
    const int per = (N + a.P - 1) / a.P;
    const int t0 = p * per, t1 = min(N, t0 + per);
    const int64_t so = (int64_t)p * a.stride;
    // slab index codes: bits 31..30 = 0 W element, 1 bias element, 2 four W elements
    auto rec = [&](uint32_t code) { s_list[atomicAdd(&s_n, 1)] = code; };
    auto emit = [&](int which, int64_t idx, float v) {
      if (which == 0) J.outW[so + idx] = v;
      else J.outB[so + idx] = v;
      rec(((uint32_t)which << 30) | (uint32_t)idx);
    };
    auto emit4 = [&](int64_t idx, float4 v) {
      *reinterpret_cast<float4*>(J.outW + so + idx) = v;
      rec((2u << 30) | (uint32_t)idx);
    };
    if (J.mfma == 1) wgrad_tile_mfma<false>(J, tile, t0, t1, emit, emit4);
    else if (J.mfma == 2) wgrad_tile_mfma<true>(J, tile, t0, t1, emit, emit4);
    else wgrad_tile(J, tile, t0, t1, a.D, emit);
    if (!arrive_last(a.cnt + J.tile0 + tile, (uint32_t)a.P, &s_flag)) return;
    const int n = s_n;
    float* P = a.tl.flat;
    float* M = a.tl.flat_m;
    float* V = a.tl.flat_v;
    for (int k = tid; k < n; k += GTR_BLOCK) {
      const uint32_t code = s_list[k];
      const uint32_t kind = code >> 30;
      const int64_t idx = code & 0x3FFFFFFFu;
      const float* src = kind == 1 ? J.outB : J.outW;
      const int64_t f0 = kind == 1 ? J.fB : J.fW;
      const int cnt = kind == 2 ? 4 : 1;
      for (int c = 0; c < cnt; ++c) {
        float g = 0.0f;
        for (int q = 0; q < a.P; ++q) g += src[(int64_t)q * a.stride + idx + c];
        const int64_t e = f0 + idx + c;
        float pv = P[e], mv = M[e], vv = V[e];
        st.apply(pv, mv, vv, g);
        P[e] = pv;
        M[e] = mv;
        V[e] = vv;
      }
    }
    if (tid == 0) reset_counter(a.cnt + J.tile0 + tile);
    return;
  }
  blk -= a.nb_wg;
  if (blk < a.nb_rows) {
    rows_body<D>(blk * GTR_BLOCK + tid, a.bt, a.T, a.tl.skeys, a.tl.svals, a.tl.dx0, a.tl.se, a.tl.coef_tgt,
                 a.tl.coef_neg, a.tl.table, a.tl.table_m, a.tl.table_v, nullptr, st,
                 a.tl.lazy_consts ? a.tl.stamp : nullptr, s_t);
    return;
  }
  blk -= a.nb_rows;
  if (blk < a.nb_small) {
    int64_t i = (int64_t)blk * GTR_BLOCK + tid;  // index into the concatenated segments
    if (i < a.small_total) {
      int sg = 0;
      while (i >= a.segs[sg].len) { i -= a.segs[sg].len; ++sg; }
      const gtr_segment& S = a.segs[sg];
      float g = 0.0f;
      for (int q = 0; q < S.nparts; ++q) g += S.src[(int64_t)q * S.pstride + i];
      const int64_t e = S.begin + i;
      float pv = a.tl.flat[e], mv = a.tl.flat_m[e], vv = a.tl.flat_v[e];
      st.apply(pv, mv, vv, g);
      a.tl.flat[e] = pv;
      a.tl.flat_m[e] = mv;
      a.tl.flat_v[e] = vv;
    }
    if (blk == 0 && a.tl.loss_part) {  // loss of the step: the readout's partials, fixed order
      float acc = 0.0f;
      for (int q = tid; q < a.tl.loss_nparts; q += GTR_BLOCK)
        acc += a.tl.loss_part[(size_t)q * 2] + a.tl.loss_part[(size_t)q * 2 + 1];
      s_acc[tid] = acc;
      __syncthreads();
      if (tid == 0) {
        float t = 0.0f;
        for (int q = 0; q < GTR_BLOCK; ++q) t += s_acc[q];
        a.tl.loss_out[0] = t;
        if (a.tl.loss_acc) a.tl.loss_acc[0] += (double)t;
      }
    } else if (blk == 0 && a.tl.loss_acc && tid == 0) {
      a.tl.loss_acc[0] += (double)a.tl.loss_out[0];
    }
  }
}

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_scatter_rows(gtr_batch bt, int mode, const float* src,
                                                            const float* coef_tgt, const float* coef_neg,
                                                            float* dense) {
  constexpr int VPL = D >= 64 ? D / 64 : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * GTR_WAVES + wave;
  const int d0 = lane * VPL;
  if (d0 >= D) return;
  const int N = bt.hdr[0], B = bt.hdr[1];
  int key;
  const float* s;
  float c;
  if (mode == 0) {
    if (r >= N) return;
    key = bt.node_item[r];
    s = src + (size_t)r * D;
    c = 1.0f;
  } else {
    if (r >= B * (1 + bt.n_neg)) return;
    if (r < B) {
      key = bt.target[r];
      s = src + (size_t)r * D;
      c = coef_tgt[r];
    } else {
      const int q = r - B;
      key = bt.negatives[q];
      s = src + (size_t)(q / bt.n_neg) * D;
      c = coef_neg[q];
    }
  }
  if (key <= 0) return;  // padding_idx = 0
#pragma unroll
  for (int q = 0; q < VPL; ++q) atomicAdd(dense + (size_t)key * D + d0 + q, c * s[d0 + q]);
}

// Step epilogue: advance the step / dropout-stream counters and (optionally) sum the
// readout's pre-scaled loss partials [nparts][2] in fixed order.
__global__ void k_step_end(int64_t* step_dev, uint32_t* rng_ctr, const float* loss_part, int nparts,
                           float* loss_out) {
  __shared__ float s_acc[64];
  const int tid = threadIdx.x;
  float acc = 0.0f;
  if (loss_part)
    for (int q = tid; q < nparts; q += 64) acc += loss_part[(size_t)q * 2] + loss_part[(size_t)q * 2 + 1];
  s_acc[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    if (loss_part && loss_out) {
      float t = 0.0f;
      for (int q = 0; q < 64; ++q) t += s_acc[q];
      loss_out[0] = t;
    }
    if (step_dev) *step_dev += 1;
    if (rng_ctr) *rng_ctr += 1;
  }
}


// ---- data-parallel step: pack (local gradients) and tail (rank-averaged update) ----------
struct DpPackK {
  gtr_batch bt;
  gtr_tail tl;
  gtr_dp_layout lay;
  float* pack;
  int T, nb_rows, nb_small, nseg;
  int windowed, pad0;  // 1 (m_cap > GTR_BEGIN_MCAP): rows part = one block per TW-slot window
  gtr_segment segs[GTR_SMALL_MAX_SEG];
};

// Windowed rows part of the pack (large batches): window w's keys, its segment sums (the
// single-GPU tail's windowed order: bitwise its gradient rows) at the segments' first
// slots, zero rows at every other slot.
template <int D>
__device__ __forceinline__ void dp_pack_window(int w, const DpPackK& a, int32_t* keys, float* rows) {
  constexpr int C4 = D / 4, NG = GTR_BLOCK / C4;
  __shared__ int s_bnd[TW + 1];
  const int tid = threadIdx.x;
  const int m_cap = a.lay.m_cap;
  const int w0 = w * TW, w1 = min(w0 + TW, m_cap);
  const int32_t* sk = a.tl.skeys;
  if (tid < TW && w0 + tid < w1) keys[w0 + tid] = sk[w0 + tid];
  for (int idx = tid; idx < (w1 - w0) * C4; idx += GTR_BLOCK) {
    const int i = w0 + idx / C4;
    if (i > 0 && sk[i - 1] == sk[i])
      reinterpret_cast<float4*>(rows + (size_t)i * D)[idx % C4] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __shared__ WinSlots s_ws;
  if (GTR_WIN_LDS) window_decode(a.bt, sk, a.tl.svals, a.tl.coef_tgt, a.tl.coef_neg, w0, w1, s_ws);
  const int nb = window_bounds<GTR_BLOCK>(sk, w0, w1, s_bnd);
  const int grp = tid / C4, gl = tid % C4, gb = grp * C4 % 64;
  for (int q = grp; q < nb; q += NG) {
    const int s0 = s_bnd[q];
    const int key = GTR_WIN_LDS ? s_ws.key[s0 - w0] : sk[s0];
    const int e = q + 1 < nb ? s_bnd[q + 1] : w1;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (key > 0 && key < a.T)
      g = window_segment_sum<D>(a.bt, sk, a.tl.svals, a.tl.dx0, a.tl.se, a.tl.coef_tgt, a.tl.coef_neg, a.tl.carry, w,
                                s0, e, w1, m_cap, key, gl, gb, &s_ws);
    reinterpret_cast<float4*>(rows + (size_t)s0 * D)[gl] = g;
  }
}

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_dp_pack(DpPackK a) {
  constexpr int C4 = D / 4;
  __shared__ float s_acc[GTR_BLOCK];
  const int tid = threadIdx.x;
  const int blk = blockIdx.x;
  const int m_cap = a.lay.m_cap;
  int32_t* keys = reinterpret_cast<int32_t*>(a.pack + a.lay.keys_off);
  float* rows = a.pack + a.lay.rows_off;
  if (blk < a.nb_rows && a.windowed) {
    dp_pack_window<D>(blk, a, keys, rows);
    return;
  }
  if (blk < a.nb_rows) {
    const int gid = blk * GTR_BLOCK + tid;
    const int i = gid / C4, c = gid - i * C4;
    if (i >= m_cap) return;
    const int key = a.tl.skeys[i];
    if (c == 0) keys[i] = key;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool start = key > 0 && key < a.T && (i == 0 || a.tl.skeys[i - 1] != key);
    if (start) {
      const gtr_batch& bt = a.bt;
      int k = i;
      do {
        const int j = a.tl.svals[k];
        const float* src;
        float cf;
        if (j < bt.n_cap) {
          src = a.tl.dx0 + (size_t)j * D;
          cf = 1.0f;
        } else if (j < bt.n_cap + bt.b_cap) {
          const int b = j - bt.n_cap;
          src = a.tl.se + (size_t)b * D;
          cf = a.tl.coef_tgt[b];
        } else {
          const int qn = j - bt.n_cap - bt.b_cap;
          src = a.tl.se + (size_t)(qn / bt.n_neg) * D;
          cf = a.tl.coef_neg[qn];
        }
        const float4 sv = reinterpret_cast<const float4*>(src)[c];
        g.x += cf * sv.x; g.y += cf * sv.y; g.z += cf * sv.z; g.w += cf * sv.w;
        ++k;
      } while (k < m_cap && a.tl.skeys[k] == key);
    }
    reinterpret_cast<float4*>(rows + (size_t)i * D)[c] = g;
    return;
  }
  const int sb = blk - a.nb_rows;
  const AdamStep unused{};
  small_body((int64_t)sb * GTR_BLOCK + tid, a.segs, a.nseg, a.bt.hdr, nullptr, nullptr, nullptr, a.pack, unused);
  if (sb == 0) {  // local loss
    float acc = 0.0f;
    if (a.tl.loss_part)
      for (int q = tid; q < a.tl.loss_nparts; q += GTR_BLOCK)
        acc += a.tl.loss_part[(size_t)q * 2] + a.tl.loss_part[(size_t)q * 2 + 1];
    s_acc[tid] = acc;
    __syncthreads();
    if (tid == 0) {
      float t = 0.0f;
      if (a.tl.loss_part) {
        for (int q = 0; q < GTR_BLOCK; ++q) t += s_acc[q];
      } else {
        t = a.tl.loss_out[0];
      }
      a.pack[a.lay.loss_off] = t;
    }
  }
}

// Union of the ranks' touched rows: stamp them and record, per (row, rank), the
// segment-start slot holding that rank's summed gradient row.
__global__ __launch_bounds__(GTR_BLOCK) void k_dp_stamp(gtr_dp_layout lay, int T, const float* recv, int32_t* stamp,
                                                        int2* slot, const int64_t* step_dev, int step_offset) {
  const int gid = blockIdx.x * GTR_BLOCK + threadIdx.x;
  const int r = gid / lay.m_cap, i = gid - r * lay.m_cap;
  if (r >= lay.world) return;
  const int32_t* keys = reinterpret_cast<const int32_t*>(recv + (size_t)r * lay.words + lay.keys_off);
  const int k = keys[i];
  if (k <= 0 || k >= T || (i > 0 && keys[i - 1] == k)) return;
  const int32_t t = (int32_t)(*step_dev + step_offset);
  if (stamp) stamp[k] = t;  // eager: marks the row for the sweep; lazy: dp_tail stamps after catch-up
  slot[(size_t)k * lay.world + r] = make_int2(t, i);
}

// Early union stamp (data parallel): every rank's sorted contribution keys, all-gathered
// right after step_begin, mark the union of the step's touched rows before the backward
// so the untouched-row sweep can ride in the backward kernels (gtr_sweep).
__global__ __launch_bounds__(GTR_BLOCK) void k_dp_union_stamp(const int32_t* keys_all, int64_t n, int T,
                                                              int32_t* stamp, const int64_t* step_dev) {
  const int64_t i = (int64_t)blockIdx.x * GTR_BLOCK + threadIdx.x;
  if (i >= n) return;
  const int k = keys_all[i];
  if (k > 0 && k < T) stamp[k] = (int32_t)*step_dev;
}

struct DpTailK {
  gtr_tail tl;
  gtr_dp_layout lay;
  gtr_adam opt;
  const float* recv;
  const int2* slot;
  int T, nb_rows, nb_small, nb_sweep;
  int64_t nvec, vbegin;
  int vpr_log2, pad0;
};

// First slot of `key` in one rank's sorted contribution keys (sentinel-padded), or -1.
__device__ __forceinline__ int dp_find(const float* keys_f, int m_cap, int key) {
  const int32_t* kq = reinterpret_cast<const int32_t*>(keys_f);
  int lo = 0, hi = m_cap;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (kq[mid] < key) lo = mid + 1; else hi = mid;
  }
  return (lo < m_cap && kq[lo] == key) ? lo : -1;
}

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_dp_tail(DpTailK a) {
  constexpr int C4 = D / 4;
  __shared__ AdamStep s_st;
  __shared__ int32_t s_t;
  const int tid = threadIdx.x;
  if (tid == 0) {
    const int64_t t = *a.opt.step_dev + a.opt.step_offset;
    s_st.init(a.opt, t);
    s_t = (int32_t)t;
  }
  __syncthreads();
  const AdamStep st = s_st;
  const int32_t t = s_t;
  const int W = a.lay.world;
  const float inv_w = 1.0f / (float)W;
  const int blk = blockIdx.x;
  if (blk < a.nb_rows) {
    // owner = lowest rank holding the row; it sums every rank's row in rank order
    const int gid = blk * GTR_BLOCK + tid;
    const int ri = gid / C4, c = gid - ri * C4;
    const int r = ri / a.lay.m_cap, i = ri - r * a.lay.m_cap;
    if (r >= W) return;
    const int32_t* keys = reinterpret_cast<const int32_t*>(a.recv + (size_t)r * a.lay.words + a.lay.keys_off);
    const int k = keys[i];
    if (k <= 0 || k >= a.T || (i > 0 && keys[i - 1] == k)) return;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.slot) {  // slot table from k_dp_stamp
      const int2* sl = a.slot + (size_t)k * W;
      for (int q = 0; q < r; ++q)
        if (sl[q].x == t) return;
      for (int q = r; q < W; ++q) {
        const int2 e = sl[q];
        if (e.x != t) continue;
        const float4 v = reinterpret_cast<const float4*>(a.recv + (size_t)q * a.lay.words + a.lay.rows_off +
                                                         (size_t)e.y * D)[c];
        g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
      }
    } else {  // lazy stamps: no union pass; find the row in each rank's sorted keys
      for (int q = 0; q < r; ++q)
        if (dp_find(a.recv + (size_t)q * a.lay.words + a.lay.keys_off, a.lay.m_cap, k) >= 0) return;  // lower owner
      for (int q = r; q < W; ++q) {
        const int at = q == r ? i : dp_find(a.recv + (size_t)q * a.lay.words + a.lay.keys_off, a.lay.m_cap, k);
        if (at < 0) continue;
        const float4 v = reinterpret_cast<const float4*>(a.recv + (size_t)q * a.lay.words + a.lay.rows_off +
                                                         (size_t)at * D)[c];
        g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
      }
    }
    g.x *= inv_w; g.y *= inv_w; g.z *= inv_w; g.w *= inv_w;
    const size_t base = (size_t)k * C4 + c;
    float4 pv = reinterpret_cast<const float4*>(a.tl.table)[base];
    float4 mv = reinterpret_cast<const float4*>(a.tl.table_m)[base];
    float4 vv = reinterpret_cast<const float4*>(a.tl.table_v)[base];
    if (a.tl.lazy_consts) {
      const int sw = a.tl.stamp[k];
      if (sw & GTR_LAZY_CLAIM) lazy_mv_forward(mv, vv, sw, t, st);  // this rank's begin brought p forward
      else catch_up4(pv, mv, vv, sw, t - 1, a.opt, a.tl.lazy_consts);  // rows only other ranks touched
    }
    st.apply(pv.x, mv.x, vv.x, g.x);
    st.apply(pv.y, mv.y, vv.y, g.y);
    st.apply(pv.z, mv.z, vv.z, g.z);
    st.apply(pv.w, mv.w, vv.w, g.w);
    reinterpret_cast<float4*>(a.tl.table)[base] = pv;
    reinterpret_cast<float4*>(a.tl.table_m)[base] = mv;
    reinterpret_cast<float4*>(a.tl.table_v)[base] = vv;
    if (a.tl.lazy_consts) {
      __builtin_amdgcn_wave_barrier();  // the row's column lanes (one wave) read the stamp above
      if (c == 0) a.tl.stamp[k] = t;
    }
    return;
  }
  if (blk < a.nb_rows + a.nb_small) {
    const int64_t e = (int64_t)(blk - a.nb_rows) * GTR_BLOCK + tid;
    if (e < a.lay.flat_total) {
      float g = 0.0f;
      for (int q = 0; q < W; ++q) g += a.recv[(size_t)q * a.lay.words + e];
      g *= inv_w;
      float pv = a.tl.flat[e], mv = a.tl.flat_m[e], vv = a.tl.flat_v[e];
      st.apply(pv, mv, vv, g);
      a.tl.flat[e] = pv;
      a.tl.flat_m[e] = mv;
      a.tl.flat_v[e] = vv;
    } else if (e == a.lay.flat_total && a.tl.loss_out) {
      float l = 0.0f;
      for (int q = 0; q < W; ++q) l += a.recv[(size_t)q * a.lay.words + a.lay.loss_off];
      a.tl.loss_out[0] = l * inv_w;
      if (a.tl.loss_acc) a.tl.loss_acc[0] += (double)(l * inv_w);
    }
    return;
  }
  sweep_body(blk - a.nb_rows - a.nb_small, a.nb_sweep, a.nvec, a.vpr_log2, a.tl.stamp, t,
             reinterpret_cast<float4*>(a.tl.table), reinterpret_cast<float4*>(a.tl.table_m),
             reinterpret_cast<float4*>(a.tl.table_v), st, a.vbegin);
}

int key_bits(int T) {
  int b = 1;
  while ((1LL << b) <= (long long)T) ++b;
  return b;
}

bool dim_ok(int D) { return D == 32 || D == 64 || D == 128 || D == 256; }

// ---- contribution sort (large batches): own LSD radix, 10-bit digits -------------------
// keys < 2^20 (T <= 1M + 1) sort in two passes of three launches each: per-tile digit
// histograms (tile = 256 x rounds items, rounds = rs_rounds(n): 16 from ~1M items down to
// 1 below 64k, so a pass keeps ~200+ workgroups busy: C5 B = 1024's 107k contributions
// ran on 27 tiles of 4096) and digit totals, the scatter offsets of every (tile,
// digit) from them (16 workgroups), then a stable scatter.  Inside a tile items are ranked in 16 rounds of 256 (the
// original order): a round's items of equal digit are matched by 10 ballots within the
// wave, waves of the round are offset by per-(wave, digit) counts in LDS, rounds by a
// running count per digit -- no atomics on the ranks, so the sort is stable and
// deterministic, equal to any stable sort of the (key, slot) pairs.
#define RS_BITS 10
#define RS_RADIX (1 << RS_BITS)
#ifndef RS_THREADS  // 512: C3 B = 8192 sort 63.3 -> 56.8 us, C3 B = 1024 31.6 -> 29.7 us against 256 (1024: equal)
#define RS_THREADS 512
#endif
#define RS_MAX_ROUNDS 16
// digit totals are accumulated into RS_TOTC copies (tile mod RS_TOTC): one copy per address
// saw every tile's atomic add (~240-way contention at C3 B = 8192); k_rs_offs sums the copies
#ifndef RS_TOTC
#define RS_TOTC 16
#endif


int rs_rounds(int n) {  // tiles of ~n / 256 items (>= RS_THREADS)
  const int r = (n + RS_THREADS * 256 - 1) / (RS_THREADS * 256);
  return r < 1 ? 1 : (r > RS_MAX_ROUNDS ? RS_MAX_ROUNDS : r);
}

// Contribution-list build folded into the first histogram pass (gtr_step_begin): each slot's
// key is derived from the batch (contrib_key, as k_contrib_prep) and written with its slot
// id and the touched-row stamp -- one launch less per large-batch step.
struct RsPrep {
  gtr_batch bt;
  int T;
  int32_t* keys;
  int32_t* vals;
  int32_t* stamp;
  const int64_t* step_dev;
};

template <bool PREP, int BITS>
__global__ __launch_bounds__(RS_THREADS) void k_rs_hist(const int32_t* keys, int n, int shift, int32_t* hist,
                                                       int32_t* tot, int rounds, RsPrep pp) {
  constexpr int RADIX = 1 << BITS;
  __shared__ int h[RADIX];
  for (int d = threadIdx.x; d < RADIX; d += RS_THREADS) h[d] = 0;
  __syncthreads();
  const int base = blockIdx.x * RS_THREADS * rounds;
  // every round's key requested before the first count (the loads are independent)
  int kk[RS_MAX_ROUNDS];
  if (PREP) {
    const int N = pp.bt.hdr[0], B = pp.bt.hdr[1];
    const int32_t tnew = pp.stamp ? (int32_t)(*pp.step_dev + 1) : 0;
#pragma unroll
    for (int r = 0; r < RS_MAX_ROUNDS; ++r) {
      const int i = base + r * RS_THREADS + threadIdx.x;
      kk[r] = -1;
      if (r < rounds && i < n) {
        const int key = contrib_key(pp.bt, pp.T, i, N, B);
        pp.keys[i] = key;
        pp.vals[i] = i;
        if (pp.stamp && key > 0 && key < pp.T) pp.stamp[key] = tnew;
        kk[r] = key;
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < RS_MAX_ROUNDS; ++r) {
      const int i = base + r * RS_THREADS + threadIdx.x;
      kk[r] = (r < rounds && i < n) ? keys[i] : -1;
    }
  }
#pragma unroll
  for (int r = 0; r < RS_MAX_ROUNDS; ++r)
    if (kk[r] >= 0) atomicAdd(&h[((uint32_t)kk[r] >> shift) & (RADIX - 1)], 1);  // integer counts
  __syncthreads();
  const int cp = (blockIdx.x % RS_TOTC) * RADIX;
  for (int d = threadIdx.x; d < RADIX; d += RS_THREADS) {
    hist[(size_t)blockIdx.x * RADIX + d] = h[d];  // tile-major, coalesced
    if (h[d]) atomicAdd(tot + cp + d, h[d]);     // digit totals (integer: order-free)
  }
}

// Scatter offsets offs[tile][d] = (items of digits < d) + (items of digit d in earlier
// tiles): workgroup w owns digits [64 w, 64 w + 64), its 16 waves a slice of the tiles
// each (loads in flight together); slices and digits are combined in fixed order.
#define RS_OFFS_SL 16
// The digits' base offsets come from a block-wide exclusive scan of the 1024 digit totals
// (DPP wave scans + 16 wave sums), not a serial walk; a slice of <= 16
// tiles keeps its histogram column in registers between the two passes (integer sums:
// the offsets are exact whatever the order).

template <int BITS>
__global__ __launch_bounds__(1024) void k_rs_offs(const int32_t* __restrict__ hist, int32_t* __restrict__ tot,
                                                 int32_t* __restrict__ offs, int ntile) {
  // RADIX threads: thread tid scans digit tid; for the offsets, workgroup w owns digits
  // [64 w, 64 w + 64) and its NSL = RADIX / 64 waves a slice of the tiles each
  constexpr int RADIX = 1 << BITS, NSL = RADIX / 64;
  __shared__ int s_sl[NSL][64];
  __shared__ int s_dp[RADIX];  // exclusive prefix of the digit totals
  __shared__ int s_ws[RADIX / 64];
  const int tid = threadIdx.x, dl = tid & 63, sl = tid >> 6;
  const int d = blockIdx.x * 64 + dl;
  const int per = (ntile + NSL - 1) / NSL;
  const int b0 = min(ntile, sl * per), b1 = min(ntile, b0 + per);
  int v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = b0 + q < b1 ? hist[(size_t)(b0 + q) * RADIX + d] : 0;
  int tv = 0;  // RADIX threads == RADIX digits: the digit's total over the RS_TOTC copies
#pragma unroll
  for (int c = 0; c < RS_TOTC; ++c) tv += tot[c * RADIX + tid];
  const int incl = wave_incl_scan_dpp(tv);
  if (dl == 63) s_ws[sl] = incl;
  int sum = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) sum += v[q];
  for (int c = b0 + 16; c < b1; c += 16) {  // slices of more than 16 tiles (> 256 tiles)
    int w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = c + q < b1 ? hist[(size_t)(c + q) * RADIX + d] : 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += w[q];
  }
  s_sl[sl][dl] = sum;
  __syncthreads();
  int wb = 0;
  for (int w = 0; w < sl; ++w) wb += s_ws[w];
  s_dp[tid] = wb + incl - tv;
  __syncthreads();
  int run = s_dp[d];
  for (int q = 0; q < sl; ++q) run += s_sl[q][dl];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    if (b0 + q < b1) offs[(size_t)(b0 + q) * RADIX + d] = run;
    run += v[q];
  }
  for (int c = b0 + 16; c < b1; c += 16) {
    int w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = c + q < b1 ? hist[(size_t)(c + q) * RADIX + d] : 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (c + q < b1) offs[(size_t)(c + q) * RADIX + d] = run;
      run += w[q];
    }
  }
}

// tot: the pass's digit totals, read by k_rs_offs; zeroed here for the next call's same
// pass (the workspace starts zeroed), so no memset node sits in the captured step.
// Step counters advanced by the last pass of gtr_step_begin's (and the lazy begin's) sort:
// workgroup 0 advances the step and dropout counters and, for the lazy table, writes
// consts[t] -- nothing of this launch reads them, and the kernels after it see the new
// values (one launch less than a separate k_counters / k_counters_lazy).
struct RsCtr {
  int64_t* step_dev;  // null: no counters in this pass
  uint32_t* rng_ctr;
  float* consts;      // lazy table: consts[t] for the new step t
  gtr_adam opt;
};

template <int BITS>
__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(const int32_t* kin, const int32_t* vin, int32_t* kout,
                                                          int32_t* vout, int n, int shift, const int32_t* offs,
                                                          int ntile, int32_t* tot, int rounds, RsCtr ctr) {
  constexpr int RADIX = 1 << BITS;
  __shared__ int run[RADIX];
  __shared__ int wcnt[RS_THREADS / 64][RADIX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (blockIdx.x == 0 && tid == 0 && ctr.step_dev) {
    const int64_t t = *ctr.step_dev + 1;
    *ctr.step_dev = t;
    if (ctr.rng_ctr) *ctr.rng_ctr += 1;
    if (ctr.consts) lazy_consts_for(ctr.opt, t, ctr.consts);
  }
  for (int c = blockIdx.x; c < RS_TOTC; c += gridDim.x)
    for (int d = tid; d < RADIX; d += RS_THREADS) tot[c * RADIX + d] = 0;
  const int base = blockIdx.x * RS_THREADS * rounds;
  // the first round's (key, value) requested before the tables are staged
  int key_n = base + tid < n ? kin[base + tid] : 0;
  int val_n = base + tid < n ? vin[base + tid] : 0;
  for (int d = tid; d < RADIX; d += RS_THREADS) {
    run[d] = offs[(size_t)blockIdx.x * RADIX + d];
#pragma unroll
    for (int w = 0; w < RS_THREADS / 64; ++w) wcnt[w][d] = 0;
  }
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  // the next round's (key, value) are requested while this round is ranked and written
  for (int r = 0; r < rounds; ++r) {
    const int i = base + r * RS_THREADS + tid;
    const bool live = i < n;
    const int key = key_n;
    const int val = val_n;
    if (r + 1 < rounds) {
      const int i2 = i + RS_THREADS;
      key_n = i2 < n ? kin[i2] : 0;
      val_n = i2 < n ? vin[i2] : 0;
    }
    const int d = ((uint32_t)key >> shift) & (RADIX - 1);
    unsigned long long match = __ballot(live);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
      const unsigned long long bb = __ballot((d >> b) & 1);
      match &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int before = __popcll(match & lt);
    if (live && before == 0) wcnt[wave][d] = __popcll(match);  // the digit's first lane in the wave
    __syncthreads();
    if (live) {
      int pos = run[d] + before;
      for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    for (int q = tid; q < RADIX; q += RS_THREADS) {
      int t = 0;
#pragma unroll
      for (int w = 0; w < RS_THREADS / 64; ++w) { t += wcnt[w][q]; wcnt[w][q] = 0; }
      run[q] += t;
    }
    __syncthreads();
  }
}

int sort_mode() {  // 0: own radix (default), 1: hipCUB
  const char* e = getenv("GTR_SORT");
  if (e && (e[0] == 'm' || e[0] == 'M' || e[0] == 'h' || e[0] == 'H')) return 1;
  return 0;
}

size_t rs_bytes(int n) {
  const size_t tile = (size_t)RS_THREADS * rs_rounds(n);
  const size_t ntile = ((size_t)n + tile - 1) / tile;
  return 4 * (size_t)n * sizeof(int32_t) + 2 * (size_t)RS_RADIX * ntile * sizeof(int32_t) +
         4 * RS_TOTC * RS_RADIX * sizeof(int32_t) + 256;
}

hipError_t rs_sort(void* tmp, const int32_t* keys, int32_t* skeys, const int32_t* vals, int32_t* svals, int n,
                   int bits, hipStream_t s, const RsCtr* ctr = nullptr, const RsPrep* prep = nullptr) {
  const int rounds = rs_rounds(n), tile = RS_THREADS * rounds;
  const int ntile = (n + tile - 1) / tile;
  int32_t* k1 = static_cast<int32_t*>(tmp);
  int32_t* v1 = k1 + n;
  int32_t* k2 = v1 + n;
  int32_t* v2 = k2 + n;
  int32_t* hist = v2 + n;
  int32_t* offs = hist + (size_t)RS_RADIX * ntile;
  int32_t* tot = offs + (size_t)RS_RADIX * ntile;  // [passes][RS_TOTC][RS_RADIX] digit totals (kept zero between calls)
  // digit width: keys of <= 18 bits (T < 2^18: C3 / C4's 82k table) at >= 256k items in
  // two passes of 9-bit digits -- half the histogram / offset work and twice the run length
  // of a digit's scattered writes per tile (C3 B = 8192: 0.7710 -> 0.7686 ms per step; at
  // C4 B = 1024, 107k items, 10-bit digits measured 0.3324 against 0.3333); otherwise
  // 10-bit digits (two passes up to T = 1M).  Any width gives the same stable order.
  const char* rb = getenv("GTR_RS_BITS");
  const int RB = rb ? (atoi(rb) == 9 ? 9 : 10) : (bits <= 18 && n >= (1 << 18) ? 9 : 10);
  const int passes = (bits + RB - 1) / RB;  // <= 4 for int32 keys below 2^30
  if (passes > 4) return hipErrorInvalidValue;
  const int32_t* ki = keys;
  const int32_t* vi = vals;
  for (int p = 0; p < passes; ++p) {
    const bool last = p == passes - 1;
    int32_t* ko = last ? skeys : (p % 2 == 0 ? k1 : k2);
    int32_t* vo = last ? svals : (p % 2 == 0 ? v1 : v2);
    int32_t* tp = tot + p * RS_TOTC * RS_RADIX;
    const RsCtr cc = (last && ctr) ? *ctr : RsCtr{};
    if (RB == 9) {
      if (p == 0 && prep)  // the first pass builds the contribution list as it counts
        hipLaunchKernelGGL((k_rs_hist<true, 9>), dim3(ntile), dim3(RS_THREADS), 0, s, ki, n, 0, hist, tp, rounds, *prep);
      else
        hipLaunchKernelGGL((k_rs_hist<false, 9>), dim3(ntile), dim3(RS_THREADS), 0, s, ki, n, p * 9, hist, tp, rounds,
                           RsPrep{});
      hipLaunchKernelGGL(k_rs_offs<9>, dim3(512 / 64), dim3(512), 0, s, hist, tp, offs, ntile);
      hipLaunchKernelGGL(k_rs_scatter<9>, dim3(ntile), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, n, p * 9, offs, ntile,
                         tp, rounds, cc);
    } else {
      if (p == 0 && prep)
        hipLaunchKernelGGL((k_rs_hist<true, 10>), dim3(ntile), dim3(RS_THREADS), 0, s, ki, n, 0, hist, tp, rounds,
                           *prep);
      else
        hipLaunchKernelGGL((k_rs_hist<false, 10>), dim3(ntile), dim3(RS_THREADS), 0, s, ki, n, p * 10, hist, tp,
                           rounds, RsPrep{});
      hipLaunchKernelGGL(k_rs_offs<10>, dim3(1024 / 64), dim3(1024), 0, s, hist, tp, offs, ntile);
      hipLaunchKernelGGL(k_rs_scatter<10>, dim3(ntile), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, n, p * 10, offs, ntile,
                         tp, rounds, cc);
    }
    ki = ko;
    vi = vo;
  }
  return hipGetLastError();
}

// Stable (key, slot) sort of the contribution list, GTR_SORT selecting the algorithm:
//   default  the own radix above (6 launches for keys < 2^20);
//   merge    hipCUB / rocPRIM's default config: block sort + merge passes below 1M items
//            (~20 launches at m_cap ~ 855k).
// Both are stable, so they sort identically.  The workspace query and the sort MUST use
// the same algorithm (gtr_contrib_sort checks the size).  (A rocPRIM Onesweep option was
// removed in round 3: it faulted inside the C3 B = 8192 step without a found cause.)
hipError_t sort_pairs(void* tmp, size_t& bytes, const int32_t* keys, int32_t* skeys, const int32_t* vals,
                      int32_t* svals, int n, int bits, hipStream_t s) {
  if (sort_mode() == 0) {
    if (!tmp) {
      bytes = rs_bytes(n);
      return hipSuccess;
    }
    return rs_sort(tmp, keys, skeys, vals, svals, n, bits, s);
  }
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, keys, skeys, vals, svals, n, 0, bits, s);
}

}  // namespace

extern "C" {

int gtr_tail_carry_floats(int m_cap, int dim) {
  return m_cap > GTR_BEGIN_MCAP ? ((m_cap + TW - 1) / TW) * dim : 0;
}

int gtr_version(void) { return 100; }
int gtr_readout_grid(int b_cap) { return b_cap < 1 ? 1 : (b_cap > 256 ? 256 : b_cap); }
int gtr_abi_version(void) { return GTR_ABI_VERSION; }
#ifndef GTR_SRC_HASH
#define GTR_SRC_HASH "unknown"
#endif
const char* gtr_source_hash(void) { return GTR_SRC_HASH; }
const char* gtr_last_error(void) { return gtr::g_err; }

int gtr_device_check(int device) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) {
    set_error("gtr_device_check: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("gtr_device_check: device %d is %s, this library is built for gfx950", device, prop.gcnArchName);
    return GTR_E_DEVICE;
  }
  return GTR_OK;
}

int gtr_adamw_small(float* param, float* m, float* v, float* grad_out, int64_t total, const gtr_segment* segs,
                    int nseg, const gtr_adam* opt, gtr_stream_t stream) {
  if (!segs || nseg <= 0 || nseg > GTR_SMALL_MAX_SEG || total <= 0) {
    set_error("gtr_adamw_small: bad segment table (nseg=%d)", nseg);
    return GTR_E_ARG;
  }
  if (!grad_out && (!param || !m || !v || !opt || !opt->step_dev)) {
    set_error("gtr_adamw_small: missing optimizer state");
    return GTR_E_ARG;
  }
  for (int i = 0; i < nseg; ++i)
    if (segs[i].live_groups) {  // per-row-group partials need the batch's group count
      set_error("gtr_adamw_small: segment %d sums live row groups (gtr_conv_bwd wfold partials)", i);
      return GTR_E_ARG;
    }
  SmallK k{};
  k.param = param; k.m = m; k.v = v; k.grad_out = grad_out; k.total = total; k.nseg = nseg;
  if (opt) k.opt = *opt;
  for (int i = 0; i < nseg; ++i) k.segs[i] = segs[i];
  const int64_t blocks = (total + GTR_BLOCK - 1) / GTR_BLOCK;
  hipLaunchKernelGGL(k_adamw_small, dim3((unsigned)blocks), dim3(GTR_BLOCK), 0, (hipStream_t)stream, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_contrib_prep(const gtr_batch* bt, int num_items, int32_t* keys, int32_t* vals, int32_t* stamp,
                     const int64_t* step_dev, gtr_stream_t stream) {
  if (!bt || !keys || !vals || (stamp && !step_dev) || bt->n_neg <= 0) {
    set_error("gtr_contrib_prep: bad arguments");
    return GTR_E_ARG;
  }
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  const int blocks = (m_cap + GTR_BLOCK - 1) / GTR_BLOCK;
  hipLaunchKernelGGL(k_contrib_prep, dim3(blocks), dim3(GTR_BLOCK), 0, (hipStream_t)stream, *bt, num_items,
                     keys, vals, stamp, step_dev);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_contrib_sort_bytes(int m_cap, int num_items, size_t* bytes) {
  if (!bytes || m_cap <= 0) { set_error("gtr_contrib_sort_bytes: bad arguments"); return GTR_E_ARG; }
  size_t b = 0;
  hipError_t e = sort_pairs(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, (const int32_t*)nullptr,
                            (int32_t*)nullptr, m_cap, key_bits(num_items), nullptr);
  if (e != hipSuccess) { set_error("gtr_contrib_sort_bytes: %s", hipGetErrorString(e)); return (int)e; }
  *bytes = b;
  return GTR_OK;
}

int gtr_contrib_sort(const int32_t* keys, const int32_t* vals, int32_t* skeys, int32_t* svals, int m_cap,
                     int num_items, void* tmp, size_t tmp_bytes, gtr_stream_t stream) {
  // The temporary storage must be sized by the SAME algorithm and key width as this call
  // (gtr_contrib_sort_bytes): a workspace sized for another algorithm is refused.
  size_t need = 0;
  if (gtr_contrib_sort_bytes(m_cap, num_items, &need) != GTR_OK) return GTR_E_ARG;
  if (!keys || !vals || !skeys || !svals || !tmp || tmp_bytes < need) {
    set_error("gtr_contrib_sort: workspace of %zu bytes < %zu needed (m_cap %d, T %d)", tmp_bytes, need, m_cap,
              num_items);
    return GTR_E_ARG;
  }
  size_t b = tmp_bytes;
  hipError_t e = sort_pairs(tmp, b, keys, skeys, vals, svals, m_cap, key_bits(num_items), (hipStream_t)stream);
  if (e != hipSuccess) { set_error("gtr_contrib_sort: %s", hipGetErrorString(e)); return (int)e; }
  return GTR_OK;
}

int gtr_adamw_rows(const gtr_batch* bt, int num_items, int dim, const int32_t* skeys, const int32_t* svals,
                   const float* dx0, const float* se, const float* coef_tgt, const float* coef_neg, float* table,
                   float* m, float* v, float* grad_dense, const gtr_adam* opt, gtr_stream_t stream) {
  if (!bt || !dim_ok(dim) || !skeys || !svals || !dx0 || !se || !coef_tgt || !coef_neg) {
    set_error("gtr_adamw_rows: bad arguments");
    return GTR_E_ARG;
  }
  if (!grad_dense && (!table || !m || !v || !opt || !opt->step_dev)) {
    set_error("gtr_adamw_rows: missing optimizer state");
    return GTR_E_ARG;
  }
  gtr_adam o{};
  if (opt) o = *opt;
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  const int64_t threads = (int64_t)m_cap * (dim / 4);
  const int blocks = (int)((threads + GTR_BLOCK - 1) / GTR_BLOCK);
  hipStream_t s = (hipStream_t)stream;
#define GTR_ROWS(DD)                                                                                         \
  hipLaunchKernelGGL(k_adamw_rows<DD>, dim3(blocks), dim3(GTR_BLOCK), 0, s, *bt, num_items, skeys, svals, dx0, \
                     se, coef_tgt, coef_neg, table, m, v, grad_dense, o)
  switch (dim) {
    case 32: GTR_ROWS(32); break;
    case 64: GTR_ROWS(64); break;
    case 128: GTR_ROWS(128); break;
    default: GTR_ROWS(256); break;
  }
#undef GTR_ROWS
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_adamw_sweep(int num_items, int dim, const int32_t* stamp, float* table, float* m, float* v,
                    const gtr_adam* opt, gtr_stream_t stream) {
  if (!dim_ok(dim) || !stamp || !table || !m || !v || !opt || !opt->step_dev || num_items <= 0) {
    set_error("gtr_adamw_sweep: bad arguments");
    return GTR_E_ARG;
  }
  const int64_t nvec = (int64_t)num_items * dim / 4;
  int vpr_log2 = 0;
  while ((1 << vpr_log2) < dim / 4) ++vpr_log2;
  int64_t blocks = (nvec + GTR_BLOCK - 1) / GTR_BLOCK;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_adamw_sweep, dim3((unsigned)blocks), dim3(GTR_BLOCK), 0, (hipStream_t)stream, nvec, vpr_log2,
                     stamp, (float4*)table, (float4*)m, (float4*)v, *opt);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_scatter_rows(const gtr_batch* bt, int dim, int mode, const float* src, const float* coef_tgt,
                     const float* coef_neg, float* dense, gtr_stream_t stream) {
  if (!bt || !dim_ok(dim) || !src || !dense || (mode == 1 && (!coef_tgt || !coef_neg))) {
    set_error("gtr_scatter_rows: bad arguments");
    return GTR_E_ARG;
  }
  const int rows = mode == 0 ? bt->n_cap : bt->b_cap * (1 + bt->n_neg);
  const int blocks = (rows + GTR_WAVES - 1) / GTR_WAVES;
  if (blocks <= 0) return GTR_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (dim) {
    case 32: hipLaunchKernelGGL(k_scatter_rows<32>, dim3(blocks), dim3(GTR_BLOCK), 0, s, *bt, mode, src, coef_tgt, coef_neg, dense); break;
    case 64: hipLaunchKernelGGL(k_scatter_rows<64>, dim3(blocks), dim3(GTR_BLOCK), 0, s, *bt, mode, src, coef_tgt, coef_neg, dense); break;
    case 128: hipLaunchKernelGGL(k_scatter_rows<128>, dim3(blocks), dim3(GTR_BLOCK), 0, s, *bt, mode, src, coef_tgt, coef_neg, dense); break;
    default: hipLaunchKernelGGL(k_scatter_rows<256>, dim3(blocks), dim3(GTR_BLOCK), 0, s, *bt, mode, src, coef_tgt, coef_neg, dense); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_step_begin(const gtr_batch* bt, int num_items, int32_t* keys, int32_t* vals, int32_t* skeys,
                   int32_t* svals, int32_t* stamp, int64_t* step_dev, uint32_t* rng_ctr, void* tmp,
                   size_t tmp_bytes, gtr_stream_t stream) {
  if (!bt || !skeys || !svals || !step_dev || bt->n_neg <= 0 || num_items <= 0) {
    set_error("gtr_step_begin: bad arguments");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  if (m_cap <= GTR_BEGIN_MCAP && num_items < GTR_BEGIN_KEY_LIMIT) {
    hipLaunchKernelGGL(k_step_begin, dim3((m_cap + 63) / 64), dim3(GTR_BEGIN_BLOCK), 0, s, *bt, num_items, skeys,
                       svals, stamp, step_dev, rng_ctr);
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  if (!keys || !vals || !tmp) { set_error("gtr_step_begin: large batch needs keys/vals/tmp scratch"); return GTR_E_ARG; }
  if (sort_mode() == 0) {  // the own radix: its first pass builds the list, its last advances the counters
    size_t need = rs_bytes(m_cap);
    if (tmp_bytes < need) { set_error("gtr_step_begin: sort workspace of %zu bytes < %zu", tmp_bytes, need); return GTR_E_ARG; }
    RsPrep pp{};
    pp.bt = *bt; pp.T = num_items; pp.keys = keys; pp.vals = vals; pp.stamp = stamp; pp.step_dev = step_dev;
    RsCtr cc{};
    cc.step_dev = step_dev; cc.rng_ctr = rng_ctr;
    hipError_t e = rs_sort(tmp, keys, skeys, vals, svals, m_cap, key_bits(num_items), s, &cc, &pp);
    if (e != hipSuccess) { set_error("gtr_step_begin: sort: %s", hipGetErrorString(e)); return (int)e; }
    return GTR_OK;
  }
  int rc = gtr_contrib_prep(bt, num_items, keys, vals, stamp, step_dev, stream);
  if (rc) return rc;
  rc = gtr_contrib_sort(keys, vals, skeys, svals, m_cap, num_items, tmp, tmp_bytes, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_counters, dim3(1), dim3(1), 0, s, step_dev, rng_ctr);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_dp_union_stamp(const int32_t* keys_all, int64_t n, int num_items, int32_t* stamp, const int64_t* step_dev,
                       gtr_stream_t stream) {
  if (!keys_all || n < 0 || num_items <= 0 || !stamp || !step_dev) {
    set_error("gtr_dp_union_stamp: bad arguments");
    return GTR_E_ARG;
  }
  if (n == 0) return GTR_OK;
  hipLaunchKernelGGL(k_dp_union_stamp, dim3((unsigned)((n + GTR_BLOCK - 1) / GTR_BLOCK)), dim3(GTR_BLOCK), 0,
                     (hipStream_t)stream, keys_all, n, num_items, stamp, step_dev);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

// Grid of k_lazy_catchup: 8 workgroups (32 waves) per CU; GTR_CATCHUP_BLOCKS overrides.
static int lazy_catchup_blocks() {
  static int blocks = 0;
  if (blocks <= 0) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const char* e = getenv("GTR_CATCHUP_BLOCKS");
    blocks = e && atoi(e) > 0 ? atoi(e) : 8 * cus;
  }
  return blocks;
}

int gtr_step_begin_lazy(const gtr_batch* bt, int num_items, int dim, int32_t* keys, int32_t* vals, int32_t* skeys,
                        int32_t* svals, int32_t* stamp, int64_t* step_dev, uint32_t* rng_ctr, void* tmp,
                        size_t tmp_bytes, const gtr_lazy* lazy, gtr_stream_t stream) {
  if (!bt || !skeys || !svals || !step_dev || !stamp || bt->n_neg <= 0 || num_items <= 0 || !dim_ok(dim) || !lazy ||
      !lazy->consts || !lazy->cnt || !lazy->table || !lazy->m || !lazy->v) {
    set_error("gtr_step_begin_lazy: bad arguments");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  if (m_cap <= GTR_BEGIN_MCAP && num_items < GTR_BEGIN_KEY_LIMIT) {
    hipLaunchKernelGGL(k_step_begin_lazy, dim3((m_cap + 63) / 64), dim3(GTR_BEGIN_BLOCK), 0, s, *bt, num_items, dim,
                       skeys, svals, stamp, step_dev, rng_ctr, *lazy);
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  if (!keys || !vals || !tmp) { set_error("gtr_step_begin_lazy: large batch needs keys/vals/tmp scratch"); return GTR_E_ARG; }
  // own radix (default): the list is built in its first pass, the counters and consts[t]
  // advance in its last, and the catch-up reads the advanced step (adv = 1)
  const bool own = sort_mode() == 0;
  if (own) {
    size_t need = rs_bytes(m_cap);
    if (tmp_bytes < need) {
      set_error("gtr_step_begin_lazy: sort workspace of %zu bytes < %zu", tmp_bytes, need);
      return GTR_E_ARG;
    }
    RsPrep pp{};
    pp.bt = *bt; pp.T = num_items; pp.keys = keys; pp.vals = vals; pp.stamp = nullptr; pp.step_dev = step_dev;
    RsCtr cc{};
    cc.step_dev = step_dev; cc.rng_ctr = rng_ctr; cc.consts = lazy->consts; cc.opt = lazy->opt;
    hipError_t e = rs_sort(tmp, keys, skeys, vals, svals, m_cap, key_bits(num_items), s, &cc, &pp);
    if (e != hipSuccess) { set_error("gtr_step_begin_lazy: sort: %s", hipGetErrorString(e)); return (int)e; }
  } else {
    int rc = gtr_contrib_prep(bt, num_items, keys, vals, nullptr, step_dev, stream);
    if (rc) return rc;
    rc = gtr_contrib_sort(keys, vals, skeys, svals, m_cap, num_items, tmp, tmp_bytes, stream);
    if (rc) return rc;
  }
  const int adv = own ? 1 : 0;
  {
    const int blocks = lazy_catchup_blocks();
    const int64_t tasks_per_wave = 2, waves = (int64_t)blocks * (GTR_BLOCK / 64);
    int spw = 1;
    while (spw < 64 && (int64_t)spw * 2 * waves * tasks_per_wave <= m_cap) spw *= 2;
    if (const char* e = getenv("GTR_CATCHUP_SPW")) spw = std::max(1, std::min(64, atoi(e)));
    const int spb = spw * (GTR_BLOCK / 64);
    const int grid = std::max(1, std::min((m_cap + spb - 1) / spb, blocks));
    if (dim <= 64) hipLaunchKernelGGL(k_lazy_catchup<1>, dim3(grid), dim3(GTR_BLOCK), 0, s, skeys, m_cap, num_items, dim, stamp, step_dev, *lazy, spw, adv);
    else if (dim == 128) hipLaunchKernelGGL(k_lazy_catchup<2>, dim3(grid), dim3(GTR_BLOCK), 0, s, skeys, m_cap, num_items, dim, stamp, step_dev, *lazy, spw, adv);
    else hipLaunchKernelGGL(k_lazy_catchup<4>, dim3(grid), dim3(GTR_BLOCK), 0, s, skeys, m_cap, num_items, dim, stamp, step_dev, *lazy, spw, adv);
    GTR_HIP_CHECK_LAUNCH();
  }
  if (!own) {
    hipLaunchKernelGGL(k_counters_lazy, dim3(1), dim3(1), 0, s, step_dev, rng_ctr, *lazy);
    GTR_HIP_CHECK_LAUNCH();
  }
  return GTR_OK;
}

int gtr_lazy_flush(int num_items, int dim, int32_t* stamp, const int64_t* step_dev, const gtr_lazy* lazy,
                   gtr_stream_t stream) {
  if (!stamp || !step_dev || !dim_ok(dim) || num_items <= 0 || !lazy || !lazy->consts || !lazy->table ||
      !lazy->m || !lazy->v) {
    set_error("gtr_lazy_flush: bad arguments");
    return GTR_E_ARG;
  }
  const int64_t threads = (int64_t)num_items * (dim / 4);
  hipLaunchKernelGGL(k_lazy_flush, dim3((unsigned)((threads + GTR_BLOCK - 1) / GTR_BLOCK)), dim3(GTR_BLOCK), 0,
                     (hipStream_t)stream, num_items, dim, stamp, step_dev, *lazy);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_step_tail(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail, const gtr_segment* segs,
                  int nseg, const gtr_adam* opt, gtr_stream_t stream) {
  if (!bt || !tail || !opt || !opt->step_dev || !dim_ok(dim) || num_items <= 0 || nseg < 0 ||
      nseg > GTR_SMALL_MAX_SEG || (nseg > 0 && !segs)) {
    set_error("gtr_step_tail: bad arguments");
    return GTR_E_ARG;
  }
  const gtr_tail& t = *tail;
  if (!t.skeys || !t.svals || !t.dx0 || !t.se || !t.coef_tgt || !t.coef_neg || !t.table || !t.table_m ||
      !t.table_v || !t.stamp || (nseg > 0 && (!t.flat || !t.flat_m || !t.flat_v)) ||
      (t.loss_part && (!t.loss_out || t.loss_nparts < 0))) {
    set_error("gtr_step_tail: missing buffers");
    return GTR_E_ARG;
  }
  TailK k{};
  k.bt = *bt;
  k.tl = t;
  k.opt = *opt;
  k.T = num_items;
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  hipStream_t s = (hipStream_t)stream;
  k.windowed = m_cap > GTR_BEGIN_MCAP ? 1 : 0;
  if (k.windowed) {
    if (!t.carry) { set_error("gtr_step_tail: large batch (m_cap > %d) needs the carry scratch", GTR_BEGIN_MCAP); return GTR_E_ARG; }
    const int nwin = (m_cap + TW - 1) / TW;
    k.nb_rows = nwin;
    if (nwin > 1) {
#define GTR_CARRY(DD) hipLaunchKernelGGL(k_tail_carry<DD>, dim3(carry_blocks(m_cap)), dim3(GTR_BLOCK), 0, s, *bt, num_items, t)
      switch (dim) {
        case 32: GTR_CARRY(32); break;
        case 64: GTR_CARRY(64); break;
        case 128: GTR_CARRY(128); break;
        default: GTR_CARRY(256); break;
      }
#undef GTR_CARRY
      GTR_HIP_CHECK_LAUNCH();
    }
  } else {
    k.nb_rows = (int)(((int64_t)m_cap * (dim / 4) + GTR_BLOCK - 1) / GTR_BLOCK);
  }
  k.nb_small = nseg > 0 ? (int)((t.flat_total + GTR_BLOCK - 1) / GTR_BLOCK) : 0;
  if (k.nb_small == 0 && (t.loss_part || t.loss_acc)) k.nb_small = 1;
  k.nvec = (int64_t)num_items * dim / 4;
  k.vpr_log2 = 0;
  while ((1 << k.vpr_log2) < dim / 4) ++k.vpr_log2;
  const int64_t from = t.lazy_consts ? num_items  // lazy: no untouched-row sweep
                                      : (t.sweep_from < 0 ? 0 : (t.sweep_from > num_items ? num_items : t.sweep_from));
  k.vbegin = from * (dim / 4);
  int64_t sw = (k.nvec - k.vbegin + GTR_BLOCK - 1) / GTR_BLOCK;
  k.nb_sweep = (int)(sw > 2048 ? 2048 : sw);
  k.nseg = nseg;
  for (int i = 0; i < nseg; ++i) k.segs[i] = segs[i];
  const int grid = k.nb_rows + k.nb_small + k.nb_sweep;
  switch (dim) {
#define GTR_TAIL(DD) if (k.windowed) hipLaunchKernelGGL((k_step_tail<DD, false>), dim3(grid), dim3(GTR_BLOCK), 0, s, k); \
  else hipLaunchKernelGGL((k_step_tail<DD, true>), dim3(grid), dim3(GTR_TAIL_BLOCK), 0, s, k)
    case 32: GTR_TAIL(32); break;
    case 64: GTR_TAIL(64); break;
    case 128: GTR_TAIL(128); break;
    default: GTR_TAIL(256); break;
#undef GTR_TAIL
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_step_tail_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, const float* pe_tab,
                        float* const* layer_slab, float* pe_slab, int n_chunks, int64_t slab_stride,
                        const int64_t* layer_flat, const int64_t* pe_flat, int num_items, const gtr_tail* tail,
                        const gtr_segment* segs, int nseg, const gtr_adam* opt, uint32_t* tile_cnt, int tile_cnt_len,
                        gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !layer_slab || !layer_flat || !tail || !opt || !opt->step_dev || num_items <= 0 ||
      nseg < 0 || nseg > GTR_TAILW_SEGS || (nseg > 0 && !segs) || !dim_ok(cfg->dim) || n_chunks <= 0 ||
      !tile_cnt || 3 * cfg->num_layers + 1 > GTR_MAX_WJOBS) {
    set_error("gtr_step_tail_wgrad: bad arguments");
    return GTR_E_ARG;
  }
  const gtr_tail& t = *tail;
  const int D = cfg->dim;
  const int m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  if (m_cap > GTR_BEGIN_MCAP) {
    set_error("gtr_step_tail_wgrad: batch too large (m_cap %d > %d): use gtr_wgrad + gtr_step_tail", m_cap,
              GTR_BEGIN_MCAP);
    return GTR_E_ARG;
  }
  if (!t.lazy_consts && t.sweep_from < num_items) {
    set_error("gtr_step_tail_wgrad: the untouched-row sweep must run in the chain (sweep_from == num_items)");
    return GTR_E_ARG;
  }
  if (!t.skeys || !t.svals || !t.dx0 || !t.se || !t.coef_tgt || !t.coef_neg || !t.table || !t.table_m ||
      !t.table_v || !t.stamp || !t.flat || !t.flat_m || !t.flat_v || (t.loss_part && (!t.loss_out || t.loss_nparts < 0))) {
    set_error("gtr_step_tail_wgrad: missing buffers");
    return GTR_E_ARG;
  }
  TailWK k{};
  k.bt = *bt;
  k.tl = t;
  k.opt = *opt;
  k.T = num_items;
  k.D = D;
  k.P = n_chunks;
  k.stride = slab_stride;
  k.cnt = tile_cnt;
  // the same tile form k_wgrad would pick for these chunks (GTR_WGRAD=mfma|valu overrides)
  const char* wm = getenv("GTR_WGRAD");
  bool mfma = (bt->n_cap + n_chunks - 1) / n_chunks >= GTR_WGRAD_MFMA_ROWS;
  if (wm && !strcmp(wm, "mfma")) mfma = true;
  if (wm && !strcmp(wm, "valu")) mfma = false;
  if (slab_stride % 4) mfma = false;
  for (int l = 0; l < cfg->num_layers; ++l)
    if (reinterpret_cast<uintptr_t>(layer_slab[l]) % 16) mfma = false;
  int nj = 0, wblocks = 0;
  const int rc = build_wjobs(cfg, bt, layers, t.dx0, pe_tab, layer_slab, pe_slab, layer_flat, pe_flat, n_chunks, 0,
                             cfg->num_layers, k.jobs, nj, wblocks, mfma);
  if (rc) return rc;
  int tiles = 0;
  for (int i = 0; i < nj; ++i) {
    k.jobs[i].tile0 = tiles;
    tiles += k.jobs[i].nt;
    if (k.jobs[i].fW < 0 && k.jobs[i].fB < 0) { set_error("gtr_step_tail_wgrad: a job without flat offsets"); return GTR_E_ARG; }
  }
  if (tiles > tile_cnt_len) {
    set_error("gtr_step_tail_wgrad: %d tile counters needed, %d given", tiles, tile_cnt_len);
    return GTR_E_ARG;
  }
  k.njobs = nj;
  k.nb_wg = wblocks;
  k.nb_rows = (int)(((int64_t)m_cap * (D / 4) + GTR_BLOCK - 1) / GTR_BLOCK);
  int64_t tot = 0;
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].live_groups) { set_error("gtr_step_tail_wgrad: folded (per row group) weight gradients"); return GTR_E_ARG; }
    k.segs[i] = segs[i];
    tot += segs[i].len;
  }
  k.nseg = nseg;
  k.small_total = (int)tot;
  k.nb_small = (int)((tot + GTR_BLOCK - 1) / GTR_BLOCK);
  if (k.nb_small == 0 && (t.loss_part || t.loss_acc)) k.nb_small = 1;
  const int grid = k.nb_wg + k.nb_rows + k.nb_small;
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 32: hipLaunchKernelGGL(k_step_tail_wgrad<32>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_step_tail_wgrad<64>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_step_tail_wgrad<128>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_step_tail_wgrad<256>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

static bool dp_layout_ok(const gtr_dp_layout* l, int dim) {
  return l && l->world >= 1 && l->m_cap > 0 && l->flat_total >= 0 && l->loss_off >= l->flat_total &&
         l->keys_off > l->loss_off && l->rows_off >= l->keys_off + l->m_cap && (l->rows_off & 3) == 0 &&
         l->words >= l->rows_off + (int64_t)l->m_cap * dim && (l->words & 3) == 0;
}

int gtr_dp_pack(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail, const gtr_segment* segs, int nseg,
                const gtr_dp_layout* lay, float* pack, gtr_stream_t stream) {
  if (!bt || !tail || !pack || !dim_ok(dim) || !dp_layout_ok(lay, dim) || nseg < 0 || nseg > GTR_SMALL_MAX_SEG ||
      lay->m_cap != bt->n_cap + bt->b_cap * (1 + bt->n_neg) || !tail->skeys || !tail->svals || !tail->dx0 ||
      !tail->se || !tail->coef_tgt || !tail->coef_neg || (!tail->loss_part && !tail->loss_out)) {
    set_error("gtr_dp_pack: bad arguments");
    return GTR_E_ARG;
  }
  DpPackK k{};
  k.bt = *bt;
  k.tl = *tail;
  k.lay = *lay;
  k.pack = pack;
  k.T = num_items;
  hipStream_t s = (hipStream_t)stream;
  // large batches: segment sums in window pieces + carries, as the single-GPU tail sums them
  k.windowed = lay->m_cap > GTR_BEGIN_MCAP ? 1 : 0;
  if (k.windowed) {
    if (!tail->carry) { set_error("gtr_dp_pack: large batch (m_cap > %d) needs the carry scratch", GTR_BEGIN_MCAP); return GTR_E_ARG; }
    const int nwin = (lay->m_cap + TW - 1) / TW;
    k.nb_rows = nwin;
    if (nwin > 1) {
      switch (dim) {
        case 32: hipLaunchKernelGGL(k_tail_carry<32>, dim3(carry_blocks(lay->m_cap)), dim3(GTR_BLOCK), 0, s, *bt, num_items, *tail); break;
        case 64: hipLaunchKernelGGL(k_tail_carry<64>, dim3(carry_blocks(lay->m_cap)), dim3(GTR_BLOCK), 0, s, *bt, num_items, *tail); break;
        case 128: hipLaunchKernelGGL(k_tail_carry<128>, dim3(carry_blocks(lay->m_cap)), dim3(GTR_BLOCK), 0, s, *bt, num_items, *tail); break;
        default: hipLaunchKernelGGL(k_tail_carry<256>, dim3(carry_blocks(lay->m_cap)), dim3(GTR_BLOCK), 0, s, *bt, num_items, *tail); break;
      }
      GTR_HIP_CHECK_LAUNCH();
    }
  } else {
    k.nb_rows = (int)(((int64_t)lay->m_cap * (dim / 4) + GTR_BLOCK - 1) / GTR_BLOCK);
  }
  k.nb_small = (int)((lay->flat_total + GTR_BLOCK - 1) / GTR_BLOCK);
  if (k.nb_small == 0) k.nb_small = 1;
  k.nseg = nseg;
  for (int i = 0; i < nseg; ++i) k.segs[i] = segs[i];
  const int grid = k.nb_rows + k.nb_small;
  switch (dim) {
    case 32: hipLaunchKernelGGL(k_dp_pack<32>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_dp_pack<64>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_dp_pack<128>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_dp_pack<256>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_dp_tail(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail, const gtr_dp_layout* lay,
                const float* recv, int32_t* slot, const gtr_adam* opt, gtr_stream_t stream) {
  if (!bt || !tail || !recv || !slot || !opt || !opt->step_dev || !dim_ok(dim) || !dp_layout_ok(lay, dim) ||
      num_items <= 0 || !tail->table || !tail->table_m || !tail->table_v || !tail->stamp ||
      (lay->flat_total > 0 && (!tail->flat || !tail->flat_m || !tail->flat_v))) {
    set_error("gtr_dp_tail: bad arguments");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t slots = (int64_t)lay->world * lay->m_cap;
  // eager: stamp the union (the tail's sweep skips it) and build the (row, rank) slot
  // table; lazy stamps need neither -- each rank's sorted keys are binary-searched
  const bool search = tail->lazy_consts != nullptr;
  if (!search) {
    hipLaunchKernelGGL(k_dp_stamp, dim3((unsigned)((slots + GTR_BLOCK - 1) / GTR_BLOCK)), dim3(GTR_BLOCK), 0, s,
                       *lay, num_items, recv, tail->lazy_consts ? nullptr : tail->stamp,
                       reinterpret_cast<int2*>(slot), opt->step_dev, opt->step_offset);
    GTR_HIP_CHECK_LAUNCH();
  }
  DpTailK k{};
  k.tl = *tail;
  k.lay = *lay;
  k.opt = *opt;
  k.recv = recv;
  k.slot = search ? nullptr : reinterpret_cast<const int2*>(slot);
  k.T = num_items;
  k.nb_rows = (int)((slots * (dim / 4) + GTR_BLOCK - 1) / GTR_BLOCK);
  k.nb_small = (int)((lay->flat_total + 1 + GTR_BLOCK - 1) / GTR_BLOCK);
  k.nvec = (int64_t)num_items * dim / 4;
  k.vpr_log2 = 0;
  while ((1 << k.vpr_log2) < dim / 4) ++k.vpr_log2;
  // rows below sweep_from were swept inside the backward (early union stamp + gtr_sweep)
  const int64_t from = tail->sweep_from < 0 ? 0 : (tail->sweep_from > num_items ? num_items : tail->sweep_from);
  k.vbegin = from * (dim / 4);
  int64_t sw = (k.nvec - k.vbegin + GTR_BLOCK - 1) / GTR_BLOCK;
  k.nb_sweep = (tail->lazy_consts || sw <= 0) ? 0 : (int)(sw > 2048 ? 2048 : sw);  // lazy: no sweep
  const int grid = k.nb_rows + k.nb_small + k.nb_sweep;
  switch (dim) {
    case 32: hipLaunchKernelGGL(k_dp_tail<32>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_dp_tail<64>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_dp_tail<128>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_dp_tail<256>, dim3(grid), dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_step_end(int64_t* step_dev, uint32_t* rng_ctr, const float* loss_part, int nparts, float* loss_out,
                 gtr_stream_t stream) {
  if (loss_part && (nparts < 0 || !loss_out)) { set_error("gtr_step_end: bad loss partials"); return GTR_E_ARG; }
  hipLaunchKernelGGL(k_step_end, dim3(1), dim3(64), 0, (hipStream_t)stream, step_dev, rng_ctr, loss_part, nparts,
                     loss_out);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

}  // extern "C"
