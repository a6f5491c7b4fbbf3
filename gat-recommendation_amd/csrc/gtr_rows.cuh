// gtr_rows.cuh — device helpers shared by the optimizer kernels (gtr_opt.hip) and the
// row-sharded table exchange (gtr_shard.hip): small-parameter segments, the lazy-table
// catch-up of zero-gradient AdamW steps, and the segmented sum of a row's sorted
// table-gradient contributions.
#pragma once

#include "gtr_common.cuh"

namespace gtr {

#define GTR_BEGIN_MCAP 8192            // contributions ranked in LDS by the one-launch begin
#define GTR_BEGIN_KEY_LIMIT (1 << 19)  // rows a (row << 13 | slot) composite key can hold

// Contribution key of slot j (sentinel T for unused slots), see gtr_contrib_prep.
__device__ __forceinline__ int contrib_key(const gtr_batch& bt, int T, int j, int N, int B) {
  int key = T;
  if (j < bt.n_cap) {
    if (j < N) key = bt.node_item[j];
  } else if (j < bt.n_cap + bt.b_cap) {
    const int b = j - bt.n_cap;
    if (b < B) key = bt.target[b];
  } else {
    const int q = j - bt.n_cap - bt.b_cap;
    if (q / bt.n_neg < B) key = bt.negatives[q];
  }
  if (key < 0 || key > T) key = T;
  return key;
}

// No-op stand-in for the step-scalar wait of k_step_tail (bodies called with ready scalars).
struct NoWait {
  __device__ __forceinline__ void operator()() const {}
};

// Small parameters: element e of the flat buffer; its segment's gradient partials summed.
// hdr: the batch header (segments with live_groups sum only its hdr[4] row groups' partials;
// null: no such segment).  wait(): called after every load is issued, before `st` is first read.
template <class Wait = NoWait>
__device__ __forceinline__ void small_body(int64_t e, const gtr_segment* segs, int nseg, const int32_t* hdr,
                                           float* param, float* m, float* v, float* grad_out, const AdamStep& st,
                                           Wait wait = Wait{}) {
  int s = -1;
  for (int i = 0; i < nseg; ++i)
    if (e >= segs[i].begin && e < segs[i].begin + segs[i].len) s = i;
  if (s < 0) return;
  const gtr_segment& sg = segs[s];
  const int64_t off = e - sg.begin;
  float g = 0.0f;
  const int np = sg.nparts;
  // live row groups (wfold partials): the count is loaded beside the partials, not before
  // them (every partial slot is allocated; dead groups' slots are read and skipped)
  const int live = (sg.live_groups && hdr) ? hdr[4] : np;
  for (int p0 = 0; p0 < np; p0 += 8) {
    float pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pv[u] = p0 + u < np ? sg.src[(int64_t)(p0 + u) * sg.pstride + off] : 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (p0 + u < live) g += pv[u];
  }
  if (grad_out) {
    grad_out[e] = g;
    return;
  }
  float pv = param[e], mv = m[e], vv = v[e];
  wait();
  st.apply(pv, mv, vv, g);
  param[e] = pv;
  m[e] = mv;
  v[e] = vv;
}

// Lazy table: bring one float4 column of a row from its stamp to step `upto` with the
// zero-gradient update of each step in order (AdamStep with step t's scalars from
// consts[t]): the same float operations as the eager sweep applies, so bitwise equal.
__device__ __forceinline__ void catch_up4(float4& p, float4& m, float4& v, int from, int upto, const gtr_adam& o,
                                          const float* consts) {
  if (from >= upto) return;
  AdamStep st;
  st.lr = o.lr; st.b1 = o.beta1; st.b2 = o.beta2; st.eps = o.eps; st.wd = o.weight_decay;
  st.decoupled = o.decoupled;
  st.decay_mul = (float)(1.0 - (double)o.lr * (double)o.weight_decay);
  // the steps' scalars 8 at a time: one load latency per 8 steps on the chain, not per step
  for (int t0 = from + 1; t0 <= upto; t0 += 8) {
    float2 c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      c[u] = t0 + u <= upto ? reinterpret_cast<const float2*>(consts)[t0 + u] : make_float2(0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (t0 + u > upto) break;
      st.step_size = c[u].x;
      st.inv_bc2 = c[u].y;
      st.apply(p.x, m.x, v.x, 0.0f);
      st.apply(p.y, m.y, v.y, 0.0f);
      st.apply(p.z, m.z, v.z, 0.0f);
      st.apply(p.w, m.w, v.w, 0.0f);
    }
  }
}

// Lazy table, one read-modify-write of m / v per touched row (decoupled AdamW): the
// begin's catch-up claims a lagging row by setting GTR_LAZY_CLAIM in its stamp (the low
// bits keep the step the row was current through), brings p forward to t-1 and writes p
// ONLY; the tail reads the claimed stamp, re-derives m / v over the same missed steps
// (apply_zero_mv: their zero-gradient chain does not involve p, so the floats are the
// catch-up's own), applies step t and stamps t.  Plain Adam (L2 in the gradient) couples
// m to p: there the catch-up writes all three and the tail re-derives nothing.
// GTR_LAZY_PONLY=0 restores the full catch-up write (A/B).
#define GTR_LAZY_CLAIM 0x40000000
#ifndef GTR_LAZY_PONLY
#define GTR_LAZY_PONLY 1
#endif
__device__ __forceinline__ bool lazy_p_only(int decoupled) { return GTR_LAZY_PONLY && decoupled; }

// Tail side: a claimed row's m / v brought from its stamp to t-1 (no-op when the catch-up
// wrote them, or the row was current).
__device__ __forceinline__ void lazy_mv_forward(float4& m, float4& v, int32_t stamp_word, int32_t t,
                                                const AdamStep& st) {
  if (!(stamp_word & GTR_LAZY_CLAIM) || !lazy_p_only(st.decoupled)) return;
  for (int s = (stamp_word & ~GTR_LAZY_CLAIM) + 1; s <= t - 1; ++s) {
    st.apply_zero_mv(m.x, v.x);
    st.apply_zero_mv(m.y, v.y);
    st.apply_zero_mv(m.z, v.z);
    st.apply_zero_mv(m.w, v.w);
  }
}

// consts[t] exactly as AdamStep::init computes the step's scalars.
__device__ __forceinline__ void lazy_consts_for(const gtr_adam& o, int64_t t, float* consts) {
  AdamStep st;
  st.init(o, t);
  reinterpret_cast<float2*>(consts)[t] = make_float2(st.step_size, st.inv_bc2);
}

#ifndef GTR_TAIL_TW
#define GTR_TAIL_TW 128
#endif
#define TW GTR_TAIL_TW  // slots per window of the large-batch segmented sums (below)

// Sum of contributions in slots [s, e) for column float4 `gl` by the C4 = D/4 lanes of
// one group (group base lane gb): slot ids are fetched one per lane, decoded to a source
// row (dx0 node row, or se session row for target / negative slots) + coefficient,
// then broadcast QF at a time so QF row loads are in flight per lane (the sum runs in slot
// order whatever QF is: bitwise the same).
template <int D, int QF = 8>
__device__ __forceinline__ float4 piece_sum(const gtr_batch& bt, const int32_t* svals, int s, int e, const float* dx0,
                                            const float* se, const float* coef_tgt, const float* coef_neg, int gl,
                                            int gb) {
  constexpr int C4 = D / 4;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = s; base < e; base += C4) {
    const int cnt = min(C4, e - base);
    int code = 0;
    float cf = 0.0f;
    if (gl < cnt) {
      const int j = svals[base + gl];
      if (j < bt.n_cap) {
        code = j;
        cf = 1.0f;
      } else if (j < bt.n_cap + bt.b_cap) {
        const int b = j - bt.n_cap;
        code = (int)(0x80000000u | (uint32_t)b);
        cf = coef_tgt[b];
      } else {
        const int q = j - bt.n_cap - bt.b_cap;
        code = (int)(0x80000000u | (uint32_t)(q / bt.n_neg));
        cf = coef_neg[q];
      }
    }
    for (int q0 = 0; q0 < cnt; q0 += QF) {
      float4 v[QF];
      float f[QF];
#pragma unroll
      for (int u = 0; u < QF; ++u) {
        const int cq = __shfl(code, gb + ((q0 + u) & (C4 - 1)));
        f[u] = __shfl(cf, gb + ((q0 + u) & (C4 - 1)));
#ifdef GTR_DBG_TAIL_SE0  // timing probe only (wrong sums): every session-row read hits row 0
        const float* src = cq < 0 ? se : dx0 + (size_t)cq * D;
#else
        const float* src = cq < 0 ? se + (size_t)(cq & 0x7FFFFFFF) * D : dx0 + (size_t)cq * D;
#endif
        v[u] = q0 + u < cnt ? reinterpret_cast<const float4*>(src)[gl] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < QF; ++u) {
        if (q0 + u < cnt) {
          g.x += f[u] * v[u].x; g.y += f[u] * v[u].y; g.z += f[u] * v[u].z; g.w += f[u] * v[u].w;
        }
      }
    }
  }
  return g;
}

// The slots of one window decoded once, one slot per thread and all at once, into LDS:
// sort key, source code (dx0 node row, or session row with the top bit set) and
// coefficient -- exactly what piece_sum decodes per chunk.  The window's segment sums then
// start from LDS instead of two dependent global rounds (slot id, then its coefficient)
// per chunk of every segment.  No barrier here: the callers' window_bounds barriers
// publish the writes.
#ifndef GTR_WIN_LDS
#define GTR_WIN_LDS 1
#endif
struct WinSlots {
  int key[TW];
  int code[TW];
  float cf[TW];
};
__device__ __forceinline__ void window_decode(const gtr_batch& bt, const int32_t* skeys, const int32_t* svals,
                                              const float* coef_tgt, const float* coef_neg, int w0, int w1,
                                              WinSlots& ws) {
  const int tid = threadIdx.x;
  if (tid < TW && w0 + tid < w1) {
    const int j = svals[w0 + tid];
    int code;
    float cf;
    if (j < bt.n_cap) {
      code = j;
      cf = 1.0f;
    } else if (j < bt.n_cap + bt.b_cap) {
      const int b = j - bt.n_cap;
      code = (int)(0x80000000u | (uint32_t)b);
      cf = coef_tgt[b];
    } else {
      const int q = j - bt.n_cap - bt.b_cap;
      code = (int)(0x80000000u | (uint32_t)(q / bt.n_neg));
      cf = coef_neg[q];
    }
    ws.key[tid] = skeys[w0 + tid];
    ws.code[tid] = code;
    ws.cf[tid] = cf;
  }
}

// piece_sum over slots [s, e) of window w0 with the decoded slots in LDS: the same products
// added in the same slot order (bitwise piece_sum's sum); QF rows in flight per lane.
template <int D, int QF = 8>
__device__ __forceinline__ float4 piece_sum_lds(const WinSlots& ws, int w0, int s, int e, const float* dx0,
                                                const float* se, int gl) {
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int q0 = s; q0 < e; q0 += QF) {
    float4 v[QF];
    float f[QF];
#pragma unroll
    for (int u = 0; u < QF; ++u) {
      const bool in = q0 + u < e;
      const int k = in ? q0 + u - w0 : 0;
      const int cq = ws.code[k];
      f[u] = ws.cf[k];
      const float* src = cq < 0 ? se + (size_t)(cq & 0x7FFFFFFF) * D : dx0 + (size_t)cq * D;
      v[u] = in ? reinterpret_cast<const float4*>(src)[gl] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < QF; ++u) {
      if (q0 + u < e) {
        g.x += f[u] * v[u].x; g.y += f[u] * v[u].y; g.z += f[u] * v[u].z; g.w += f[u] * v[u].w;
      }
    }
  }
  return g;
}

// ---- large batches (m_cap > GTR_BEGIN_MCAP): windowed segmented sums ------------------
// The sorted contribution list is cut into windows of TW slots.  A row's segment that
// starts in window w is summed by window w's block over its in-window part; the part
// lying in each following window w' (it can span many: hot Zipf items collect thousands
// of node contributions) is a "carry" summed beforehand (tail_carry_wave), so no thread
// walks a long segment serially.  Sums run in slot order inside a piece and pieces are
// added in window order: deterministic.  The single-GPU tail, the data-parallel pack and
// the row-sharded pack all sum this way, so their segment sums are bitwise equal.

// Carry of window w (>= 1) whose first slot continues the previous window's segment:
// the sum over [w*TW, first key change in w), split over the block's groups in fixed
// contiguous pieces and combined in group order -- a whole block per window, used up to
// GTR_CARRY_WAVE_WINDOWS windows (a hot row's full-window piece then runs in 8 parallel
// pieces, the launch's critical path at a few hundred windows).  carry: [nwin][D].
// Block-uniform exit.
template <int D, int BLOCK>
__device__ __forceinline__ void tail_carry_body(int w, const gtr_batch& bt, int T, const int32_t* skeys,
                                                const int32_t* svals, const float* dx0, const float* se,
                                                const float* coef_tgt, const float* coef_neg, float* carry) {
  constexpr int C4 = D / 4, NG = BLOCK / C4;
  __shared__ int s_end;
  __shared__ __attribute__((aligned(16))) float4 s_part[NG][C4];
  const int tid = threadIdx.x;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int w0 = w * TW, w1 = min(w0 + TW, m_cap);
  const int key = skeys[w0];
  if (key <= 0 || key >= T || skeys[w0 - 1] != key) return;  // block-uniform
  if (tid == 0) s_end = w1;
  __syncthreads();
  if (tid < TW && w0 + tid < w1 && skeys[w0 + tid] != key) atomicMin(&s_end, w0 + tid);
  __syncthreads();
  const int e = s_end;
  const int grp = tid / C4, gl = tid % C4;
  const int len = e - w0, per = (len + NG - 1) / NG;
  const int ps = min(e, w0 + grp * per), pe = min(e, ps + per);
  s_part[grp][gl] = piece_sum<D>(bt, svals, ps, pe, dx0, se, coef_tgt, coef_neg, gl, grp * C4 % 64);
  __syncthreads();
  if (tid < C4) {
    float4 g = s_part[0][tid];
    for (int q = 1; q < NG; ++q) {
      const float4 t = s_part[q][tid];
      g.x += t.x; g.y += t.y; g.z += t.z; g.w += t.w;
    }
    reinterpret_cast<float4*>(carry)[(size_t)w * C4 + tid] = g;
  }
}

// Carry of window w (>= 1) whose first slot continues the previous window's segment: the
// sum over [w*TW, first key change in w), by ONE wave (the window's few slots did not fill
// a 256-thread block: round 5's block per window spent 23 us of launch at 6,680 windows).
// The wave's 64 / C4 lane groups take contiguous pieces in order and are combined in group
// order.  carry: [nwin][D].  Wave-uniform exit; s_part: this wave's [64 / C4][C4] scratch.
template <int D>
__device__ __forceinline__ void tail_carry_wave(int w, const gtr_batch& bt, int T, const int32_t* skeys,
                                                const int32_t* svals, const float* dx0, const float* se,
                                                const float* coef_tgt, const float* coef_neg, float* carry,
                                                float4* s_part) {
  constexpr int C4 = D / 4, NGW = 64 / C4;
  const int lane = threadIdx.x & 63;
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  const int w0 = w * TW, w1 = min(w0 + TW, m_cap);
  if (w0 >= m_cap) return;
  const int key = skeys[w0];
  if (key <= 0 || key >= T || skeys[w0 - 1] != key) return;  // wave-uniform
  int e = w1;  // the segment's end inside the window
  for (int b = w0; b < w1; b += 64) {
    const int k = b + lane;
    const unsigned long long bal = __ballot(k < w1 && skeys[k] != key);
    if (bal) {
      e = b + __ffsll((long long)bal) - 1;
      break;
    }
  }
  const int grp = lane / C4, gl = lane % C4;
  const int len = e - w0, per = (len + NGW - 1) / NGW;
  const int ps = min(e, w0 + grp * per), pe = min(e, ps + per);
  s_part[grp * C4 + gl] = piece_sum<D>(bt, svals, ps, pe, dx0, se, coef_tgt, coef_neg, gl, grp * C4);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < C4) {
    float4 g = s_part[lane];
    for (int q = 1; q < NGW; ++q) {
      const float4 t = s_part[q * C4 + lane];
      g.x += t.x; g.y += t.y; g.z += t.z; g.w += t.w;
    }
    reinterpret_cast<float4*>(carry)[(size_t)w * C4 + lane] = g;
  }
}

// Carries by wave (GTR_BLOCK / 64 windows per workgroup) from this many windows on, by
// block below: C3 B = 8192 (6,680 windows) tail + carry 112 -> 105 us by wave; C3 B = 1024
// (840 windows) 66 -> 71 us by wave, where a hot row's full-window piece in 2 instead of 8
// parallel pieces sets the launch.  Both variants sum every tail kind (single GPU, data
// parallel, row-sharded) the same way for a given m_cap.
#define GTR_CARRY_WAVE_WINDOWS 2048
__host__ __device__ inline bool carry_by_wave(int m_cap) { return (m_cap + TW - 1) / TW >= GTR_CARRY_WAVE_WINDOWS; }

// Launch of the carries (windows 1 .. nwin - 1): workgroups of the launch.
__host__ __device__ inline int carry_blocks(int m_cap) {
  const int nwin = (m_cap + TW - 1) / TW;
  if (nwin <= 1) return 0;
  return carry_by_wave(m_cap) ? (nwin - 1 + GTR_BLOCK / 64 - 1) / (GTR_BLOCK / 64) : nwin - 1;
}

template <int D>
__device__ __forceinline__ void tail_carry_block(const gtr_batch& bt, int T, const int32_t* skeys,
                                                 const int32_t* svals, const float* dx0, const float* se,
                                                 const float* coef_tgt, const float* coef_neg, float* carry) {
  const int m_cap = bt.n_cap + bt.b_cap * (1 + bt.n_neg);
  if (!carry_by_wave(m_cap)) {
    tail_carry_body<D, GTR_BLOCK>((int)blockIdx.x + 1, bt, T, skeys, svals, dx0, se, coef_tgt, coef_neg, carry);
    return;
  }
  __shared__ __attribute__((aligned(16))) float4 s_part[GTR_BLOCK];  // 64 per wave: (64 / C4) groups x C4
  const int wave = threadIdx.x >> 6;
  tail_carry_wave<D>((int)blockIdx.x * (GTR_BLOCK / 64) + wave + 1, bt, T, skeys, svals, dx0, se, coef_tgt,
                     coef_neg, carry, s_part + wave * 64);
}

// Segment starts (key changes) of window [w0, w1) in slot order -> s_bnd[0..nb), returns
// nb.  Every thread of the block calls it (barriers inside); BLOCK >= TW.
template <int BLOCK>
__device__ __forceinline__ int window_bounds(const int32_t* skeys, int w0, int w1, int* s_bnd) {
  __shared__ int s_nb;
  __shared__ int s_wcnt[BLOCK / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int i = w0 + tid;
  bool bnd = false;
  if (tid < TW && i < w1) bnd = (i == 0) || skeys[i] != skeys[i - 1];
  const unsigned long long bal = __ballot(bnd);
  if (lane == 0) s_wcnt[tid >> 6] = __popcll(bal);
  __syncthreads();
  int off = 0;
  for (int q = 0; q < (tid >> 6); ++q) off += s_wcnt[q];
  if (bnd) s_bnd[off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
  if (tid == 0) {
    int tot = 0;
    for (int q = 0; q < BLOCK / 64; ++q) tot += s_wcnt[q];
    s_nb = tot;
  }
  __syncthreads();
  return s_nb;
}

// Sum of the segment of `key` that starts at s0 inside window w (in-window end e): the
// in-window piece, then -- if the segment reaches the window's end -- the carries of the
// following windows in window order.
template <int D, int QF = 8>
__device__ __forceinline__ float4 window_segment_sum(const gtr_batch& bt, const int32_t* skeys, const int32_t* svals,
                                                     const float* dx0, const float* se, const float* coef_tgt,
                                                     const float* coef_neg, const float* carry, int w, int s0, int e,
                                                     int w1, int m_cap, int key, int gl, int gb,
                                                     const WinSlots* wsl) {
  constexpr int C4 = D / 4;
#if GTR_WIN_LDS
  (void)bt; (void)svals; (void)coef_tgt; (void)coef_neg; (void)gb;
  float4 g = piece_sum_lds<D, QF>(*wsl, w * TW, s0, e, dx0, se, gl);
#else
  float4 g = piece_sum<D, QF>(bt, svals, s0, e, dx0, se, coef_tgt, coef_neg, gl, gb);
#endif
  if (e == w1) {  // the segment may continue: add the carries in window order
    for (int w2 = w + 1; w2 * TW < m_cap && skeys[w2 * TW] == key; ++w2) {
      const float4 c = reinterpret_cast<const float4*>(carry)[(size_t)w2 * C4 + gl];
      g.x += c.x; g.y += c.y; g.z += c.z; g.w += c.w;
      if (skeys[min((w2 + 1) * TW, m_cap) - 1] != key) break;
    }
  }
  return g;
}

}  // namespace gtr
