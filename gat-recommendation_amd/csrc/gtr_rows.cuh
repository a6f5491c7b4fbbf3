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
  for (int t = from + 1; t <= upto; ++t) {
    const float2 c = reinterpret_cast<const float2*>(consts)[t];
    st.step_size = c.x;
    st.inv_bc2 = c.y;
    st.apply(p.x, m.x, v.x, 0.0f);
    st.apply(p.y, m.y, v.y, 0.0f);
    st.apply(p.z, m.z, v.z, 0.0f);
    st.apply(p.w, m.w, v.w, 0.0f);
  }
}

// consts[t] exactly as AdamStep::init computes the step's scalars.
__device__ __forceinline__ void lazy_consts_for(const gtr_adam& o, int64_t t, float* consts) {
  AdamStep st;
  st.init(o, t);
  reinterpret_cast<float2*>(consts)[t] = make_float2(st.step_size, st.inv_bc2);
}

#define TW 128

// Sum of contributions in slots [s, e) for column float4 `gl` by the C4 = D/4 lanes of
// one group (group base lane gb): slot ids are fetched one per lane, decoded to a source
// row (dx0 node row, or se session row for target / negative slots) + coefficient,
// then broadcast 8 at a time so 8 row loads are in flight per lane.
template <int D>
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
    for (int q0 = 0; q0 < cnt; q0 += 8) {
      float4 v[8];
      float f[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int cq = __shfl(code, gb + ((q0 + u) & (C4 - 1)));
        f[u] = __shfl(cf, gb + ((q0 + u) & (C4 - 1)));
        const float* src = cq < 0 ? se + (size_t)(cq & 0x7FFFFFFF) * D : dx0 + (size_t)cq * D;
        v[u] = q0 + u < cnt ? reinterpret_cast<const float4*>(src)[gl] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (q0 + u < cnt) {
          g.x += f[u] * v[u].x; g.y += f[u] * v[u].y; g.z += f[u] * v[u].z; g.w += f[u] * v[u].w;
        }
      }
    }
  }
  return g;
}

}  // namespace gtr
