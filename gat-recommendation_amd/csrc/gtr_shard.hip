// gtr_shard.hip — row-sharded item table for the multi-GPU step (SURVEY.md §8e ii).
//
// The reference keeps one dense nn.Embedding(T, d) (base.py:36) updated by a dense AdamW
// (train_baseline.py:252-256).  Across P ranks the table and its AdamW moments are
// row-sharded: global row r lives on rank r % P as local row r / P (cyclic ownership
// spreads the Zipf-hot items over every owner).  One step per rank:
//
//   gtr_step_begin   (sorted contribution list of the rank's batch, global keys)
//   gtr_shard_route  unique requested rows per owner -> send_ids [P][cap]; the batch's
//                    ids remapped to "compact" rows q*cap + 1 + j of the fetched-row buffer
//   all-to-all ids   (RCCL)
//   gtr_shard_serve  owner: requested rows as of step t-1 (lazy zero-gradient AdamW applied
//                    in registers, bitwise the dense update) -> send_rows [P][cap][D]
//   all-to-all rows  == the "halo" fetch of source embeddings at layer 0
//   forward / loss / backward on the compact rows (unchanged layer kernels)
//   gtr_shard_pack   per requested row the summed table-gradient row -> send_grads
//                    [P][cap][D] (the rank's contributions in sorted order, as the
//                    single-GPU tail sums them) + the small-parameter gradient and loss
//   all-to-all grads + all-gather of the small packs
//   gtr_shard_update owner: every requested row's gradient summed over the requesting
//                    ranks in rank order / P, AdamW at step t (the same arithmetic as
//                    gtr_dp_tail); small parameters from the gathered packs.
//
// Slot 0 of every peer block carries the block's count; capacities are fixed so that the
// collectives and kernels replay from one captured hipGraph.  A block that would overflow
// its capacity sets status[0] (sticky in status[1]); the flag travels in the small pack, so
// every owner applies such a step as a zero-gradient step and every rank's host raises.

#include "gtr_rows.cuh"

namespace {

using namespace gtr;

#define RB_THREADS 256
#define RB_MAX_BLOCKS 512  // route workgroups: rounds of RB_THREADS slots each, <= this many workgroups
#define SH_MAXP 16

// Rounds of RB_THREADS slots per route workgroup: one round up to RB_MAX_BLOCKS workgroups
// (round 5: single-round blocks, C4 B = 1024 route 24.5 -> 18.5 us), more past that -- at
// 855k slots (C4 B = 8192) single-round blocks were 3,340 workgroups whose arrival tickets
// on ONE counter serialized (k_route_count 45.8 us).
__host__ __device__ inline int route_rounds(int m_cap) {
  const int r = (m_cap + RB_THREADS * RB_MAX_BLOCKS - 1) / (RB_THREADS * RB_MAX_BLOCKS);
  return r < 1 ? 1 : r;
}
__host__ __device__ inline int route_blocks(int m_cap) {
  const int slots = RB_THREADS * route_rounds(m_cap);
  return (m_cap + slots - 1) / slots;
}

struct RouteK {
  gtr_batch bt;
  const int32_t* skeys;
  const int32_t* svals;
  int32_t* send_ids;
  int32_t* ckeys;
  int32_t* node_item_c;
  int32_t* target_c;
  int32_t* negatives_c;
  const float* pe_tab;
  float* node_pe;
  int32_t* bcnt;    // [nblk][2P] first-occurrence counts per (class, owner), then exclusive offsets
  int32_t* rcnt;    // [nblk * rounds][2P] the same counts per 256-slot round (k_route_write's workgroups)
  int32_t* status;
  uint32_t* ticket; // arrival counter of k_route_count (scratch tail; zero between launches)
  int32_t* node_mark;  // [T] (cap_s > 0): rows a node reads, stamped with the step
  int T, P, cap, pe_k, m_cap, nblk, rounds, pad_r;
  int cap_s, blk, ncls, n_cap;  // class-1 slots per peer, id-block stride, classes (1 / 2)
  const int64_t* step_dev;      // this step (node_mark stamps): *step_dev + step_offset
  int step_offset, pad_t;
};

__device__ __forceinline__ int32_t route_step(const RouteK& a) { return (int32_t)(*a.step_dev + a.step_offset); }

__device__ __forceinline__ bool slot_info(const RouteK& a, int i, int& key, int& owner, bool& first) {
  key = i < a.m_cap ? a.skeys[i] : a.T;
  const bool valid = key >= 0 && key < a.T;
  owner = valid ? key % a.P : 0;
  first = valid && (i == 0 || a.skeys[i - 1] != key);
  return valid;
}

// Class of slot i's row: 0 if a node of the batch reads the row, 1 if only the scoring
// readout does (targets / negatives).  Within a row's segment of the sorted list the node
// slots come first (slots ascending), so a segment's first slot decides; k_route_count
// stamps node_mark[row] for class-0 segments, which later slots of the segment read.
__device__ __forceinline__ int slot_class(const RouteK& a, int i, int key, bool first) {
  if (a.ncls == 1) return 0;
  if (a.svals[i] < a.n_cap) return 0;
  if (first) return 1;
  return a.node_mark[key] == route_step(a) ? 0 : 1;
}

__device__ void route_scan_body(const RouteK& a);

// Pass 1: first occurrences (segment starts of the sorted list) per owner and block; the
// last arriving block then runs pass 2 (the scan) -- one launch for both (the counts are
// written through and the arrival is a relaxed ticket: no release fence per block).
__global__ __launch_bounds__(RB_THREADS) void k_route_count(RouteK a) {
  __shared__ int s_cnt[2 * SH_MAXP];
  __shared__ int s_rc[2 * SH_MAXP];
  __shared__ int s_flag;
  const int NQ = a.ncls * a.P;
  if (threadIdx.x < 2 * SH_MAXP) { s_cnt[threadIdx.x] = 0; s_rc[threadIdx.x] = 0; }
  __syncthreads();
  for (int r = 0; r < a.rounds; ++r) {
    const int i = (blockIdx.x * a.rounds + r) * RB_THREADS + threadIdx.x;
    int key, q;
    bool first;
    slot_info(a, i, key, q, first);
    if (first) {
      const int c = slot_class(a, i, key, true);
      if (a.ncls == 2 && c == 0) a.node_mark[key] = route_step(a);  // read by k_route_write (next launch)
      atomicAdd(&s_cnt[c * a.P + q], 1);  // integer counts: order-independent
      atomicAdd(&s_rc[c * a.P + q], 1);
    }
    __syncthreads();
    if (threadIdx.x < NQ) {  // the round's counts (read by the next launch)
      a.rcnt[((size_t)blockIdx.x * a.rounds + r) * NQ + threadIdx.x] = s_rc[threadIdx.x];
      s_rc[threadIdx.x] = 0;
    }
    __syncthreads();
  }
  if (threadIdx.x < a.ncls * a.P)
    __hip_atomic_store(a.bcnt + (size_t)blockIdx.x * a.ncls * a.P + threadIdx.x, s_cnt[threadIdx.x], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (!arrive_last_wt(a.ticket, (uint32_t)a.nblk, &s_flag)) return;
  route_scan_body(a);
  if (threadIdx.x == 0) reset_counter(a.ticket);
}

// Pass 2 (one workgroup): exclusive offsets of every block per owner, the owners' totals
// into the count slots, overflow status.  Thread t owns a contiguous chunk of blocks; each
// (class, owner) counter's 256 chunk sums are scanned across the threads by DPP wave scans
// plus the 4 wave totals (a serial walk over the 256 chunk sums per counter was a chain of
// 256 dependent LDS reads, ~10 us of k_route_count at 420 blocks).
__device__ void route_scan_body(const RouteK& a) {
  constexpr int NW = RB_THREADS / 64;
  __shared__ int s_sum[2 * SH_MAXP][RB_THREADS];
  __shared__ int s_wsum[2 * SH_MAXP][NW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NQ = a.ncls * a.P;  // (class, owner) counters, class-major
  if (tid == 0) a.status[0] = 0;  // this step's flag (a kernel write: no memset node in the captured step)
  const int per = (a.nblk + RB_THREADS - 1) / RB_THREADS;
  const int b0 = min(a.nblk, tid * per), b1 = min(a.nblk, b0 + per);
  for (int q = 0; q < NQ; ++q) {
    int sq = 0;
    for (int b = b0; b < b1; ++b) sq += a.bcnt[(size_t)b * NQ + q];
    s_sum[q][tid] = sq;
  }
  for (int q = 0; q < NQ; ++q) {  // wave-uniform
    const int x = s_sum[q][tid];
    const int incl = wave_incl_scan_dpp(x);
    s_sum[q][tid] = incl - x;
    if (lane == 63) s_wsum[q][wave] = incl;
  }
  __syncthreads();
  if (tid < NQ) {  // counter tid's total: the owner block's count slot, overflow status
    int tot = 0;
    for (int w = 0; w < NW; ++w) tot += s_wsum[tid][w];
    const int c = tid / a.P, q = tid - c * a.P;
    const int lim = (c ? a.cap_s : a.cap) - 1;
    a.send_ids[(size_t)q * a.blk + (c ? a.cap : 0)] = min(tot, lim);
    if (tot > lim) {
      a.status[0] = 1;
      atomicOr(a.status + 1, 1);
    }
  }
  for (int q = 0; q < NQ; ++q) {
    int run = s_sum[q][tid];
    for (int w = 0; w < wave; ++w) run += s_wsum[q][w];
    for (int b = b0; b < b1; ++b) {
      const int v = a.bcnt[(size_t)b * NQ + q];
      a.bcnt[(size_t)b * NQ + q] = run;
      run += v;
    }
  }
}

// Pass 3: inclusive first-occurrence rank of each slot among its owner's rows (slot
// order), compact row q*cap + rank, owner lists, remapped batch ids (+ PE rows).  One
// workgroup per 256-slot round (the count's workgroups hold several rounds past 512 of
// them): its offsets are its count block's plus the earlier rounds' counts of that block.
__global__ __launch_bounds__(RB_THREADS) void k_route_write(RouteK a) {
  __shared__ int s_run[2 * SH_MAXP];
  __shared__ int s_wt[RB_THREADS / 64][2 * SH_MAXP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NQ = a.ncls * a.P;
  const int cb = blockIdx.x / a.rounds, r0 = blockIdx.x - cb * a.rounds;
  if (tid < NQ) {
    int off = a.bcnt[(size_t)cb * NQ + tid];
    for (int r = 0; r < r0; ++r) off += a.rcnt[((size_t)cb * a.rounds + r) * NQ + tid];
    s_run[tid] = off;
  }
  __syncthreads();
  const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
  {
    const int i = blockIdx.x * RB_THREADS + tid;
    int key, q;
    bool first;
    const bool valid = slot_info(a, i, key, q, first);
    const int c = valid ? slot_class(a, i, key, first) : 0;
    const int cq = c * a.P + q;  // this slot's (class, owner) counter
    int mine = 0;
    for (int o = 0; o < NQ; ++o) {
      const unsigned long long bal = __ballot(first && cq == o);
      if (lane == 0) s_wt[wave][o] = __popcll(bal);
      if (cq == o) mine = __popcll(bal & le);
    }
    __syncthreads();
    int base = s_run[cq];
    for (int w = 0; w < wave; ++w) base += s_wt[w][cq];
    if (valid) {
      const int incl = base + mine;  // first occurrences of (class c, owner q) in [0, i]
      const int lim = (c ? a.cap_s : a.cap) - 1;
      // the fetched-row ("compact table") row and the id / gradient block slot
      int compact = c ? a.P * a.cap + q * a.cap_s + incl : q * a.cap + incl;
      int gslot = q * a.blk + (c ? a.cap : 0) + incl;
      if (incl > lim) {
        compact = q * a.cap;  // in bounds; the step is flagged invalid
        gslot = q * a.blk;
        a.status[0] = 1;
        atomicOr(a.status + 1, 1);
      } else if (first) {
        a.send_ids[gslot] = key;
      }
      a.ckeys[i] = gslot;
      const int s = a.svals[i];
      const gtr_batch& bt = a.bt;
      if (s < bt.n_cap) {
        a.node_item_c[s] = compact;
        if (a.node_pe)
          for (int k = 0; k < a.pe_k; ++k) a.node_pe[(size_t)s * a.pe_k + k] = a.pe_tab[(size_t)key * a.pe_k + k];
      } else if (s < bt.n_cap + bt.b_cap) {
        a.target_c[s - bt.n_cap] = compact;
      } else {
        a.negatives_c[s - bt.n_cap - bt.b_cap] = compact;
      }
    } else if (i < a.m_cap) {
      a.ckeys[i] = -1;
    }
  }
}

// Count of a class block starting at ids[off] with `cap` slots (count included).
__device__ __forceinline__ int block_count(const int32_t* ids, size_t off, int cap) {
  const int c = ids[off];
  return c < 0 ? 0 : (c > cap - 1 ? cap - 1 : c);
}

// Entry e of the [P][blk] id / gradient blocks: peer r, class c, slot j of the class
// block (1.. its count), and its count; false for count slots and unused slots.
__device__ __forceinline__ bool entry_of(const gtr_shard& sh, const int32_t* ids, int64_t e, int& r, int& c, int& j) {
  const int blk = sh.cap + sh.cap_s;
  r = (int)(e / blk);
  const int jj = (int)(e - (int64_t)r * blk);
  c = jj >= sh.cap ? 1 : 0;
  j = c ? jj - sh.cap : jj;
  if (r >= sh.world || j < 1) return false;
  return j <= block_count(ids, (size_t)r * blk + (c ? sh.cap : 0), c ? sh.cap_s : sh.cap);
}

// Owner side, step t: every requested row as it stands after step t-1, into its slot of
// send_rows.  A row whose stamp lags (< t-1) is brought forward IN REGISTERS with the
// zero-gradient update of every missed step (the consts chain of the lazy table, bitwise
// the dense sweep); the table itself is not written here.  The owner's update
// (k_shard_update) recomputes the same chain and writes p / m / v once, together with the
// step-t update: one read-modify-write of a touched row per step, and no write in this
// kernel, so several ranks' requests of one row need no claim (one launch, read-only on
// the table).  C4 lanes per entry.
template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_shard_serve(gtr_shard sh, const int32_t* recv_ids, float* send_rows) {
  constexpr int C4 = D / 4;
  const int64_t gid = (int64_t)blockIdx.x * GTR_BLOCK + threadIdx.x;
  const int64_t e = gid / C4;
  const int c = (int)(gid - e * C4);
  int r, cls, j;
  if (!entry_of(sh, recv_ids, e, r, cls, j)) return;
  const int local = recv_ids[e] / sh.world;
  // class 0 rows -> send_rows [P][cap][D], class 1 -> send_rows + P cap D, [P][cap_s][D]
  const int64_t orow = cls ? (int64_t)sh.world * sh.cap + (int64_t)r * sh.cap_s + j : (int64_t)r * sh.cap + j;
  const int32_t t = (int32_t)(*sh.opt.step_dev + sh.opt.step_offset);
  const int old = sh.stamp[local];
  const size_t at = (size_t)local * C4 + c;
  float4 p = reinterpret_cast<const float4*>(sh.table)[at];
  if (old < t - 1) {
    float4 m = reinterpret_cast<const float4*>(sh.m)[at];
    float4 v = reinterpret_cast<const float4*>(sh.v)[at];
    catch_up4(p, m, v, old, t - 1, sh.opt, sh.consts);
  }
  reinterpret_cast<float4*>(send_rows)[orow * C4 + c] = p;
}

// The gradient row of id-block slot g ([P][blk] slots) in a [P][grad_stride] buffer.
__device__ __forceinline__ int64_t grad_row_off(int64_t g, int blk, int64_t grad_stride, int D) {
  const int64_t q = g / blk;
  return q * grad_stride + (g - q * blk) * D;
}

struct PackK {
  gtr_batch bt;
  gtr_tail tl;
  const int32_t* ckeys;
  float* send_grads;
  float* small_pack;
  int64_t grad_stride, small_stride;
  int blk, world, rows_part, small_part;
  const int32_t* status;  // this rank's overflow flag of the step (status[0]) -> small_pack[F + 1]
  int T, nb_rows, nseg, m_cap;
  int windowed, pad0;  // 1 (m_cap > GTR_BEGIN_MCAP): rows part = one block per TW-slot window
  gtr_segment segs[GTR_SMALL_MAX_SEG];
};

// Large batches: carries of the windows (gtr_rows.cuh), summed before k_shard_pack.
template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_shard_carry(gtr_batch bt, int T, gtr_tail tl) {
  tail_carry_block<D>(bt, T, tl.skeys, tl.svals, tl.dx0, tl.se, tl.coef_tgt, tl.coef_neg, tl.carry);
}

// Windowed rows part (large batches): the segments starting in window w, each summed as
// the single-GPU tail sums it (in-window piece + carries of the following windows), so no
// thread walks a hot row's thousands of contributions serially.
template <int D>
__device__ __forceinline__ void shard_pack_window(int w, const PackK& a) {
  constexpr int C4 = D / 4, NG = GTR_BLOCK / C4;
  __shared__ int s_bnd[TW + 1];
  const int tid = threadIdx.x;
  const int w0 = w * TW, w1 = min(w0 + TW, a.m_cap);
  const int32_t* sk = a.tl.skeys;
  __shared__ WinSlots s_ws;
  if (GTR_WIN_LDS) window_decode(a.bt, sk, a.tl.svals, a.tl.coef_tgt, a.tl.coef_neg, w0, w1, s_ws);
  const int nb = window_bounds<GTR_BLOCK>(sk, w0, w1, s_bnd);
  const int grp = tid / C4, gl = tid % C4, gb = grp * C4 % 64;
  for (int q = grp; q < nb; q += NG) {
    const int s0 = s_bnd[q];
    const int key = GTR_WIN_LDS ? s_ws.key[s0 - w0] : sk[s0];
    if (key < 0 || key >= a.T) continue;
    const int ck = a.ckeys[s0];
    if (ck < 0) continue;
    const int e = q + 1 < nb ? s_bnd[q + 1] : w1;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (key > 0)  // padding_idx = 0: no gradient (the owner still applies g = 0)
      g = window_segment_sum<D>(a.bt, sk, a.tl.svals, a.tl.dx0, a.tl.se, a.tl.coef_tgt, a.tl.coef_neg, a.tl.carry, w,
                                s0, e, w1, a.m_cap, key, gl, gb, &s_ws);
    reinterpret_cast<float4*>(a.send_grads + grad_row_off(ck, a.blk, a.grad_stride, D))[gl] = g;
  }
}

// Requester side: the summed gradient row of every requested row (segment of the sorted
// contribution list, summed in slot order like the single-GPU tail) -> its compact slot;
// then the summed small-parameter gradient and the local loss -> small_pack.
template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_shard_pack(PackK a) {
  constexpr int C4 = D / 4, NG = GTR_BLOCK / C4;
  __shared__ float s_acc[GTR_BLOCK];
  const int tid = threadIdx.x, lane = tid & 63;
  if ((int)blockIdx.x < a.nb_rows && a.windowed) {
    shard_pack_window<D>(blockIdx.x, a);
    return;
  }
  if ((int)blockIdx.x < a.nb_rows) {
    const int grp = tid / C4, gl = tid % C4, gb = grp * C4 % 64;
    const int i = blockIdx.x * NG + grp;
    const int key = i < a.m_cap ? a.tl.skeys[i] : a.T;
    const bool start = key >= 0 && key < a.T && (i == 0 || a.tl.skeys[i - 1] != key);
    // segment end: the group's lanes probe C4 slots per round (ballot inside the wave)
    int e = i + 1;
    bool more = start;
    while (__ballot(more) != 0ull) {  // wave-uniform loop; groups of the wave step together
      const int k = e + gl;
      const bool same = more && k < a.m_cap && a.tl.skeys[k] == key;
      const unsigned long long bal = __ballot(!same && more) >> gb;
      const unsigned long long gm = C4 == 64 ? ~0ull : ((1ull << C4) - 1ull);
      if (more) {
        const unsigned long long stop = bal & gm;
        if (stop) { e += __ffsll((long long)stop) - 1; more = false; }
        else e += C4;
      }
    }
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (start && key > 0)  // padding_idx = 0: no gradient (the owner still applies g = 0)
      g = piece_sum<D>(a.bt, a.tl.svals, i, e, a.tl.dx0, a.tl.se, a.tl.coef_tgt, a.tl.coef_neg, gl, gb);
    if (start) {
      const int ck = a.ckeys[i];
      if (ck >= 0) reinterpret_cast<float4*>(a.send_grads + grad_row_off(ck, a.blk, a.grad_stride, D))[gl] = g;
    }
    (void)lane;
    return;
  }
  const int sb = blockIdx.x - a.nb_rows;
  const AdamStep unused{};
  small_body((int64_t)sb * GTR_BLOCK + tid, a.segs, a.nseg, a.bt.hdr, nullptr, nullptr, nullptr, a.small_pack,
             unused);
  if (a.small_stride > 0) {  // the small pack rides in every peer's gradient block
    __syncthreads();
    const int64_t e = (int64_t)sb * GTR_BLOCK + tid;
    if (e < a.tl.flat_total) {
      const float v = a.small_pack[e];  // this thread's own write above (same thread)
      for (int q = 1; q < a.world; ++q) a.small_pack[q * a.small_stride + e] = v;
    }
  }
  if (sb == 0) {  // local loss after the flat gradient
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
      const float flag = a.status[0] != 0 ? 1.0f : 0.0f;
      for (int q = 0; q < (a.small_stride > 0 ? a.world : 1); ++q) {
        a.small_pack[q * a.small_stride + a.tl.flat_total] = t;
        a.small_pack[q * a.small_stride + a.tl.flat_total + 1] = flag;
      }
    }
  }
}

// Position of `key` in a class block of ascending ids (slots 1..count) at ids[off], or -1.
__device__ __forceinline__ int block_find(const int32_t* ids, size_t off, int cap, int key) {
  const int32_t* p = ids + off + 1;
  int lo = 0, hi = block_count(ids, off, cap);
  const int n = hi;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p[mid] < key) lo = mid + 1; else hi = mid;
  }
  return (lo < n && p[lo] == key) ? lo + 1 : -1;
}

// Slot of `key` in peer r's id block (either class), or -1.
__device__ __forceinline__ int peer_find(const gtr_shard& sh, const int32_t* ids, int r, int key) {
  const int blk = sh.cap + sh.cap_s;
  const int p0 = block_find(ids, (size_t)r * blk, sh.cap, key);
  if (p0 >= 0 || sh.cap_s == 0) return p0;
  const int p1 = block_find(ids, (size_t)r * blk + sh.cap, sh.cap_s, key);
  return p1 >= 0 ? sh.cap + p1 : -1;
}

struct UpdateK {
  gtr_shard sh;
  gtr_tail tl;
  const int32_t* recv_ids;
  const float* recv_grads;
  const float* small_all;
  int64_t small_words;
  int nb_rows, pad0;
};

template <int D>
__global__ __launch_bounds__(GTR_BLOCK) void k_shard_update(UpdateK a) {
  constexpr int C4 = D / 4;
  __shared__ AdamStep s_st;
  __shared__ int32_t s_t;
  const int tid = threadIdx.x;
  const gtr_shard& sh = a.sh;
  if (tid == 0) {
    const int64_t t = *sh.opt.step_dev + sh.opt.step_offset;
    s_st.init(sh.opt, t);
    s_t = (int32_t)t;
    if (blockIdx.x == 0 && t < sh.consts_cap) lazy_consts_for(sh.opt, t, sh.consts);
  }
  __syncthreads();
  const AdamStep st = s_st;
  const int32_t t = s_t;
  const int W = sh.world;
  const float inv_w = 1.0f / (float)W;
  // a step on which ANY rank overflowed an exchange block carries incomplete gradients: it
  // is applied as a zero-gradient step (touched rows stay at t - 1 and are caught up with
  // g = 0 when next read; the small parameters take g = 0), and every rank's sticky status
  // records it, so the host raises on every rank and no partial update is ever applied
  bool bad = false;
  for (int q = 0; q < W; ++q) bad = bad || a.small_all[(size_t)q * a.small_words + a.tl.flat_total + 1] != 0.0f;
  if (bad && blockIdx.x == 0 && tid == 0) atomicOr(sh.status + 1, 2);
  if ((int)blockIdx.x < a.nb_rows) {
    if (bad) return;
    const int64_t gid = (int64_t)blockIdx.x * GTR_BLOCK + tid;
    const int64_t e = gid / C4;
    const int c = (int)(gid - e * C4);
    int r, cls, j;
    if (!entry_of(sh, a.recv_ids, e, r, cls, j)) return;
    const int blk = sh.cap + sh.cap_s;
    const int key = a.recv_ids[e];
    for (int q = 0; q < r; ++q)
      if (peer_find(sh, a.recv_ids, q, key) >= 0) return;  // a lower rank leads this row
    const int64_t gs = sh.grad_stride > 0 ? sh.grad_stride : (int64_t)blk * D;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = r; q < W; ++q) {
      const int at = q == r ? (int)(e - (int64_t)r * blk) : peer_find(sh, a.recv_ids, q, key);
      if (at < 0) continue;
      const float4 v = reinterpret_cast<const float4*>(a.recv_grads + q * gs + (int64_t)at * D)[c];
      g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
    }
    g.x *= inv_w; g.y *= inv_w; g.z *= inv_w; g.w *= inv_w;
    const int local = key / W;
    const size_t base = (size_t)local * C4 + c;
    const int old = sh.stamp[local];
    float4 pv = reinterpret_cast<const float4*>(sh.table)[base];
    float4 mv = reinterpret_cast<const float4*>(sh.m)[base];
    float4 vv = reinterpret_cast<const float4*>(sh.v)[base];
    catch_up4(pv, mv, vv, old, t - 1, sh.opt, sh.consts);  // the chain k_shard_serve applied in registers
    st.apply(pv.x, mv.x, vv.x, g.x);
    st.apply(pv.y, mv.y, vv.y, g.y);
    st.apply(pv.z, mv.z, vv.z, g.z);
    st.apply(pv.w, mv.w, vv.w, g.w);
    reinterpret_cast<float4*>(sh.table)[base] = pv;
    reinterpret_cast<float4*>(sh.m)[base] = mv;
    reinterpret_cast<float4*>(sh.v)[base] = vv;
    __builtin_amdgcn_wave_barrier();  // the row's column lanes (one wave) read the stamp above
    if (c == 0) sh.stamp[local] = t;
    return;
  }
  const int64_t e = (int64_t)(blockIdx.x - a.nb_rows) * GTR_BLOCK + tid;
  const int64_t F = a.tl.flat_total;
  if (e < F) {
    float g = 0.0f;
    for (int q = 0; q < W; ++q) g += a.small_all[(size_t)q * a.small_words + e];
    g = bad ? 0.0f : g * inv_w;
    float pv = a.tl.flat[e], mv = a.tl.flat_m[e], vv = a.tl.flat_v[e];
    st.apply(pv, mv, vv, g);
    a.tl.flat[e] = pv;
    a.tl.flat_m[e] = mv;
    a.tl.flat_v[e] = vv;
  } else if (e == F && a.tl.loss_out) {
    float l = 0.0f;
    for (int q = 0; q < W; ++q) l += a.small_all[(size_t)q * a.small_words + F];
    a.tl.loss_out[0] = l * inv_w;
    if (a.tl.loss_acc) a.tl.loss_acc[0] += (double)(l * inv_w);
  }
}

bool shard_ok(const gtr_shard* s) {
  return s && s->world >= 1 && s->world <= SH_MAXP && s->rank >= 0 && s->rank < s->world && s->cap >= 2 &&
         (s->cap_s == 0 || (s->cap_s >= 2 && s->node_mark)) && s->grad_stride >= 0 && s->small_stride >= 0 &&
         s->num_items > 0 && s->local_rows == (s->num_items - s->rank + s->world - 1) / s->world &&
         (s->dim == 32 || s->dim == 64 || s->dim == 128 || s->dim == 256) && s->table && s->m && s->v && s->stamp &&
         s->consts && s->consts_cap > 0 && s->status && s->opt.step_dev;
}

}  // namespace

extern "C" {

int gtr_shard_route_scratch(int m_cap, int world, size_t* bytes) {
  if (!bytes || m_cap <= 0 || world < 1 || world > SH_MAXP) {
    set_error("gtr_shard_route_scratch: bad arguments");
    return GTR_E_ARG;
  }
  // [nblk][2P] block counts, [nblk * rounds][2P] round counts, the arrival ticket (64-byte
  // aligned slots)
  const size_t nb = (size_t)route_blocks(m_cap), nr = nb * route_rounds(m_cap);
  *bytes = ((nb * 2 * world * sizeof(int32_t) + 63) & ~(size_t)63) + ((nr * 2 * world * sizeof(int32_t) + 63) &
                                                                      ~(size_t)63) + 64;
  return GTR_OK;
}

int gtr_shard_route(const gtr_batch* bt, const int32_t* skeys, const int32_t* svals, const gtr_shard* sh,
                    int32_t* send_ids, int32_t* ckeys, int32_t* node_item_c, int32_t* target_c, int32_t* negatives_c,
                    const float* pe_tab, int pe_k, float* node_pe, void* scratch, size_t scratch_bytes,
                    gtr_stream_t stream) {
  if (!bt || !skeys || !svals || !shard_ok(sh) || !send_ids || !ckeys || !node_item_c || !target_c || !negatives_c ||
      !scratch || (node_pe && (!pe_tab || pe_k <= 0))) {
    set_error("gtr_shard_route: bad arguments");
    return GTR_E_ARG;
  }
  RouteK k{};
  k.bt = *bt;
  k.skeys = skeys; k.svals = svals; k.send_ids = send_ids; k.ckeys = ckeys;
  k.node_item_c = node_item_c; k.target_c = target_c; k.negatives_c = negatives_c;
  k.pe_tab = pe_tab; k.node_pe = node_pe; k.pe_k = node_pe ? pe_k : 0;
  k.status = sh->status;
  k.T = sh->num_items; k.P = sh->world; k.cap = sh->cap;
  k.cap_s = sh->cap_s; k.blk = sh->cap + sh->cap_s; k.ncls = sh->cap_s > 0 ? 2 : 1; k.n_cap = bt->n_cap;
  k.node_mark = sh->node_mark;
  k.step_dev = sh->opt.step_dev;
  k.step_offset = (int)sh->opt.step_offset;
  k.m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  k.rounds = route_rounds(k.m_cap);
  k.nblk = route_blocks(k.m_cap);
  const size_t cnt_bytes = ((size_t)k.nblk * k.ncls * k.P * sizeof(int32_t) + 63) & ~(size_t)63;
  const size_t rcnt_bytes = ((size_t)k.nblk * k.rounds * k.ncls * k.P * sizeof(int32_t) + 63) & ~(size_t)63;
  if (scratch_bytes < cnt_bytes + rcnt_bytes + 64) {
    set_error("gtr_shard_route: scratch of %zu bytes < %zu", scratch_bytes, cnt_bytes + rcnt_bytes + 64);
    return GTR_E_ARG;
  }
  k.bcnt = static_cast<int32_t*>(scratch);
  k.rcnt = reinterpret_cast<int32_t*>(static_cast<char*>(scratch) + cnt_bytes);
  k.ticket = reinterpret_cast<uint32_t*>(static_cast<char*>(scratch) + cnt_bytes + rcnt_bytes);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_route_count, dim3(k.nblk), dim3(RB_THREADS), 0, s, k);  // + the scan (last arriver)
  GTR_HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_route_write, dim3(k.nblk * k.rounds), dim3(RB_THREADS), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_shard_serve(const gtr_shard* sh, const int32_t* recv_ids, float* send_rows, gtr_stream_t stream) {
  if (!shard_ok(sh) || !recv_ids || !send_rows) {
    set_error("gtr_shard_serve: bad arguments");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t entries = (int64_t)sh->world * (sh->cap + sh->cap_s);
  const int64_t threads = entries * (sh->dim / 4);
  const dim3 grid((unsigned)((threads + GTR_BLOCK - 1) / GTR_BLOCK));
  switch (sh->dim) {
    case 32: hipLaunchKernelGGL(k_shard_serve<32>, grid, dim3(GTR_BLOCK), 0, s, *sh, recv_ids, send_rows); break;
    case 64: hipLaunchKernelGGL(k_shard_serve<64>, grid, dim3(GTR_BLOCK), 0, s, *sh, recv_ids, send_rows); break;
    case 128: hipLaunchKernelGGL(k_shard_serve<128>, grid, dim3(GTR_BLOCK), 0, s, *sh, recv_ids, send_rows); break;
    default: hipLaunchKernelGGL(k_shard_serve<256>, grid, dim3(GTR_BLOCK), 0, s, *sh, recv_ids, send_rows); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_shard_pack(const gtr_batch* bt, const gtr_shard* sh, const gtr_tail* tail, const int32_t* ckeys,
                   const gtr_segment* segs, int nseg, float* send_grads, float* small_pack, gtr_stream_t stream) {
  if (!bt || !shard_ok(sh) || !tail || !ckeys || !send_grads || !small_pack || nseg < 0 ||
      nseg > GTR_SMALL_MAX_SEG || (nseg > 0 && !segs) || !tail->skeys || !tail->svals || !tail->dx0 || !tail->se ||
      !tail->coef_tgt || !tail->coef_neg || (!tail->loss_part && !tail->loss_out)) {
    set_error("gtr_shard_pack: bad arguments");
    return GTR_E_ARG;
  }
  PackK k{};
  k.bt = *bt;
  k.tl = *tail;
  k.ckeys = ckeys;
  k.send_grads = send_grads;
  k.small_pack = small_pack;
  k.blk = sh->cap + sh->cap_s;
  k.world = sh->world;
  k.grad_stride = sh->grad_stride > 0 ? sh->grad_stride : (int64_t)k.blk * sh->dim;
  k.small_stride = sh->small_stride;
  k.rows_part = sh->pack_parts == 0 || (sh->pack_parts & 1);
  k.small_part = sh->pack_parts == 0 || (sh->pack_parts & 2);
  k.status = sh->status;
  k.T = sh->num_items;
  k.m_cap = bt->n_cap + bt->b_cap * (1 + bt->n_neg);
  hipStream_t s = (hipStream_t)stream;
  // large batches: windowed segment sums (one block per window + carries), bitwise the
  // single-GPU tail's and the data-parallel pack's order
  k.windowed = k.m_cap > GTR_BEGIN_MCAP ? 1 : 0;
  if (!k.rows_part) {
    k.nb_rows = 0;  // the small part only (launched after the weight gradients)
  } else if (k.windowed) {
    if (!tail->carry) {
      set_error("gtr_shard_pack: large batch (m_cap > %d) needs the carry scratch", GTR_BEGIN_MCAP);
      return GTR_E_ARG;
    }
    const int nwin = (k.m_cap + TW - 1) / TW;
    k.nb_rows = nwin;
    if (nwin > 1) {
      const dim3 cg(carry_blocks(k.m_cap));
      switch (sh->dim) {
        case 32: hipLaunchKernelGGL(k_shard_carry<32>, cg, dim3(GTR_BLOCK), 0, s, *bt, sh->num_items, *tail); break;
        case 64: hipLaunchKernelGGL(k_shard_carry<64>, cg, dim3(GTR_BLOCK), 0, s, *bt, sh->num_items, *tail); break;
        case 128: hipLaunchKernelGGL(k_shard_carry<128>, cg, dim3(GTR_BLOCK), 0, s, *bt, sh->num_items, *tail); break;
        default: hipLaunchKernelGGL(k_shard_carry<256>, cg, dim3(GTR_BLOCK), 0, s, *bt, sh->num_items, *tail); break;
      }
      GTR_HIP_CHECK_LAUNCH();
    }
  } else {
    const int NG = GTR_BLOCK / (sh->dim / 4);
    k.nb_rows = (k.m_cap + NG - 1) / NG;
  }
  k.nseg = nseg;
  for (int i = 0; i < nseg; ++i) k.segs[i] = segs[i];
  int nb_small = (int)((tail->flat_total + GTR_BLOCK - 1) / GTR_BLOCK);
  if (nb_small == 0) nb_small = 1;
  if (!k.small_part) nb_small = 0;
  if (k.nb_rows + nb_small == 0) return GTR_OK;
  const dim3 grid(k.nb_rows + nb_small);
  switch (sh->dim) {
    case 32: hipLaunchKernelGGL(k_shard_pack<32>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_shard_pack<64>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_shard_pack<128>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_shard_pack<256>, grid, dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

int gtr_shard_update(const gtr_shard* sh, const gtr_tail* tail, const int32_t* recv_ids, const float* recv_grads,
                     const float* small_all, int64_t small_words, gtr_stream_t stream) {
  if (!shard_ok(sh) || !tail || !recv_ids || !recv_grads || !small_all || small_words < tail->flat_total + 2 ||
      (tail->flat_total > 0 && (!tail->flat || !tail->flat_m || !tail->flat_v))) {
    set_error("gtr_shard_update: bad arguments");
    return GTR_E_ARG;
  }
  UpdateK k{};
  k.sh = *sh;
  k.tl = *tail;
  k.recv_ids = recv_ids;
  k.recv_grads = recv_grads;
  k.small_all = small_all;
  k.small_words = small_words;
  const int64_t entries = (int64_t)sh->world * (sh->cap + sh->cap_s);
  k.nb_rows = (int)((entries * (sh->dim / 4) + GTR_BLOCK - 1) / GTR_BLOCK);
  const int nb_small = (int)((tail->flat_total + 1 + GTR_BLOCK - 1) / GTR_BLOCK);
  const dim3 grid(k.nb_rows + nb_small);
  hipStream_t s = (hipStream_t)stream;
  switch (sh->dim) {
    case 32: hipLaunchKernelGGL(k_shard_update<32>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    case 64: hipLaunchKernelGGL(k_shard_update<64>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    case 128: hipLaunchKernelGGL(k_shard_update<128>, grid, dim3(GTR_BLOCK), 0, s, k); break;
    default: hipLaunchKernelGGL(k_shard_update<256>, grid, dim3(GTR_BLOCK), 0, s, k); break;
  }
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

}  // extern "C"
