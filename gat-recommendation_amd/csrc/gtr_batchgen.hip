// gtr_batchgen.hip — GPU batch constructor: SessionDataset.__getitem__ + collate_fn
// (etpgt/train/dataloader.py:64-202) writing the packed batch image the layer kernels
// consume (gtr_batch; etpgt/data/batch.py:blob_layout), so a training step can run
// from resident session / graph data without a host round trip.
//
//   per session (dataloader.py:64-124): the last max_len clicks; target = the last;
//     context = the rest; nodes = sorted unique context ids (collate_fn's unique());
//     edges = co-occurrence graph edges (item_i <= item_j) with both endpoints in the
//     context, directed item_i -> item_j, in (src, dst) order; n negatives drawn
//     uniformly from [1, T) rejecting the session's clicks (with replacement across
//     draws) from a counter-based hash stream (seed, batch position, draw).
//   per batch (collate_fn / Batch.from_data_list): node / edge offsets, CSR by
//     destination and by source, row-group ranges, header, zeroed tails.
//
// Graph membership is one open-addressing hash probe sequence per (a, b) pair
// (keys a*T + b, built once by gtr_edge_hash_build), not a binary search.
// Launches per batch: k_bb_scan (one workgroup: offsets from the per-session counts of
// gtr_session_counts, ranges, header, tails; records the batch start and advances the
// device cursor) and k_bb_write (wave per session).  The batch's sessions are
// order[(start + b) % S], so a captured graph replays the epoch batch after batch.

#include "gtr_common.cuh"

namespace {

using namespace gtr;

#define BB_WAVES 4
#define BB_BLOCK (64 * BB_WAVES)
#define BB_NEG_ROUNDS (1u << 20)  // rejection rounds before a session is declared unsatisfiable
#define BB_SCAN_BLOCK 1024
#define BB_BMAX 16384  // sessions per batch (k_bb_scan keeps node_ptr in LDS)
#define EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ bool edge_member(const uint64_t* slots, uint64_t mask, uint64_t key) {
  uint64_t h = mix64(key) & mask;
  while (true) {
    const uint64_t v = slots[h];
    if (v == key) return true;
    if (v == EMPTY_KEY) return false;
    h = (h + 1) & mask;
  }
}

__global__ __launch_bounds__(256) void k_edge_hash_build(const int64_t* keys, int64_t E, uint64_t* slots,
                                                         uint64_t mask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= E) return;
  const uint64_t key = (uint64_t)keys[i];
  uint64_t h = mix64(key) & mask;
  while (true) {
    const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(slots + h),
                                              (unsigned long long)EMPTY_KEY, (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) return;
    h = (h + 1) & mask;
  }
}

struct BBK {
  gtr_batch bt;                 // output image (pointers into the caller's blob)
  const int32_t* sess_ptr;      // [S+1] click offsets
  const int32_t* sess_items;    // clicks, click order
  const int32_t* sess_nodes;    // [S] unique context items of each session
  const int32_t* sess_edges;    // [S] induced edges of each session
  const int32_t* order;         // epoch order of session ids (cyclic)
  int64_t* cursor;              // position in order of the next batch's first session
  int64_t* start;               // [1] this batch's first position (written by k_bb_scan)
  const uint64_t* slots;        // edge hash
  uint64_t mask;
  int32_t* scratch;             // [2 * b_cap]: edge offset, node offset per session
  int32_t* status;              // [2]: this batch's code (1 over capacity, 2 negatives unsatisfiable), sticky OR
  int32_t B, T, max_len, R, S, seed;
  int64_t stride;               // cursor advance per batch (B; the global batch across ranks)
};

// The session's last max_len clicks (one per lane, lanes >= len hold INT_MAX), its
// target, and the sorted unique context (lane r < u holds the r-th id).  Whole wave.
__device__ __forceinline__ int session_nodes(const int32_t* sess_ptr, const int32_t* sess_items, int max_len,
                                             int s, int lane, int* s_uq, int& uq, int& len, int& tgt, int& click) {
  const int c0 = sess_ptr[s], c1 = sess_ptr[s + 1];
  len = min(c1 - c0, max_len);
  const int base = c1 - len;
  click = lane < len ? sess_items[base + lane] : 0x7FFFFFFF;
  tgt = __shfl(click, len > 0 ? len - 1 : 0);
  int v = lane < len - 1 ? click : 0x7FFFFFFF;  // context = all but the last
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {           // bitonic sort across the wave
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = __shfl_xor(v, j);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      v = (lower == up) ? min(v, o) : max(v, o);
    }
  }
  const int prev = __shfl_up(v, 1);
  const bool first = v != 0x7FFFFFFF && (lane == 0 || prev != v);
  const unsigned long long bal = __ballot(first);
  const int rank = __popcll(bal & ((1ull << lane) - 1ull));
  const int u = __popcll(bal);
  if (first) s_uq[rank] = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uq = lane < u ? s_uq[lane] : 0;
  return u;
}

// Induced adjacency of the u unique ids in s_uq: row[x] bit y / col[y] bit x for every
// graph edge (s_uq[x], s_uq[y]), x <= y.  Whole wave; returns the edge count.
__device__ __forceinline__ int session_adjacency(const uint64_t* slots, uint64_t mask, int T, int u, int lane,
                                                 const int* s_uq, unsigned long long* s_row,
                                                 unsigned long long* s_col) {
  s_row[lane] = 0ull;
  s_col[lane] = 0ull;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int q = lane; q < u * u; q += 64) {
    const int x = q / u, y = q - x * u;
    if (x > y) continue;
    const uint64_t key = (uint64_t)s_uq[x] * (uint64_t)T + (uint64_t)s_uq[y];
    if (edge_member(slots, mask, key)) {
      atomicOr(&s_row[x], 1ull << y);
      atomicOr(&s_col[y], 1ull << x);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int e = lane < u ? __popcll(s_row[lane]) : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
  return e;
}

// Per-session node / edge counts of sessions [0, S) (capacity planning + offsets).
__global__ __launch_bounds__(BB_BLOCK) void k_bb_count(const int32_t* sess_ptr, const int32_t* sess_items, int S,
                                                       int max_len, const uint64_t* slots, uint64_t mask, int T,
                                                       int32_t* nodes, int32_t* edges) {
  __shared__ int s_uq[BB_WAVES][64];
  __shared__ unsigned long long s_row[BB_WAVES][64];
  __shared__ unsigned long long s_col[BB_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s = blockIdx.x * BB_WAVES + w;
  if (s >= S) return;
  int uq, len, tgt, click;
  const int u = session_nodes(sess_ptr, sess_items, max_len, s, lane, s_uq[w], uq, len, tgt, click);
  const int e = session_adjacency(slots, mask, T, u, lane, s_uq[w], s_row[w], s_col[w]);
  if (lane == 0) { nodes[s] = u; edges[s] = e; }
}

template <int BLK>
__device__ void write_header_tails(const BBK& a, const int* np, const int* ep, int es, int N, int E, bool over,
                                   int64_t cur);

// Single workgroup: node / edge offsets of the batch, header, session offsets (PyG
// ptr), row-group ranges, CSR tails and zeroed unused regions (as pack_batch writes);
// records the batch start and advances the cursor.
__global__ __launch_bounds__(BB_SCAN_BLOCK) void k_bb_scan(BBK a) {
  __shared__ int s_np[BB_BMAX + 1];
  __shared__ int s_wsum[2][BB_SCAN_BLOCK / 64];
  __shared__ int s_tot[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = a.B;
  const int64_t cur = *a.cursor;
  const int per = (B + BB_SCAN_BLOCK - 1) / BB_SCAN_BLOCK;
  const int b0 = min(B, tid * per), b1 = min(B, b0 + per);
  int sn = 0, se = 0;
  for (int b = b0; b < b1; ++b) {
    const int s = a.order[(cur + b) % a.S];
    sn += a.sess_nodes[s];
    se += a.sess_edges[s];
  }
  int in = sn, ie = se;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int tn = __shfl_up(in, o), te = __shfl_up(ie, o);
    if (lane >= o) { in += tn; ie += te; }
  }
  if (lane == 63) { s_wsum[0][wave] = in; s_wsum[1][wave] = ie; }
  __syncthreads();
  if (tid == 0) {
    int an = 0, ae = 0;
    for (int w = 0; w < BB_SCAN_BLOCK / 64; ++w) {
      const int xn = s_wsum[0][w], xe = s_wsum[1][w];
      s_wsum[0][w] = an; s_wsum[1][w] = ae;
      an += xn; ae += xe;
    }
    s_tot[0] = an; s_tot[1] = ae;
  }
  __syncthreads();
  int on = s_wsum[0][wave] + in - sn, oe = s_wsum[1][wave] + ie - se;
  for (int b = b0; b < b1; ++b) {
    const int s = a.order[(cur + b) % a.S];
    s_np[b] = on;
    a.scratch[2 * b] = oe;
    a.scratch[2 * b + 1] = on;
    on += a.sess_nodes[s];
    oe += a.sess_edges[s];
  }
  const int N = s_tot[0], E = s_tot[1];
  if (tid == 0) s_np[B] = N;
  __syncthreads();  // every thread has read *cursor
  const gtr_batch& bt = a.bt;
  const bool over = N > bt.n_cap || E > bt.e_cap || B > bt.b_cap;
  if (tid == 0) *a.cursor = cur + a.stride;
  write_header_tails<BB_SCAN_BLOCK>(a, s_np, a.scratch, 2, N, E, over, cur);
}

// LDS of one wave's session (k_bb_write / k_bb_one)
struct BBWave {
  int uq[64];
  int clk[64];
  unsigned long long row[64];
  unsigned long long col[64];
  int inoff[64];
};

// One wave writes session b (epoch position pos, first edge e0, first node n0): nodes,
// induced edges, CSR by destination and by source, target, negatives.
__device__ void write_session(const BBK& a, int b, int64_t pos, int e0, int n0, BBWave& L) {
  const int lane = threadIdx.x & 63;
  const int s = a.order[pos % a.S];
  int uq, len, tgt, click;
  const int u = session_nodes(a.sess_ptr, a.sess_items, a.max_len, s, lane, L.uq, uq, len, tgt, click);
  session_adjacency(a.slots, a.mask, a.T, u, lane, L.uq, L.row, L.col);
  unsigned long long* s_row_w = L.row;
  unsigned long long* s_col_w = L.col;
  int* s_inoff_w = L.inoff;
  int* s_clk_w = L.clk;
  const gtr_batch& bt = a.bt;
  const unsigned long long row = lane < u ? s_row_w[lane] : 0ull;
  const unsigned long long col = lane < u ? s_col_w[lane] : 0ull;
  const int indeg = __popcll(col), outdeg = __popcll(row);
  int iin = indeg, iout = outdeg;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int ti = __shfl_up(iin, o), to = __shfl_up(iout, o);
    if (lane >= o) { iin += ti; iout += to; }
  }
  const int in_off = iin - indeg, out_off = iout - outdeg;
  s_inoff_w[lane] = in_off;
  s_clk_w[lane] = click;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < u) {
    const_cast<int32_t*>(bt.node_item)[n0 + lane] = uq;
    const_cast<int32_t*>(bt.in_ptr)[n0 + lane] = e0 + in_off;
    const_cast<int32_t*>(bt.out_ptr)[n0 + lane] = e0 + out_off;
    int32_t* in_src = const_cast<int32_t*>(bt.in_src) + e0 + in_off;
    unsigned long long c = col;
    for (int k = 0; c; ++k) {  // in-edges of destination `lane`, sources ascending
      const int x = __ffsll((unsigned long long)c) - 1;
      c &= c - 1ull;
      in_src[k] = n0 + x;
    }
    int32_t* oe = const_cast<int32_t*>(bt.out_edge) + e0 + out_off;
    int32_t* od = const_cast<int32_t*>(bt.out_dst) + e0 + out_off;
    unsigned long long r = row;
    for (int k = 0; r; ++k) {  // out-edges of source `lane`, destinations ascending
      const int y = __ffsll((unsigned long long)r) - 1;
      r &= r - 1ull;
      oe[k] = e0 + s_inoff_w[y] + __popcll(s_col_w[y] & ((1ull << lane) - 1ull));
      od[k] = n0 + y;
    }
  }
  if (lane == 0) const_cast<int32_t*>(bt.target)[b] = tgt;
  // negatives: uniform in [1, T) rejecting the session's clicks, 64 candidates a round,
  // rejected for as long as it takes (dataloader.py:107-124 loops until it has n).  Only a
  // session holding (nearly) every catalog item could exhaust BB_NEG_ROUNDS rounds; the
  // wave then stops (no GPU hang where the reference would spin forever) and flags
  // status 2, which the host turns into an error.
  const int n = bt.n_neg;
  int32_t* negs = const_cast<int32_t*>(bt.negatives) + (size_t)b * n;
  int filled = 0;
  for (uint32_t round = 0; filled < n; ++round) {
    if (round == BB_NEG_ROUNDS) {
      if (lane == 0) {
        __hip_atomic_store(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or(a.status + 1, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    const uint32_t h = mix3((uint32_t)a.seed, (uint32_t)pos, round * 64u + (uint32_t)lane);
    const int cand = 1 + (int)(h % (uint32_t)(a.T - 1));
    bool seen = false;
    for (int i = 0; i < len; ++i) seen |= s_clk_w[i] == cand;
    const unsigned long long ok = __ballot(!seen);
    const int rk = __popcll(ok & ((1ull << lane) - 1ull));
    if (!seen && filled + rk < n) negs[filled + rk] = cand;
    filled += __popcll(ok);
  }
}

// Wave per session, offsets from k_bb_scan.
__global__ __launch_bounds__(BB_BLOCK) void k_bb_write(BBK a) {
  __shared__ BBWave s_w[BB_WAVES];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * BB_WAVES + w;
  if (a.status[0] != 0 || b >= a.B) return;
  write_session(a, b, *a.start + b, a.scratch[2 * b], a.scratch[2 * b + 1], s_w[w]);
}

// The header / tails part of the build (k_bb_scan's, or k_bb_one's last workgroup):
// node_ptr, row-group ranges, CSR tails and zeroed unused regions.  np[b] / ep[b]: node /
// edge offset of session b (np[B] = N).
template <int BLK>
__device__ void write_header_tails(const BBK& a, const int* np, const int* ep, int es, int N, int E, bool over,
                                   int64_t cur) {
  const int tid = threadIdx.x;
  const int B = a.B;
  const gtr_batch& bt = a.bt;
  const int R = a.R;
  const int G = (N + R - 1) / R;
  const int g_cap = (bt.n_cap + R - 1) / R;
  int32_t* hdr = const_cast<int32_t*>(bt.hdr);
  if (tid == 0) {
    hdr[0] = over ? 0 : N; hdr[1] = over ? 0 : B; hdr[2] = over ? 0 : E; hdr[3] = bt.n_neg;
    hdr[4] = over ? 0 : G; hdr[5] = R; hdr[6] = 0; hdr[7] = 0;
    a.status[0] = over ? 1 : 0;
    if (over) a.status[1] |= 1;  // sticky over the batches built since the host cleared it
    *a.start = cur;
  }
  if (over) return;
  int32_t* node_ptr = const_cast<int32_t*>(bt.node_ptr);
  for (int b = tid; b <= bt.b_cap; b += BLK) node_ptr[b] = b <= B ? np[b] : N;
  int32_t* grp_row = const_cast<int32_t*>(bt.grp_row);
  int32_t* grp_edge = const_cast<int32_t*>(bt.grp_edge);
  for (int g = tid; g <= g_cap; g += BLK) {
    int r = N, e = E;
    if (g < G) {  // first session whose first node is >= g*R
      const int v = g * R;
      int lo = 0, hi = B;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (np[mid] < v) lo = mid + 1; else hi = mid;
      }
      r = lo < B ? np[lo] : N;
      e = lo < B ? ep[(size_t)lo * es] : E;
    }
    grp_row[g] = r;
    grp_edge[g] = e;
  }
  int32_t* node_item = const_cast<int32_t*>(bt.node_item);
  int32_t* in_ptr = const_cast<int32_t*>(bt.in_ptr);
  int32_t* out_ptr = const_cast<int32_t*>(bt.out_ptr);
  for (int i = N + tid; i <= bt.n_cap; i += BLK) {
    if (i < bt.n_cap) node_item[i] = 0;
    in_ptr[i] = E;
    out_ptr[i] = E;
  }
  int32_t* in_src = const_cast<int32_t*>(bt.in_src);
  int32_t* out_edge = const_cast<int32_t*>(bt.out_edge);
  int32_t* out_dst = const_cast<int32_t*>(bt.out_dst);
  for (int i = E + tid; i < bt.e_cap; i += BLK) { in_src[i] = 0; out_edge[i] = 0; out_dst[i] = 0; }
  int32_t* target = const_cast<int32_t*>(bt.target);
  int32_t* negs = const_cast<int32_t*>(bt.negatives);
  for (int b = B + tid; b < bt.b_cap; b += BLK) target[b] = 0;
  for (int i = B * bt.n_neg + tid; i < bt.b_cap * bt.n_neg; i += BLK) negs[i] = 0;
}

// Batches of up to BB_BLOCK sessions in ONE launch (round 5; the Trainer's C2 steps build
// B = 32): every workgroup reads the cursor and scans the B sessions' node / edge counts
// itself (B <= BB_BLOCK: one value per thread), its waves then write their sessions; the
// last workgroup writes the header, node_ptr, row-group ranges and the zeroed tails.  The
// last workgroup to ARRIVE (after every workgroup has read the cursor) advances it; the
// arrival ticket is scratch[2 * b_cap] (zero-initialised, reset by that workgroup).  One
// launch instead of k_bb_scan + k_bb_write: the single-workgroup scan and its dependent
// launch boundary go.
__global__ __launch_bounds__(BB_BLOCK) void k_bb_one(BBK a) {
  __shared__ BBWave s_w[BB_WAVES];
  __shared__ int s_np[BB_BLOCK + 1], s_ep[BB_BLOCK + 1];
  __shared__ int s_ws[2][BB_WAVES];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int B = a.B;
  const int64_t cur = *a.cursor;
  int cn = 0, ce = 0;
  if (tid < B) {
    const int s = a.order[(cur + tid) % a.S];
    cn = a.sess_nodes[s];
    ce = a.sess_edges[s];
  }
  int in = cn, ie = ce;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int tn = __shfl_up(in, o), te = __shfl_up(ie, o);
    if (lane >= o) { in += tn; ie += te; }
  }
  if (lane == 63) { s_ws[0][w] = in; s_ws[1][w] = ie; }
  __syncthreads();
  int bn = 0, be = 0, N = 0, E = 0;
#pragma unroll
  for (int q = 0; q < BB_WAVES; ++q) {
    if (q < w) { bn += s_ws[0][q]; be += s_ws[1][q]; }
    N += s_ws[0][q];
    E += s_ws[1][q];
  }
  s_np[tid] = bn + in - cn;  // past B: N (the counts there are 0)
  s_ep[tid] = be + ie - ce;
  if (tid == 0) { s_np[BB_BLOCK] = N; s_ep[BB_BLOCK] = E; }
  // every workgroup has read *cursor once its scan is in LDS: the last to arrive advances it
  uint32_t* ticket = reinterpret_cast<uint32_t*>(a.scratch + 2 * a.bt.b_cap);
  if (arrive_last_wt(ticket, gridDim.x, &s_flag) && tid == 0) {
    *a.cursor = cur + a.stride;
    reset_counter(ticket);
  }
  const gtr_batch& bt = a.bt;
  const bool over = N > bt.n_cap || E > bt.e_cap || B > bt.b_cap;
  if ((int)blockIdx.x == (int)gridDim.x - 1) {
    write_header_tails<BB_BLOCK>(a, s_np, s_ep, 1, N, E, over, cur);
    return;
  }
  const int b = blockIdx.x * BB_WAVES + w;
  if (over || b >= B) return;
  write_session(a, b, cur + b, s_ep[b], s_np[b], s_w[w]);
}

}  // namespace

extern "C" int gtr_edge_hash_slots(int64_t num_edges, int64_t* slots) {
  if (!slots || num_edges < 0) { set_error("gtr_edge_hash_slots: bad arguments"); return GTR_E_ARG; }
  int64_t n = 1024;
  while (n < 2 * num_edges) n <<= 1;
  *slots = n;
  return GTR_OK;
}

extern "C" int gtr_edge_hash_build(const int64_t* keys, int64_t num_edges, uint64_t* slots, int64_t num_slots,
                                   gtr_stream_t stream) {
  if (!slots || num_slots < 1024 || (num_slots & (num_slots - 1)) != 0 || num_slots < 2 * num_edges ||
      (num_edges > 0 && !keys)) {
    set_error("gtr_edge_hash_build: bad arguments (slots must be a power of two >= 2 * edges)");
    return GTR_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(slots, 0xFF, (size_t)num_slots * sizeof(uint64_t), s);
  if (e != hipSuccess) { set_error("gtr_edge_hash_build: %s", hipGetErrorString(e)); return (int)e; }
  if (num_edges > 0) {
    hipLaunchKernelGGL(k_edge_hash_build, dim3((unsigned)((num_edges + 255) / 256)), dim3(256), 0, s, keys,
                       num_edges, slots, (uint64_t)(num_slots - 1));
    GTR_HIP_CHECK_LAUNCH();
  }
  return GTR_OK;
}

extern "C" int gtr_session_counts(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots, int max_len,
                                  int32_t* nodes, int32_t* edges, gtr_stream_t stream) {
  if (!ss || !ss->sess_ptr || !ss->sess_items || !slots || !nodes || !edges || max_len < 2 || max_len > 64 ||
      ss->num_items < 2 || ss->num_sessions <= 0) {
    set_error("gtr_session_counts: bad arguments (2 <= max_len <= 64)");
    return GTR_E_ARG;
  }
  hipLaunchKernelGGL(k_bb_count, dim3((ss->num_sessions + BB_WAVES - 1) / BB_WAVES), dim3(BB_BLOCK), 0,
                     (hipStream_t)stream, ss->sess_ptr, ss->sess_items, ss->num_sessions, max_len, slots,
                     (uint64_t)(num_slots - 1), ss->num_items, nodes, edges);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_build_batch_strided(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots,
                                       int max_len, const int32_t* order, int64_t* cursor, int B, int64_t stride,
                                       int row_group, uint32_t seed, const gtr_batch* out, int32_t* scratch,
                                       int64_t* start, int32_t* status, gtr_stream_t stream) {
  if (!ss || !ss->sess_ptr || !ss->sess_items || !ss->sess_nodes || !ss->sess_edges || !slots || !order ||
      !cursor || !out || !scratch || !start || !status || B <= 0 || B > BB_BMAX || B > out->b_cap ||
      max_len < 2 || max_len > 64 || row_group <= 0 || ss->num_items < 2 || ss->num_sessions <= 0 ||
      out->n_neg <= 0 || stride < B) {
    set_error("gtr_build_batch: bad arguments (1 <= B <= min(b_cap, %d), 2 <= max_len <= 64, stride >= B)",
              BB_BMAX);
    return GTR_E_ARG;
  }
  BBK k{};
  k.bt = *out;
  k.sess_ptr = ss->sess_ptr; k.sess_items = ss->sess_items; k.sess_nodes = ss->sess_nodes;
  k.sess_edges = ss->sess_edges;
  k.order = order; k.cursor = cursor; k.start = start;
  k.slots = slots; k.mask = (uint64_t)(num_slots - 1);
  k.scratch = scratch; k.status = status;
  k.B = B; k.T = ss->num_items; k.max_len = max_len; k.R = row_group; k.S = ss->num_sessions;
  k.seed = (int32_t)seed;
  k.stride = stride;
  hipStream_t s = (hipStream_t)stream;
  const char* one = getenv("GTR_BB_ONE");  // 0: always the scan + write pair
  if (B <= BB_BLOCK && !(one && one[0] == '0')) {  // one launch (k_bb_one)
    hipLaunchKernelGGL(k_bb_one, dim3((B + BB_WAVES - 1) / BB_WAVES + 1), dim3(BB_BLOCK), 0, s, k);
    GTR_HIP_CHECK_LAUNCH();
    return GTR_OK;
  }
  hipLaunchKernelGGL(k_bb_scan, dim3(1), dim3(BB_SCAN_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_bb_write, dim3((B + BB_WAVES - 1) / BB_WAVES), dim3(BB_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_build_batch(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots, int max_len,
                               const int32_t* order, int64_t* cursor, int B, int row_group, uint32_t seed,
                               const gtr_batch* out, int32_t* scratch, int64_t* start, int32_t* status,
                               gtr_stream_t stream) {
  return gtr_build_batch_strided(ss, slots, num_slots, max_len, order, cursor, B, (int64_t)B, row_group, seed, out,
                                 scratch, start, status, stream);
}
