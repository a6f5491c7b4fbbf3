// gtr_bwd.hip — backward kernels of the GraphTransformer hot path (gfx950).
//
// k_conv_bwd<D>: autograd of graph_transformer.py:171-177 for one layer
//   (BatchNorm backward from finalized batch sums, beta-gate backward, attention
//   softmax backward, dK/dV gathered over out-edges (CSR by source — no float
//   atomics, deterministic), dX = dQKVS . W_all on MFMA, residual add, previous
//   layer's dropout mask and BatchNorm backward sums).  Same row groups as the
//   forward: every edge of a processed destination stays inside the workgroup.
// k_wgrad: lin_{query,key,value,skip} weight/bias, lin_beta and LapPE projection
//   gradients as deterministic per-chunk partial slabs (summed by the optimizer).

#include <string.h>

#include "gtr_layer.cuh"
#include "gtr_wgrad.cuh"

namespace {

using namespace gtr;

GTR_PH_DECL

#include "gtr_bwd_body.cuh"

template <int D, bool SPLIT>
__global__ __launch_bounds__(CONV_BLOCK) void k_conv_bwd(ConvBwdK a) {
  const int rb = role_block(a.main_grid, a.xpack);
  if (rb >= a.main_grid) {  // extra workgroups: untouched-row AdamW slice
    sweep_slice(a.sw, a.sw_slot, rb - a.main_grid, gridDim.x - a.main_grid);
    return;
  }
  conv_bwd_body<D, SPLIT>(a, rb);
}

// Split path (large batches): the attention backward of one row group per workgroup
// (gtr_attn_bwd); dX runs in k_dx (gtr_qkvs_bwd).
template <int D>
__global__ __launch_bounds__(CONV_BLOCK) void k_attn_bwd(ConvBwdK a) {
  conv_bwd_body<D, false, false>(a, blockIdx.x);
}

// ------------------------------------------------------------------------------------
// weight gradients
// ------------------------------------------------------------------------------------


__global__ __launch_bounds__(GTR_BLOCK) void k_wgrad(WgradK a) {
  const int blk = blockIdx.x;
  int jid = 0;
  while (jid + 1 < a.njobs && blk >= a.jobs[jid + 1].blk0) ++jid;
  const WJob& J = a.jobs[jid];
  const int local = blk - J.blk0;
  const int tile = local / a.P, p = local - tile * a.P;
  const int N = a.hdr[0];
  const int per = (N + a.P - 1) / a.P;
  const int t0 = p * per;
  const int t1 = min(N, t0 + per);
  const int64_t so = (int64_t)p * a.stride;
  auto emit = [&](int which, int64_t idx, float v) {
    if (which == 0) J.outW[so + idx] = v;
    else J.outB[so + idx] = v;
  };
  auto emit4 = [&](int64_t idx, float4 v) { *reinterpret_cast<float4*>(J.outW + so + idx) = v; };
  if (J.mfma == 1) wgrad_tile_mfma<false>(J, tile, t0, t1, emit, emit4);
  else if (J.mfma == 2) wgrad_tile_mfma<true>(J, tile, t0, t1, emit, emit4);
  else wgrad_tile(J, tile, t0, t1, a.D, emit);
}

}  // namespace

GTR_PH_READER(gtr_dbg_bwd_phases)

extern "C" int gtr_conv_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            float* dx0, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_conv_bwd: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim;
  ConvBwdK k;
  if (const int rc = make_bwd_args(cfg, bt, layers, l, dx0, k)) return rc;
  int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
  {
    const int slot = 2 * cfg->num_layers - l;  // after the forward slots and the readout's
    if (cfg->sweep && slot < GTR_SWEEP_SLOTS && cfg->sweep->bounds[slot + 1] > cfg->sweep->bounds[slot]) {
      k.sw = *cfg->sweep;
      k.sw_slot = slot;
      grid += sweep_blocks(cfg->sweep, grid);
    }
  }
  k.xpack = xcd_pack(k.main_grid, grid);
  hipStream_t s = (hipStream_t)stream;
#define GTR_BWD(DD, SP) set_lds_limit<DD>(k_conv_bwd<DD, SP>, (size_t)LayerGeom<DD>::B_WORDS * 4); \
  hipLaunchKernelGGL((k_conv_bwd<DD, SP>), dim3(grid), dim3(CONV_BLOCK), \
                                       (size_t)LayerGeom<DD>::B_WORDS * 4, s, k)
  const bool sp = gemm_split(D) != 0;
  switch (D) {
    case 32: if (sp) { GTR_BWD(32, true); } else { GTR_BWD(32, false); } break;
    case 64: if (sp) { GTR_BWD(64, true); } else { GTR_BWD(64, false); } break;
    case 128: if (sp) { GTR_BWD(128, true); } else { GTR_BWD(128, false); } break;
    default: GTR_BWD(256, false); break;  // no LDS-staged rows at D = 256: f32 MFMA from L2
  }
#undef GTR_BWD
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_attn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                            gtr_stream_t stream) {
  if (!cfg || !bt || !layers || l < 0 || l >= cfg->num_layers) {
    set_error("gtr_attn_bwd: bad arguments");
    return GTR_E_ARG;
  }
  if (cfg->sync_bn ? !cfg->split_sync : cfg->consumer_reduce) {
    set_error("gtr_attn_bwd: the split path reads producer-finalized BatchNorm sums (consumer_reduce 0) or, "
              "under sync_bn, the gathered per-rank sums (split_sync)");
    return GTR_E_ARG;
  }
  ConvBwdK k;
  float dummy = 0.0f;  // dx0 is written by gtr_qkvs_bwd, not here
  if (const int rc = make_bwd_args(cfg, bt, layers, l, &dummy, k)) return rc;
  k.dx0 = nullptr;
  const int grid = (bt->n_cap + cfg->row_group - 1) / cfg->row_group;
  if (grid <= 0) return GTR_OK;
  k.main_grid = grid;
  hipStream_t s = (hipStream_t)stream;
#define GTR_ABW(DD) set_lds_limit<DD>(k_attn_bwd<DD>, (size_t)LayerGeom<DD>::B_WORDS * 4); \
  hipLaunchKernelGGL((k_attn_bwd<DD>), dim3(grid), dim3(CONV_BLOCK), (size_t)LayerGeom<DD>::B_WORDS * 4, s, k)
  switch (cfg->dim) {
    case 32: GTR_ABW(32); break;
    case 64: GTR_ABW(64); break;
    case 128: GTR_ABW(128); break;
    default: GTR_ABW(256); break;
  }
#undef GTR_ABW
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}

extern "C" int gtr_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers,
                         const float* dx0, const float* pe_tab, float* const* layer_slab, float* pe_slab,
                         int n_chunks, int64_t slab_stride, int l_begin, int l_end, gtr_stream_t stream) {
  if (!cfg || !bt || !layers || !layer_slab || n_chunks <= 0) {
    set_error("gtr_wgrad: bad arguments");
    return GTR_E_ARG;
  }
  const int D = cfg->dim, Lc = cfg->num_layers;
  if (3 * Lc + 1 > GTR_MAX_WJOBS) { set_error("gtr_wgrad: too many layers"); return GTR_E_ARG; }
  WgradK k{};
  k.hdr = bt->hdr;
  k.P = n_chunks;
  k.D = D;
  k.stride = slab_stride;
  if (l_begin < 0 || l_end > Lc || l_begin > l_end) { set_error("gtr_wgrad: bad layer range"); return GTR_E_ARG; }
  int nj = 0, blocks = 0;
  // MFMA tiles for the QKVS weight once a chunk holds enough rows to amortize them
  // (GTR_WGRAD=mfma|valu overrides; the float4 slab stores need 16 B aligned slabs)
  const char* wm = getenv("GTR_WGRAD");
  const int rows_per_chunk = (bt->n_cap + n_chunks - 1) / n_chunks;
  bool mfma = rows_per_chunk >= GTR_WGRAD_MFMA_ROWS;
  if (wm && !strcmp(wm, "mfma")) mfma = true;
  if (wm && !strcmp(wm, "valu")) mfma = false;
  if (slab_stride % 4) mfma = false;
  for (int l = l_begin; l < l_end; ++l)
    if (reinterpret_cast<uintptr_t>(layer_slab[l]) % 16) mfma = false;
  const int rc = build_wjobs(cfg, bt, layers, dx0, pe_tab, layer_slab, pe_slab, nullptr, nullptr, n_chunks, l_begin,
                             l_end, k.jobs, nj, blocks, mfma);
  if (rc) return rc;
  if (const char* jm = getenv("GTR_WGRAD_JOBS")) {  // diagnostics (timing only): keep job types in the mask
    const int mask = atoi(jm);
    int kept = 0;
    blocks = 0;
    for (int i = 0; i < nj; ++i) {
      const bool pe = k.jobs[i].type == WJ_MM && k.jobs[i].M1 == D;
      const int bit = pe ? 8 : 1 << k.jobs[i].type;
      if (!(mask & bit)) continue;
      WJob j = k.jobs[i];
      j.blk0 = blocks;
      blocks += j.nt * n_chunks;
      k.jobs[kept++] = j;
    }
    nj = kept;
  }
  k.njobs = nj;
  if (nj == 0 || blocks == 0) return GTR_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_wgrad, dim3(blocks), dim3(GTR_BLOCK), 0, s, k);
  GTR_HIP_CHECK_LAUNCH();
  return GTR_OK;
}
