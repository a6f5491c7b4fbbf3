/*
 * gtr.h — C ABI of libgtr_hip.so, the MI355X (gfx950) training hot path of the
 * GraphTransformer session recommender (Axionis47/GAT-Recommendation).
 *
 * The reference has NO native boundary: its hot path is a Python module API
 * (etpgt.model / etpgt.train).  These entry points are what a
 * maintainer's FFI for that path binds (the ctypes stub in INTEGRATION.md).
 * Each one replaces a span of reference Python (file:line in /root/reference):
 *
 *   gtr_conv_fwd      graph_transformer.py:140-152 (embedding + LapPE add, layer 0)
 *                     + graph_transformer.py:171-177 (TransformerConv -> BatchNorm
 *                     -> residual -> dropout) for one layer, fused; PyG
 *                     TransformerConv semantics per SURVEY.md Appendix A.
 *   gtr_readout_loss  base.py:136-155 (mean SessionReadout) + base.py:80-113 /
 *                     losses.py:8-228 (BPR / listwise / dual scoring loss), forward
 *                     and backward, fused; trainer.py:86-122 loss dispatch.
 *   gtr_conv_bwd      autograd of graph_transformer.py:171-177 for one layer.
 *   gtr_wgrad         weight/bias gradients of lin_{query,key,value,skip},
 *                     lin_beta and laplacian_pe.projection (laplacian_pe.py:194-197).
 *   gtr_contrib_prep  embedding-row gradient bookkeeping (nn.Embedding(padding_idx=0)
 *     gtr_contrib_sort  backward, base.py:35-37) as a sorted-segment reduction.
 *   gtr_adamw_rows / gtr_adamw_sweep / gtr_adamw_small
 *                     torch.optim.AdamW(lr, wd) step of train_baseline.py:252-256
 *                     (trainer.py:125-127) over the item table and the dense params.
 *   gtr_scatter_rows  eager (autograd) path: dense table gradient.
 *   gtr_step_end      step / dropout-stream counters.
 *   gtr_step_begin / gtr_step_tail
 *                     one whole Trainer.train_epoch iteration (trainer.py:80-133)
 *                     is begin -> conv_fwd.. -> readout_loss -> conv_bwd.. -> wgrad
 *                     -> tail: zero_grad/backward/optimizer.step() of trainer.py:
 *                     123-127 without a dense table gradient.
 *   gtr_dp_pack / gtr_dp_tail
 *                     the data-parallel version of that step (one process per GPU);
 *                     the reference has no multi-GPU path.
 *   gtr_readout_grid  partial count of gtr_readout_loss (host sizing).
 *   gtr_score_topk    base.py:59-78 predict (full-catalog scores + top-k), the
 *                     Recall@K / NDCG@K evaluation of trainer.py:138-173.
 *   gtr_build_batch   dataloader.py:64-202 SessionDataset.__getitem__ + collate_fn on
 *                     the device (+ gtr_edge_hash_build, gtr_session_counts).
 *
 * Conventions: plain pointers + sizes, no torch types; every
 * pointer is a device pointer unless marked (host); stream is a hipStream_t;
 * every function returns 0 on success or a non-zero code (hipError_t value,
 * or GTR_E_* below) and never throws; gtr_last_error() returns a message.
 * Functions never allocate: workspace is caller-provided.  Indices are int32
 * on device.  Live batch sizes (N, B, E) are read from device memory (hdr) so
 * that a captured hipGraph can be replayed over batches of varying shape
 * within fixed capacities.
 */
#ifndef GTR_H
#define GTR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GTR_ABI_VERSION 8 /* 8: gtr_shard.cap_s / grad_stride / small_stride / pack_parts / node_mark (two-class exchange); 7: gtr_tail.loss_acc; 6: gtr_layer.ffn + gtr_ffn_fwd / gtr_ffn_bwd / gtr_ffn_wgrad (the FFN variant); 5: gtr_config.loss_batch / wfold_stride, gtr_layer.wfold, gtr_segment.live_groups, hdr[6] halo source rows; 4: gtr_step_tail_wgrad on split-K slabs; 3: gtr_config.begin / ctr_add, gtr_tail.rng_inc */

#define GTR_OK 0
#define GTR_E_ARG 1001      /* bad argument / unsupported shape */
#define GTR_E_DEVICE 1002   /* not a gfx950 device */

typedef void* gtr_stream_t; /* hipStream_t */

/* Batch in HBM: fixed-capacity arrays, live sizes in hdr[] on device.
 * hdr[0] = N (nodes), hdr[1] = B (sessions), hdr[2] = E (edges),
 * hdr[4] = G (row groups), hdr[5] = R (row-group width, == gtr_config.row_group),
 * hdr[6] = source rows of a halo batch (0: N; etpgt.train.halo): rows [N, hdr[6]) are
 * ghost copies of other ranks' nodes -- sources of local edges (their K / V rows arrive
 * by the halo exchange, gtr_attn_bwd writes their dK / dV for the owner) and the tail of
 * a session that straddles the cut (read by the readout).
 * Row group g owns every session whose first node lies in [g*R, (g+1)*R):
 * rows [grp_row[g], grp_row[g+1]) and dst-ordered edges [grp_edge[g], grp_edge[g+1]).  */
typedef struct gtr_batch {
  const int32_t* hdr;
  const int32_t* node_item; /* [n_cap]   global item id of each node          */
  const int32_t* node_ptr;  /* [b_cap+1] first node of each session (PyG ptr)  */
  const int32_t* in_ptr;    /* [n_cap+1] CSR by destination                    */
  const int32_t* in_src;    /* [e_cap]   source node of dst-ordered edge        */
  const int32_t* out_ptr;   /* [n_cap+1] CSR by source                         */
  const int32_t* out_edge;  /* [e_cap]   dst-order position of src-ordered edge */
  const int32_t* out_dst;   /* [e_cap]   destination node of src-ordered edge   */
  const int32_t* target;    /* [b_cap]                                          */
  const int32_t* negatives; /* [b_cap * n_neg]                                  */
  const float* node_pe;     /* optional [n_cap, pe_k] batch.laplacian_pe, or NULL */
  const int32_t* grp_row;   /* [g_cap+1] first row of each row group             */
  const int32_t* grp_edge;  /* [g_cap+1] first dst-ordered edge of each row group */
  int32_t n_cap, b_cap, e_cap, n_neg;
} gtr_batch;

typedef struct gtr_sweep gtr_sweep;

/* gtr_step_begin's work (stamps of the touched rows, *step_dev += 1, the rank-sorted
 * contribution list) run by extra workgroups of gtr_conv_fwd(layer 0) instead of a launch
 * of its own (gtr_config.begin; m_cap <= 8192, num_items < 2^19).  The dropout counter is
 * then NOT advanced there: every kernel of the step reads *rng_ctr + gtr_config.ctr_add
 * (1) and the step tail advances it at its end (gtr_tail.rng_inc).                      */
typedef struct gtr_begin {
  int32_t* skeys;
  int32_t* svals;
  int32_t* stamp;      /* or NULL */
  int64_t* step_dev;
  int32_t num_items;
  int32_t pad;
} gtr_begin;

typedef struct gtr_config {
  int32_t num_items;  /* T: table rows                          */
  int32_t dim;        /* D = embedding_dim = hidden_dim          */
  int32_t heads;      /* H (C = D / H)                           */
  int32_t pe_k;       /* LapPE k, 0 = no LapPE                   */
  int32_t num_layers; /* L                                       */
  int32_t row_group;  /* R: sessions are grouped by first node / R */
  int32_t training;   /* 1 = train mode (batch BN stats, dropout) */
  float dropout;      /* p                                       */
  float bn_eps;       /* 1e-5                                    */
  float bn_momentum;  /* 0.1                                     */
  uint32_t seed;      /* dropout stream seed                     */
  const uint32_t* rng_ctr; /* device counter mixed into dropout masks */
  int32_t consumer_reduce; /* 1: a BatchNorm's batch statistics (fwd) and backward sums are
                              reduced from the producer's per-group partials by the CONSUMING
                              kernel (no inter-workgroup fences; for <= 64 row groups);
                              0: the producer's last-arriving workgroup finalises them */
  int32_t sync_bn;         /* 1: BatchNorm statistics over every rank's batch (SyncBN): the
                              consumers reduce gtr_layer.bn_part_all / bn_gpart_all (the
                              all-gathered partials of all ranks; requires consumer_reduce)
                              and producers zero the partial rows of their empty groups */
  const gtr_sweep* sweep;  /* optional (fused single-GPU step): untouched-row AdamW
                              slices run by extra workgroups of the layer kernels */
  const gtr_begin* begin;  /* optional: gtr_conv_fwd(layer 0) also runs the step begin */
  int32_t ctr_add;         /* added to *rng_ctr by every kernel (1 with a fused begin)    */
  int32_t split_sync;      /* 1: SyncBN on the split layer path: gtr_attn_fwd merges its
                              partials into ONE (count, mean, M2) row (bn_part row 0), the
                              readout and gtr_qkvs_bwd finalize their local backward sums
                              (bn_gsum); the ranks all-gather those single rows, so
                              bn_part_all is [P][1 + 2D] and bn_gpart_all [P][2D]
                              (nparts_fwd = nparts_bwd = P), and the consumers
                              (gtr_qkvs_fwd, the readout, gtr_attn_bwd) fold P rows     */
  float loss_batch;        /* > 0: the loss means divide by this many sessions instead of
                              the batch's own B (a halo cut gives ranks unequal session
                              counts: loss_batch = global B / P makes the rank average of
                              the gradients the global batch's mean)                      */
  int64_t wfold_stride;    /* > 0: weight gradients folded into gtr_conv_bwd (gtr_layer.wfold;
                              the segments read them with live_groups = 1); 0: gtr_wgrad    */
} gtr_config;



/* Parameters + saved activations of one TransformerConv/BatchNorm layer.
 * w_all = [lin_query; lin_key; lin_value; lin_skip].weight stacked [4D, D],
 * b_all the matching biases [4D]; w_beta = lin_beta.weight [3D].             */
typedef struct gtr_layer {
  const float* w_all;
  const float* b_all;
  const float* w_beta;
  const float* bn_gamma;
  const float* bn_beta;
  float* bn_rmean;
  float* bn_rvar;
  int64_t* bn_nbt;
  float* xin;      /* [n_cap, D]  layer input (x_{l-1})            */
  float* qkvs;     /* [n_cap, 4D] query | key | value | skip        */
  float* alpha;    /* [e_cap, H]  attention probabilities            */
  float* agg;      /* [n_cap, D]  attention aggregate               */
  float* gate;     /* [n_cap]     beta gate                         */
  float* out;      /* [n_cap, D]  conv output (pre BatchNorm)        */
  float* bn_stats; /* [2D] batch mean, rstd                         */
  float* bn_part;  /* [max(g_cap, ceil(n_cap/8)), 1+2D] forward (count, mean, M2) partials
                      per row group (per 8 rows on the split path's gtr_attn_fwd).
                      consumer_reduce = 0 with > 32 row groups: the forward's bucket
                      mergers overwrite row 32*b with bucket b's merged row, so after
                      such a forward bn_part is NOT per-group partials any more      */
  float* bn_gsum;  /* [2D] sum(dy), sum(dy*xhat)                     */
  float* bn_gpart; /* [max(g_cap, 256), 2D] backward partials         */
  uint32_t* cnt;   /* [8 + 2*max(ceil(partials/32), 8)] arrival counters (zero-initialised
                      once; past 32 partial rows -- row groups, 8-row blocks, or the
                      <= 256 gtr_qkvs_bwd workgroups -- they are merged per bucket of 32) */
  float* dy;       /* [n_cap, D]  grad wrt BN(out)+x_{l-1} (pre dropout) */
  float* dqkvs;    /* [n_cap, 4D]                                    */
  float* du;       /* [n_cap]     grad wrt gate logit                 */
  float* dlogit;   /* [e_cap, H]                                     */
  float* dagg;     /* [n_cap, D]                                     */
  const float* bn_part_all;  /* sync_bn: every rank's forward partials [nparts_fwd][1+2D]  */
  const float* bn_gpart_all; /* sync_bn: every rank's backward partials [nparts_bwd][2D]   */
  int32_t nparts_fwd;
  int32_t nparts_bwd;
  float* wfold;              /* gtr_config.wfold_stride > 0: gtr_conv_bwd writes each row group's
                                split-K partial of this layer's weight gradients (w_all | b_all |
                                w_beta at the gtr_wgrad slab offsets) at wfold + g * stride     */
  const struct gtr_ffn* ffn; /* NULL, or this layer's feed-forward block (use_ffn=True; split
                                layer path only): the next layer's gtr_qkvs_fwd then takes its
                                input rows from ffn->z as they are, and its gtr_qkvs_bwd writes
                                d/dz into ffn->dz (no dropout mask, no BatchNorm sums)         */
} gtr_layer;

/* Feed-forward block of one layer (graph_transformer.py:88-100 _make_ffn, applied at
 * :160-170): with y = dropout(BN(conv out) + x) the layer's output rows,
 *   a = y W1^T + b1,  h = dropout(GELU(a)),  z = y + dropout(h W2^T + b2)   (F = 4 D).
 * GELU is the exact (erf) form of nn.GELU().  Dropout streams: kind 2 = h (element
 * row*F + j), kind 3 = the block output (row*D + j), per layer and step counter.       */
typedef struct gtr_ffn {
  const float* w1;  /* [F, D] ffns.{l}.0.weight  */
  const float* b1;  /* [F]    ffns.{l}.0.bias    */
  const float* w2;  /* [D, F] ffns.{l}.3.weight  */
  const float* b2;  /* [D]    ffns.{l}.3.bias    */
  float* y;         /* [n_cap, D] block input (saved)                         */
  float* a;         /* [n_cap, F] pre-activation (saved)                      */
  float* z;         /* [n_cap, D] block output                                */
  float* dz;        /* [n_cap, D] d loss / d z                                */
  float* g2;        /* [n_cap, D] dz * output dropout mask (d / d(h W2^T + b2)) */
  float* da;        /* [n_cap, F] d loss / d a                                */
  int32_t expansion; /* F / D: 4 (the factory default)                       */
  int32_t pad;
} gtr_ffn;

/* Embedding + LapPE inputs of layer 0. */
typedef struct gtr_embed {
  const float* table;  /* [T, D] item_embedding.weight              */
  const float* pe_tab; /* [T, pe_k] laplacian_pe._cached_pe or NULL  */
  const float* wpe;    /* [D, pe_k] laplacian_pe.projection.weight    */
  const float* bpe;    /* [D]                                        */
} gtr_embed;

/* Loss head. */
#define GTR_LOSS_NONE 0
#define GTR_LOSS_BPR 1
#define GTR_LOSS_LISTWISE 2
#define GTR_LOSS_DUAL 3
#define GTR_RO_FWD 1
#define GTR_RO_LOSS 2
#define GTR_RO_BWD 4

typedef struct gtr_head {
  int32_t flags;       /* GTR_RO_* */
  int32_t loss_kind;   /* GTR_LOSS_* */
  float temperature;
  float dual_alpha;
  float* se;           /* [b_cap, D] session embeddings (out if FWD, in otherwise) */
  const float* dse_in; /* [b_cap, D] upstream grad (BWD without LOSS)  */
  float* dse_out;      /* [b_cap, D] d loss / d se (LOSS; optional)    */
  float* coef_tgt;     /* [b_cap]     d loss / d pos score              */
  float* coef_neg;     /* [b_cap*n]   d loss / d neg score              */
  float* loss_part;    /* [512] per-workgroup (listwise, bpr) partial sums */
  float* loss_out;     /* [1]                                           */
  uint32_t* cnt;       /* [4]                                           */
} gtr_head;

int gtr_version(void);
int gtr_abi_version(void);
/* Hash of the sources the library was built from (etpgt/backend/_srchash.py). */
const char* gtr_source_hash(void);
const char* gtr_last_error(void);
/* 0 if `device` is a gfx950 (MI355X) device. */
int gtr_device_check(int device);

/* Forward of layer `l`; l == 0 gathers table rows (+LapPE), l > 0 applies the
 * previous layer's BatchNorm + residual + dropout in its prologue.  In training
 * mode the last arriving workgroup finalises this layer's BatchNorm statistics
 * and updates running_mean / running_var / num_batches_tracked.               */
int gtr_conv_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb,
                 const gtr_layer* layers, int l, gtr_stream_t stream);

/* Mean readout of the last layer (+ scoring loss forward/backward, + readout
 * backward into layers[L-1].dy and the last BatchNorm's backward sums).         */
int gtr_readout_loss(const gtr_config* cfg, const gtr_batch* bt, const float* table,
                     const gtr_layer* layers, const gtr_head* head, gtr_stream_t stream);

/* Backward of layer `l` given layers[l].dy and layers[l].bn_gsum.  Writes
 * layers[l].dqkvs/du and either layers[l-1].dy (+ its BN sums) or dx0.        */
int gtr_conv_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                 float* dx0, gtr_stream_t stream);

/* ---- large-batch ("split") layer path: the same layer as gtr_conv_fwd / gtr_conv_bwd
 * in two launches each, the dense GEMMs over ALL node rows (persistent f32-MFMA kernels
 * that keep W_all in registers per CU) and the per-row-group attention apart.  qkvs and
 * dX are bitwise those of the fused kernels (same k order); the BatchNorm backward sums
 * are summed in another (fixed) order.  Training needs consumer_reduce = 0 and no
 * sync_bn; D in {64, 128} for the GEMMs.  Order per layer:
 *   forward   gtr_qkvs_fwd(l) -> gtr_attn_fwd(l)
 *   backward  gtr_attn_bwd(l) -> gtr_qkvs_bwd(l)                                     */
/* X (layer 0: item row + LapPE projection, graph_transformer.py:140-152; l > 0: dropout(
 * BN(prev out) + prev in), :175-177) -> layers[l].xin; qkvs = X . W_all^T + b_all (PyG
 * TransformerConv lin_query/key/value/skip) -> layers[l].qkvs.                        */
int gtr_qkvs_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_embed* emb,
                 const gtr_layer* layers, int l, gtr_stream_t stream);
/* Attention over in-edges, beta gate and this layer's BatchNorm partials / statistics
 * from layers[l].qkvs (PyG TransformerConv message/softmax/aggregate). */
int gtr_attn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                 gtr_stream_t stream);
/* BatchNorm backward, gate backward, softmax backward, dQ / dK / dV -> layers[l].dqkvs,
 * du, dlogit (given layers[l].dy and bn_gsum).                                        */
int gtr_attn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                 gtr_stream_t stream);
/* dX = dQKVS . W_all + dy, the previous layer's dropout mask -> layers[l-1].dy and its
 * BatchNorm backward sums (bn_gsum), or dx0 at l == 0.                                */
int gtr_qkvs_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                 float* dx0, gtr_stream_t stream);

/* ---- feed-forward block (gtr_layer.ffn; D in {64, 128}, F = 4 D).  Order per layer l:
 *   forward   gtr_qkvs_fwd(l) -> gtr_attn_fwd(l) -> gtr_ffn_fwd(l)
 *   backward  gtr_ffn_bwd(l) -> gtr_attn_bwd(l) -> gtr_qkvs_bwd(l)
 * The readout of a model whose last layer has an FFN reads ffn->z through an identity
 * BatchNorm layer struct (statistics 0 / 1, gamma 1, beta 0, zero residual, dropout 0). */
/* y = dropout(BN(out) + xin) of layer l -> ffn->y; a = y W1^T + b1 -> ffn->a;
 * z = y + dropout(dropout(GELU(a)) W2^T + b2) -> ffn->z.                               */
int gtr_ffn_fwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                gtr_stream_t stream);
/* From ffn->dz: g2 -> ffn->g2, da -> ffn->da, and dy = (dz + da W1) * the layer's output
 * dropout mask -> layers[l].dy with its BatchNorm backward sums (bn_gsum).              */
int gtr_ffn_bwd(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                gtr_stream_t stream);
/* Weight-gradient partials of layer l's FFN over n_chunks row chunks:
 * slab[p * slab_stride + ...] = [dW1 F*D | db1 F | dW2 D*F | db2 D].                    */
int gtr_ffn_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, int l,
                  float* slab, int n_chunks, int64_t slab_stride, gtr_stream_t stream);

/* Weight-gradient partial slabs for layers [l_begin, l_end) (+ LapPE projection
 * when l_begin == 0).
 * Slab layout matches the flat parameter layout of each layer block:
 *   [w_all 4D*D | b_all 4D | w_beta 3D] and PE [wpe D*k | bpe D].
 * slabs[p * slab_stride + offset]; n_chunks partials over the node range.     */
int gtr_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers,
              const float* dx0, const float* pe_tab, float* const* layer_slab, float* pe_slab,
              int n_chunks, int64_t slab_stride, int l_begin, int l_end, gtr_stream_t stream);

/* One segment of the flat dense-parameter buffer for gtr_adamw_small. */
typedef struct gtr_segment {
  int64_t begin;      /* element offset in the flat buffer (multiple of 256) */
  int64_t len;
  const float* src;   /* gradient partials                                  */
  int64_t pstride;    /* distance between partials                           */
  int32_t nparts;
  int32_t live_groups; /* 1: sum only the batch's live row groups (min(nparts, hdr[4])):
                          partials written per row group by gtr_conv_bwd (wfold)     */
} gtr_segment;

typedef struct gtr_adam {
  float lr, beta1, beta2, eps, weight_decay;
  int32_t decoupled;          /* 1 = AdamW, 0 = Adam (L2 into the gradient)            */
  int32_t step_offset;        /* the update is step t = *step_dev + step_offset:
                                 1 when *step_dev counts completed steps (eager entry
                                 points), 0 after gtr_step_begin advanced it           */
  const int64_t* step_dev;    /* optimizer step counter (device)                       */
} gtr_adam;

/* AdamW (g = 0) of the item-table rows NOT touched by the step, spread over the layer
 * kernels of the fused step: launch slot s (conv_fwd of layer l -> slot l, conv_bwd of
 * layer l -> slot 2L-1-l) appends `blocks` workgroups that update rows
 * [bounds[s], bounds[s+1]) whose stamp != step, on the CUs the latency-bound row
 * groups leave idle.  The forward/backward never reads those rows (only touched rows
 * are gathered), so the slices are race-free; gtr_tail.sweep_from then skips them.    */
#define GTR_SWEEP_SLOTS 8
typedef struct gtr_sweep {
  float* table;
  float* m;
  float* v;
  int32_t* stamp;
  gtr_adam opt;       /* by value: the kernels copy it (opt.step_dev is a device pointer) */
  int64_t bounds[GTR_SWEEP_SLOTS + 1];
  int32_t dim;
  int32_t blocks;     /* workgroups per launch; <= 0: the CUs the launch's own workgroups leave */
  /* lag = 1 (lazy-table stamps, "current through step s"): the launches of step t bring
   * every row with stamp < t-1 forward to t-1 (the previous step's zero-gradient update,
   * older steps from consts as gtr_lazy) and stamp it; the rows the step reads were
   * brought forward by gtr_step_begin_lazy.  Used when the previous step's touched rows
   * are only known after the kernels that sweep (data parallel: the ranks' union).      */
  const float* consts;
  int32_t lag;
  int32_t pad;
} gtr_sweep;

#define GTR_SMALL_MAX_SEG 48
/* Sum each segment's gradient partials and apply (Adam|AdamW) — or, when
 * grad_out != NULL, only write the summed gradient there (eager path).        */
int gtr_adamw_small(float* param, float* m, float* v, float* grad_out, int64_t total,
                    const gtr_segment* segs, int nseg, const gtr_adam* opt, gtr_stream_t stream);

/* Contribution list of the item-table gradient: j < n_cap node rows (dx0),
 * then b_cap target rows, then b_cap*n negative rows (coef * se[b]).
 * Writes keys/vals (sentinel key = T for unused slots) and marks touched rows
 * stamp[row] = step+1.  m_cap = n_cap + b_cap*(1+n).                          */
int gtr_contrib_prep(const gtr_batch* bt, int num_items, int32_t* keys, int32_t* vals,
                     int32_t* stamp, const int64_t* step_dev, gtr_stream_t stream);
/* tmp (gtr_contrib_sort_bytes) must be zero-initialised once and otherwise left to the
 * sort: the default radix keeps per-pass digit totals there, zero between calls.       */
int gtr_contrib_sort_bytes(int m_cap, int num_items, size_t* bytes);
int gtr_contrib_sort(const int32_t* keys, const int32_t* vals, int32_t* skeys, int32_t* svals,
                     int m_cap, int num_items, void* tmp, size_t tmp_bytes, gtr_stream_t stream);

/* Touched rows: segmented sum of contributions in sorted (stable) order, then
 * AdamW on the row.  grad_dense != NULL: write the row gradient instead.      */
int gtr_adamw_rows(const gtr_batch* bt, int num_items, int dim, const int32_t* skeys,
                   const int32_t* svals, const float* dx0, const float* se, const float* coef_tgt,
                   const float* coef_neg, float* table, float* m, float* v, float* grad_dense,
                   const gtr_adam* opt, gtr_stream_t stream);

/* Untouched rows (stamp[row] != step+1): AdamW with zero gradient.            */
int gtr_adamw_sweep(int num_items, int dim, const int32_t* stamp, float* table, float* m, float* v,
                    const gtr_adam* opt, gtr_stream_t stream);

/* Eager path: dense[key_j] += coef_j * src_j over a contribution range.
 * mode 0: node rows (src = dx0, coef 1); mode 1: score rows (src = se).       */
int gtr_scatter_rows(const gtr_batch* bt, int dim, int mode, const float* src, const float* coef_tgt,
                     const float* coef_neg, float* dense, gtr_stream_t stream);

/* ---- fused training step (etpgt.train.fused.FusedTrainStep) ------------------
 * gtr_step_begin: advance the step (*step_dev += 1) and dropout-stream counters,
 * stamp the touched table rows (stamp[row] = new step) and build the sorted
 * contribution list skeys/svals (keys/vals/tmp: scratch for large batches, sized
 * by gtr_contrib_sort_bytes).  One launch (rank sort, 64 slots per workgroup) when
 * m_cap <= 8192 and T < 2^19; else contrib_prep + radix sort + counter update.  */
int gtr_step_begin(const gtr_batch* bt, int num_items, int32_t* keys, int32_t* vals, int32_t* skeys,
                   int32_t* svals, int32_t* stamp, int64_t* step_dev, uint32_t* rng_ctr, void* tmp,
                   size_t tmp_bytes, gtr_stream_t stream);

/* ---- deferred zero-gradient AdamW ("lazy" table, bitwise-identical) ---------------
 * The reference's dense AdamW updates every table row every step; a row the batch does
 * not touch takes the g = 0 update, whose only inputs are the row's own p, m, v and the
 * step's scalars.  In lazy mode those updates are deferred: stamp[row] = the step through
 * which the row is current, and a row is brought forward -- the same per-step update,
 * applied step by step with that step's scalars, so the floats are identical to eager
 * sweeping -- right before it is read (gtr_step_begin_lazy, gtr_dp_tail) or on demand
 * (gtr_lazy_flush: evaluation, checkpoints).  The step tail then updates only the
 * touched rows.  consts[t] = {lr / (1 - beta1^t), 1 / sqrt(1 - beta2^t)} (fp32 of the
 * double expressions, exactly as the eager kernels compute them), filled by the begin
 * kernel of step t; cap = its capacity in steps.                                      */
typedef struct gtr_lazy {
  float* consts;   /* [cap][2] */
  int32_t cap;
  int32_t pad;
  uint32_t* cnt;   /* [1] arrival counter (zero-initialised once) */
  float* table;
  float* m;
  float* v;
  gtr_adam opt;    /* by value */
} gtr_lazy;

/* gtr_step_begin + the lazy catch-up of every touched row and consts[t]; the step
 * counter advances after every workgroup has read it.  A touched row is claimed by
 * setting bit 30 of its stamp (the low bits keep the step it was current through) and p
 * is brought to t-1; under AdamW (decoupled) only p is written and the tail re-derives
 * m / v over the same missed steps, so the row's moments take one read-modify-write per
 * step.  The tail stamps the row with t.                                             */
int gtr_step_begin_lazy(const gtr_batch* bt, int num_items, int dim, int32_t* keys, int32_t* vals, int32_t* skeys,
                        int32_t* svals, int32_t* stamp, int64_t* step_dev, uint32_t* rng_ctr, void* tmp,
                        size_t tmp_bytes, const gtr_lazy* lazy, gtr_stream_t stream);
/* Bring every row forward to step *step_dev (stamp[row] = *step_dev).               */
int gtr_lazy_flush(int num_items, int dim, int32_t* stamp, const int64_t* step_dev, const gtr_lazy* lazy,
                   gtr_stream_t stream);

/* Inputs of the optimizer tail of a fused step.                                  */
typedef struct gtr_tail {
  const int32_t* skeys;   /* sorted contribution list (gtr_step_begin)             */
  const int32_t* svals;
  const float* dx0;       /* [n_cap, D] layer-0 input gradient                      */
  const float* se;        /* [b_cap, D] session embeddings                          */
  const float* coef_tgt;  /* [b_cap] d loss / d score(target)                        */
  const float* coef_neg;  /* [b_cap*n] d loss / d score(negative)                    */
  float* table;           /* [T, D] item table, its AdamW moments                    */
  float* table_m;
  float* table_v;
  int32_t* stamp;         /* [T] last step each row was touched (dp_tail writes) */
  float* flat;            /* flat small-parameter buffer + moments                   */
  float* flat_m;
  float* flat_v;
  int64_t flat_total;
  const float* loss_part; /* [loss_nparts, 2] pre-scaled loss partials (or NULL)     */
  float* loss_out;        /* [1] loss of the step                                   */
  int32_t loss_nparts;
  int32_t pad0;
  float* carry;           /* large batches (m_cap > 8192): [gtr_tail_carry_floats] scratch
                             for segment pieces spanning windows of the sorted list; else NULL */
  int64_t sweep_from;     /* untouched rows below this were updated during the chain (gtr_sweep) */
  const float* lazy_consts; /* lazy mode (gtr_lazy.consts): no untouched-row sweep; touched rows
                               are stamped with the step; the dp tail catches rows up first */
  uint32_t* rng_inc;        /* optional: += 1 at the end of the tail (fused begin, gtr_begin) */
  double* loss_acc;         /* optional: += the step's loss (one thread, after loss_out is final):
                               a device-side running sum over the steps of an epoch, so steps
                               chained in one hipGraph need no per-step loss read (trainer.py:130) */
} gtr_tail;

/* Floats of gtr_tail.carry needed at contribution capacity m_cap (0: not used).      */
int gtr_tail_carry_floats(int m_cap, int dim);

/* One launch: AdamW of the touched table rows (segmented sums), of the untouched
 * rows (zero gradient) and of every small parameter (segments), plus the loss sum.
 * Large batches (m_cap > 8192) add a first launch summing the segment pieces that
 * span windows of the sorted list (tail->carry); the rows part then runs per window.
 * opt->step_offset must be 0 (runs after gtr_step_begin).                        */
int gtr_step_tail(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail,
                  const gtr_segment* segs, int nseg, const gtr_adam* opt, gtr_stream_t stream);

/* Small batches (m_cap <= 8192, untouched-row sweep in the chain or a lazy table):
 * gtr_wgrad + gtr_step_tail as ONE launch (trainer.py:123-127: backward +
 * optimizer.step()).  The weight-gradient tiles write their split-K partial slabs
 * (layer_slab / pe_slab, n_chunks, slab_stride as gtr_wgrad); each tile's last arriving
 * chunk sums the n_chunks partials of its outputs in chunk order and applies AdamW;
 * touched rows and the bn_gsum segments run beside the tiles.  layer_flat [L][3] =
 * element offsets into tail->flat of each layer's w_all / b_all / w_beta; pe_flat [2] =
 * offsets of the LapPE projection weight / bias (NULL without LapPE); segs = the other
 * dense segments (BatchNorm gamma / beta from bn_gsum, <= 16); tile_cnt = tile_cnt_len
 * zeroed counters (one per tile; each launch leaves them zero).  Bitwise equal to
 * gtr_wgrad + gtr_step_tail.                                                          */
int gtr_step_tail_wgrad(const gtr_config* cfg, const gtr_batch* bt, const gtr_layer* layers, const float* pe_tab,
                        float* const* layer_slab, float* pe_slab, int n_chunks, int64_t slab_stride,
                        const int64_t* layer_flat, const int64_t* pe_flat, int num_items, const gtr_tail* tail,
                        const gtr_segment* segs, int nseg, const gtr_adam* opt, uint32_t* tile_cnt, int tile_cnt_len,
                        gtr_stream_t stream);

/* ---- data-parallel step (one process per GPU; etpgt.train.distributed) --------
 * Each rank packs its gradients into `pack` (words per rank = layout.words):
 *   [0, flat_total)          summed small-parameter gradient (flat layout)
 *   [loss_off]               local loss
 *   [keys_off, +m_cap)       sorted contribution keys (int32 bits; sentinel T)
 *   [rows_off, +m_cap*D)     per-segment-start summed table-gradient rows
 * After an all-gather of the packs (RCCL), every rank runs gtr_dp_tail on the
 * same [world][words] buffer: AdamW with the rank-averaged gradient on the union
 * of touched rows, the untouched rows and the small parameters — replicas stay
 * identical without exchanging parameters.                                       */
typedef struct gtr_dp_layout {
  int64_t flat_total, loss_off, keys_off, rows_off, words;
  int32_t m_cap, world;
} gtr_dp_layout;

int gtr_dp_pack(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail, const gtr_segment* segs,
                int nseg, const gtr_dp_layout* lay, float* pack, gtr_stream_t stream);

/* Early union stamp: keys_all = every rank's sorted contribution keys (all-gathered
 * right after gtr_step_begin, n = world * m_cap): stamp[key] = *step_dev, so that the
 * untouched-row sweep can run inside the backward kernels (gtr_sweep slots of the
 * readout / conv_bwd) and gtr_dp_tail sweeps only rows >= tail->sweep_from.          */
int gtr_dp_union_stamp(const int32_t* keys_all, int64_t n, int num_items, int32_t* stamp, const int64_t* step_dev,
                       gtr_stream_t stream);

/* slot: [T][world] int2 {step, segment-start index} scratch (init to -1).          */
int gtr_dp_tail(const gtr_batch* bt, int num_items, int dim, const gtr_tail* tail, const gtr_dp_layout* lay,
                const float* recv, int32_t* slot, const gtr_adam* opt, gtr_stream_t stream);

/* ---- row-sharded item table (etpgt.train.sharded; SURVEY.md §8e ii) ---------------
 * Replaces, across P ranks, the one dense nn.Embedding(T, d) of base.py:36 and its dense
 * AdamW state (train_baseline.py:252-256): global row r lives on rank r % P as local row
 * r / P, with its exp_avg / exp_avg_sq and a lazy-table stamp (gtr_lazy semantics: the
 * step through which the row is current).  A step:
 *   gtr_step_begin (global keys, stamp NULL) -> gtr_shard_route -> all-to-all send_ids
 *   -> gtr_shard_serve -> all-to-all send_rows -> forward/backward on the compact batch
 *   (table = fetched rows) -> gtr_shard_pack -> all-to-all send_grads + all-gather of
 *   small_pack -> gtr_shard_update.
 * Rows come in two classes when cap_s > 0: class 0 = rows some node of the batch reads
 * (needed by layer 0), class 1 = rows only the scoring readout reads (targets /
 * negatives: needed after the layers), so the class-1 rows can travel during the forward.
 * Per peer q, the id and gradient blocks hold blk = cap + cap_s slots: class 0 at
 * [0, cap) (slot 0 its count), class 1 at [cap, blk) (slot cap its count); ids ascending
 * per class.  The fetched-row buffer ("compact table") is [P*cap + P*cap_s][D]: class-0
 * row j of owner q at q*cap + j, class-1 row j at P*cap + q*cap_s + j, so each class is
 * one [P][cap_c][D] all-to-all.  cap_s = 0: one class, blk = cap (all rows class 0).   */
typedef struct gtr_shard {
  int32_t num_items;   /* T (global rows)                                       */
  int32_t world;       /* P (<= 16)                                             */
  int32_t rank;
  int32_t cap;         /* slots per peer block, the count slot included        */
  int32_t local_rows;  /* (T - rank + P - 1) / P                                */
  int32_t dim;
  float* table;        /* [local_rows, D] this rank's rows, exp_avg, exp_avg_sq */
  float* m;
  float* v;
  int32_t* stamp;      /* [local_rows] step through which the row is current   */
  float* consts;       /* [consts_cap][2] per-step AdamW scalars (gtr_lazy)     */
  int32_t consts_cap;
  int32_t cap_s;       /* class-1 slots per peer block (count included); 0: one class */
  int32_t* status;     /* [2]: [0] this step overflowed a block, [1] sticky:
                        * bit 0 this rank overflowed, bit 1 some rank did      */
  gtr_adam opt;        /* by value; step_offset 0 (runs after gtr_step_begin)   */
  int32_t* node_mark;  /* [T] scratch (cap_s > 0): step stamp of the rows a node reads */
  int64_t grad_stride; /* floats per peer block of send_grads / recv_grads (0: blk*D) */
  int64_t small_stride;/* > 0: gtr_shard_pack writes small_pack P times, q*small_stride
                          apart (the small pack riding in each peer's gradient block) */
  int32_t pack_parts;  /* gtr_shard_pack: 1 the rows part, 2 the small part, 0 / 3 both */
  int32_t pad1;
} gtr_shard;

/* Bytes of route scratch at contribution capacity m_cap.                            */
int gtr_shard_route_scratch(int m_cap, int world, size_t* bytes);
/* Requester: from the sorted contribution list (skeys / svals of gtr_step_begin), the
 * unique rows per owner -> send_ids [P][cap]; ckeys [m_cap] = compact row of each sorted
 * slot (-1: unused); the batch's node / target / negative ids as compact rows (the
 * arrays of the batch the layer kernels then read); node_pe [n_cap][pe_k] = pe_tab rows
 * of the nodes when given (LapPE: the layer kernels read node_pe, not pe_tab[id]).     */
int gtr_shard_route(const gtr_batch* bt, const int32_t* skeys, const int32_t* svals, const gtr_shard* sh,
                    int32_t* send_ids, int32_t* ckeys, int32_t* node_item_c, int32_t* target_c, int32_t* negatives_c,
                    const float* pe_tab, int pe_k, float* node_pe, void* scratch, size_t scratch_bytes,
                    gtr_stream_t stream);
/* Owner: the rows every peer requested (recv_ids = the all-to-all of send_ids) as they
 * stand after step t-1 (a lagging row's zero-gradient steps applied in registers; the
 * table is only read), into send_rows [P][cap][D] (row j of block r = recv_ids[r][j]). */
int gtr_shard_serve(const gtr_shard* sh, const int32_t* recv_ids, float* send_rows, gtr_stream_t stream);
/* Requester: summed table-gradient row of every requested row -> send_grads [P][cap][D]
 * at its compact slot; summed small-parameter gradient [flat_total] + local loss +
 * this step's overflow flag -> small_pack [flat_total + 2].                           */
int gtr_shard_pack(const gtr_batch* bt, const gtr_shard* sh, const gtr_tail* tail, const int32_t* ckeys,
                   const gtr_segment* segs, int nseg, float* send_grads, float* small_pack, gtr_stream_t stream);
/* Owner: every requested row caught up from its stamp to step t-1 and AdamW-updated at
 * step t in ONE read-modify-write, with the rank-averaged gradient (peers
 * summed in rank order), stamps t, consts[t]; small parameters from small_all
 * [P][small_words >= flat_total + 2] (rank-averaged) and the rank-averaged loss ->
 * tail->loss_out.  If any rank's pack carries the overflow flag, the step is applied
 * with zero gradients (rows unstamped, caught up later) and status[1] |= 2.          */
int gtr_shard_update(const gtr_shard* sh, const gtr_tail* tail, const int32_t* recv_ids, const float* recv_grads,
                     const float* small_all, int64_t small_words, gtr_stream_t stream);

/* ---- evaluation: full-catalog scoring + top-k (etpgt.model.base.predict) ---------
 * Replaces base.py:59-78 (scores = se @ item_embedding.weight.T; torch.topk(scores, k))
 * as called by Trainer.evaluate (trainer.py:138-173) for Recall@K / NDCG@K.
 * se [B, dim], table [num_items, dim] fp32 row-major; out_idx [B, k] int64 item ids and
 * out_score [B, k] fp32 scores, best first (score descending, item id ascending on ties;
 * row 0 and seen items are not masked, as in the reference).  1 <= k <= 128, k <= T.
 * Workspace (device, caller-provided) of gtr_topk_workspace_bytes(B, T, k) bytes.      */
int gtr_topk_workspace_bytes(int B, int num_items, int k, size_t* bytes);
int gtr_score_topk(const float* se, int B, int dim, const float* table, int num_items, int k,
                   int64_t* out_idx, float* out_score, void* ws, size_t ws_bytes, gtr_stream_t stream);
/* Same with per-session excluded ids (serving, etpgt/serving/recommender.py:126-131:
 * the session's items and the padding row never come back): session b excludes the
 * ascending ids excl_ids[excl_ptr[b] .. excl_ptr[b+1]).  If fewer than k ids remain,
 * the tail of out_idx is -1 (score -inf).                                           */
int gtr_score_topk_masked(const float* se, int B, int dim, const float* table, int num_items, int k,
                          const int32_t* excl_ptr, const int32_t* excl_ids, int64_t* out_idx, float* out_score,
                          void* ws, size_t ws_bytes, gtr_stream_t stream);

/* ---- GPU batch constructor (etpgt.data.gpu_batch) ----------------------------------
 * SessionDataset.__getitem__ + collate_fn (dataloader.py:64-202) on the device, writing
 * the packed batch image (gtr_batch) the training step consumes.  Per session: the last
 * max_len clicks, target = the last, nodes = sorted unique context ids, edges = graph
 * edges (item_i <= item_j, directed item_i -> item_j) with both ends in the context in
 * (src, dst) order, n_neg negatives uniform in [1, T) rejecting the session's clicks
 * (counter-based hash stream of (seed, batch position, draw)).                          */
typedef struct gtr_sessions {
  const int32_t* sess_ptr;   /* [S+1] click offsets                              */
  const int32_t* sess_items; /* clicks in click order                            */
  const int32_t* sess_nodes; /* [S] unique context ids (gtr_session_counts)      */
  const int32_t* sess_edges; /* [S] induced edges (gtr_session_counts)           */
  int32_t num_sessions;      /* S                                                */
  int32_t num_items;         /* T (table rows)                                   */
} gtr_sessions;

/* Power-of-two slot count (>= 2 * num_edges) of the edge hash.                        */
int gtr_edge_hash_slots(int64_t num_edges, int64_t* slots);
/* Open-addressing hash of the edge keys item_i * T + item_j.                           */
int gtr_edge_hash_build(const int64_t* keys, int64_t num_edges, uint64_t* slots, int64_t num_slots,
                        gtr_stream_t stream);
/* nodes[s], edges[s] of every session (capacity planning and batch offsets).           */
int gtr_session_counts(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots, int max_len,
                       int32_t* nodes, int32_t* edges, gtr_stream_t stream);
/* One batch of the B sessions order[(*cursor + b) % S] into *out (device blob arrays;
 * hdr sizes live), then *cursor += B.  scratch: [2 * b_cap + 2] int32, zero-initialised
 * (word 2 * b_cap: the arrival ticket of the one-launch build for B <= 256, reset by the
 * build itself); start: [1] int64;
 * status [2]: status[0] = this batch's code -- 1 (and an empty header) if the batch exceeds
 * out's capacities, 2 if a session leaves no item to sample negatives from (it holds
 * nearly the whole catalog: the reference would reject forever); status[1] |= each code
 * (sticky until the caller clears it).
 * row_group = the layer kernels' R for out's n_cap.  B <= 16384, max_len <= 64.        */
int gtr_build_batch(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots, int max_len,
                    const int32_t* order, int64_t* cursor, int B, int row_group, uint32_t seed,
                    const gtr_batch* out, int32_t* scratch, int64_t* start, int32_t* status,
                    gtr_stream_t stream);
/* The same with the cursor advancing by ``stride`` >= B per batch instead of B: rank r of
 * P data-parallel ranks, its cursor started at r*B, builds sessions [i*P*B + r*B, +B) of
 * the epoch order -- its share of global batch i, with the same position-keyed negatives
 * a single GPU draws for that global batch (stride = P*B).                            */
int gtr_build_batch_strided(const gtr_sessions* ss, const uint64_t* slots, int64_t num_slots, int max_len,
                            const int32_t* order, int64_t* cursor, int B, int64_t stride, int row_group,
                            uint32_t seed, const gtr_batch* out, int32_t* scratch, int64_t* start, int32_t* status,
                            gtr_stream_t stream);

/* ---- Laplacian positional-encoding precompute (etpgt.encodings.laplacian_gpu) ------
 * Replaces the host eigsh of compute_laplacian_pe (etpgt/encodings/laplacian_pe.py:19-66:
 * PyG get_laplacian(normalization="sym") + eigsh(k+1, which="SM"), reference
 * scripts/train/train_etpgt.py's LapPE precompute) for a symmetric adjacency in CSR
 * (ptr [n+1], col [nnz]):
 *   gtr_lap_build writes the off-diagonal values of L = I - D^-1/2 A D^-1/2 (dis [n] =
 *     deg^-1/2, val [nnz]; self loops 0; the unit diagonal is implicit).
 *   gtr_lap_plan (HOST pointers) cuts the rows into an nnz-balanced work list: items
 *     [n_items][4] = (row, e0, e1, part or -1), splits [n_splits][4] = (row, p0, p1, 0)
 *     for rows longer than `chunk`; call with items = splits = NULL to get the counts.
 *   gtr_lap_spmm computes Y = alpha * L X + beta * X for b <= 256 vectors (X, Y [n, b]
 *     row-major, X != Y) from the plan (device copies) and a part [n_parts, b] scratch —
 *     the block eigen-solver's operator; deterministic.                              */
int gtr_lap_build(const int32_t* ptr, const int32_t* col, int n, float* dis, float* val, gtr_stream_t stream);
int gtr_lap_plan(const int32_t* ptr, int n, int chunk, int32_t* items, int64_t* n_items, int32_t* splits,
                 int64_t* n_splits, int64_t* n_parts);
int gtr_lap_spmm(const int32_t* col, const float* val, int n, int b, const int32_t* items, int64_t n_items,
                 const int32_t* splits, int64_t n_splits, float* part, const float* X, float* Y, float alpha,
                 float beta, gtr_stream_t stream);
/* The solver's Gram matrices: out [2][64][64] fp64 = S^T S | S^T Y for S, Y [n, m] fp32
 * row-major, m <= 64 (entries past m are 0), accumulated in fp64 and summed in a fixed
 * order; part: P * 8192 doubles of scratch (P row chunks).                           */
int gtr_lap_gram(const float* S, const float* Y, int n, int m, double* part, int P, double* out,
                 gtr_stream_t stream);

/* Workgroups of gtr_readout_loss = the number of its loss / BatchNorm-sum partials
 * (gtr_tail.loss_nparts; the last layer's bn_gpart rows).                         */
int gtr_readout_grid(int b_cap);

/* step_dev += 1 (if non-NULL); rng_ctr += 1 (if non-NULL); if loss_part != NULL,
 * loss_out[0] = sum of the 2*nparts (already scaled) loss partials in order.     */
int gtr_step_end(int64_t* step_dev, uint32_t* rng_ctr, const float* loss_part, int nparts, float* loss_out,
                 gtr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GTR_H */
