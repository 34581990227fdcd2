/*
 * mirec.h — C-ABI of libmirec.so, the MI355X (gfx950) native hot path behind
 * recbole_amd (a drop-in for ghazalehnt/RecBole's embedding-lookup +
 * negative-sampling train loop and full-sort evaluator).
 *
 * Conventions:
 *   - every tensor argument is a DEVICE pointer owned by the caller (the PyTorch
 *     caching allocator); the library never allocates or frees caller memory;
 *   - scratch comes from a caller buffer sized by the matching *_workspace_size();
 *   - every call is stream-ordered on `stream` (a hipStream_t passed as void*),
 *     re-entrant, and does not synchronise the host (graph-capturable);
 *   - return 0 on success, <0 on error (argument error = -1, HIP error = -(1000+hipError_t));
 *     mirec_last_error() gives a thread-local message.
 *
 * The reference is pure Python/PyTorch: there is no FFI in it. Each entry
 * below cites the reference function whose arithmetic it replaces; the host
 * binding (ctypes) lives in recbole_amd/_native.py.
 */
#ifndef MIREC_H
#define MIREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIREC_ABI_VERSION 18

int mirec_abi_version(void);
const char* mirec_last_error(void);

/* ---------------------------------------------------------------------------
 * K4  Negative sampler: cyclic walk over a pre-shuffled list + rejection.
 * Replaces AbstractSampler.random_num / sample_by_key_ids
 *   (recbole/sampler/sampler.py:82-101, 103-154) as driven by
 *   Sampler.sample_by_user_ids (:246-265) and RepeatableSampler (:341-420).
 * Bit-exact: out[j*Kb + k] is the j-th negative of key k of a batch of Kb keys;
 * round 0 takes random_list[(pr + t) mod L] for slot t, and every slot whose
 * value is in used[key] is refilled IN ASCENDING SLOT ORDER from the
 * continuing walk until none is left. *pr_dev is advanced (kept mod L) and
 * persists across calls exactly like `random_pr`.
 *
 * Processes n_batches consecutive batches in ONE launch: batch b uses keys
 * keys[b*batch_keys .. min((b+1)*batch_keys, n_keys)) and writes its
 * Kb*num values at out + b*out_stride (out_stride 0 = batch_keys*num), so the
 * trainer can sample a chunk of future batches straight into their
 * [pos | neg] key rows.  used_ptr[n_key_space+1]/used_cols is a CSR of the
 * phase's used item ids per key, each row sorted ascending; used_bits (or
 * NULL) the same sets as a [n_key_space, ceil(n_bits/32)] bitmap built by
 * mirec_used_bitmap_build — one load per membership test instead of a binary
 * search; either representation gives identical results. reject==0 skips
 * the rejection (RepeatableSampler).  Status -2: a key is out of range
 * (the reference raises ValueError in sample_by_user_ids); -3: the walk did
 * not terminate within 4*L+1024 refill rounds (the reference loops forever).
 * ------------------------------------------------------------------------- */
size_t mirec_sample_walk_workspace_size(int64_t batch_keys, int64_t num);
int mirec_sample_walk(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                      const int64_t* keys, int64_t n_keys, int64_t batch_keys,
                      int64_t n_batches, int64_t num,
                      const int64_t* used_ptr, const int32_t* used_cols,
                      const uint32_t* used_bits, int64_t n_bits,
                      int64_t n_key_space, int reject,
                      int64_t* out, int64_t out_stride, int32_t* status_dev,
                      void* ws, size_t ws_bytes, void* stream);

/* Successive sample_by_key_ids calls of DIFFERENT sizes in one launch (the
 * evaluation loaders' one call per user, general_dataloader.py:210-221 ->
 * sampler.py:246-265): call s uses keys[seg_ptr[s] .. seg_ptr[s+1]) and writes
 * its K_s*num values (layout j*K_s + k) at out + seg_ptr[s]*num; the walk
 * continues from call to call. seg_ptr: device int64 [n_seg+1]; K_s <=
 * max_seg_keys; workspace = mirec_sample_walk_workspace_size(max_seg_keys, num).
 * Same status codes as mirec_sample_walk. */
int mirec_sample_walk_segments(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                               const int64_t* keys, const int64_t* seg_ptr, int64_t n_seg,
                               int64_t max_seg_keys, int64_t num,
                               const int64_t* used_ptr, const int32_t* used_cols,
                               const uint32_t* used_bits, int64_t n_bits,
                               int64_t n_key_space, int reject, int64_t* out,
                               int32_t* status_dev, void* ws, size_t ws_bytes, void* stream);

/* Alias-table FAST MODE (labelled non-parity; north_star (c)): i.i.d. draws from
 * the same distribution the walk follows — p(v) proportional to counts[v], i.e.
 * the number of times v appears in random_list (uniform: 1 for ids 1..n-1;
 * popularity: item frequency, sampler.py:197-201) — with the same rejection of
 * used ids, but NOT the reference's value sequence. Replaces random_num's
 * cyclic walk (sampler.py:82-101) when Sampler.enable_alias() was called.
 *
 * mirec_alias_build (HOST pointers, host-side setup): Vose's alias method in
 * exact integer arithmetic over n columns; thr[c] in units of 2^-32.
 * mirec_sample_alias: draw id = counter + g for the g-th value of the call
 * (batches in order, slot j*Kb + k inside batch b, values at out + b*out_stride
 * like mirec_sample_walk); random bits = splitmix64(seed ^ splitmix64(id*4096 +
 * attempt)); a used value is redrawn with attempt+1 (status -3 after 4096
 * attempts, -2 for a key outside [0, n_key_space)). The caller advances counter
 * by n_keys*num per call. Deterministic for a given (seed, counter). */
int mirec_alias_build(const int64_t* counts, int64_t n, uint32_t* thr, int32_t* alias);
int mirec_sample_alias(const uint32_t* thr, const int32_t* alias, int64_t n_cols,
                       uint64_t seed, uint64_t counter, const int64_t* keys,
                       int64_t n_keys, int64_t batch_keys, int64_t num,
                       const int64_t* used_ptr, const int32_t* used_cols,
                       const uint32_t* used_bits, int64_t n_bits, int64_t n_key_space,
                       int reject, int64_t* out, int64_t out_stride,
                       int32_t* status_dev, void* stream);

/* Host data-pipeline primitives (CPU, HOST pointers):
 * mirec_host_counting_order: order = stable sort permutation of keys in
 *   [0, key_space) (grouping rows by user: dataset.py:1249-1256 _grouped_index);
 * mirec_host_csr_build: CSR of the distinct (key, value) pairs, rows ascending
 *   (the per-phase used-id sets, sampler.py:206-227); cols sized n by the caller;
 *   returns the number of distinct pairs. */
int mirec_host_counting_order(const int64_t* keys, int64_t n, int64_t key_space, int64_t* order);
int64_t mirec_host_csr_build(const int64_t* keys, const int64_t* vals, int64_t n, int64_t n_keys,
                             int64_t* ptr, int32_t* cols);

/* Used-id bitmap of a CSR (sampler.py:206-227 used_ids as bits):
 * bits[k * ceil(n_bits/32) + v/32] bit v%32 set iff v in used[k], v < n_bits. */
/* K4s — the same walk (values, pointer, status: bit for bit mirec_sample_walk's) of
 * n_batches fixed-size batches by speculation: every batch is walked at every start its
 * window admits (R = refill draws of the batches before it, windows b*r_mean -+
 * (4.5*r_sd*sqrt(b) + 3) from the caller's per-batch rejection statistics, b < 16) in one
 * chip-wide launch, a second launch chains the exact starts and writes each batch from
 * its chosen start; a batch outside its window and every batch after it are walked by the
 * single-block walk. Two launches per 16 batches instead of one serial walk. keys =
 * users (batch b at users + b*batch_keys); out / out_stride as mirec_sample_walk. With
 * user_keys (and items, item_keys, key_stride >= batch_keys) it also copies each batch's
 * keys to user_keys + b*batch_keys and its items to item_keys + b*key_stride (the chunk
 * preparation's key rows). batch_keys <= 1024, batch_keys * num <= 4096. Workspace:
 * mirec_sample_walk_spec_workspace_size(batch_keys, num, min(n_batches, 16), r_mean, r_sd). */
size_t mirec_sample_walk_spec_workspace_size(int64_t batch_keys, int64_t num,
                                             int64_t max_batches, double r_mean, double r_sd);
int mirec_sample_walk_spec(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                           const int64_t* users, const int64_t* items, int64_t n_batches,
                           int64_t batch_keys, int64_t num, const int64_t* used_ptr,
                           const int32_t* used_cols, const uint32_t* used_bits, int64_t n_bits,
                           int64_t n_key_space, int reject, double r_mean, double r_sd,
                           int64_t* out, int64_t out_stride, int64_t* user_keys,
                           int64_t* item_keys, int64_t key_stride, int32_t* status_dev, void* ws,
                           size_t ws_bytes, void* stream);
size_t mirec_used_bitmap_bytes(int64_t n_keys, int64_t n_bits);
int mirec_used_bitmap_build(const int64_t* used_ptr, const int32_t* used_cols, int64_t n_keys,
                            int64_t n_bits, uint32_t* bits, void* stream);

/* ---------------------------------------------------------------------------
 * K1  Row gather (any row width, 16-B vectorised when aligned).
 * Replaces nn.Embedding forward / index_select (bpr.py:58-72 via
 *   torch.nn.functional.embedding) and the column gathers of Interaction
 *   slicing / shuffle (interaction.py:260-276).
 * out[i, :] = table[idx[i], :];  idx must lie in [0, n_rows).
 * ------------------------------------------------------------------------- */
int mirec_gather_rows(const void* table, int64_t n_rows, int64_t row_bytes,
                      const int64_t* idx, int64_t n, void* out, void* stream);
int mirec_gather_rows_i32idx(const void* table, int64_t n_rows, int64_t row_bytes,
                             const int32_t* idx, int64_t n, void* out, void* stream);

/* Sliding-window gather (SequentialDataLoader.augmentation,
 * recbole/data/dataloader/sequential_dataloader.py:95-127, on the device):
 * out[i, t] = col[start[i] + t] for t < len[i], else 0 (elements of 4 or 8 bytes). */
int mirec_window_gather(const void* col, int32_t elem_bytes, const int64_t* start,
                        const int64_t* len, int64_t n, int32_t L, void* out, void* stream);

/* ---------------------------------------------------------------------------
 * K3  Fused BPR forward + backward.
 * Replaces BPR.calculate_loss (recbole/model/general_recommender/bpr.py:74-83),
 *   BPRLoss.forward (recbole/model/loss.py:47-49) and their autograd backward.
 * Pairwise layout of GeneralNegSampleDataLoader (general_dataloader.py:235-241):
 *   row r = j*B + k pairs (user[k], pos[k], neg[j*B+k]) for j < times.
 * Per row: x = <u,p> - <u,n>;  loss_r = -log(gamma + sigmoid(x));
 *   dloss/dx_r = grad_scale * (-(s*(1-s)) / (gamma + s)),  s = sigmoid(x)
 *   (grad_scale = 1/(B*times) reproduces .mean()).
 * Outputs (any may be NULL):
 *   loss_k[B]          = sum_j loss_{j*B+k}       (fixed j order)
 *   pos_score[B], neg_score[times*B]
 *   gU[B,d]            = sum_j dx_jk * (p_k - n_jk)      (d loss / d u_k)
 *   gI[(1+times)*B,d]  rows 0..B-1: (sum_j dx_jk) * u_k  (d loss / d p_k)
 *                      rows B+r   : -dx_r * u_k          (d loss / d n_r)
 * d in {32, 64, 128, 256}.
 * ------------------------------------------------------------------------- */
int mirec_bpr_fwd_bwd_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                          int32_t d, const int64_t* user, const int64_t* pos,
                          const int64_t* neg, int64_t B, int32_t times,
                          float gamma, float grad_scale,
                          float* loss_k, float* pos_score, float* neg_score,
                          float* gU, float* gI, void* stream);

/* K3 forward only, for the data-parallel step: the same per-row computation as
 * mirec_bpr_fwd_bwd_f32 (loss_k as there) plus coef[times*B], coef[r] = dloss/dx_r
 * of row r = j*B + k — the ONLY per-row quantity the backward needs besides the
 * rows themselves. Ranks exchange these (4 B per row instead of a d-float row). */
/* K3 on a row-sharded step's received rows (csrc/shard.hip): E holds the rows every slot
 * reads (users and items alike), ids index E, and each slot's gradient row is written at
 * grad + id * d — the message position it returns in — instead of at its slot: K3 and the
 * backward gather (mirec_gather_rows_i32idx) in one launch. The ids of a batch's slots
 * must be distinct. Arithmetic: mirec_bpr_fwd_bwd_f32's, bit for bit. */
int mirec_bpr_fwd_bwd_at_ids_f32(const float* E, int64_t nE, int32_t d, const int64_t* user,
                                 const int64_t* pos, const int64_t* neg, int64_t B,
                                 int32_t times, float gamma, float grad_scale, float* loss_k,
                                 float* grad, void* stream);
int mirec_bpr_fwd_coef_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                           int32_t d, const int64_t* user, const int64_t* pos,
                           const int64_t* neg, int64_t B, int32_t times,
                           float gamma, float grad_scale, float* loss_k, float* coef,
                           void* stream);

/* The gradient rows gU / gI of mirec_bpr_fwd_bwd_f32 for a (global) batch of B
 * positives rebuilt from the rows and the coefficients, bit-identical to what
 * mirec_bpr_fwd_bwd_f32 writes for the same batch on one GPU. Coefficient of row
 * (j, k): coef[(k / coef_block) * coef_stride + j * coef_block + k % coef_block]
 * (coef_block = positives per rank, coef_stride >= times * coef_block: the rank
 * blocks of an all-gathered exchange buffer; one block of stride times*B is the
 * single-rank layout). Replaces the backward half of the same reference path. */
int mirec_bpr_contrib_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                          int32_t d, const int64_t* user, const int64_t* pos,
                          const int64_t* neg, int64_t B, int32_t times,
                          const float* coef, int64_t coef_block, int64_t coef_stride,
                          float* gU, float* gI, void* stream);

/* score[r] = <EU[u[r]], EI[i[r]]>  — BPR.predict (bpr.py:85-89), used by the
 * sampled-evaluation loaders (trainer.py:400-406). d in {32,64,128,256}. */
int mirec_dot_rows_f32(const float* EU, int64_t nU, const float* EI, int64_t nI, int32_t d,
                       const int64_t* u, const int64_t* i, int64_t n, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Deterministic reductions used by the trainer loop (trainer.py:157-174).
 * out[0] = sum(x[0..n)) in a fixed tree order (launch-shape independent).
 * ------------------------------------------------------------------------- */
int mirec_sum_f32(const float* x, int64_t n, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * K2  Segment sort: group contribution rows by table row id, deterministic.
 * Replaces the index_add in torch's embedding_dense_backward for
 *   nn.Embedding(sparse=False) (bpr.py:40-41; trainer.py:170).
 * Stable sort of (keys[c], c): perm[i] = c sorted by (key, c); one workgroup in LDS
 * up to 8,192 keys, a device-wide 4-bit LSD radix sort above (single batch);
 *   uniq[u] = distinct keys ascending, seg[u]..seg[u+1] their slice of perm,
 *   *n_uniq_dev = number of distinct keys. Keys must lie in [0, key_space).
 * ------------------------------------------------------------------------- */
size_t mirec_segment_sort_workspace_size(int64_t n, int64_t key_space);
int mirec_segment_sort(const int64_t* keys, int64_t n, int64_t key_space,
                       int32_t* perm, int32_t* uniq, int32_t* seg,
                       int32_t* n_uniq_dev, void* ws, size_t ws_bytes, void* stream);

/* Batched form: batch b groups keys[b*batch_n, min((b+1)*batch_n, n)) into
 * perm/uniq + b*batch_n, seg + b*(batch_n+1), n_uniq_dev[b]; one workgroup per
 * batch, so a whole chunk of future training batches is grouped in one launch.
 * Workspace: mirec_segment_sort_workspace_size(n_batches*batch_n, key_space). */
int mirec_segment_sort_batched(const int64_t* keys, int64_t n, int64_t batch_n,
                               int64_t key_space, int32_t* perm, int32_t* uniq, int32_t* seg,
                               int32_t* n_uniq_dev, void* ws, size_t ws_bytes, void* stream);

/* The single sort of mirec_segment_sort for n > 8,192 keys in 2 + ceil(bits / 8)
 * launches (global digit histograms; per 8-bit pass a stable LDS ranking of 2,048-key
 * tiles whose digit offsets come from a decoupled look-back; the segments by a look-back
 * scan). Same perm / uniq / seg / n_uniq; pos_seg (nullable, int32[n]) = the segment of
 * each sorted position. ws: >= 16 * n bytes. status: int32[n_status >=
 * mirec_segment_sort_onesweep_status_words(n)], zero before the first call, left zero
 * (one buffer per stream). 0 < n < 2^30. The grouping K2 of every gradient reduction
 * (reference: torch's embedding backward in recbole/model/sequential_recommender/
 * sasrec.py:107-141 and abstract_recommender.py's embedding lookups). */
int64_t mirec_segment_sort_onesweep_status_words(int64_t n);
int mirec_segment_sort_onesweep(const int64_t* keys, int64_t n, int64_t key_space,
                                int32_t* perm, int32_t* uniq, int32_t* seg, int32_t* n_uniq_dev,
                                int32_t* pos_seg, void* ws, size_t ws_bytes, int32_t* status,
                                int64_t n_status, void* stream);

/* The same single sort (mirec_segment_sort outputs) for keys that come in blocks of
 * block_n (<= 8,192) with every key of block b below every key of block b+1 (e.g.
 * DeepFM's token keys, field-major at increasing table offsets): each block sorted
 * in LDS, then concatenated — two launches instead of a device-wide radix sort.
 * Workspace: mirec_segment_sort_blocks_workspace_size(n, block_n). */
size_t mirec_segment_sort_blocks_workspace_size(int64_t n, int64_t block_n);
int mirec_segment_sort_blocks(const int64_t* keys, int64_t n, int64_t block_n, int64_t key_space,
                              int32_t* perm, int32_t* uniq, int32_t* seg, int32_t* n_uniq_dev,
                              void* ws, size_t ws_bytes, void* stream);
/* The same in ONE launch for block_n <= 4,096 and at most 256 blocks: each block sorts
 * in LDS (8-bit digits over its own key span) and writes straight into the
 * concatenated outputs after summing the unique counts of the blocks before it.
 * status: int32[n_status >= n_blocks + 1], all zero before the first call; every call
 * leaves it zero again (reuse one buffer per stream; two calls in flight at once need
 * two buffers). pos_seg (nullable, int32[n]): pos_seg[p] = the segment of sorted
 * position p (seg[pos_seg[p]] <= p < seg[pos_seg[p] + 1]) for the *_pos_seg reductions.
 * The grouping of the token-field embedding gradient rows of
 * reference recbole/model/layers.py:121-141 (FMEmbedding, called from
 * abstract_recommender.py:260 embed_token_fields) before the deferred Adam. */
int mirec_segment_sort_blocks_chained(const int64_t* keys, int64_t n, int64_t block_n,
                                      int64_t key_space, int32_t* perm, int32_t* uniq,
                                      int32_t* seg, int32_t* n_uniq_dev, int32_t* status,
                                      int64_t n_status, int32_t* pos_seg, void* stream);
/* The same for keys given as fields (mirec_offset_keys' inputs: block f = cols[f][0..B)
 * + offsets[f], ranges increasing with f): the launch forms the keys, writes them to
 * keys_out [n_fields * B] and sorts them — mirec_offset_keys + the chained sort in one
 * launch. 1 <= n_fields <= 64, B <= 4,096; status >= n_fields + 1 words (as above). */
int mirec_segment_sort_fields_chained(const int64_t* const* cols, const int64_t* offsets,
                                      int32_t n_fields, int64_t B, int64_t key_space,
                                      int64_t* keys_out, int32_t* perm, int32_t* uniq,
                                      int32_t* seg, int32_t* n_uniq_dev, int32_t* status,
                                      int64_t n_status, int32_t* pos_seg, void* stream);

/* Look-ahead lists of the deferred Adam: for b < n_batches-1,
 * out[b*stride ..) = uniq(b+1) \ uniq(b) ascending, n_out[b] its length, where
 * uniq(b) = uniq[b*stride .. + n_uniq[b]) (the batched segment-sort layout);
 * n_out[n_batches-1] = 0. */
int mirec_uniq_ahead_diff(const int32_t* uniq, const int32_t* n_uniq, int64_t stride,
                          int64_t n_batches, int32_t* out, int32_t* n_out, void* stream);

/* ---------------------------------------------------------------------------
 * Chunk preparation of the fused pairwise train step (the data side of
 * Trainer._train_epoch, trainer.py:157-174, for n_batches consecutive batches of
 * the shuffled train table: GeneralNegSampleDataLoader._next_batch_data +
 * _neg_sampling, general_dataloader.py:181-251) in ONE call, stream-ordered:
 *   keys     user_keys[b*Bc + k] = users[s0 + b*Bc + k];
 *            item_keys[b*(1+T)*Bc + k] = items[s0 + b*Bc + k]   (row 0: positives)
 *   K4 walk  negatives of each batch into item_keys rows 1..T (mirec_sample_walk)
 *   K2       groupings of the user keys and of the [pos | neg] item keys per batch
 *            (mirec_segment_sort_batched, key spaces n_users / n_items)
 *   ahead    look-ahead lists (mirec_uniq_ahead_diff), when u_ahead != NULL
 * Every pointer is a device pointer except the struct itself (host). sort_ws:
 * mirec_segment_sort_workspace_size(n_batches*(1+T)*Bc, n_items) bytes. */
typedef struct mirec_chunk_prep {
  const int64_t* users;  const int64_t* items;  int64_t s0;
  int64_t n_batches, Bc, T;
  int64_t* user_keys;    int64_t* item_keys;
  const int32_t* random_list; int64_t L; int64_t* pr_dev;
  const int64_t* used_ptr; const int32_t* used_cols; const uint32_t* used_bits; int64_t n_bits;
  int64_t n_users, n_items; int32_t reject; int32_t* status;
  void* walk_ws; size_t walk_ws_bytes; void* sort_ws; size_t sort_ws_bytes;
  int32_t *u_perm, *u_uniq, *u_seg, *u_nu, *i_perm, *i_uniq, *i_seg, *i_nu;
  int32_t *u_ahead, *u_nah, *i_ahead, *i_nah;
  /* alias fast mode (alias_thr != NULL): mirec_sample_alias replaces the walk */
  const uint32_t* alias_thr; const int32_t* alias_idx; int64_t n_alias;
  uint64_t alias_seed, alias_counter;
  /* K35 records (u_rec != NULL): mirec_step_records after the groupings */
  int32_t *u_rec, *u_crec, *i_rec, *i_crec;
  /* K4s (spec_ws != NULL, walk only): the chunk's walk and key rows by
   * mirec_sample_walk_spec with the rejection statistics r_mean / r_sd */
  void* spec_ws; size_t spec_ws_bytes; double r_mean, r_sd;
} mirec_chunk_prep;
int mirec_prepare_chunk(const mirec_chunk_prep* p, void* stream);
/* The two halves of mirec_prepare_chunk, for two streams (the caller orders
 * group after walk, e.g. with an event): keys + K4 walk (or alias draws), then the
 * K2 groupings + look-ahead lists. Splitting lets chunk c+1's walk run while
 * chunk c is grouped. */
int mirec_prepare_chunk_walk(const mirec_chunk_prep* p, void* stream);
int mirec_prepare_chunk_group(const mirec_chunk_prep* p, void* stream);
/* K36 — a prepared chunk's grouping side in ONE launch, one workgroup per (table,
 * batch): the K2 groupings (perm / uniq / seg / n_uniq, identical to
 * mirec_segment_sort_batched's), the K35 records (identical to mirec_step_records';
 * u_rec.. NULL: none) and the look-ahead lists (identical to mirec_uniq_ahead_diff's;
 * u_ahead.. NULL: none). Keys are clamped to [0, n) as the records clamp them.
 * Returns 1 when done, 0 when the shapes are outside its one-workgroup form (Bc >
 * 2,048, (1+T)*Bc > 4,096, key and position bits > 32, or look-ahead key spaces >
 * 2^18 rows) — nothing was launched, the caller groups by the general path — and
 * < 0 on bad arguments. mirec_prepare_chunk_group uses it when it applies. */
int mirec_chunk_group(const int64_t* user_keys, const int64_t* item_keys, int64_t n_batches,
                      int64_t Bc, int32_t T, int64_t n_users, int64_t n_items, int32_t* u_perm,
                      int32_t* u_uniq, int32_t* u_seg, int32_t* u_nu, int32_t* i_perm,
                      int32_t* i_uniq, int32_t* i_seg, int32_t* i_nu, int32_t* u_rec,
                      int32_t* u_crec, int32_t* i_rec, int32_t* i_crec, int32_t* u_ahead,
                      int32_t* u_nah, int32_t* i_ahead, int32_t* i_nah, void* stream);
/* 1 when mirec_chunk_group takes chunks of batches of Bc positives with T negatives over
 * n_users x n_items tables (ahead: look-ahead lists asked for), else 0. Host only. */
int mirec_chunk_group_fits(int64_t Bc, int32_t T, int64_t n_users, int64_t n_items,
                           int32_t ahead);

/* dense[uniq[u], :] += sum_{i in seg[u]..seg[u+1]} rows[perm[i], :] — the
 * dense-gradient form used by the autograd-compatible path. n = number of
 * contributions (seg[n_uniq] <= n). The sorted contributions are summed in chunks
 * of 32 (8 when d = 1) positions in a fixed order (hot rows are split over many lane groups and
 * their partials added in chunk order by a fixup pass): deterministic, no atomics.
 * Workspace: mirec_segment_scatter_add_workspace_size(n, d). 1 <= d <= 256. */
size_t mirec_segment_scatter_add_workspace_size(int64_t n, int32_t d);
int mirec_segment_scatter_add_f32(const float* rows, int32_t d, const int32_t* perm,
                                  const int32_t* uniq, const int32_t* seg,
                                  const int32_t* n_uniq_dev, int64_t n, float* dense,
                                  int64_t n_rows, void* ws, size_t ws_bytes, void* stream);
/* The deferred optimizer's second level for two reduced sources of one table: A =
 * (uA[0..*nA_dev) ascending distinct, rowsA [capA, d]), B likewise. uniq_out / rows_out
 * get the union rows ascending, *n_out_dev their count, and each row the sum the
 * second-level mirec_segment_reduce_f32 of [A; B] gives ((0 + a) + b, 0 + a, 0 + b; with
 * a_pre = 1, a already carries its 0 +: a previous merge's output) — bit for bit,
 * without sorting the concatenated keys. ws: >= 8 * (capA + capB) bytes; status:
 * >= (capA + capB) / 512 + 2 int32, zero before the call, left zero. Two launches. */
int mirec_segment_merge2_f32(const int32_t* uA, const int32_t* nA_dev, int64_t capA,
                             const float* rowsA, const int32_t* uB, const int32_t* nB_dev,
                             int64_t capB, const float* rowsB, int32_t d, int32_t a_pre,
                             int32_t* uniq_out, int32_t* n_out_dev, float* rows_out, void* ws,
                             size_t ws_bytes, int32_t* status, int64_t n_status, void* stream);
/* Compact form: out[u, :] = sum of segment u's contributions (u < n_uniq), the same
 * chunked fixed-order summation; out needs n rows. Lets K5 take each touched row's
 * gradient as one row (hot Zipf rows would otherwise be summed serially in K5). */
int mirec_segment_reduce_f32(const float* rows, int32_t d, const int32_t* perm,
                             const int32_t* uniq, const int32_t* seg, const int32_t* n_uniq_dev,
                             int64_t n, float* out, void* ws, size_t ws_bytes, void* stream);
/* mirec_segment_reduce_f32 with pos_seg[n] (the segment of every sorted position, from
 * mirec_segment_sort_onesweep / _blocks_chained): the same outputs bit for bit (same
 * pieces, same order), without a search per chunk of positions. 1 <= d <= 256. */
int mirec_segment_reduce_pos_seg_f32(const float* rows, int32_t d, const int32_t* perm,
                                     const int32_t* pos_seg, const int32_t* uniq,
                                     const int32_t* seg, const int32_t* n_uniq_dev, int64_t n,
                                     float* out, void* ws, size_t ws_bytes, void* stream);
/* Two sources grouped by the same segments in one pass (DeepFM's [V, d] token rows and
 * [V, 1] first-order weights): out = mirec_segment_reduce_f32(rows, d, ...) and out1 =
 * the same for rows1 with d = 1, bit for bit. 2 <= d <= 16; ws: at least
 * mirec_segment_scatter_add_workspace_size(n, d + 1) bytes. */
int mirec_segment_reduce2_f32(const float* rows, int32_t d, const float* rows1,
                              const int32_t* perm, const int32_t* uniq, const int32_t* seg,
                              const int32_t* n_uniq_dev, int64_t n, float* out, float* out1,
                              void* ws, size_t ws_bytes, void* stream);
/* mirec_segment_reduce2_f32 with pos_seg[n] (the segment of every sorted position, from
 * mirec_segment_sort_blocks_chained): the same outputs bit for bit, without a search per
 * chunk of positions. */
int mirec_segment_reduce2_pos_seg_f32(const float* rows, int32_t d, const float* rows1,
                                      const int32_t* perm, const int32_t* pos_seg,
                                      const int32_t* uniq, const int32_t* seg,
                                      const int32_t* n_uniq_dev, int64_t n, float* out,
                                      float* out1, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * K5  Dense Adam over every row, with the gradient supplied in compact form.
 * Replaces optim.Adam.step (trainer.py:109-130, 173; torch optim/adam.py
 *   _single_tensor_adam) for a table whose dense gradient would be zero
 *   except on the rows in `uniq` — i.e. exactly the dense Adam the reference
 *   runs over nn.Embedding(sparse=False) weights, in ONE streaming pass over
 *   p, m, v (no dense gradient buffer).
 * g[row] = sum_{i in seg[u]..seg[u+1]} rows[perm[i]]  if row == uniq[u], else 0
 * (+ dense_grad[row] when dense_grad != NULL; the grouped part may be omitted
 * with n_uniq_dev == NULL) (+ wd*p).  d in {4,16,32,64,128,256} floats per row
 * (any tensor whose numel % 4 == 0 can be viewed as [numel/4, 4]).
 * Per element (torch's order and rounding, see adam.hip):
 *   g = fma(p, wd, g);  m = fma(1-b1, g-m, m);  v = fma((1-b2)*g, g, v*b2);
 *   p = p + ((-step_size) * m) / (sqrt(v)/bc2_sqrt + eps)
 * step_consts_dev (16-byte aligned) holds 4 floats per 0-based step index s:
 * {step_size, bc2_sqrt, RN(1/bc2_sqrt), step_size*bc2_sqrt*(1+2^-20) rounded up},
 * precomputed on the host in double
 * like torch does; step s = step_idx_dev[0] is a device counter (advanced by
 * mirec_step_finish) so that a captured graph replays successive steps.
 * ------------------------------------------------------------------------- */
int mirec_adam_sparse_grad_f32(float* p, float* m, float* v, int64_t n_rows, int32_t d,
                               const float* rows, const int32_t* perm,
                               const int32_t* uniq, const int32_t* seg,
                               const int32_t* n_uniq_dev, int64_t n_max_uniq,
                               const float* dense_grad,
                               const float* step_consts_dev, const int32_t* step_idx_dev,
                               double beta1, double beta2, double eps, double weight_decay,
                               void* stream);

/* Flat form for parameters of any size (biases, [n,1] tables, MLP weights):
 * n elements, dense gradient, the same per-element arithmetic as above. */
int mirec_adam_flat_f32(float* p, float* m, float* v, int64_t n, const float* grad,
                        const float* step_consts_dev, const int32_t* step_idx_dev,
                        double beta1, double beta2, double eps, double weight_decay,
                        void* stream);
/* Up to 16 flat parameters with dense gradients in one launch (the same per-element
 * step as mirec_adam_flat_f32 / the streamed K5: bit-identical results). */
typedef struct mirec_flat_param {
  float* p;
  float* m;
  float* v;
  const float* g;
  int64_t n;
} mirec_flat_param;
int mirec_adam_flat_multi_f32(const mirec_flat_param* params, int32_t n_params,
                              const float* step_consts_dev, const int32_t* step_idx_dev,
                              double beta1, double beta2, double eps, double weight_decay,
                              void* stream);
/* The same with step_idx_dev = step_counter_dev, which the launch then advances by one
 * after every block has read it (graph mode's device step; ticket_dev: one int32, zero
 * before the first call, left zero) — the optimizer step's last launch, no separate
 * increment. */
int mirec_adam_flat_multi_advance_f32(const mirec_flat_param* params, int32_t n_params,
                                      const float* step_consts_dev, int32_t* step_counter_dev,
                                      int32_t* ticket_dev, double beta1, double beta2,
                                      double eps, double weight_decay, void* stream);

/* Several tables in ONE launch (e.g. the user and the item embedding of BPR),
 * same arithmetic per table. `tables` is a HOST array of n_tables <= 4
 * descriptors; every pointer inside is a device pointer. */
typedef struct mirec_adam_table {
  float* p;
  float* m;
  float* v;
  int64_t n_rows;
  const float* rows;        /* grouped gradient rows (or NULL)             */
  const int32_t* perm;      /* K2 grouping of `rows` by table row          */
  const int32_t* uniq;
  const int32_t* seg;
  const int32_t* n_uniq;    /* device counter; NULL = no grouped gradient  */
  const float* dense_grad;  /* optional dense gradient [n_rows, d] or NULL */
  int32_t* last;            /* deferred schedule: steps applied per row    */
  const int32_t* ahead_uniq;   /* deferred: rows the next batch reads, sorted */
  const int32_t* ahead_n_uniq; /* device count of ahead_uniq (NULL = none)    */
  float* p_alt;             /* deferred / flush: parity buffer of p (or NULL): the
                               state after t applied steps lives in t & 1 ? p_alt : p
                               (mirec_bpr_adam_step_f32); the flush also completes p */
} mirec_adam_table;

/* Streamed schedule: every row of every table, step index
 * s = step_base_dev[0] + step_off (consts at 2s, 2s+1). `last` is ignored. */
int mirec_adam_multi_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                         const float* step_consts_dev, const int32_t* step_base_dev,
                         int32_t step_off, double beta1, double beta2, double eps,
                         double weight_decay, void* stream);

/* Deferred schedule — bit-identical to the streamed one. Only the rows in each
 * table's `uniq` are touched at step s = step_base_dev[0] + step_off: row r
 * first replays steps last[r]..s-1 with a zero gradient (exactly the updates
 * the streamed kernel would have applied), then applies step s with its
 * gradient; last[r] = s + 1. Look-ahead: rows in ahead_uniq (the rows the
 * next batch's forward pass reads) and not in uniq replay steps last[r]..s with
 * a zero gradient; last[r] = s + 1 — so the next forward reads complete rows.
 * A row with last[r] > s (already complete through s) is left unchanged.
 * n_max_uniq[q] (host array) bounds table q's n_uniq and ahead count (grid
 * size). dense_grad must be NULL. Rows never touched lag until
 * mirec_adam_flush_f32.
 * last[r] == MIREC_ADAM_ZERO_STATE marks a row whose m and v are all +0 (the
 * caller sets it, only with weight_decay == 0): every zero-gradient step is then
 * the identity on p, m and v, bit for bit, so the row is current at any step —
 * look-ahead and flush leave it untouched; its first gradient step applies
 * directly (no replay) and ends the mark (last[r] = s + 1). */
#define MIREC_ADAM_ZERO_STATE 0x7fffffff
int mirec_adam_deferred_f32(const mirec_adam_table* tables, int32_t n_tables,
                            const int64_t* n_max_uniq, int32_t d,
                            const float* step_consts_dev, const int32_t* step_base_dev,
                            int32_t step_off, double beta1, double beta2, double eps,
                            double weight_decay, void* stream);
/* The deferred schedule (same semantics, same results) for a PAIR of tables in one
 * launch: tables[0] of width d (4..256) and tables[1] of width 1 — DeepFM's token
 * embeddings and first-order weights, which share the rows, the grouping and the step
 * (replaces FusedAdam's two mirec_adam_deferred_f32 launches, at the forward's catch-up
 * and at the step; reference: the optim.Adam.step of trainer.py:173 over both tables of
 * deepfm.py / layers.py FMEmbedding + FMFirstOrderLinear). n_max_uniq: HOST array of 2. */
int mirec_adam_deferred_pair_f32(const mirec_adam_table* tables, const int64_t* n_max_uniq,
                                 int32_t d, const float* step_consts_dev,
                                 const int32_t* step_base_dev, int32_t step_off, double beta1,
                                 double beta2, double eps, double weight_decay, void* stream);

/* Flush of the deferred schedule: every row r of every table with
 * last[r] < t = step_base_dev[0] + step_off replays steps last[r]..t-1 with a
 * zero gradient; last[r] = t. After it, p, m, v equal the streamed result.
 * With p_alt (parity buffers, d >= 64): rows are read from their state's buffer and
 * written to t & 1 ? p_alt : p and to p; rows already current at an odd t are copied
 * p_alt -> p — afterwards p holds every row (the parameter tensor is complete). */
int mirec_adam_flush_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                         const float* step_consts_dev, const int32_t* step_base_dev,
                         int32_t step_off, double beta1, double beta2, double eps,
                         double weight_decay, void* stream);
/* The same flush (same results) for tables whose rows mostly need nothing (the zero
 * state, or current): each wave owns rows_per_wave[q] (1..64, HOST array per table)
 * consecutive rows of table q and completes those that lag one after another, so the
 * grid has rows / (4 * R) workgroups instead of one per row (the workgroup dispatcher,
 * not the replay, bounds a one-per-row flush of a mostly idle table). d >= 64. */
int mirec_adam_flush_rows_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                              const int32_t* rows_per_wave, const float* step_consts_dev,
                              const int32_t* step_base_dev, int32_t step_off, double beta1,
                              double beta2, double eps, double weight_decay, void* stream);
/* K35 — one training step of the fused BPR path in ONE launch: BPR forward + backward
 * (mirec_bpr_fwd_bwd_f32's arithmetic) and the deferred Adam step
 * (mirec_adam_deferred_f32's arithmetic) of every touched row, and the look-ahead
 * replays — results bit-identical to those two launches. Replaces, as one kernel,
 * BPR.calculate_loss + BPRLoss + the embedding backward + optim.Adam.step (bpr.py:74-83,
 * loss.py:43-49, trainer.py:157-174). tables[0] = users (grouping of the batch's user
 * keys, contribution k = positive k), tables[1] = items (grouping of its (1+T)*Bc item
 * keys, the pairwise slots: positive k at k, negative j of k at Bc + j*Bc + k); each
 * table needs p and p_alt (parity buffers: the state after t steps lives in
 * t & 1 ? p_alt : p), m, v, last, n_uniq and optionally the look-ahead list (n_max_uniq:
 * bounds of both, the grid is sized by them); `rows` and
 * `dense_grad` are unused / NULL. The touched rows come as the records of
 * mirec_step_records (u_rec / i_rec: the batch's record region; u_crec / i_crec: one per
 * grouped position) of this batch. Rows with more than 2 contributions are split: their
 * contributions are formed by several blocks of the launch, which hand the vectors over
 * through u_part / i_part (scratch, Bc / (1+T)*Bc positions x d floats) and count in on
 * u_join / i_join (2*Bc / 2*(1+T)*Bc int32; the first half counts the arrivals per row
 * slot, the second is spare: all ZERO before the first launch, every launch leaves them
 * zero). The sums keep
 * the grouping order, so split rows give the same bits.
 * The step s = step_base_dev[0] + step_off reads every
 * row from buffer s & 1 (all rows the batch reads must be complete through s - 1) and
 * writes touched + look-ahead rows at state s + 1 to buffer (s + 1) & 1; zero-state rows
 * must hold the same p in both buffers. loss_k[k] = sum_j -log(gamma + sigmoid(x_kj)).
 * items = the batch's item keys (read only for negatives past the 4th). d in
 * {64, 128, 256}; T >= 1. */
int mirec_bpr_adam_step_f32(const mirec_adam_table* tables, const int64_t* n_max_uniq,
                            int32_t d, const int64_t* items, int64_t Bc, int32_t T, float gamma,
                            float grad_scale, float* loss_k, const int32_t* u_rec,
                            const int32_t* u_crec, const int32_t* i_rec, const int32_t* i_crec,
                            float* u_part, int32_t* u_join, float* i_part, int32_t* i_join,
                            const float* step_consts_dev, const int32_t* step_base_dev,
                            int32_t step_off, double beta1, double beta2, double eps,
                            double weight_decay, void* stream);
/* The K35 records of n_batches consecutive batches (strides per batch: Bc user keys,
 * (1+T)*Bc item keys; the groupings of mirec_segment_sort_batched / the chunk
 * preparation). Contribution record (8 int32) per grouped position i: positive k,
 * negative slot j (-1 for a user slot or a positive slot), user id, positive item id,
 * the first 4 negatives' ids (ids clamped to the table as K3 clamps them). Record
 * region per batch and table (mirec_step_record_ints(per) int32, per = Bc or
 * (1+T)*Bc): per row records (20 int32: row id, first position, contribution count,
 * share count, the records of its first two contributions), then 256 share records of
 * split rows (24 int32: row slot, share, first position, count, row id, share count,
 * 0, 0, the share's two contribution records), then the number of share records.
 * u_crec / i_crec: per batch Bc / (1+T)*Bc positions x 8 int32. u_ahead .. i_nah
 * (all four or none): the look-ahead lists of mirec_uniq_ahead_diff, formed in the same
 * launch (one launch of three block roles after the groupings). */
int mirec_step_records(const int64_t* user_keys, const int64_t* item_keys, int64_t n_batches,
                       int64_t Bc, int32_t T, int64_t n_users, int64_t n_items,
                       const int32_t* u_perm, const int32_t* u_uniq, const int32_t* u_seg,
                       const int32_t* u_nu, const int32_t* i_perm, const int32_t* i_uniq,
                       const int32_t* i_seg, const int32_t* i_nu, int32_t* u_rec,
                       int32_t* u_crec, int32_t* i_rec, int32_t* i_crec, int32_t* u_ahead,
                       int32_t* u_nah, int32_t* i_ahead, int32_t* i_nah, void* stream);
/* int32 per batch of one table's record region for per keys per batch (-1 if per < 0). */
int64_t mirec_step_record_ints(int64_t per);

int mirec_copy_many(const void* const* src, void* const* dst, const int64_t* bytes, int n,
                    void* stream);

/* Copy n_bytes (a multiple of 4, at most a few KiB: e.g. the mirec_ctx_field
 * descriptors of a batch) from host memory to dst_dev through kernel arguments:
 * stream-ordered, and recorded BY VALUE when the stream is being captured into a
 * graph (a host-to-device memcpy node would re-read the host buffer at replay). */
int mirec_write_bytes(void* dst_dev, const void* src_host, size_t n_bytes, void* stream);

/* Self-test of the K5 replay's fast correctly rounded sqrt and division
 * (csrc/adam_math.h) against sqrtf / IEEE division, bitwise, on this GPU:
 * every sqrt_stride-th float of [2^-96, FLT_MAX] plus the floats near each power
 * of two, and n_div pseudo-random pairs of the fast division range. out4_dev
 * (device) receives {sqrt mismatches, sqrt tested, div mismatches, div tested}.
 * (tools/check_adam_math.hip is the exhaustive / 2^34-pair version.) */
int mirec_selftest_adam_math(uint64_t sqrt_stride, uint64_t n_div, uint64_t seed,
                             unsigned long long* out4_dev, void* stream);

/* End-of-step bookkeeping of Trainer._train_epoch (trainer.py:161-169):
 * loss_hist[step] = (sum of loss_k[0..n), fixed order) / denom, then
 * step_idx_dev[0] += 1.  Keeps the per-batch `losses.item()` on the device
 * (read once per epoch) instead of a host sync per batch. */
int mirec_step_finish(const float* loss_k, int64_t n, float denom, float* loss_hist,
                      int32_t* step_idx_dev, void* stream);

/* The same for n_steps consecutive steps whose losses sit at
 * loss_k[c*stride .. c*stride+n): loss_hist[step_base + c] (same reduction
 * order as mirec_step_finish), then step_base_dev[0] += n_steps. One workgroup
 * per step; ticket_dev is one device int32, zero before the call and zero
 * again after it (it orders the last workgroup's counter update after every
 * workgroup has read the counter). */
int mirec_chunk_finish(const float* loss_k, int64_t n, int64_t stride, int32_t n_steps,
                       float denom, float* loss_hist, int32_t* step_base_dev,
                       int32_t* ticket_dev, void* stream);

/* ---------------------------------------------------------------------------
 * K6  Full-sort scorer + mask + top-K + positive flags, fused (no [n,I] matrix).
 * Replaces BPR.full_sort_predict (bpr.py:91-96) + Trainer._full_sort_batch_eval
 *   (trainer.py:328-353: pad column and history set to -inf, positives swapped
 *   to the front) + TopKEvaluator.collect (evaluators.py:53-76: flip + topk) +
 *   the pos_idx test of TopKEvaluator._calculate_metrics (:134).
 * For query q with user vector Uq[q,:]: score(i) = <Uq[q], EI[i]> for
 *   i in [1, I) not in hist[q]; top_ids[q, 0..K) = the K best items ordered by
 *   (score desc, item asc); pos_flags[q, r] = top_ids[q, r] in pos[q].
 *   Slots beyond the number of unmasked items get id -1, score -inf, flag 0.
 * hist/pos: CSR over queries, column ids sorted ascending per query.
 * FP32 MFMA (v_mfma_f32_32x32x2_f32), exact f32 products.
 * d in {32, 64, 128, 256};  1 <= K <= 50.
 * ------------------------------------------------------------------------- */
int mirec_fullsort_topk_f32(const float* Uq, int64_t nq, const float* EI, int64_t I,
                            int32_t d, const int64_t* hist_ptr, const int32_t* hist_cols,
                            const int64_t* pos_ptr, const int32_t* pos_cols, int32_t K,
                            float* top_scores, int32_t* top_ids, uint8_t* pos_flags,
                            void* stream);

/* mirec_fullsort_topk_f32 with the item range split over n_split workgroups per user
 * block (partial top-K lists in the workspace, then a per-user merge by (score desc,
 * id asc) — the same total order, so the same outputs). For launches too small to
 * fill the chip (the last user block of an evaluation). Same reference code as
 * mirec_fullsort_topk_f32. */
size_t mirec_fullsort_topk_split_workspace_size(int64_t nq, int32_t K, int32_t n_split);
int mirec_fullsort_topk_split_f32(const float* Uq, int64_t nq, const float* EI, int64_t I,
                                  int32_t d, const int64_t* hist_ptr, const int32_t* hist_cols,
                                  const int64_t* pos_ptr, const int32_t* pos_cols, int32_t K,
                                  int32_t n_split, void* ws, size_t ws_bytes,
                                  float* top_scores, int32_t* top_ids, uint8_t* pos_flags,
                                  void* stream);

/* Plain score matrix S[q, i] = <Uq[q], EI[i]> (FP32 MFMA) for the
 * full_sort_predict API contract (flat [nq*I] scores, bpr.py:91-96). */
int mirec_score_matrix_f32(const float* Uq, int64_t nq, const float* EI, int64_t I,
                           int32_t d, float* S, void* stream);

/* ---------------------------------------------------------------------------
 * K7  Graph propagation (LightGCN): CSR SpMM with a fused epilogue.
 * Replaces torch.sparse.mm(norm_adj_matrix, E) in LightGCN.forward
 *   (recbole/model/general_recommender/lightgcn.py:118-124), the layer mean
 *   (:125-126) and their autograd backward (A_hat is symmetric, so the same CSR
 *   propagates gradients).
 * A "rows reference" names a [n_rows, d] fp32 matrix stored as two blocks:
 *   row r at lo + r*d for r < split, else hi + (r - split)*d (hi NULL = lo);
 *   lo NULL = operand absent. This maps the ego matrix cat(E_U, E_I) (:107-113)
 *   onto the two parameter tensors without a copy.
 * Per row r (nonzeros in ascending CSR order):
 *   y = sum_j vals[j] * X[cols[j]];  if add: y += add_scale * ADD[r];
 *   if y: Y[r] = y;  if acc_out: ACC_OUT[r] = (ACC_IN[r] (0 if absent) + y) * acc_scale.
 * Load balance: the host plan (recbole_amd/ops.py `SpmmPlan`) cuts row r into
 *   min(ceil(deg/piece), 1024) units of near-equal length (at least one);
 *   unit u covers nonzeros [unit_beg[u], unit_beg[u+1]) of row unit_row[u]
 *   (unit_beg has n_units+1 entries, the last = nnz; piece = the base unit length,
 *   informational); unit_slot[u] = -1 when it is the row's only unit, else the
 *   row of `partial` [n_slots, d] it writes; fix_row[f] / fix_ptr[f..f+1] list the
 *   split rows and their slots, summed in slot order (deterministic).
 * d in {32, 64, 128, 256}; Y / ACC_OUT must not alias X.
 * ------------------------------------------------------------------------- */
typedef struct mirec_rows_ref {
  float* lo;
  float* hi;
  int64_t split;
} mirec_rows_ref;

typedef struct mirec_spmm_epilogue {
  mirec_rows_ref add;
  float add_scale;
  mirec_rows_ref y;
  mirec_rows_ref acc_in;
  mirec_rows_ref acc_out;
  float acc_scale;
} mirec_spmm_epilogue;

int mirec_spmm_csr_f32(const int64_t* row_ptr, const int32_t* cols, const float* vals,
                       int64_t n_rows, int32_t d, const int32_t* unit_row,
                       const int64_t* unit_beg, const int32_t* unit_slot, int64_t n_units,
                       int32_t piece, const int32_t* fix_row, const int32_t* fix_ptr,
                       int64_t n_fix, float* partial, const mirec_rows_ref* x,
                       const mirec_spmm_epilogue* ep, void* stream);

/* EmbLoss helpers (recbole/model/loss.py:79-84, used by LightGCN.calculate_loss
 * lightgcn.py:148-152): sq[i] = sum_k table[idx[i],k]^2 (fixed order);
 * out[i,:] = scale_dev[0] * table[idx[i],:] (the norm's gradient rows). */
int mirec_gather_sqnorm_f32(const float* table, int64_t n_rows, int32_t d, const int64_t* idx,
                            int64_t n, float* sq, void* stream);
int mirec_gather_scale_rows_f32(const float* table, int64_t n_rows, int32_t d,
                                const int64_t* idx, int64_t n, const float* scale_dev,
                                float* out, void* stream);

/* ---------------------------------------------------------------------------
 * K8  Context-aware fields + factorization machine (DeepFM's embedding side).
 * Replaces ContextRecommender.embed_input_fields / concat_embed_input_fields
 *   (recbole/model/abstract_recommender.py:199-412), FMEmbedding
 *   (model/layers.py:121-144), BaseFactorizationMachine (:147-171),
 *   FMFirstOrderLinear (:905-1062) and DeepFM's y_fm (context_aware_recommender/
 *   deepfm.py:58-70), with their autograd backward.
 * fields_dev: DEVICE array of n_fields descriptors in concat order
 *   (token fields, then token_seq fields, then float fields):
 *   kind 0 token:     row = ids[b] + offset of the shared token table;
 *   kind 1 token_seq: ids [B, seq_len] into the field's own table, masked mean
 *                     sum(e * (id != 0)) / (count + 1e-8);
 *   kind 2 float:     e = table[offset] * vals[b].
 *   table1 is the matching first-order table (width 1, same rows).
 * Forward:  concat[b, f*d + k] = e_bfk;  keys[b] = token row (kind 0, if keys);
 *   y_fm[b] = (sum float w*x + sum token w + sum token_seq masked w) + bias[0]
 *             + 0.5 * sum_k ((sum_f e_bfk)^2 - sum_f e_bfk^2).
 * Backward (g_concat may be NULL): ge = g_concat + g_fm[b] * (S_bk - e_bfk);
 *   token: grad[b*grad_ld + k] = ge, grad1[b*grad1_ld] = g_fm[b];
 *   token_seq: grad[(b*L + t)*d + k] = mask * ge / (count + 1e-8), grad1[b*L+t] = mask*g_fm[b];
 *   float: grad[b*grad_ld + k] = ge * x_b, grad1[b*grad1_ld] = g_fm[b] * x_b
 *          (column-sum them over b).
 * 1 <= d <= 64. work: mirec_ctx_fm_work_floats(B, n_fields, d) floats written by the
 * forward (per-field first-order terms, then S_bk) and read by the backward of the same
 * batch. The forward is two launches (a gather over every (sample, field) pair, then
 * the per-sample sums in field order), the backward one over every (sample, field).
 * ------------------------------------------------------------------------- */
typedef struct mirec_ctx_field {
  int32_t kind;
  int32_t seq_len;
  const int64_t* ids;
  const float* vals;
  int64_t offset;
  const float* table;
  const float* table1;
  int64_t n_rows;
  float* grad;
  float* grad1;
  int64_t* keys;
  int64_t grad_ld;   /* row stride (floats) of grad for kinds 0 and 2 */
  int64_t grad1_ld;  /* stride of grad1 for kinds 0 and 2 */
} mirec_ctx_field;

size_t mirec_ctx_fm_work_floats(int64_t B, int32_t n_fields, int32_t d);
int mirec_ctx_fm_fwd_f32(const mirec_ctx_field* fields_dev, int32_t n_fields, int64_t B,
                         int32_t d, const float* bias, float* concat, float* y_fm, float* work,
                         void* stream);
int mirec_ctx_fm_bwd_f32(const mirec_ctx_field* fields_dev, int32_t n_fields, int64_t B,
                         int32_t d, const float* concat, const float* g_concat,
                         const float* g_fm, const float* work, void* stream);

/* sigmoid + nn.BCELoss (DeepFM.forward / calculate_loss, deepfm.py:66-73):
 * z = y_fm + y_deep (y_deep may be NULL); prob = sigmoid(z);
 * loss[b] = (t-1)*max(log(1-p),-100) - t*max(log p,-100)  (mean = sum/B);
 * dz[b] = grad_scale*(p-t)/max((1-p)p, 1e-12) * (1-p)*p. Any output may be NULL;
 * label may be NULL when only prob is requested. */
int mirec_sigmoid_bce_f32(const float* y_fm, const float* y_deep, const float* label, int64_t B,
                          float grad_scale, float* prob, float* loss, float* dz, void* stream);
/* The training loss of DeepFM in one launch: dz as mirec_sigmoid_bce_f32, loss_b
 * (nullable) the per-sample terms, loss_mean[0] = their fixed-order sum (mirec_sum_f32's
 * order) / B — nn.BCELoss's mean (reference deepfm.py:66-73). 0 < B <= 2^24. */
int mirec_sigmoid_bce_mean_f32(const float* y_fm, const float* y_deep, const float* label,
                               int64_t B, float grad_scale, float* loss_b, float* loss_mean,
                               float* dz, void* stream);

/* out[j] = sum_{i<n} x[i*m + j] in row order (fixed; float-field / bias grads). */
int mirec_colsum_f32(const float* x, int64_t n, int64_t m, float* out, void* stream);
/* The tail of nn.Linear's backward over a tall input (reference: torch's Linear backward
 * under SASRec's layers, layers.py:338-461): dW = sum_c P[c] (C split-K partials of n_w
 * floats, summed in c order; skipped when C == 1 and P == dW) and db = the column sum of
 * g [K, n_out] (NULL: none; rows in chunks of 2048, each in row order, chunks in order) in
 * ONE launch. n_w and n_out multiples of 4, 16-B aligned P / dW / g. scratch: floats of
 * mirec_linear_grad_finish_scratch(K, n_out); ticket: one int32, zero before a call and
 * left zero. */
int64_t mirec_linear_grad_finish_scratch(int64_t K, int32_t n_out);
int mirec_linear_grad_finish_f32(const float* P, int32_t C, int64_t n_w, float* dW,
                                 const float* g, int64_t K, int32_t n_out, float* db,
                                 float* scratch, int32_t* ticket, void* stream);
/* Several column sums in ONE launch (up to 4 jobs: out[q][j] = sum_i x[q][i*m[q] + j],
 * x[q] of n[q] rows): each job summed exactly as mirec_colsum_f32 sums it (same tile, same
 * order), the three of a DeepFM backward (float fields, their first-order terms, the bias)
 * in one launch. HOST arrays of device pointers and sizes. */
int mirec_colsum_multi_f32(const float* const* x, const int64_t* n, const int64_t* m,
                           float* const* out, int32_t n_jobs, void* stream);
/* keys[f*B + i] = cols[f][i] + offsets[f] for n_fields <= 64 int64 id columns (HOST array of
 * device pointers; HOST offsets): DeepFM's token keys in the shared table, one launch. */
int mirec_offset_keys(const int64_t* const* cols, const int64_t* offsets, int32_t n_fields,
                      int64_t B, int64_t* out, void* stream);

/* ---------------------------------------------------------------------------
 * K10  DeepFM's deep part (recbole/model/layers.py:30-86 MLPLayers: Dropout -> Linear
 * -> ReLU per hidden layer; deepfm.py:40-43,61 deep_predict_layer) on fp32 MFMA:
 * one forward launch and two backward launches (data gradient through every layer,
 * then every dW / db tile; fixed summation orders). Layer l maps dims[l] -> dims[l+1]
 * with W[l] the nn.Linear weight [dims[l+1], dims[l]] (16-B aligned) and b[l] its
 * bias (or NULL); dropout[l]: Dropout(p) before layer l; relu[l]: ReLU after it (every
 * hidden layer must have it). Widths <= 1024, multiples of 4 except dims[n_layers].
 * Dropout (training): element e of layer l's input is kept iff
 *   splitmix64(splitmix64(seed + counter[0]) ^ (e*8 + l)) >> 32 < keep_threshold
 * and scaled by `scale`; the forward advances counter[0] by one (last block; `arrive`
 * is zero-initialised device scratch). Saved for the backward: xs[l] = layer l's input
 * after its dropout [B, dims[l]] (xs[0] may be NULL when layer 0 has no dropout: the
 * backward then reads x), mask0 = layer 0's keep flags [B, dims[0]] (dropout[0] only).
 * Backward: dy = d loss / d y [B, dims[n_layers]]; gz[l] [B, dims[l+1]] scratch for
 * l < n_layers - 1; writes gx [B, dims[0]], dW[l], db[l] (when non-NULL).
 * ------------------------------------------------------------------------- */
#define MIREC_MLP_MAX_LAYERS 6
typedef struct mirec_mlp {
  int32_t n_layers;
  int32_t dims[MIREC_MLP_MAX_LAYERS + 1];
  int32_t dropout[MIREC_MLP_MAX_LAYERS];
  int32_t relu[MIREC_MLP_MAX_LAYERS];
  int32_t tile_start[MIREC_MLP_MAX_LAYERS];   /* set by mirec_mlp_bwd_f32 */
  uint32_t keep_threshold;
  float scale;
  uint64_t seed;
  int64_t* counter;
  int32_t* arrive;
  const float* W[MIREC_MLP_MAX_LAYERS];
  const float* b[MIREC_MLP_MAX_LAYERS];
  float* xs[MIREC_MLP_MAX_LAYERS];
  uint8_t* mask0;
  float* gz[MIREC_MLP_MAX_LAYERS];
  float* dW[MIREC_MLP_MAX_LAYERS];
  float* db[MIREC_MLP_MAX_LAYERS];
  /* the wide backward's scratch (mirec_mlp_bwd_workspace: floats, and int32 counters that
   * must be zero before a call and are left zero); NULL: the row-block backward */
  float* wscratch;
  int32_t* wcount;
} mirec_mlp;

int mirec_mlp_fwd_f32(const mirec_mlp* mlp, const float* x, int64_t B, float* y, int32_t train,
                      void* stream);
int mirec_mlp_bwd_f32(const mirec_mlp* mlp, const float* x, const float* dy, int64_t B, float* gx,
                      void* stream);
/* Wide layer 0 (dims[0] >= 256, >= 2 layers): the forward runs layer 0 over the whole chip
 * (16 rows x 32 columns per 4-wave block, K split in two halves added in a fixed order)
 * when xs[1] is given, then layers 1.. in row blocks; the backward (with wscratch /
 * wcount) runs layers L-1..1 in row blocks, then layer 0's data gradient and every weight
 * gradient as 64-column wave tiles over the whole chip (the batch in 4 x 4 slices summed
 * in a fixed order). Returns 1 and the scratch sizes when the shapes take the wide
 * backward, 0 otherwise, < 0 on bad arguments. */
int mirec_mlp_bwd_workspace(const mirec_mlp* mlp, int64_t B, int64_t* scratch_floats,
                            int64_t* counters);

/* ---------------------------------------------------------------------------
 * K9  Sequential recommender (SASRec) embedding block and sampled softmax.
 * seq_embed_ln replaces the input block of SASRec.forward
 *   (recbole/model/sequential_recommender/sasrec.py:107-117):
 *   out[r] = LayerNorm(item_table[item_seq[r]] + pos_table[r % L]) (gamma, beta, eps),
 *   r = b*L + t over [B, L]; mean / rstd [B*L] saved for the backward.
 * Backward: dx[r] = LayerNorm input gradient (may be NULL); ditem[r] = dx[r], or 0
 *   where item_seq[r] == 0 (nn.Embedding(padding_idx=0)); part_gamma / part_beta
 *   [mirec_seq_embed_ln_partials(B*L), d] per-block partial sums of g*xhat and g,
 *   to be finished by mirec_colsum_f32 (fixed order). d in {32,64,128,256}.
 * sampled_softmax (the C3 configuration's loss, a build extension; pinned by the
 *   oracle's torch restatement): per sequence b, logits over [pos[b],
 *   neg[j*B + b] for j < n_neg] (the sampler's layout), loss[b] =
 *   logsumexp - logit_0, g_seq[b] = grad_scale * (sum_j p_j E_j - E_0),
 *   g_items rows [(1+n_neg)*B, d]: row b = grad_scale*(p_0 - 1)*s_b,
 *   row j*B + b = grad_scale*p_j*s_b. d in {64,128,256}, n_neg <= 4095.
 * ------------------------------------------------------------------------- */
int mirec_seq_embed_ln_fwd_f32(const float* item_table, int64_t n_items, const float* pos_table,
                               const int64_t* item_seq, int64_t B, int32_t L, int32_t d,
                               const float* gamma, const float* beta, float eps, float* out,
                               float* mean, float* rstd, void* stream);
int64_t mirec_seq_embed_ln_partials(int64_t n_rows);
int mirec_seq_embed_ln_bwd_f32(const float* item_table, int64_t n_items, const float* pos_table,
                               const int64_t* item_seq, int64_t B, int32_t L, int32_t d,
                               const float* gamma, const float* mean, const float* rstd,
                               const float* grad_out, float* dx, float* ditem,
                               float* part_gamma, float* part_beta, void* stream);
/* K9a with SASRec's embedding dropout after the LayerNorm (sasrec.py:107-114) folded in:
 * out = drop_p(LayerNorm(...)); the backward masks grad_out with the same flags. Draws as
 * mirec_add_ln_drop_fwd_f32 (the forward records the counter value in drawn[0], the backward
 * redraws from it and sets counter = drawn[0] + 1). */
int mirec_seq_embed_ln_drop_fwd_f32(const float* item_table, int64_t n_items,
                                    const float* pos_table, const int64_t* item_seq, int64_t B,
                                    int32_t L, int32_t d, const float* gamma, const float* beta,
                                    float eps, float p, uint64_t seed, int64_t* counter,
                                    int64_t* drawn, float* out, float* mean, float* rstd,
                                    void* stream);
int mirec_seq_embed_ln_drop_bwd_f32(const float* item_table, int64_t n_items,
                                    const float* pos_table, const int64_t* item_seq, int64_t B,
                                    int32_t L, int32_t d, const float* gamma, const float* mean,
                                    const float* rstd, const float* grad_out, float p,
                                    uint64_t seed, int64_t* drawn, int64_t* counter, float* dx,
                                    float* ditem, float* part_gamma, float* part_beta,
                                    void* stream);
/* K9d  LayerNorm(a + b) of the transformer blocks' residual connections (layers.py
 * MultiHeadAttention / FeedForward, reference layers.py:338-552) in one pass, and its
 * backward (dx = d(a + b), per-block dgamma / dbeta partials as K9a, summed with
 * mirec_colsum_f32). a, b, out, grad_out, dx: [n, d] rows; d in {32,64,128,256}. */
int mirec_add_ln_fwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                         const float* gamma, const float* beta, float eps, float* out,
                         float* mean, float* rstd, void* stream);
/* K11  nn.Linear over tall inputs on fp32 MFMA (SASRec's transformer Linears, reference
 * layers.py:338-461: B x L rows of width 64..256): y[M, N] = x[M, K] w[N, K]^T (+ bias[N])
 * and the data gradient gx[M, n_in] = gy[M, n_out] w[n_out, n_in] (accumulate != 0: added
 * to what gx holds — the sum of several Linears' input gradients). Row-major, x / gy / w
 * 16-byte aligned; widths with mirec_linear_shape_ok(K, N) != 0 ({64,128,256}^2 except
 * 256 x 256: the weight stays in one workgroup's LDS). */
int mirec_linear_shape_ok(int32_t K, int32_t N);
int mirec_linear_fwd_f32(const float* x, int64_t M, int32_t K, int32_t N, const float* w,
                         const float* bias, float* y, void* stream);
int mirec_linear_bwd_data_f32(const float* gy, int64_t M, int32_t n_out, int32_t n_in,
                              const float* w, float* gx, int32_t accumulate, void* stream);
/* gx = acc + gy W (the residual gradient of a block's input plus the Linear's data
 * gradient, one pass; acc may equal gx). Replaces autograd's add of the two input
 * gradients where x feeds both a Linear and a residual (reference layers.py:338-461). */
int mirec_linear_bwd_data_acc_f32(const float* gy, int64_t M, int32_t n_out, int32_t n_in,
                                  const float* w, const float* acc, float* gx, void* stream);
/* K9e  The attention core of MultiHeadAttention (reference layers.py:338-407, the lines
 * scores = q k^T / sqrt(dh); + attention_mask; softmax; attn_dropout; @ v), L <= 64 and
 * dh = 64, one workgroup per (sequence, head), fp32 MFMA. q, k, v, out / dout, dq, dk, dv:
 * [B, L, H*64] row-major (the Linear outputs before transpose_for_scores; the context is
 * written back in the same layout, i.e. after the reference's permute + view); mask:
 * [B, L, L] additive (SASRec's [B, 1, L, L] extended mask); lse: [B*H, 64] floats (the
 * forward writes each query row's log-sum-exp, the backward reads it). Dropout p > 0:
 * counter-based draws (csrc/attn.hip header: seed, the device int64 counter — read by the
 * forward, advanced by one by the backward when it gets the counter; a forward without a
 * backward leaves the advance to the caller), the keep bits written to keep_words [B*H, 64]
 * uint64 and read back by the backward.
 * Replaces torch's fused scaled_dot_product_attention and the context permute copy. */
int mirec_attn_fwd_f32(const float* q, const float* k, const float* v, const float* mask,
                       int64_t B, int32_t L, int32_t H, float dropout_p, uint64_t seed,
                       int64_t* counter, float* out, float* lse, uint64_t* keep_words,
                       void* stream);
int mirec_attn_bwd_f32(const float* q, const float* k, const float* v, const float* mask,
                       const float* dout, const float* lse, const uint64_t* keep_words,
                       int64_t* counter, int64_t B, int32_t L, int32_t H, float dropout_p,
                       float* dq, float* dk, float* dv, void* stream);
/* SASRec.get_attention_mask (sasrec.py:91-105) in one launch: mask [B, 1, L, L] float =
 * (1 - [item_seq[b][j] > 0] * [j <= i]) * -10000, the reference's values bit for bit (-0.0
 * where attention is allowed). item_seq: [B, L] int64. */
int mirec_seq_attn_mask_f32(const int64_t* item_seq, int64_t B, int32_t L, float* mask,
                            void* stream);
/* GELU (erf form) of the feed-forward block, forward and backward, elementwise. */
int mirec_gelu_fwd_f32(const float* x, int64_t n, float* y, void* stream);
int mirec_gelu_bwd_f32(const float* x, const float* g, int64_t n, float* dx, void* stream);
int mirec_add_ln_bwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                         const float* gamma, const float* mean, const float* rstd,
                         const float* grad_out, float* dx, float* part_gamma, float* part_beta,
                         void* stream);
/* K9d with the hidden dropout folded in (layers.py:338-461: LayerNorm(dropout(hidden) +
 * input_tensor), the MultiHeadAttention out_dropout / FeedForward dropout): y =
 * LayerNorm(drop_p(a) + b). Counter-based draws (csrc/seq.hip K9d header): the forward reads
 * the device int64 `counter` and writes the value it used to drawn[0]; the backward redraws
 * the same keep flags from drawn[0], sets counter = drawn[0] + 1 (a forward without a
 * backward leaves the advance to the caller) and writes dx_a = dLN * keep / (1 - p) (the
 * gradient of `a`) and dx_b = dLN (of `b`). 0 < p < 1. */
int mirec_add_ln_drop_fwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                              const float* gamma, const float* beta, float eps, float p,
                              uint64_t seed, int64_t* counter, int64_t* drawn, float* out,
                              float* mean, float* rstd, void* stream);
int mirec_add_ln_drop_bwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                              const float* gamma, const float* mean, const float* rstd,
                              const float* grad_out, float p, uint64_t seed, int64_t* drawn,
                              int64_t* counter, float* dx_a, float* dx_b, float* part_gamma,
                              float* part_beta, void* stream);

/* K9c: sampled evaluation (uni-N) of a sequential model — rank[q] = number of the
 * m sampled items neg[q*m .. q*m+m) (row-major: the sampler's per-row walk order)
 * whose score <seq_out[q], E[i]> is greater than or equal to the positive's (exact
 * ties — sampled copies of the positive item — counted ahead of it; torch.topk
 * leaves their order unspecified). pos_idx[q, r] = (rank[q] == r) for r < K — Trainer.evaluate's
 * repeat / sample_collect / topk sequence (trainer.py:384-409, abstract_evaluator.py
 * :65-75) for one positive per query. d in {32,64,128,256}. */
int mirec_rank_of_pos_f32(const float* seq_out, const float* item_table, int64_t n_items,
                          int32_t d, const int64_t* pos, const int64_t* neg, int64_t n, int32_t m,
                          int32_t* rank, void* stream);
/* x *= g[0] in place (n % 4 == 0, 16-byte aligned x; a device scalar g), a no-op when
 * g[0] == 1: a loss Function's backward scaling its saved gradient rows by the incoming
 * gradient (reference: autograd's grad_output * saved). */
int mirec_scale_by_f32(float* x, int64_t n, const float* g, void* stream);
int mirec_sampled_softmax_f32(const float* seq_out, const float* item_table, int64_t n_items,
                              int32_t d, const int64_t* pos, const int64_t* neg, int64_t B,
                              int32_t n_neg, float grad_scale, float* loss, float* g_seq,
                              float* g_items, void* stream);

/* ---------------------------------------------------------------------------
 * Row-sharded tables over G ranks (replaces the single-process
 * nn.Embedding tables of bpr.py:40-41 + the dense optim.Adam state of
 * trainer.py:109-130 by G shards). Ownership: row id on rank id % G, local row
 * id / G; S = rows per shard. Global slots of a batch of Bc positives (the
 * pairwise layout, general_dataloader.py:235-241): user slot t = k, item slot
 * t = Bc + j*Bc + k; slot t belongs to slice g = k / B (rank g's positives).
 * Message (g, o) = the slots of slice g whose row rank o owns, ascending t; a
 * slot's place in it is idx(t) < cap (else status -4).
 * ------------------------------------------------------------------------- */
/* keys[i] = (ids[i] % G) * S + ids[i] / G: owner-major sort keys for K2. */
int mirec_shard_keys(const int64_t* ids, int64_t n, int32_t G, int64_t S, int64_t* keys,
                     void* stream);
/* Exchange plans of n_batches batches (users [nb, Bc], items [nb, (1+T)*Bc], original
 * ids) for rank `rank`:
 *   fwd_rows[nb, G*cap]  owner side: message (g, rank) entry idx = the slot's local
 *                        row (user shard: row >= 0; item shard: -(row+1)); padding 0
 *   map2[nb, Bc + (1+T)*Bc]  owner side: slot t of a row it owns -> g*cap + idx(t)
 *   pos[nb, (2+T)*B]     requester side (slice = rank): local slot ls (users k',
 *                        items n + j*n + k', n = this slice's positives) -> o*cap + idx
 *   bwd_src[nb, G*cap]   requester side: message (rank, o) entry idx -> local slot ls;
 *                        padding 0.
 *   status[2]            (accumulated, zero it first) [0] = -4 if any message of any
 *                        rank exceeded cap, [1] = max over launches of the largest
 *                        message (rows). Every rank counts every message, so all ranks
 *                        see the same status. An overflowing slot gets position 0 in
 *                        map2 / pos (in range, never read out of bounds); its batch must
 *                        be re-planned with cap >= status[1] before it runs. */
int mirec_shard_plan(const int64_t* users, const int64_t* items, int64_t n_batches, int64_t Bc,
                     int64_t B, int32_t T, int32_t G, int32_t rank, int64_t cap,
                     int64_t* fwd_rows, int32_t* map2, int64_t* pos, int32_t* bwd_src,
                     int32_t* status, void* stream);
/* Rank `rank`'s slice of the K2 grouping of each batch (uniq keyed by
 * mirec_shard_keys, sorted; per-batch strides per_batch / per_batch + 1): the key
 * range [rank*S, (rank+1)*S) -> own_uniq (local rows), own_seg (its segment
 * offsets, n+1 entries), own_n; perm2[p] = map2[map_off + perm[p]] for the
 * positions p of those segments (the contribution's place in the backward receive
 * buffer); the same range of the look-ahead list (ahead may be NULL). */
int mirec_shard_own(const int32_t* uniq, const int32_t* seg, const int32_t* n_uniq,
                    const int32_t* perm, int64_t per_batch, int64_t n_batches,
                    const int32_t* ahead, const int32_t* n_ahead, const int32_t* map2,
                    int64_t map_stride, int64_t map_off, int64_t S, int32_t rank,
                    int32_t* own_uniq, int32_t* own_seg, int32_t* own_n, int32_t* perm2,
                    int32_t* own_ahead, int32_t* own_nah, void* stream);
/* The owner-filtered grouping input (each rank sorts only the slots it owns, ~1/G of the
 * global batch): per batch (ids [n_batches, per]), the slots i with ids[i] % G == rank in
 * slot order, keyed rank*S + ids[i]/G (the mirec_shard_keys key) -> keys [n_batches,
 * cap_sel], their positions -> sel_pos; padded with the key (rank+1)*S. sel_most[0] =
 * max(sel_most[0], the largest owned count): over cap_sel, the batch was truncated and
 * must be re-selected with a larger cap_sel. Sort keys with mirec_segment_sort_batched
 * (stride cap_sel, key space G*S + 1), then mirec_shard_own_sel. */
int mirec_shard_select(const int64_t* ids, int64_t n_batches, int64_t per, int32_t G, int64_t S,
                       int32_t rank, int64_t cap_sel, int64_t* keys, int32_t* sel_pos,
                       int32_t* sel_most, void* stream);
/* mirec_shard_own on the owner-filtered grouping: input lists of stride cap_sel, a grouped
 * position p's slot is sel_pos[perm[p]]; outputs with the global lists' stride per. Same
 * owned lists and the same per-row contribution order as mirec_shard_own on the global
 * grouping (the compaction keeps slot order; the sort is stable). */
int mirec_shard_own_sel(const int32_t* uniq, const int32_t* seg, const int32_t* n_uniq,
                        const int32_t* perm, int64_t cap_sel, int64_t n_batches,
                        const int32_t* ahead, const int32_t* n_ahead, const int32_t* map2,
                        int64_t map_stride, int64_t map_off, int64_t S, int32_t rank,
                        const int32_t* sel_pos, int64_t per, int32_t* own_uniq, int32_t* own_seg,
                        int32_t* own_n, int32_t* perm2, int32_t* own_ahead, int32_t* own_nah,
                        void* stream);
/* Where each entry of step c's owned lists (mirec_shard_own: own / own_ahead) sits in
 * step c+1's owned list, for c < n_batches - 1: next_t[c*per_batch + i] = that index
 * (-1: step c+1 does not read the row), next_a[c*per_batch + a] likewise for the
 * look-ahead list — the push lists of mirec_comm_adam_deferred_f32. */
int mirec_shard_next(const int32_t* own, const int32_t* own_n, const int32_t* own_ahead,
                     const int32_t* own_nah, int64_t per_batch, int64_t n_batches,
                     int32_t* next_t, int32_t* next_a, void* stream);
/* out[i] = idx[i] >= 0 ? U[idx[i]] : I[-idx[i]-1] (rows of d floats; d in
 * {32,64,128,256}): an owner's forward message from its two shards. */
int mirec_shard_gather_f32(const float* U, const float* I, int32_t d, const int64_t* idx,
                           int64_t n, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Cross-GPU exchange (SURVEY.md §8b comm entry points, §8e; csrc/comm.hip). One
 * process per GPU; every rank's receive WINDOW (one uncached device allocation) is
 * mapped into every other rank through HIP IPC over xGMI, and the exchanges are
 * kernels storing straight into the peers' windows with one flag per (source,
 * exchange set) — replacing the row-sharded step's two RCCL all-to-alls per step
 * (reference: the DDP-style exchange the survey maps trainer.py:157-173 onto).
 * Setup (host): mirec_comm_init -> mirec_comm_window (this rank's window + its IPC
 * handle) -> the caller shares the handles (e.g. torch.distributed all_gather_object)
 * -> mirec_comm_connect. Window: [fwd rows: world x wcap x d][bwd rows: same][flags];
 * an exchange with a plan cap <= wcap puts source src's block at src * cap rows.
 * Ordering: a pushing launch's last block raises the flags (system-scope release);
 * the consuming launch's blocks poll this rank's flags (bounded: status -5 on a lost
 * peer) and acquire. Step sets 0 / 1 alternate (each push of a set needs the other
 * set's flags, which need the reader's consumption); the generic calls (sets 2, 3)
 * are bracketed by a barrier (set 4) on entry and exit, so they may follow or precede
 * a step chunk or each other on the stream. Graph-capturable. Design: DESIGN.md §7.
 * ------------------------------------------------------------------------- */
typedef struct mirec_comm mirec_comm;
int mirec_comm_init(int rank, int world, const void* unique_id, mirec_comm** out);
int64_t mirec_comm_handle_bytes(void);
int mirec_comm_window(mirec_comm* comm, int64_t wcap, int32_t d, void** local, void* handle_out);
int mirec_comm_connect(mirec_comm* comm, const void* handles);
int mirec_comm_layout(const mirec_comm* comm, int64_t* fwd_off, int64_t* bwd_off,
                      int32_t** status_dev);
/* The device status word (after a device synchronize), then cleared: 0, or -5 when a
 * wait gave up on a peer since the last read. */
int mirec_comm_status(mirec_comm* comm, int32_t* out);
int mirec_comm_destroy(mirec_comm* comm);
/* MIREC_COMM_PREWAIT: a one-block wait kernel ahead of each step launch (ranks that
 * share a device: the launch's blocks must not spin on CUs the peer needs). */
#define MIREC_COMM_PREWAIT 1
int mirec_comm_config(mirec_comm* comm, int32_t flags);
/* A stand-alone wait of set 0 / 1 that advances the set's counter (diagnostics; the
 * step launches below wait by themselves — do not combine the two). */
int mirec_comm_wait(mirec_comm* comm, int32_t set, void* stream);
/* The row-sharded step's forward exchange: entry g*cap + j of idx (mirec_shard_plan's
 * fwd_rows: >= 0 a row of U, < 0 row -id-1 of I) into rank g's forward region at
 * me*cap + j; raises set 0. */
int mirec_comm_push_rows_f32(mirec_comm* comm, const float* U, const float* I,
                             const int64_t* idx, int64_t cap, void* stream);
/* K3 on this rank's slice reading the forward region at the plan's positions (user
 * [B], pos [B], neg [times x B] message positions o*cap + j), each gradient row into
 * owner o's backward region at me*cap + j (where its perm2 reads it); per-positive
 * losses to loss_k. Its blocks first wait for set 0 (no separate mirec_comm_wait); its
 * last block raises set 1. Same arithmetic as mirec_bpr_fwd_bwd_at_ids_f32. */
int mirec_comm_bpr_f32(mirec_comm* comm, const int64_t* user, const int64_t* pos,
                       const int64_t* neg, int64_t B, int32_t times, float gamma,
                       float grad_scale, float* loss_k, int64_t cap, void* stream);
/* The owner's deferred Adam of a row-sharded step with both exchanges folded in (one
 * launch; mirec_adam_deferred_f32's rows, arithmetic and bits): its blocks wait for
 * set 1 (the readers' gradient rows: tables' `rows` = this rank's backward region);
 * with push lists, every row of the next step (each is in this step's touched or
 * look-ahead list) is stored, right after its update, into each reader's forward
 * region at its message positions, and the last block raises set 0. next[2q] / [2q+1]:
 * mirec_shard_next's next_t / next_a of table q for this step; next_seg[q] / next_dst[q]:
 * the next step's own_seg / perm2 of table q (message positions g*cap + idx); next
 * NULL: no push (a chunk's last step: the next chunk's first rows go by
 * mirec_comm_push_rows_f32 after its entry catch-up). n_max: host bounds of the lists. */
int mirec_comm_adam_deferred_f32(mirec_comm* comm, const mirec_adam_table* tables,
                                 int32_t n_tables, const int64_t* n_max, int32_t d,
                                 const float* step_consts_dev, const int32_t* step_base_dev,
                                 int32_t step_off, double beta1, double beta2, double eps,
                                 double weight_decay, const int32_t* const* next,
                                 const int32_t* const* next_seg, const int32_t* const* next_dst,
                                 int64_t cap, void* stream);
/* All-to-all of ragged row blocks: send [world x wcap x d] (block g to rank g, its first
 * send_counts[g] rows; device int64 [world], NULL = all wcap); afterwards recv [world x
 * wcap x d] (the caller's buffer) holds block src at src * wcap rows, its first
 * recv_counts[src] rows (device int64 [world], written when non-NULL) as rank src sent
 * them; rows past a count are left as they were. Entry / exit barriers included. */
int mirec_alltoallv_rows_f32(mirec_comm* comm, const float* send, const int64_t* send_counts,
                             float* recv, int64_t* recv_counts, int32_t d, void* stream);
/* buf[n] <- the sum of every rank's buf, added in rank order (the same bits on every
 * rank); n <= wcap*d, a multiple of 4, buf 16-B aligned. Entry / exit barriers included. */
int mirec_allreduce_sum_f32(mirec_comm* comm, float* buf, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MIREC_H */
