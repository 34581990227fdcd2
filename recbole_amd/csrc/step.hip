// K35 — the whole model side of one C2 training step in ONE launch: BPR forward +
// backward (K3's arithmetic) and the deferred dense-Adam step (K5's arithmetic) of
// every touched row, plus the look-ahead replays — without gradient rows in HBM and
// without the K3 -> K5 kernel boundary.
//
// Reference: BPR.calculate_loss (bpr.py:74-83) + BPRLoss (loss.py:43-49), the
// nn.Embedding backward (index_add into a dense gradient) and optim.Adam.step over
// every row (trainer.py:157-174; torch optim/adam.py _single_tensor_adam).
//
// Who computes what. K3 formed one gradient row per contribution (per positive for the
// user table, per pos / neg slot for the item table) and K5 summed them per table row
// in the K2 grouping's order. Here the OWNER of a touched row forms its own
// contributions: for each one it gathers the rows of that contribution's positive
// (u, p, the T negatives), recomputes the scores and coefficients with K3's exact
// arithmetic (bpr_math.h; same lane layout, same reductions), builds the contribution
// vector, and the block adds them in grouping order and applies the Adam step — the
// same sums and the same bits as K3 + K5. The scores of a positive are recomputed by
// each of its rows' owners (≈ 3x the dot products, ≈ 4x the row reads of K3; the rows
// sit in L2 / MALL: 2.5 MB of a batch's rows against 84.6 MB tables).
//
// Parity double buffer. A touched row's new p cannot overwrite the row other blocks
// are reading as a partner in the same launch, so p lives in two buffers: the state
// after t applied steps is in P[t & 1]. Step s reads partners (and its own rows) from
// P[s & 1] — every row a step reads is complete through s - 1 (look-ahead of step s-1,
// the chunk entry catch-up, or a flush) — and writes the touched and look-ahead rows
// at state s + 1 into P[(s + 1) & 1]. m and v are private to a row's owner: one
// buffer. Zero-state rows (never updated, adam.hip) are valid in both buffers (the
// caller copies P[0] to P[1] when it marks them). mirec_adam_flush_f32 with p_alt set
// completes every row into P[t & 1] and, for an odd t, also into P[0] (the parameter).
//
// Block = one table row (D in {64, 128, 256}). Touched rows: the block's D/4-lane groups
// take the row's contributions in turn (float4 slices, K3's layout), write them to LDS;
// every thread adds its elements of each contribution in order, then replays (if
// behind) and applies the step. Look-ahead rows: the deferred kernel's replay of steps
// last..s. Per element the arithmetic is adam_deferred_kernel's (adam_core.h), whatever
// the number of elements a thread holds.
#include "adam_core.h"
#include "bpr_math.h"
#include "ahead.h"

namespace mirec {

struct StepLaunch {
  mirec_adam_table t[2];       // [0] users, [1] items: p (+ p_alt), m, v, last, grouping
  const int32_t* rec[2];       // row records per touched-row slot (mirec_step_records)
  const int32_t* crec[2];      // contribution records per grouped position
  float* part[2];              // contribution vectors of split rows, per position x D
  int32_t* join[2];            // arrivals per row slot of split rows (zero between launches)
  int64_t block_start[7];      // segments: shares U, I, look-ahead U, I, touched U, I, end
  int32_t seg_rows[6];         // rows each segment is sized for (the buffers' bound)
};

// rows of one contribution of the positive k: u = EU[user[k]], p = EI[items[k]],
// n_j = EI[items[Bc + j*Bc + k]] (ids clamped as K3 clamps them)
__device__ __forceinline__ int64_t clamp_id(int64_t id, int64_t n) {
  return id < 0 ? 0 : (id >= n ? n - 1 : id);
}


// Contribution records, built per chunk on the prep stream (mirec_step_records, after
// the K2 grouping) so that a step's touched row reaches its partner rows in two
// dependent loads (its record, then the rows) instead of four (segment, perm, ids,
// rows). Contribution record (8 int32): positive k, negative slot j (-1: the positive
// or the user slot), user id, positive item id, the negatives' ids (the first 4; more
// are read from the keys). Row record (kRowRec int32) per touched-row slot x: row id,
// first position i0, contribution count nc, share count nsh, then the records of its
// first kRecInline contributions; the others are at crec[i0 + c].
//
// Split rows. A row with more than kShare contributions (a hot item: its positives and
// negative slots) would take ceil(nc / NG) dependent rounds in one block — the long
// pole of the launch. Its contributions are dealt out in shares of kShare: share 0 to
// the row's own block, shares 1..nsh-1 to blocks of the launch's "share" segment (task
// records below, one per share, carrying the share's contribution records inline).
// Every participant writes its contribution vectors to part[(i0 + c) * D] and counts
// itself in on join[x]; the last to arrive sums ALL nc vectors in grouping order (the
// same sequential sum as an unsplit row) and applies the Adam step. At most
// kSplitCap shares per (table, batch) are dealt out; the contributions of shares past
// the cap stay with the row's own block.
//
// Record region per (table, batch), rec_ints(per) int32: per row records, kSplitCap
// task records {x, share j, i0, nc}, {row, nsh, 0, 0}, the share's contribution
// records, then the task count.
constexpr int kRecInts = 8;
constexpr int kRecInline = 2;
constexpr int kRowRec = 4 + kRecInline * kRecInts;
constexpr int kShare = kRecInline;      // contributions per share of a split row
constexpr int kTaskRec = 8 + kShare * kRecInts;
constexpr int kSplitCap = 256;          // shares dealt out per (table, batch)
constexpr int kStepExtraCap = 62;       // extra records staged in LDS per touched row

__host__ __device__ constexpr int64_t rec_ints(int64_t per) {
  return per * kRowRec + (int64_t)kSplitCap * kTaskRec + 4;
}

__device__ __forceinline__ void contrib_record(int q, int tb, int Bc, int T,
                                               const int64_t* __restrict__ user,
                                               const int64_t* __restrict__ items, int64_t nU,
                                               int64_t nI, int32_t* __restrict__ out) {
  int kk = q, jn = -1;
  if (tb == 1 && q >= Bc) {                      // item row as a negative slot
    const int r = q - Bc;
    jn = r / Bc;
    kk = r - jn * Bc;
  }
  int32_t r[kRecInts];
  r[0] = kk;
  r[1] = jn;
  r[2] = (int32_t)clamp_id(user[kk], nU);
  r[3] = (int32_t)clamp_id(items[kk], nI);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int jj = jn >= 0 ? (j == 0 ? jn : -1) : (j < T ? j : -1);
    r[4 + j] = jj >= 0 ? (int32_t)clamp_id(items[Bc + (int64_t)jj * Bc + kk], nI) : 0;
  }
  reinterpret_cast<int4*>(out)[0] = make_int4(r[0], r[1], r[2], r[3]);
  reinterpret_cast<int4*>(out)[1] = make_int4(r[4], r[5], r[6], r[7]);
}

struct RecJob {   // one table's groupings, record buffers and look-ahead lists
  const int32_t* perm; const int32_t* uniq; const int32_t* seg; const int32_t* nu;
  int32_t* rec; int32_t* crec; int32_t* ahead; int32_t* nah;
};

// The K35 side of a chunk's preparation, after its K2 groupings, in ONE launch of
// kPrepThreads-lane blocks with three roles (no role reads another's output):
//   [0, 2nb)          look-ahead list of (table, batch) (ahead.h; skipped without lists);
//   [2nb, 4nb)        row records of (table, batch) and the share records of its split
//                     rows, shares dealt in row-slot order by a block scan; the inline
//                     contribution records are formed here from the keys;
//   [4nb, 4nb + 2nb*PC) contribution records of PC position blocks per (table, batch).
constexpr int kPrepThreads = 512;
__global__ __launch_bounds__(kPrepThreads) void step_prep_kernel(
    const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ikeys, int n_batches, int Bc,
    int T, int64_t nU, int64_t nI, RecJob U, RecJob I, int PC) {
  __shared__ int32_t a_lds[kDiffLds];
  __shared__ int scan_lds[kPrepThreads / 64 + 1];
  const int nb2 = 2 * n_batches;
  const int role = blockIdx.x < (unsigned)nb2 ? 0 : blockIdx.x < (unsigned)(2 * nb2) ? 1 : 2;
  const int q = role < 2 ? blockIdx.x - role * nb2 : (blockIdx.x - 2 * nb2) / PC;
  const int tb = q >= n_batches;
  const int b = tb ? q - n_batches : q;
  const RecJob& J = tb ? I : U;
  const int KI = (1 + T) * Bc;
  const int per = tb ? KI : Bc;
  const int64_t* __restrict__ user = ukeys + (int64_t)b * Bc;
  const int64_t* __restrict__ items = ikeys + (int64_t)b * KI;
  if (role == 0) {
    if (J.ahead)
      uniq_ahead_diff_batch(J.uniq, J.nu, per, n_batches, J.ahead, J.nah, b, a_lds, scan_lds);
    return;
  }
  const int32_t* __restrict__ perm = J.perm + (int64_t)b * per;
  const int32_t* __restrict__ seg = J.seg + (int64_t)b * (per + 1);
  const int nu = J.nu[b];
  if (role == 2) {
    const int i = ((blockIdx.x - 2 * nb2) % PC) * kPrepThreads + threadIdx.x;
    if (i < per && i < seg[nu])
      contrib_record(perm[i], tb, Bc, T, user, items, nU, nI,
                     J.crec + ((int64_t)b * per + i) * kRecInts);
    return;
  }
  const int32_t* __restrict__ uniq = J.uniq + (int64_t)b * per;
  int32_t* __restrict__ rec = J.rec + (int64_t)b * rec_ints(per);
  int32_t* __restrict__ task = rec + (int64_t)per * kRowRec;
  int dealt = 0;                                   // shares dealt out so far (block-uniform)
  for (int x0 = 0; x0 < nu; x0 += kPrepThreads) {
    const int x = x0 + threadIdx.x;
    int i0 = 0, nc = 0, row = 0;
    if (x < nu) {
      i0 = seg[x];
      nc = seg[x + 1] - i0;
      row = uniq[x];
    }
    const int want = nc > kShare ? (nc + kShare - 1) / kShare - 1 : 0;
    int total;
    const int base = dealt + block_exclusive_scan(want, scan_lds, &total);
    dealt += total;
    if (x >= nu) continue;
    const int got = max(0, min(want, kSplitCap - base));
    const int nsh = 1 + got;
    int32_t* r = rec + (int64_t)x * kRowRec;
    reinterpret_cast<int4*>(r)[0] = make_int4(row, i0, nc, nsh);
    for (int c = 0; c < kRecInline && c < nc; ++c)
      contrib_record(perm[i0 + c], tb, Bc, T, user, items, nU, nI, r + 4 + c * kRecInts);
    for (int j = 1; j <= got; ++j) {
      int32_t* tr = task + (int64_t)(base + j - 1) * kTaskRec;
      reinterpret_cast<int4*>(tr)[0] = make_int4(x, j, i0, nc);
      reinterpret_cast<int4*>(tr)[1] = make_int4(row, nsh, 0, 0);
      for (int c = 0; c < kShare && j * kShare + c < nc; ++c)
        contrib_record(perm[i0 + j * kShare + c], tb, Bc, T, user, items, nU, nI,
                       tr + 8 + c * kRecInts);
    }
  }
  if (threadIdx.x == 0) task[(int64_t)kSplitCap * kTaskRec] = min(dealt, kSplitCap);
}

// ---- K36: a chunk's whole grouping side in ONE launch (replaces the K2 LDS sort launch
// and step_prep_kernel on the C2 path). One 512-lane workgroup per (table, batch):
//  1. the batch's user and item keys into LDS (ids clamped as the records clamp them);
//  2. a sort of the 32-bit composites key << pbits | position (the stable sort by key IS
//     the sort of these distinct composites): bucket counts by the key's top 12 bits in
//     LDS, one scan, a scatter, a rank inside each bucket — no per-digit passes;
//  3. segment heads -> uniq / seg / perm (the K2 outputs, identical to the radix sort's);
//  4. K35 row / share records and the contribution records from LDS (step_prep_kernel's
//     roles 1 and 2, the same share dealing in 512-slot chunks: identical records);
//  5. the look-ahead list of the PREVIOUS batch, uniq(b) \ uniq(b-1) in ascending order,
//     from a bitmap of batch b-1's keys (step_prep_kernel's role 0 as a membership test).
// The radix sort's latency was set by its fixed per-pass cost (C2: user / item sorts of
// a batch 14.7 / 20.3 us), the records launch by three dependent global load levels.
constexpr int kGrpThreads = 512;                    // = kPrepThreads: same share dealing
constexpr int kGrpEpt = 8;                          // composites per lane
constexpr int kGrpMax = kGrpThreads * kGrpEpt;      // keys per (table, batch)
constexpr int kGrpUserMax = kGrpMax / 2;            // user keys per batch (T >= 1)
constexpr int kGrpBitmapWords = 8192;               // look-ahead bitmap: key spaces <= 2^18
constexpr int kGrpBucketBits = 12;                  // sort buckets: the key's top 12 bits
constexpr int kGrpBuckets = 1 << kGrpBucketBits;
static_assert(kGrpThreads == kPrepThreads, "share dealing must match step_prep_kernel");

struct GroupJob {
  int32_t *perm, *uniq, *seg, *nu;   // K2 grouping of the table's batches
  int32_t *rec, *crec;               // K35 records (nullptr: none)
  int32_t *ahead, *nah;              // look-ahead lists (nullptr: none)
  int64_t space;                     // key space (table rows)
  int pbits;                         // bits of a position (per - 1)
};

struct GroupLds {
  uint32_t xa[kGrpMax], xb[kGrpMax];     // xa = the sorted composites, xb = by bucket
  int32_t hist[kGrpBuckets], bstart[kGrpBuckets];
  int32_t uk[kGrpUserMax], ik[kGrpMax];  // the batch's keys (clamped)
  int32_t srow[kGrpMax], sseg[kGrpMax + 1];
  uint32_t bits[kGrpBitmapWords];
  int scan[kGrpThreads / 64 + 1];
};
static_assert(sizeof(GroupLds) <= 160 * 1024, "GroupLds exceeds the gfx950 LDS");

// contrib_record from the LDS copies of the keys (ids already clamped)
__device__ __forceinline__ void contrib_record_lds(int q, int tb, int Bc, int T,
                                                   const int32_t* uk, const int32_t* ik,
                                                   int32_t* __restrict__ out) {
  int kk = q, jn = -1;
  if (tb == 1 && q >= Bc) {
    const int r = q - Bc;
    jn = r / Bc;
    kk = r - jn * Bc;
  }
  int32_t r[kRecInts];
  r[0] = kk;
  r[1] = jn;
  r[2] = uk[kk];
  r[3] = ik[kk];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int jj = jn >= 0 ? (j == 0 ? jn : -1) : (j < T ? j : -1);
    r[4 + j] = jj >= 0 ? ik[Bc + jj * Bc + kk] : 0;
  }
  reinterpret_cast<int4*>(out)[0] = make_int4(r[0], r[1], r[2], r[3]);
  reinterpret_cast<int4*>(out)[1] = make_int4(r[4], r[5], r[6], r[7]);
}

__global__ __launch_bounds__(kGrpThreads) void chunk_group_kernel(
    const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ikeys, int n_batches, int Bc,
    int T, GroupJob U, GroupJob I) {
  __shared__ GroupLds L;
  const int tb = blockIdx.x >= (unsigned)n_batches;
  const int b = tb ? blockIdx.x - n_batches : blockIdx.x;
  const GroupJob& J = tb ? I : U;
  const int KI = (1 + T) * Bc;
  const int per = tb ? KI : Bc;
  const int tid = threadIdx.x;
  const int64_t nU = U.space, nI = I.space;
  // 1. keys (both tables: the records need the user and the item ids of every position)
  const int64_t* __restrict__ user = ukeys + (int64_t)b * Bc;
  const int64_t* __restrict__ items = ikeys + (int64_t)b * KI;
  for (int i = tid; i < Bc; i += kGrpThreads) L.uk[i] = (int32_t)clamp_id(user[i], nU);
  for (int i = tid; i < KI; i += kGrpThreads) L.ik[i] = (int32_t)clamp_id(items[i], nI);
  const bool ahead = J.ahead != nullptr && b > 0;   // this block lists batch b-1's look-ahead
  if (ahead) {
    const int words = (int)((J.space + 31) >> 5);
    for (int w = tid; w < words; w += kGrpThreads) L.bits[w] = 0u;
  }
  if (J.ahead != nullptr && b == 0 && tid == 0) J.nah[n_batches - 1] = 0;   // nothing after
  __syncthreads();
  if (ahead) {                                      // batch b-1's keys of this table
    const int64_t* __restrict__ prev = tb ? ikeys + (int64_t)(b - 1) * KI
                                          : ukeys + (int64_t)(b - 1) * Bc;
    for (int i = tid; i < per; i += kGrpThreads) {
      const int32_t k = (int32_t)clamp_id(prev[i], J.space);
      atomicOr(&L.bits[k >> 5], 1u << (k & 31));
    }
  }
  // 2. sort of the composites key << pbits | position (distinct values: stability comes
  //    free). Bucket by the key's top bits (<= 4,096 buckets, LDS counters: atomics give
  //    each element a slot in its bucket in any order), scan the counts, scatter, then
  //    rank each element inside its bucket (its rank = the bucket's smaller composites;
  //    a bucket holds one or a few keys — a Zipf head key's many positions among them).
  const int pbits = J.pbits;
  const int32_t* keys = tb ? L.ik : L.uk;
  int kbits = 0;
  while (kbits < 31 && ((int64_t)1 << kbits) < J.space) ++kbits;
  const int shift = kbits > kGrpBucketBits ? kbits - kGrpBucketBits : 0;
  const int nbk = (int)(((J.space - 1) >> shift) + 1);
  for (int q = tid; q < nbk; q += kGrpThreads) L.hist[q] = 0;
  __syncthreads();
  uint32_t x[kGrpEpt];
  int slot_in[kGrpEpt];
#pragma unroll
  for (int r = 0; r < kGrpEpt; ++r) {
    const int e = tid + r * kGrpThreads;
    x[r] = 0u;
    slot_in[r] = 0;
    if (e < per) {
      x[r] = ((uint32_t)keys[e] << pbits) | (uint32_t)e;
      slot_in[r] = atomicAdd(&L.hist[keys[e] >> shift], 1);
    }
  }
  __syncthreads();
  {                                               // exclusive scan of the bucket counts
    constexpr int kPer = kGrpBuckets / kGrpThreads;
    int c[kPer], sum = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int q = tid * kPer + j;
      c[j] = q < nbk ? L.hist[q] : 0;
      sum += c[j];
    }
    int tot;
    int run = block_exclusive_scan(sum, L.scan, &tot);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int q = tid * kPer + j;
      if (q < nbk) L.bstart[q] = run;
      run += c[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kGrpEpt; ++r) {
    const int e = tid + r * kGrpThreads;
    if (e < per) L.xb[L.bstart[keys[e] >> shift] + slot_in[r]] = x[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kGrpEpt; ++r) {
    const int e = tid + r * kGrpThreads;
    if (e < per) {
      const int bk = keys[e] >> shift;
      const int b0 = L.bstart[bk], n = L.hist[bk];
      int rank = 0;
      for (int f = 0; f < n; ++f) rank += L.xb[b0 + f] < x[r] ? 1 : 0;
      L.xa[b0 + rank] = x[r];
    }
  }
  __syncthreads();
  // 3. segments: heads of equal-key runs, uniq / seg / perm
  const uint32_t* S = L.xa;
  int32_t* __restrict__ perm = J.perm + (int64_t)b * per;
  int32_t* __restrict__ uniq = J.uniq + (int64_t)b * per;
  int32_t* __restrict__ seg = J.seg + (int64_t)b * (per + 1);
  int hm = 0, cnt = 0;
#pragma unroll
  for (int r = 0; r < kGrpEpt; ++r) {
    const int e = kGrpEpt * tid + r;
    if (e < per) {
      const uint32_t k = S[e] >> pbits;
      const int h = (e == 0 || (S[e - 1] >> pbits) != k) ? 1 : 0;
      hm |= h << r;
      cnt += h;
      perm[e] = (int32_t)(S[e] & ((1u << pbits) - 1u));
    }
  }
  int nu;
  int slot = block_exclusive_scan(cnt, L.scan, &nu);
#pragma unroll
  for (int r = 0; r < kGrpEpt; ++r) {
    if ((hm >> r) & 1) {
      const int e = kGrpEpt * tid + r;
      const int32_t k = (int32_t)(S[e] >> pbits);
      L.srow[slot] = k;
      L.sseg[slot] = e;
      uniq[slot] = k;
      seg[slot] = e;
      ++slot;
    }
  }
  if (tid == 0) {
    L.sseg[nu] = per;
    seg[nu] = per;
    J.nu[b] = nu;
  }
  __syncthreads();
  // 4. K35 records (step_prep_kernel roles 1 and 2, from LDS)
  if (J.rec != nullptr) {
    int32_t* __restrict__ rec = J.rec + (int64_t)b * rec_ints(per);
    int32_t* __restrict__ task = rec + (int64_t)per * kRowRec;
    const uint32_t pm = (1u << pbits) - 1u;
    int dealt = 0;
    for (int x0 = 0; x0 < nu; x0 += kGrpThreads) {
      const int xs = x0 + tid;
      int i0 = 0, nc = 0, row = 0;
      if (xs < nu) {
        i0 = L.sseg[xs];
        nc = L.sseg[xs + 1] - i0;
        row = L.srow[xs];
      }
      const int want = nc > kShare ? (nc + kShare - 1) / kShare - 1 : 0;
      int total;
      const int base = dealt + block_exclusive_scan(want, L.scan, &total);
      dealt += total;
      if (xs >= nu) continue;
      const int got = max(0, min(want, kSplitCap - base));
      const int nsh = 1 + got;
      int32_t* r = rec + (int64_t)xs * kRowRec;
      reinterpret_cast<int4*>(r)[0] = make_int4(row, i0, nc, nsh);
      for (int c = 0; c < kRecInline && c < nc; ++c)
        contrib_record_lds((int)(S[i0 + c] & pm), tb, Bc, T, L.uk, L.ik, r + 4 + c * kRecInts);
      for (int jj = 1; jj <= got; ++jj) {
        int32_t* tr = task + (int64_t)(base + jj - 1) * kTaskRec;
        reinterpret_cast<int4*>(tr)[0] = make_int4(xs, jj, i0, nc);
        reinterpret_cast<int4*>(tr)[1] = make_int4(row, nsh, 0, 0);
        for (int c = 0; c < kShare && jj * kShare + c < nc; ++c)
          contrib_record_lds((int)(S[i0 + jj * kShare + c] & pm), tb, Bc, T, L.uk, L.ik,
                             tr + 8 + c * kRecInts);
      }
    }
    if (tid == 0) task[(int64_t)kSplitCap * kTaskRec] = min(dealt, kSplitCap);
    int32_t* __restrict__ crec = J.crec + (int64_t)b * per * kRecInts;
    for (int e = tid; e < per; e += kGrpThreads)
      contrib_record_lds((int)(S[e] & pm), tb, Bc, T, L.uk, L.ik, crec + (int64_t)e * kRecInts);
  }
  // 5. look-ahead list of batch b-1: this batch's rows that batch b-1 does not touch
  if (ahead) {
    int32_t* __restrict__ out = J.ahead + (int64_t)(b - 1) * per;
    int base = 0;
    for (int x0 = 0; x0 < nu; x0 += kGrpThreads) {
      const int xs = x0 + tid;
      int f = 0;
      int32_t k = 0;
      if (xs < nu) {
        k = L.srow[xs];
        f = ((L.bits[k >> 5] >> (k & 31)) & 1u) ? 0 : 1;
      }
      int tot;
      const int ex = block_exclusive_scan(f, L.scan, &tot);
      if (f) out[base + ex] = k;
      base += tot;
    }
    if (tid == 0) J.nah[b - 1] = base;
  }
}

// Hand-off of a split row's contribution vectors between the blocks of one launch
// (MI355X_MICROARCH.md, inter-workgroup visibility, first hand-off form): the vectors go
// out as agent-scope atomic stores (write-through: past this XCD's L2), every storing
// wave drains them (vmcnt(0)) before the row's threads meet and ONE lane counts the row
// in with an agent-scope add; the last adder takes an agent-scope acquire and the row's
// threads read the vectors back with agent-scope loads (sc1: from past the L2).
//
// Measured alternatives (round 4; the probe builds live on branch probes/k35-r4):
// - the C++ memory model's own producer form — each thread an agent-scope release fence
//   before the meeting, acq_rel adds (here and at the look-ahead half-join). Bit-identical,
//   but the release is `buffer_wbl2 sc1`: it writes back every dirty line of the XCD's L2
//   (K35's row-state stores), once per wave — C2 driver window 23.5-23.9 M -> 5.6 M
//   positives/s. Not adopted.
// - a release on the counting lane only (the drains removed): a workgroup barrier does not
//   wait for the other wave's stores, and test_gpu_e2e's bit-identity failed at d = 256 (a
//   two-wave row) — the drain in every wave is what the hand-off rests on.
__device__ __forceinline__ void part_store(float* p, float4 a) {
  auto q = (__attribute__((address_space(1))) unsigned long long*)(p);
  const unsigned long long lo =
      (unsigned long long)__float_as_uint(a.x) | ((unsigned long long)__float_as_uint(a.y) << 32);
  const unsigned long long hi =
      (unsigned long long)__float_as_uint(a.z) | ((unsigned long long)__float_as_uint(a.w) << 32);
  __hip_atomic_store(q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void part_load(const float* p, float& a) {
  auto q = (const __attribute__((address_space(1))) unsigned int*)(p);
  a = __uint_as_float(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void part_load(const float* p, float2& a) {
  auto q = (const __attribute__((address_space(1))) unsigned long long*)(p);
  const unsigned long long w = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a = make_float2(__uint_as_float((unsigned)w), __uint_as_float((unsigned)(w >> 32)));
}

constexpr int kJoinOrder = __ATOMIC_RELAXED;

// Row-state stores of K35 (plain stores; write-through stores measured no better)
template <typename V>
__device__ __forceinline__ void state_store(V* p, const V& x) {
  *p = x;
}

template <int D> struct StepVec { using T = float2; };
template <> struct StepVec<64> { using T = float; };
// Rows per workgroup: a row of D <= 128 is one wave, and RPB of them share a workgroup
// (each wave works alone: wave-level synchronisation only), so the dispatcher hands out
// RPB times fewer workgroups (it deals ~2-3 per ns: ~10 K one-row workgroups were ~3 us
// of a launch). D = 256 rows span two waves: one row per workgroup.
#ifndef MIREC_STEP_RPB
#define MIREC_STEP_RPB 4
#endif
template <int D> struct StepRows { static constexpr int n = D <= 128 ? MIREC_STEP_RPB : 1; };
#ifndef MIREC_STEP_SUM_LOADS
#define MIREC_STEP_SUM_LOADS 8           // a split row's vectors loaded at once by its last
#endif                                   // arriver (one dependent round per group)
constexpr int kSumLoads = MIREC_STEP_SUM_LOADS;
#ifndef MIREC_STEP_WAVES
#define MIREC_STEP_WAVES 5               // waves per SIMD the register budget allows (6: 80
#endif                                   // VGPRs, 28 B/lane spilled; 5: 86, no spill)

template <int D>
__global__ __launch_bounds__(D / Lanes<typename StepVec<D>::T>::n * StepRows<D>::n,
                             MIREC_STEP_WAVES)
void bpr_adam_step_kernel(
    const StepLaunch L, const int64_t* __restrict__ items, int Bc, int T, float gamma,
    float grad_scale, float* __restrict__ loss_k, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  using V = typename StepVec<D>::T;
  constexpr int EPT = Lanes<V>::n;         // elements per thread
  constexpr int TPB = D / EPT;             // threads per row
  constexpr int RPB = StepRows<D>::n;      // rows per workgroup
  static_assert(RPB == 1 || TPB == 64, "several rows per workgroup need one wave per row");
  constexpr int LPR = D / 4;               // lanes per contribution (float4 each, K3's layout)
  constexpr int NG = TPB / LPR;            // contributions in flight per row
  __shared__ float cont_all[RPB][NG][D];
  __shared__ int s_last_all[RPB];
  // the row of this wave: wave-uniform, so the row's indices stay in scalar registers
  const int wv = RPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x / TPB)) : 0;
  auto& cont = cont_all[wv];
  int& s_last = s_last_all[wv];
  // the row's threads in step: a workgroup barrier for a two-wave row, else the wave
  auto row_sync = [&]() {
    if (RPB == 1) {
      __syncthreads();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };
  int si = 0;
#pragma unroll
  for (int q = 1; q < 6; ++q)
    if ((int64_t)blockIdx.x >= L.block_start[q]) si = q;
  const int kind = si >> 1;                // 0 share of a split row, 1 look-ahead, 2 touched
  const bool ahead = kind == 1;
  const int tb = si & 1;                   // 0 users, 1 items
  const mirec_adam_table& T_ = L.t[tb];
  const int u = (int)(((int64_t)blockIdx.x - L.block_start[si]) * RPB) + wv;
  if (u >= L.seg_rows[si]) return;         // past the segment's bound (wave-uniform)
  const int t = threadIdx.x - wv * TPB;
  const int grp = t / LPR;
  const int l = t - grp * LPR;
  // first load level, all independent of each other: the count and the row id (look-
  // ahead), the row record (touched: row, i0, nc, nsh and this lane group's inline
  // contribution record) or the task record (share j of row slot x); u < the
  // launch's bound, so the loads stay in the buffers even past the count
  const int per = tb ? (1 + T) * Bc : Bc;
  const int32_t* __restrict__ R = L.rec[tb];
  int4 h0 = make_int4(0, 0, 0, 0), h1 = h0, ra = h0, rb = h0;
  int n;
  int64_t row;
  if (ahead) {
    n = T_.ahead_n_uniq[0];
    row = T_.ahead_uniq[u];
  } else {
    const int32_t* __restrict__ Q;
    if (kind == 2) {
      n = T_.n_uniq[0];
      Q = R + (int64_t)u * kRowRec;
      h0 = reinterpret_cast<const int4*>(Q)[0];              // row, i0, nc, nsh
      row = h0.x;
      Q += 4;
    } else {
      const int32_t* __restrict__ task = R + (int64_t)per * kRowRec;
      n = task[(int64_t)kSplitCap * kTaskRec];
      Q = task + (int64_t)u * kTaskRec;
      h0 = reinterpret_cast<const int4*>(Q)[0];              // x, j, i0, nc
      h1 = reinterpret_cast<const int4*>(Q)[1];              // row, nsh
      row = h1.x;
      Q += 8;
    }
    if (grp < kRecInline) {
      ra = reinterpret_cast<const int4*>(Q + grp * kRecInts)[0];
      rb = reinterpret_cast<const int4*>(Q + grp * kRecInts)[1];
    }
  }
  const int st = step_base[0] + step_off;
  if (u >= n) return;                      // wave-uniform (row-uniform)
  const float* __restrict__ Pr[2] = {T_.p, T_.p_alt};
  float* __restrict__ Pw = ((st + 1) & 1) ? T_.p_alt : T_.p;
  const int raw = T_.last[row];
  const int64_t off = row * (D / EPT) + t;           // in units of V

  if (ahead) {
    // rows the next step reads and this one does not touch: replay last..st (zero
    // gradient), as adam_deferred_kernel's look-ahead segment; whole rows, four steps'
    // chains in flight (round 5: rows split over two half-row slots with eight in flight
    // measured 4 % slower in the C2 driver window — more waves for the same work)
    if (raw == kZeroState || raw > st) return;    // current at every step / already done
    V p = reinterpret_cast<const V*>(Pr[raw & 1])[off];
    V m = reinterpret_cast<const V*>(T_.m)[off];
    V v = reinterpret_cast<const V*>(T_.v)[off];
    replay<V, true, 4>(p, m, v, raw, st, consts, k);
    V z;
    memset(&z, 0, sizeof(V));
    adam_vec(p, m, v, z, step_consts(consts, st), k);   // step st: zero gradient
    MIREC_WORK(3, EPT * MIREC_WORK_LANES());
    MIREC_WORK(5, 1);
    state_store(reinterpret_cast<V*>(Pw) + off, p);
    state_store(reinterpret_cast<V*>(T_.m) + off, m);
    state_store(reinterpret_cast<V*>(T_.v) + off, v);
    row_sync();                                    // every thread read `last`
    if (t == 0) T_.last[row] = st + 1;
    return;
  }

  // ---- touched row (or one share of it): own state in flight while the contributions
  // are formed. Every row a step reads is complete through st - 1 (look-ahead / entry
  // catch-up / flush) or in the zero state (the same p in both buffers), so its p is in
  // buffer st & 1; a row behind (never, by that invariant) reloads from its own buffer.
  const int last = raw == kZeroState ? st : raw;
  V p = reinterpret_cast<const V*>(Pr[st & 1])[off];
  V m = reinterpret_cast<const V*>(T_.m)[off];
  V v = reinterpret_cast<const V*>(T_.v)[off];
  const float* __restrict__ EU = L.t[0].p;         // partner rows at state st
  const float* __restrict__ EI = L.t[1].p;
  if (st & 1) {
    EU = L.t[0].p_alt;
    EI = L.t[1].p_alt;
  }
  // this block's contributions: i = 0..cnt-1 -> grouping position c(i). Share j >= 1:
  // c = j*kShare + i. The row's own block (j = 0): share 0, then the contributions past
  // the dealt-out shares (c = i + (nsh-1)*kShare for i >= kShare).
  const int x = kind == 2 ? u : h0.x;
  const int j = kind == 2 ? 0 : h0.y;
  const int i0 = kind == 2 ? h0.y : h0.z;
  const int nc = kind == 2 ? h0.z : h0.w;
  const int nsh = kind == 2 ? h0.w : h1.y;
  const bool split = nsh > 1;                      // block-uniform
  const int cnt = j ? min(kShare, nc - j * kShare)
                    : min(kShare, nc) + max(0, nc - nsh * kShare);
  const int cskip = (nsh - 1) * kShare;
  const float ng = -grad_scale;
  float* __restrict__ part = L.part[tb] + (int64_t)i0 * D;
  V g;
  memset(&g, 0, sizeof(V));
  // records of contributions kRecInline.. into LDS (one level, beside round 0's rows)
  __shared__ int4 xrec_all[RPB][kStepExtraCap][2];
  auto& xrec = xrec_all[wv];
  if (cnt > kRecInline) {                          // row-uniform (own row only)
    const int32_t* __restrict__ C = L.crec[tb] + (int64_t)(i0 + cskip) * kRecInts;
    for (int c = kRecInline + t; c < min(cnt, kRecInline + kStepExtraCap); c += TPB) {
      xrec[c - kRecInline][0] = reinterpret_cast<const int4*>(C + (int64_t)c * kRecInts)[0];
      xrec[c - kRecInline][1] = reinterpret_cast<const int4*>(C + (int64_t)c * kRecInts)[1];
    }
    row_sync();
  }
  for (int base = 0; base < cnt; base += NG) {
    const int i = base + grp;
    if (i < cnt) {
      int4 r0 = ra, r1 = rb;                        // contribution i's record
      if (i >= kRecInline) {
        if (i - kRecInline < kStepExtraCap) {
          r0 = xrec[i - kRecInline][0];
          r1 = xrec[i - kRecInline][1];
        } else {
          const int32_t* C = L.crec[tb] + (int64_t)(i0 + cskip + i) * kRecInts;
          r0 = reinterpret_cast<const int4*>(C)[0];
          r1 = reinterpret_cast<const int4*>(C)[1];
        }
      }
      const int kk = r0.x, jn = r0.y;
      if (l == 0) {
        if (jn >= 0) { MIREC_WORK(8, 1); } else if (tb == 0) { MIREC_WORK(6, 1); } else { MIREC_WORK(7, 1); }
      }
      const float4 uv = reinterpret_cast<const float4*>(EU + (int64_t)r0.z * D)[l];
      const float4 pv = reinterpret_cast<const float4*>(EI + (int64_t)r0.w * D)[l];
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (jn >= 0) {                                  // item row as the negative jn
        const float4 nv = reinterpret_cast<const float4*>(EI + (int64_t)r1.x * D)[l];
        const float sp = group_sum<LPR>(dot4(uv, pv));
        const float sn = group_sum<LPR>(dot4(uv, nv));
        acc = contrib_n(bpr_coef(sp, sn, gamma, ng).dx, uv);
      } else {                                        // user row, or item row as the positive
        const int nid4[4] = {r1.x, r1.y, r1.z, r1.w};
        float lsum = 0.f;
        for (int j0 = 0; j0 < T; j0 += 4) {
          float4 nv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int jj = j0 + e;
            nv[e] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (jj < T) {
              const int64_t nid = jj < 4 ? (int64_t)nid4[e]
                                         : clamp_id(items[Bc + (int64_t)jj * Bc + kk],
                                                    L.t[1].n_rows);
              nv[e] = reinterpret_cast<const float4*>(EI + nid * D)[l];
            }
          }
          const float sp = group_sum<LPR>(dot4(uv, pv));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int jj = j0 + e;
            if (jj < T) {
              const float sn = group_sum<LPR>(dot4(uv, nv[e]));
              const BprCoef cf = bpr_coef(sp, sn, gamma, ng);
              lsum += cf.nll;
              if (tb == 0)
                contrib_u(acc, cf.dx, pv, nv[e]);
              else
                contrib_p(acc, cf.dx, uv);
            }
          }
        }
        if (tb == 0 && l == 0 && loss_k) loss_k[kk] = lsum;   // one user slot per positive
      }
      if (split) {
        const int c = i < kShare ? j * kShare + i : cskip + i;
        part_store(part + (int64_t)c * D + 4 * l, acc);
      } else {
        *reinterpret_cast<float4*>(&cont[grp][4 * l]) = acc;
      }
    }
    if (!split) {
      row_sync();
#pragma unroll
      for (int h = 0; h < NG; ++h)
        if (base + h < cnt) {
          const V cv = *reinterpret_cast<const V*>(&cont[h][EPT * t]);
#pragma unroll
          for (int e = 0; e < EPT; ++e) Lanes<V>::at(g, e) += Lanes<V>::at(cv, e);
        }
      row_sync();                                    // cont is rewritten next round
    }
  }
  if (split) MIREC_WORK(9, 1);
  if (split) {
    // Hand-off (see part_store): drain this wave's write-through stores, meet, one lane
    // counts the row in on join[x]; the add that returns nsh - 1 is the last, whose lane
    // takes an agent-scope acquire before the row's threads load the vectors.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    row_sync();
    if (t == 0) {
      const int arrived =
          __hip_atomic_fetch_add(L.join[tb] + x, 1, kJoinOrder, __HIP_MEMORY_SCOPE_AGENT);
      s_last = arrived == nsh - 1;
      if (s_last) {                                  // every participant has counted in
        __hip_atomic_store(L.join[tb] + x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    row_sync();
    if (!s_last) return;                             // row-uniform
    const float* __restrict__ pe = part + EPT * t;
    int c = 0;
    for (; c + kSumLoads <= nc; c += kSumLoads) {
      V cv[kSumLoads];
#pragma unroll
      for (int h = 0; h < kSumLoads; ++h) part_load(pe + (int64_t)(c + h) * D, cv[h]);
#pragma unroll
      for (int h = 0; h < kSumLoads; ++h)
#pragma unroll
        for (int e = 0; e < EPT; ++e) Lanes<V>::at(g, e) += Lanes<V>::at(cv[h], e);
    }
    for (; c < nc; ++c) {
      V cv;
      part_load(pe + (int64_t)c * D, cv);
#pragma unroll
      for (int e = 0; e < EPT; ++e) Lanes<V>::at(g, e) += Lanes<V>::at(cv, e);
    }
  }
  if (last < st) {                                   // behind (not expected): own buffer
    p = reinterpret_cast<const V*>(Pr[last & 1])[off];
  }

  // ---- Adam step of the row (replaying skipped zero-gradient steps first)
  replay<V, true>(p, m, v, last, st, consts, k);
  const bool fresh = last <= st;
  if (fresh) adam_vec(p, m, v, g, step_consts(consts, st), k);
  if (fresh) {
    MIREC_WORK(2, EPT * MIREC_WORK_LANES());
    MIREC_WORK(4, 1);
  }
  row_sync();
  if (!fresh) return;
  state_store(reinterpret_cast<V*>(Pw) + off, p);
  state_store(reinterpret_cast<V*>(T_.m) + off, m);
  state_store(reinterpret_cast<V*>(T_.v) + off, v);
  if (t == 0) T_.last[row] = st + 1;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_step_records(const int64_t* user_keys, const int64_t* item_keys,
                                  int64_t n_batches, int64_t Bc, int32_t T, int64_t n_users,
                                  int64_t n_items, const int32_t* u_perm, const int32_t* u_uniq,
                                  const int32_t* u_seg, const int32_t* u_nu,
                                  const int32_t* i_perm, const int32_t* i_uniq,
                                  const int32_t* i_seg, const int32_t* i_nu, int32_t* u_rec,
                                  int32_t* u_crec, int32_t* i_rec, int32_t* i_crec,
                                  int32_t* u_ahead, int32_t* u_nah, int32_t* i_ahead,
                                  int32_t* i_nah, void* stream) {
  if (n_batches < 0 || n_batches > 32767 || Bc < 0 || T < 1 ||
      (int64_t)(1 + T) * Bc > INT32_MAX || n_users <= 0 || n_items <= 0 || !user_keys || !item_keys || !u_perm || !u_uniq || !u_seg || !u_nu ||
      !i_perm || !i_uniq || !i_seg || !i_nu || !u_rec || !u_crec || !i_rec || !i_crec ||
      !u_ahead != !u_nah || !u_ahead != !i_ahead || !i_ahead != !i_nah) {
    set_error("mirec_step_records: bad arguments");
    return -1;
  }
  if (n_batches == 0 || Bc == 0) return 0;
  const RecJob U = {u_perm, u_uniq, u_seg, u_nu, u_rec, u_crec, u_ahead, u_nah};
  const RecJob I = {i_perm, i_uniq, i_seg, i_nu, i_rec, i_crec, i_ahead, i_nah};
  const int64_t KI = (1 + T) * Bc;
  const int PC = (int)((KI + kPrepThreads - 1) / kPrepThreads);
  hipLaunchKernelGGL(step_prep_kernel, dim3((unsigned)(4 * n_batches + 2 * n_batches * PC)),
                     dim3(kPrepThreads), 0, (hipStream_t)stream, user_keys, item_keys,
                     (int)n_batches, (int)Bc, T, n_users, n_items, U, I, PC);
  return launch_status("mirec_step_records");
}

extern "C" int64_t mirec_step_record_ints(int64_t per) { return per < 0 ? -1 : rec_ints(per); }

#if defined(MIREC_STEP_COUNT)
// diagnostic build only: copy (and clear) this unit's executed-work counters (16 x u64)
extern "C" int mirec_work_counters(unsigned long long* dst, int clear) {
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_work), sizeof(g_work)) != hipSuccess) return -1;
  if (clear) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_work), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

namespace mirec {
static int bits_for(int64_t n) {        // bits of n - 1 (n >= 1)
  int b = 0;
  while (b < 40 && ((int64_t)1 << b) < n) ++b;
  return b;
}
}  // namespace mirec

namespace mirec {
// the shapes K36's one-workgroup form takes (else the K2 sort + mirec_step_records)
static bool chunk_group_fits(int64_t Bc, int32_t T, int64_t n_users, int64_t n_items,
                             bool ahead) {
  if (Bc <= 0 || T < 1 || n_users <= 0 || n_items <= 0) return false;
  const int64_t KI = (int64_t)(1 + T) * Bc;
  const int pu = bits_for(Bc), pi = bits_for(KI);
  return !(Bc > kGrpUserMax || KI > kGrpMax || bits_for(n_users) + pu > 32 ||
           bits_for(n_items) + pi > 32 ||
           (ahead && (n_users > 32 * (int64_t)kGrpBitmapWords ||
                      n_items > 32 * (int64_t)kGrpBitmapWords)));
}
}  // namespace mirec

extern "C" int mirec_chunk_group_fits(int64_t Bc, int32_t T, int64_t n_users, int64_t n_items,
                                      int32_t ahead) {
  return chunk_group_fits(Bc, T, n_users, n_items, ahead != 0) ? 1 : 0;
}

// K36 on a prepared chunk (include/mirec.h): 1 = done, 0 = shapes outside the one-
// workgroup form (the caller runs the K2 sort + mirec_step_records), < 0 = error.
extern "C" int mirec_chunk_group(const int64_t* user_keys, const int64_t* item_keys,
                                 int64_t n_batches, int64_t Bc, int32_t T, int64_t n_users,
                                 int64_t n_items, int32_t* u_perm, int32_t* u_uniq,
                                 int32_t* u_seg, int32_t* u_nu, int32_t* i_perm,
                                 int32_t* i_uniq, int32_t* i_seg, int32_t* i_nu,
                                 int32_t* u_rec, int32_t* u_crec, int32_t* i_rec,
                                 int32_t* i_crec, int32_t* u_ahead, int32_t* u_nah,
                                 int32_t* i_ahead, int32_t* i_nah, void* stream) {
  if (n_batches < 0 || n_batches > 32767 || Bc < 0 || T < 1 || n_users <= 0 || n_items <= 0 ||
      !user_keys || !item_keys || !u_perm || !u_uniq || !u_seg || !u_nu || !i_perm || !i_uniq ||
      !i_seg || !i_nu || !u_rec != !u_crec || !u_rec != !i_rec || !i_rec != !i_crec ||
      !u_ahead != !u_nah || !u_ahead != !i_ahead || !i_ahead != !i_nah) {
    set_error("mirec_chunk_group: bad arguments");
    return -1;
  }
  if (n_batches == 0 || Bc == 0) return 1;
  const int64_t KI = (int64_t)(1 + T) * Bc;
  const int pu = bits_for(Bc), pi = bits_for(KI);
  if (!chunk_group_fits(Bc, T, n_users, n_items, u_ahead != nullptr)) return 0;
  GroupJob U = {u_perm, u_uniq, u_seg, u_nu, u_rec, u_crec, u_ahead, u_nah, n_users, pu};
  GroupJob I = {i_perm, i_uniq, i_seg, i_nu, i_rec, i_crec, i_ahead, i_nah, n_items, pi};
  hipLaunchKernelGGL(chunk_group_kernel, dim3((unsigned)(2 * n_batches)), dim3(kGrpThreads), 0,
                     (hipStream_t)stream, user_keys, item_keys, (int)n_batches, (int)Bc, T, U, I);
  const int rc = launch_status("mirec_chunk_group");
  return rc ? rc : 1;
}


extern "C" int mirec_bpr_adam_step_f32(const mirec_adam_table* tables,
                                       const int64_t* n_max_uniq, int32_t d,
                                       const int64_t* items, int64_t Bc, int32_t T, float gamma,
                                       float grad_scale, float* loss_k, const int32_t* u_rec,
                                       const int32_t* u_crec, const int32_t* i_rec,
                                       const int32_t* i_crec, float* u_part, int32_t* u_join,
                                       float* i_part, int32_t* i_join,
                                       const float* step_consts_dev,
                                       const int32_t* step_base_dev, int32_t step_off,
                                       double beta1, double beta2, double eps,
                                       double weight_decay, void* stream) {
  const char* what = "mirec_bpr_adam_step_f32";
  if (!tables || !n_max_uniq || !items || Bc < 0 || T < 1 || !step_consts_dev ||
      (int64_t)(1 + T) * Bc > INT32_MAX || !u_rec || !u_crec || !i_rec || !i_crec ||
      !u_part || !u_join || !i_part || !i_join || !step_base_dev || ((uintptr_t)step_consts_dev & 15) != 0) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  if (d != 64 && d != 128 && d != 256) {
    set_error("%s: embedding_size %d not in {64,128,256}", what, d);
    return -1;
  }
  StepLaunch L;
  memset(&L, 0, sizeof(L));
  for (int q = 0; q < 2; ++q) {
    const mirec_adam_table& t = tables[q];
    if (!t.p || !t.p_alt || !t.m || !t.v || !t.last || !t.n_uniq || t.n_rows <= 0 ||
        n_max_uniq[q] < 0 || t.dense_grad ||
        (t.ahead_uniq == nullptr) != (t.ahead_n_uniq == nullptr)) {
      set_error("%s: bad table %d", what, q);
      return -1;
    }
    L.t[q] = t;
  }
  L.rec[0] = u_rec;
  L.crec[0] = u_crec;
  L.rec[1] = i_rec;
  L.crec[1] = i_crec;
  L.part[0] = u_part;
  L.join[0] = u_join;
  L.part[1] = i_part;
  L.join[1] = i_join;
  // segments: the shares of split rows first (their row's step waits for them), then
  // the look-ahead rows (their replays are long chains), then the touched rows
  if (n_max_uniq[0] == 0 && n_max_uniq[1] == 0) return 0;
  const int64_t rows[6] = {kSplitCap, kSplitCap,
                           L.t[0].ahead_uniq ? n_max_uniq[0] : 0,
                           L.t[1].ahead_uniq ? n_max_uniq[1] : 0,
                           n_max_uniq[0], n_max_uniq[1]};
  const int rpb = d <= 128 ? MIREC_STEP_RPB : 1;  // StepRows<d>
  int64_t b = 0;
  for (int q = 0; q < 6; ++q) {
    L.block_start[q] = b;
    L.seg_rows[q] = (int32_t)rows[q];
    b += (rows[q] + rpb - 1) / rpb;
  }
  L.block_start[6] = b;
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grd((unsigned)b);
#define MIREC_STEP_CASE(DD)                                                                  \
  case DD:                                                                                   \
    hipLaunchKernelGGL(bpr_adam_step_kernel<DD>, grd,                                        \
                       dim3(DD / Lanes<typename StepVec<DD>::T>::n * StepRows<DD>::n), 0, st,\
                       L, items,                                                             \
                       (int)Bc, T, gamma, grad_scale, loss_k, step_consts_dev, step_base_dev,\
                       step_off, k);                                                         \
    break;
  switch (d) {
    MIREC_STEP_CASE(64)
    MIREC_STEP_CASE(128)
    MIREC_STEP_CASE(256)
  }
#undef MIREC_STEP_CASE
  return launch_status(what);
}

