// kernels.hpp — host-callable launchers for the HIP kernels in query_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devtypes.hpp"

namespace sb {

// The slice-query kernel: one wavefront per query.  Each wave finds its exact
// [lo, hi) record bounds from the segment's coarse POS index, filters the
// records with the reference's predicates, reproduces its order-dependent
// early exits and writes packed hits into its host-planned region at
// q.hit_off, per-query totals into res and, for the sample path, a carrier
// bitset per query into samples_out.
// qidx (optional) lists the queries this launch covers (n of them); max_words
// = 0 compiles out the sample path; nonneg selects the monotone call_count path;
// mode (MODE_*) picks the predicate specialisation every listed query fits.
void launch_scan(const DStore &st, const QDev *q, const uint32_t *qidx, uint32_t n, bool nonneg, uint32_t max_words,
                 int mode, const uint8_t *qbytes, const uint64_t *subsets, QRes *res, uint64_t *hits,
                 uint64_t *samples_out, hipStream_t s);

// Several sample-free groups (each a list of queries fitting one MODE_*) in
// one launch, in the order given (put the longest-running first).
constexpr int kFusedMax = 5;
struct FusedGroup {
    const QDev *q;  // the group's n queries, contiguous in launch order
    uint32_t n;
    int mode;
};
void launch_fused(const DStore &st, const FusedGroup *groups, int count, bool nonneg,
                  const uint8_t *qbytes, const uint64_t *subsets, QRes *res, uint64_t *hits, hipStream_t s);

// Slice chains (devtypes.hpp ChainDev): runs of chains of consecutive
// variantType slices of one request per wave; corig[s] = batch index of the
// chain-ordered slice s.  launch_chain_src writes the hit-region offset of
// every chained slice (dense per chain) into src[batch index].
void launch_chains(const DStore &st, const ChainDev *chains, uint32_t n_chains, const uint32_t *runs, uint32_t n_runs,
                   const uint32_t *corig, QRes *res, uint64_t *hits, ReqPartial *cpart, hipStream_t s);
// chain runs (one wave each): at most pack_run_max() chains and pack_slots_max() slices per run
uint32_t pack_run_max();
uint32_t pack_slots_max();
void launch_chain_src(const ChainDev *chains, uint32_t n_chains, const uint32_t *corig, const QRes *res,
                      uint64_t *src, hipStream_t s);

// summariseSlice: phase A = one workgroup per chunk of kSumChunk records
// (chunk_slice[c] = its slice), reducing the records' (numVariants, numCalls)
// contributions into part[c] and writing the overshoot bitmap; phase B = one
// wave per slice replaying the skip heuristic over the (rare) overshooting
// records.  bitmap needs ceil((hi - lo) / 64) words per slice.
void launch_summarise(const SStore &ss, const SDev *slices, uint32_t ns, const uint32_t *chunk_slice, uint32_t nchunks,
                      uint64_t *bitmap, SPart *part, SRes *out, hipStream_t s);

// Per-request partials of one shard (sb_batch_reduce_requests): row w sums
// the answers of queries [seg[w], seg[w+1]).  wide (optional, per query) =
// the query's counts needed more than 64 bits (mark_wide, from the general
// path's big list); row_flag (optional, per row) = 1 when the row's
// call_count / all_alleles_count are not exact in int64 (low 64 bits kept).
void mark_wide(const uint32_t *big_n, const GenBig *big, uint32_t cap, uint8_t *wide, hipStream_t s);
void launch_request_reduce(const QRes *res, const uint32_t *seg, const uint8_t *host_err, const uint8_t *wide,
                           uint32_t n_rows, ReqPartial *out, uint8_t *row_flag, hipStream_t s);

// Dense per-query hit lists on the device: dense[q] = exclusive prefix of the
// queries' hit counts (dense[nq] = total), out[dense[q] ..] = query q's hits
// (from its region at src[q]) + rec_base; row_off[w] = dense[seg[w]] for
// w <= n_rows when seg is given.  tsum needs hit_scan_words(nq) words.
size_t hit_scan_words(uint32_t nq);
void launch_hit_lists(const QRes *res, uint32_t nq, const uint64_t *src, const uint64_t *hits, uint64_t rec_base,
                      const uint32_t *seg, uint32_t n_rows, uint64_t *tsum, uint64_t *dense, uint64_t *out,
                      uint64_t *row_off, hipStream_t s);

// Request rows by pieces (chains + unchained queries; piece bit 31 = chain):
// row_reduce sums each row's pieces (chain partials from chain_kernel's
// cpart, QRes otherwise); row_hit_lists scans the rows' n_variants into
// row_off (n_rows + 1) and copies each row's pieces' hits to out[row_off[w]..]
// with rec_base added.  tsum needs hit_scan_words(n_rows) words.
// rowsrc (n_rows x {hit region, count}; {~0, 0} = several pieces) is written
// by row_reduce and read by row_hit_lists.
void launch_row_reduce(const ReqPartial *cpart, const ChainDev *chains, const uint64_t *hoff, const QRes *res,
                       const uint8_t *host_err, const uint32_t *poff, const uint32_t *piece, uint32_t n_rows,
                       ReqPartial *out, ulonglong2 *rowsrc, hipStream_t s);
// sb_batch_deliver (row pieces): rows + dense n_variants / tile sums, the
// offset scan over them, then the segmented gather; rowout (optional, built
// at sb_batch_set_owners) = each single-piece row's hit region (~0: several
// pieces) in place of the rowsrc the reduction would write
void launch_row_deliver(const ReqPartial *cpart, const ChainDev *chains, const uint64_t *hoff, const QRes *res,
                        const uint8_t *host_err, const uint32_t *poff, const uint32_t *piece, uint32_t n_rows,
                        ReqPartial *rows, ulonglong2 *rowsrc, const uint64_t *rowout, int64_t *nv, uint64_t *tsum,
                        const uint64_t *hits, uint64_t rec_base, uint64_t *row_off, uint64_t *out, hipStream_t s);
void launch_row_hit_lists(const ReqPartial *rows, const ulonglong2 *rowsrc, const uint32_t *poff,
                          const uint32_t *piece, uint32_t n_rows, const ChainDev *chains, const ReqPartial *cpart,
                          const QRes *res, const uint64_t *hoff, const uint64_t *hits, uint64_t rec_base,
                          uint64_t *tsum, uint64_t *row_off, uint64_t *out, hipStream_t s);

// General records (devtypes.hpp GenRec): one wave per slice of the work list
// (work[0] = count, then launch indices into st.q_all) written by the scan
// kernels; `grid` single-wave workgroups loop over it, each with
// general_wave_bytes() of scratch.  Slices whose counts need more than 64
// bits append {orig} to big (count in *big_n, at most big_cap) and their
// limbs to big_limbs (2 x kGenAccMax u32 per entry: call_count, all_alleles_count).
uint64_t general_wave_bytes(const GStore &gs, uint32_t *hwords, uint32_t *tcap);
void launch_general(const DStore &st, const GStore &gs, const uint32_t *work, uint32_t grid, const uint8_t *qbytes,
                    const uint64_t *subsets, QRes *res, uint64_t *hits, uint64_t *samples_out, uint8_t *scratch,
                    uint32_t *big_n, GenBig *big, uint32_t *big_limbs, uint32_t big_cap, hipStream_t s);

// Request batches (devtypes.hpp RowRun): rows + row offsets + dense hits in
// row order, one wave per run, offsets by decoupled look-back (ticket and
// status zeroed by the caller; status n_runs words).  sres..shits: the
// batch's per-slice part (rows of it already reduced into `rows`), or null.
void launch_request_rows(const DStore &st, const ReqChain *chains, RowRun *runs, uint32_t n_runs,
                         unsigned long long *status, unsigned long long *tstatus, const QRes *sres,
                         const uint32_t *sseg, const uint64_t *shoff, const uint8_t *sherr, const uint64_t *shits,
                         ReqPartial *rows, uint64_t *row_off, uint64_t *row_src, uint32_t *stage, uint64_t *out,
                         uint32_t n_rows, uint64_t rec_base, uint32_t n_lut, uint32_t run, unsigned int *err,
                         int compact, bool rec_staged, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                         const ReqIn *plan_in, uint32_t n_in, uint64_t stride, int inject, bool tile_scan,
                         const ReqEsc &esc, bool lab7);
// lab7: the store holds a record with 8 ALTs (a chain hit can carry the label
// 7, which the compact hit form escapes; store_has_label7)
// chain slots per run (kReqRun)
uint32_t req_run_max();
// Request planning on the device: rows in runs of kRunRows (n_runs =
// ceil(n / 64)); chains gets kReqRun ReqChain slots per run, runs the RowRuns
// with staging offsets, rcap one word per run; counters (4 words, zeroed by
// the caller) = chain rows, their slices, the staging total, the largest run
// capacity.  stride != 0 (a re-planning pass of a batch laid out at a fixed
// stride): run w stages at w x stride, no staging scan, *err bit 0 when a
// run would not fit.
void launch_request_plan(const DStore &st, const ReqIn *in, uint32_t n, ReqChain *chains, RowRun *runs,
                         unsigned long long *rcap, unsigned long long *counters, hipStream_t s, uint64_t stride = 0,
                         unsigned int *err = nullptr);
size_t request_plan_words(uint32_t n_runs);  // planning scratch: per-run and per-workgroup totals + counters
uint32_t request_tiles(uint32_t n_runs);
size_t request_tstatus_words(uint32_t n_runs);  // tile offsets + eval workgroup totals

// Fetch-time gather of every query's hits into one dense array.
void launch_compact(const uint64_t *hit_off, const uint64_t *dense_off, const QRes *res, uint32_t nq,
                    const uint64_t *hits, uint64_t *out, hipStream_t s);

// duplicateVariantSearch (dedup_kernels.hip).  gather takes host-planned
// tiles (segment, key offset) of dedup_gather_tile() keys and splits each
// tile's keys into the exact stream ke (words only) and the hashed stream
// (kh, key ids vh), compacted at the start of the tile's own slot region;
// tcnt[t] / tcnt[ntiles + t] = the tile's exact / hashed counts.  pos_bits = 0
// disables the exact stream; mask trims the hash (tests force collisions).
// The radix sort ping-pongs (k0, v0) <-> (k1, v1) over ceil(bits / 8) passes
// (v0 = nullptr: keys only; tile_n = the per-tile counts of a gathered,
// sparse input, made dense by the first pass) and returns 1 when the result
// ends in (k1, v1); hist needs 256 words per tile of the largest pass and
// bsum radix_bsum_words of that.  unique writes per-block partial counts
// part[b] = {job_first, n_first, job_last, n_last} (jobs strictly inside a
// block are added into counts[]); with verify it confirms equal words on the
// key strings and lists (into coll, capacity n) every sorted position whose
// string differs from its equal-word neighbour.
size_t radix_hist_words(uint64_t n);
size_t radix_bsum_words(uint64_t n);
uint32_t dedup_gather_tile();
uint32_t dedup_unique_blocks(uint64_t n);
void launch_dedup_gather(const KStore &ks, const KSeg *segs, const uint2 *tiles, uint32_t ntiles, uint32_t pos_bits,
                         uint32_t exact_job_shift, uint32_t job_bits, uint64_t mask, uint64_t *ke, uint64_t *kh,
                         uint32_t *vh, uint32_t *tcnt, hipStream_t s);
int launch_radix_sort(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t bits,
                      uint32_t *hist, uint32_t *bsum, hipStream_t s, const uint32_t *tile_n = nullptr,
                      uint32_t sparse_tiles = 0);
// a stream by hash buckets instead of a full sort (exact words; or, with
// vals = key ids, the hashed stream, equal words confirmed on the strings and
// any collision raising *overflow): two radix passes on
// the top 16 bits of a mix of the word, then an LDS hash set per workgroup
// of buckets adds each job's distinct words to counts[job].  Sets
// *overflow (leaving counts partial) when a workgroup's buckets outgrow its
// set: the caller then recounts the stream with the radix path.
int launch_bucket_dedupe(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, const KStore &ks,
                         uint32_t job_shift, uint32_t nj, unsigned long long *counts, uint32_t *overflow,
                         uint32_t *hist, uint32_t *bsum, hipStream_t s, const uint32_t *tile_n, uint32_t sparse_tiles);
// window dedup: dedup_plan_kernel cuts every job (devtypes.hpp KJob; nj of
// them, windows [w0, w0 + nw) each, nw in all) into window records (rec:
// nw records of rec_words u32 each = the KWin header, then each run's piece
// [lo, hi) of the window's keys; rec_words = kWinRecHead + 2 x the call's
// largest run count, rounded to 4); then one workgroup per window (runs at most kWinPieces, keys at most
// kWinCap), then one lane per deferred displaced key (list: cap entries,
// *n_list zeroed by the caller; runs = every job's KRun table); adds each
// job's distinct keys to counts[job] (each window's count to wfresh[w], nw
// entries, then one fold per job); *overflow = the window path cannot
// answer this call exactly
void launch_window_dedupe(const KStore &ks, const KJob *jobs, uint32_t nj, uint32_t *rec, uint32_t rec_words, uint32_t nw,
                          const KRun *runs, unsigned long long *counts, uint2 *list, uint32_t *n_list, uint32_t cap,
                          uint32_t *overflow, uint32_t *wfresh, hipStream_t s);
void launch_dedup_unique(const uint64_t *keys, const uint32_t *vals, uint64_t n, const KStore &ks, uint32_t job_shift,
                         bool verify, unsigned long long *counts, uint4 *part, uint32_t *coll, uint32_t *ncoll,
                         hipStream_t s);

}  // namespace sb
