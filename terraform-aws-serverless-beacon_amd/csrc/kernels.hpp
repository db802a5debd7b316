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
// = 0 compiles out the sample path; nonneg selects the monotone call_count path.
void launch_scan(const DStore &st, const QDev *q, const uint32_t *qidx, uint32_t n, bool nonneg, uint32_t max_words,
                 const uint8_t *qbytes, const uint64_t *subsets, QRes *res, uint64_t *hits, uint64_t *samples_out,
                 hipStream_t s);

// summariseSlice: one workgroup per slice — a reduction of the records'
// (numVariants, numCalls) contributions plus an overshoot bitmap, then one
// wave replays the skip heuristic over the (rare) overshooting records.
// bitmap needs sum over slices of ceil((hi - lo) / 256) * 4 words.
void launch_summarise(const SStore &ss, const SDev *slices, uint32_t ns, uint64_t *bitmap, SRes *out,
                      hipStream_t s);

// Fetch-time gather of every query's hits into one dense array.
void launch_compact(const QDev *q, const uint64_t *dense_off, const QRes *res, uint32_t nq, const uint64_t *hits,
                    uint64_t *out, hipStream_t s);

}  // namespace sb
