// kernels.hpp — host-callable launchers for the HIP kernels in query_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devtypes.hpp"

namespace sb {

// Wave-cooperative 64-ary lower/upper bound of every slice query over its
// (vcf, contig) segment; writes [lo, hi) record bounds and the alt-row
// capacity (upper bound on hits) per query.
void launch_bounds(const DStore &st, const QDev *q, uint32_t nq, uint32_t *lohi, uint32_t *caps,
                   hipStream_t s);

// Exclusive prefix sum u32 -> u64 (out has n + 1 entries; out[n] = total).
// tmp must hold scan_tmp_words(n) u64 words.
size_t scan_tmp_words(uint32_t n);
void launch_exclusive_scan(const uint32_t *in, uint32_t n, uint64_t *out, uint64_t *tmp, hipStream_t s);

// The range-scan kernel: per query, filters the records of [lo, hi) with the
// reference's predicates, reproduces its order-dependent early exits and
// writes compacted (record, alt) hits at hit_off[q], per-query totals and,
// for the sample path, a carrier bitset per query.
void launch_scan(const DStore &st, const QDev *q, uint32_t nq, const uint32_t *lohi,
                 const uint64_t *hit_off, const uint8_t *qbytes, const uint64_t *subsets,
                 uint32_t max_words, QRes *res, uint32_t *nhits, uint32_t *hit_rec, uint32_t *hit_alt,
                 uint64_t *samples_out, hipStream_t s);

// Gather per-query hit runs from their capacity-sized slots into a dense array.
void launch_compact(const uint64_t *hit_off, const uint64_t *dense_off, const uint32_t *nhits, uint32_t nq,
                    const uint32_t *hit_rec, const uint32_t *hit_alt, uint32_t *out_rec, uint32_t *out_alt,
                    hipStream_t s);

}  // namespace sb
