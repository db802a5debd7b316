/*
 * sbeacon.h — C ABI of the MI355X-native sBeacon variant-query engine
 * (libsbeacon_hip.so).
 *
 * Drop-in boundary for the reference's genomic-variant query path
 * (SURVEY.md §8b).  In the reference, each performQuery Lambda shells out to
 * `bcftools query --regions chrom:a-b ...` and filters the text in a Python
 * loop (lambda/performQuery/search_variants.py:33-271,
 * search_variants_in_samples.py:31-259).  Here the VCFs are ingested once into
 * a position-sorted columnar store resident in HBM and every slice query of a
 * request is answered by one batched HIP launch sequence.
 *
 * Conventions: every function returns 0 on success or a negative SB_E* code;
 * sb_last_error() then holds a thread-local message.  Strings are
 * (pointer, length) pairs — no NUL requirement.  The library owns everything
 * it returns until the matching *_free call.  Inputs are borrowed for the
 * duration of the call.  All entry points are re-entrant; concurrent queries
 * on one store are serialised per device internally, except request batches
 * (sb_requests_*): each owns its device buffers, so passes of different
 * batches on different streams overlap on the device.
 */
#ifndef SBEACON_H
#define SBEACON_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SB_ABI_VERSION 2

/* ---- error codes ------------------------------------------------------- */
enum {
    SB_OK = 0,
    SB_EINVAL = -1,     /* malformed argument / payload */
    SB_ENOSTORE = -2,   /* unknown vcf id / store not built */
    SB_EHIP = -3,       /* HIP runtime failure */
    SB_EIO = -4,        /* file / decompression failure */
    SB_EPARSE = -5,     /* VCF text the store cannot represent exactly */
    SB_ENOMEM = -6,
    SB_ESTALE = -7,     /* a persisted store's source VCF changed since it was saved */
    SB_EINTERNAL = -8,  /* a device pass failed its own consistency checks (a bug, never a wrong answer) */
};

/* per-query error: the Python exception the reference raises on this input
 * (sb_result_view.error); the query's other fields are then undefined */
enum {
    SB_QERR_NONE = 0,
    SB_QERR_UNBOUND_LOCAL = 1, /* search_variants.py:101 (variantType, strict mode) */
    SB_QERR_INDEX = 2,         /* search_variants.py:207 / :223 */
    SB_QERR_VALUE = 3,         /* search_variants.py:199 int(AN) / :206 int(AC) */
    SB_QERR_ATTRIBUTE = 4,     /* search_variants_in_samples.py:89 None.replace */
    SB_QERR_RUNTIME = 5,       /* a C++ runtime_error of the reference (readVcfData.cpp:35,50; gzip.cpp:85) */
    SB_QERR_UNSUPPORTED = 9,   /* regex metacharacters in referenceBases */
};

enum { SB_GRAN_BOOLEAN = 0, SB_GRAN_COUNT = 1, SB_GRAN_AGGREGATED = 2, SB_GRAN_RECORD = 3 };

const char *sb_last_error(void);
int sb_abi_version(void);

/* ---- store build (ingest) ---------------------------------------------- */
/* Replaces: the VCF-on-S3 + CSI/TBI + bcftools region retrieval the reference
 * performs per slice (search_variants.py:42-50; init.sh:73-91 builds htslib). */
typedef struct sb_builder sb_builder;
typedef struct sb_store sb_store;

typedef struct {
    int32_t keep_genotypes; /* build per-alt carrier bitplanes (sample path) */
    int32_t n_threads;      /* host parse threads (0 = all) */
} sb_build_opts;

int sb_builder_new(const sb_build_opts *opts, sb_builder **out);
/* register one VCF; `location` is the string payloads carry as vcf_location */
int sb_builder_begin_vcf(sb_builder *b, const char *location, size_t location_len, uint32_t *vcf_id);
/* feed VCF text (header and/or whole records; chunks must end on '\n') */
int sb_builder_add_text(sb_builder *b, uint32_t vcf_id, const char *text, size_t len);
/* convenience: plain or gzip/BGZF file from disk (zlib) */
int sb_builder_add_file(sb_builder *b, uint32_t vcf_id, const char *path);
/* genotypes of a sites-only VCF from a separate carrier bit-matrix (config 5,
 * gnomAD-shape sites + a cohort's genotypes): one row of ceil(n_samples/64)
 * u64 words per ALT in record-then-ALT order, bit s of ALT k = sample s has
 * a GT token equal to str(k+1) -- the set search_variants.py:233-236 collects
 * from GT text.  Call after the VCF's last text; every record needs AC and AN
 * (else SB_EINVAL: the reference's GT-count fallbacks, :215-226,:244-250,
 * need the GT text itself).  Replaces the `[%GT,]` columns bcftools would emit
 * (search_variants.py:45). */
int sb_builder_attach_carriers(sb_builder *b, uint32_t vcf_id, const char *const *names, const uint32_t *name_len,
                               uint32_t n_samples, const uint64_t *planes, uint64_t n_rows);
/* Shard builds (one rank's part of a VCF, sbeacon/sharding.py): keep only
 * records [lo, hi) of the file (0-based, file order); call before any text
 * of that VCF. */
int sb_builder_set_record_range(sb_builder *b, uint32_t vcf_id, uint64_t lo, uint64_t hi);
/* CHROM / POS of every record of a VCF file (plain, gzip or BGZF) without
 * building a store: the input of a shard plan.  Contigs in file order with
 * their record ranges [lo, hi); pos[r] = POS of record r. */
typedef struct sb_vcf_scan sb_vcf_scan;
int sb_vcf_scan_file(const char *path, sb_vcf_scan **out);
int sb_vcf_scan_info(const sb_vcf_scan *s, uint64_t *n_records, uint32_t *n_contigs, const uint32_t **pos);
int sb_vcf_scan_contig(const sb_vcf_scan *s, uint32_t i, const char **name, size_t *len, uint64_t *lo, uint64_t *hi);
void sb_vcf_scan_free(sb_vcf_scan *s);
/* upload to device `device` (HIP ordinal) and return an immutable store.
 * device = SB_HOST_ONLY builds every host-side column without a device
 * image (no HIP call): request planning, region files, CSI/TBI and
 * sb_store_save work on it; a query or pass returns SB_EHIP. */
#define SB_HOST_ONLY (-1)
int sb_builder_finish(sb_builder *b, int device, sb_store **out);
void sb_builder_free(sb_builder *b);
void sb_store_close(sb_store *s);
/* Free the device and pinned buffers a store keeps for reuse by request
 * batches (at most 64 of each, 4 GiB device / 2 GiB pinned; batches in
 * flight keep theirs). */
int sb_store_trim(sb_store *s);
/* Persisted stores.  sb_store_save writes the finished store to directory
 * `dir` (created if absent): manifest.json, host.bin (host columns, VCF
 * metadata) and device.bin (the device image; empty for a host-only store).
 * sb_store_open re-creates it on `device` (or SB_HOST_ONLY: the host side
 * only) from `dir` or `dir`/manifest.json without re-reading any VCF;
 * if a source file of the store (sb_builder_add_file) changed since the save
 * it returns SB_ESTALE and sb_last_error() lists the changed paths, one per
 * line -- re-ingest that store.  Replaces the reference's persisted ingest
 * state (region files in S3, lambda/summariseSlice/source/
 * write_data_to_s3.h:39-92; toUpdate in DynamoDB, main.cpp:360-438). */
int sb_store_save(sb_store *s, const char *dir);
int sb_store_open(const char *path, int device, sb_store **out);

typedef struct {
    uint64_t n_records;
    uint64_t n_alt_rows;
    uint32_t n_vcfs;
    uint32_t n_segments; /* (vcf, contig) position-sorted segments */
    uint64_t device_bytes;
    uint32_t max_samples;
    int32_t device;
} sb_store_info;
int sb_store_get_info(const sb_store *s, sb_store_info *out);
/* variantType candidates of every (segment, kind) list of the store and the
 * bytes of the two columns request_eval_kernel reads per candidate (the
 * 16-byte VcQ word and the 4-byte record id): the working set of the
 * config-3 request pass, to set against the 256 MiB Infinity Cache. */
int sb_store_candidates(const sb_store *s, uint64_t *n, uint64_t *bytes);
/* vcf id for a vcf_location string, or SB_ENOSTORE */
int sb_store_find_vcf(const sb_store *s, const char *location, size_t len, uint32_t *vcf_id);
int sb_store_n_samples(const sb_store *s, uint32_t vcf_id, uint32_t *n);
/* header-order sample name i of a VCF */
int sb_store_sample_name(const sb_store *s, uint32_t vcf_id, uint32_t i, const char **p, size_t *len);

/* ---- query batch --------------------------------------------------------
 * One sb_query = one PerformQueryPayload
 * (shared_resources/payloads/lambda_payloads.py:46-77) after splitQuery has
 * cut the request into 10 kb slices (lambda/splitQuery/lambda_function.py:74-110).
 * Strings: ptr == NULL means Python None. */
typedef struct {
    uint32_t vcf_id;
    uint32_t _pad0;
    const char *region; size_t region_len; /* "chrom:a-b" exactly as in the payload */
    int64_t end_min, end_max;
    const char *reference_bases; size_t reference_len;
    const char *alternate_bases; size_t alternate_len;
    const char *variant_type; size_t variant_type_len;
    int64_t variant_min_length, variant_max_length; /* max < 0 = infinity */
    uint8_t granularity;           /* SB_GRAN_* */
    uint8_t include_details;       /* splitQuery: includeResultsetResponses in {HIT, ALL} */
    uint8_t include_samples;       /* passthrough.includeSamples */
    uint8_t selected_samples_only; /* passthrough.selectedSamplesOnly -> samples variant */
    uint8_t strict_variant_type;   /* 1 = reproduce the reference's UnboundLocalError */
    uint8_t _pad1[3];
    const char *sample_names; size_t sample_names_len; /* ','-joined passthrough.sampleNames, NULL = ['_'] */
} sb_query;

typedef struct sb_result_set sb_result_set;

/* Runs the whole batch on the store's device.  Results stay valid until
 * sb_result_free. */
int sb_query_batch(sb_store *s, const sb_query *q, size_t nq, uint32_t flags, sb_result_set **out);

typedef struct {
    int32_t error;      /* SB_QERR_* */
    int32_t exists;
    int64_t call_count;
    int64_t all_alleles_count;
    uint64_t n_variants;      /* hits = (record, alt) pairs, reference order */
    const uint32_t *hit_record; /* global record ids */
    const uint32_t *hit_alt;    /* alt index used for the label (0-based) */
    uint64_t n_sample_indices;  /* indices into the emitted sample list */
    const uint32_t *sample_indices;
    /* Python ints are unbounded (search_variants.py:199,206,214,245): when
     * call_count or all_alleles_count needs more than 64 bits, both exact
     * values are here as big_limbs 32-bit limbs each, two's complement,
     * little-endian (the int64 fields then hold their low 64 bits);
     * big_limbs = 0 otherwise */
    uint32_t big_limbs;
    uint32_t _pad;
    const uint32_t *big_call_count;
    const uint32_t *big_all_alleles_count;
} sb_result_view;

int sb_result_get(const sb_result_set *r, size_t i, sb_result_view *out);
/* views of queries 0 .. n-1 in one call (n <= the batch's queries) */
int sb_result_get_all(const sb_result_set *r, sb_result_view *out, size_t n);
/* Reference-format strings for query i: variants '\n'-joined
 * (f'{chrom}\t{POS}\t{REF}\t{ALT}\t{VT}', search_variants.py:210) and
 * sample names ','-joined.  Pointers valid until sb_result_free. */
int sb_result_variants_text(sb_result_set *r, size_t i, const char **p, size_t *len);
int sb_result_sample_names_text(sb_result_set *r, size_t i, const char **p, size_t *len);
/* The g_variants route aggregation (lambda/getGenomicVariants/
 * route_g_variants.py:153-171: variants.update(...) over the responses) in
 * the library: the distinct variant strings of the listed queries (errored
 * queries skipped), '\n'-joined in first-seen order, *count of them.
 * Pointer valid until the next call on r or sb_result_free. */
int sb_result_distinct_variants(sb_result_set *r, const uint32_t *queries, size_t n, const char **p, size_t *len,
                                uint64_t *count);

typedef struct {
    uint64_t n_queries;
    uint64_t records_scanned; /* records with POS inside each slice, summed */
    uint64_t hits;
    double device_ms;         /* HIP-event time of the kernel sequence */
    uint64_t chained_slices;  /* slices answered by the chain kernel (one chain = one request's slices) */
    uint64_t chains;
    /* variantType candidates of the chains: read from the coarse-index superset
     * (cand_loaded), inside the chain windows (cand_window), and in the union
     * of the windows (cand_unique: each candidate counted once) */
    uint64_t cand_loaded, cand_window, cand_unique;
} sb_batch_stats;
int sb_result_stats(const sb_result_set *r, sb_batch_stats *out);
void sb_result_free(sb_result_set *r);

/* ---- summariseSlice --------------------------------------------------------
 * One sb_slice = one summariseSlice SNS message {"location", "virtual_start",
 * "virtual_end"} (lambda/summariseSlice/source/main.cpp:446-453); the result
 * is its RegionStats {numVariants, numCalls} (main.cpp:43-49, 195-245),
 * including the reference's record-skip heuristic (main.cpp:226,234-235).
 * The VCF must have been ingested from its BGZF file (sb_builder_add_file)
 * so virtual offsets resolve.  Slices must start on a record and must not cut
 * one (CSI/TBI chunk boundaries do neither); otherwise error =
 * SB_QERR_UNSUPPORTED. */
typedef struct {
    uint32_t vcf_id;
    uint32_t _pad;
    uint64_t virtual_start, virtual_end; /* BGZF virtual offsets (coffset << 16 | uoffset) */
} sb_slice;

typedef struct {
    int32_t error;
    int32_t _pad;
    uint64_t num_variants;
    uint64_t num_calls;
    uint64_t records; /* records the reference reader visits */
} sb_slice_stats;

/* device_ms (optional): HIP-event time of the summarise kernel */
int sb_summarise_slices(sb_store *s, const sb_slice *slices, size_t n, sb_slice_stats *out, double *device_ms);
/* BGZF block count and text-stream length of an ingested VCF */
int sb_store_vcf_stream(const sb_store *s, uint32_t vcf_id, uint64_t *n_blocks, uint64_t *stream_len);
/* contigs (CHROM values) of an ingested VCF, in file order */
int sb_store_n_contigs(const sb_store *s, uint32_t vcf_id, uint32_t *n);
int sb_store_contig_name(const sb_store *s, uint32_t vcf_id, uint32_t i, const char **p, size_t *len);
/* Chunk boundaries of one contig for summariseVcf's partition_chunks
 * (lambda/summariseVcf/lambda_function.py:90-104,197-214): the virtual
 * offsets of every stride-th record start of the contig, then the offset just
 * past its last record.  The reference takes them from the CSI/TBI index
 * (chunk_beg/chunk_end of non-pseudo bins), which are record starts too; the
 * store knows every record start.  *n = count (voffs gets min(count, cap)). */
int sb_store_chunk_boundaries(const sb_store *s, uint32_t vcf_id, const char *contig, size_t contig_len,
                              uint32_t stride, uint64_t *voffs, size_t cap, size_t *n);

/* ---- summariseSlice region files ---------------------------------------------
 * What summariseSlice writes to S3 besides its counts
 * (lambda/summariseSlice/source/write_data_to_s3.h:30-228): one entry
 * {pos u64 LE, len u16 LE, ref' '_' alt'} per ALT of every record the reader
 * visits (skip heuristic included), split into files at POS gaps above
 * MAX_SLICE_GAP (100,000) and above VCF_S3_OUTPUT_SIZE_LIMIT (50,000,000)
 * entries (main.tf:17,215-216).  A file's S3 key is
 * vcf-summaries/contig/{CHROM}/{bucket%key}/regions/{first_pos}-{last_pos}-{bytes}
 * (the caller formats it; contig = index into sb_store_contig_name).
 * with_data = 1: the files' uncompressed bytes are concatenated in file order;
 * with_data = 2: the bytes of each file as the reference stores it -- one
 * gzip member (level 9, header name "c", write_data_to_s3.h:49-67 /
 * gzip.cpp:19-59) per buffer, a buffer closed when the next entry's
 * pos + ref' + alt' bytes would take it past VCF_S3_OUTPUT_SIZE_LIMIT.
 * data_bytes = the file's length in the data buffer.  status[i] =
 * SB_QERR_UNSUPPORTED for a slice the reference throws on (compressSeq of an
 * IUPAC code, reads past a line) or that is not record-aligned. */
typedef struct {
    uint32_t slice;     /* index into the slices argument */
    uint32_t contig;    /* contig index of the slice's VCF */
    uint64_t first_pos, last_pos;
    uint64_t bytes;     /* uncompressed file length (the S3 key's last field) */
    uint64_t entries;
    uint64_t data_bytes; /* this file's bytes in the data buffer (0 without data) */
} sb_region_file;
typedef struct sb_region_files sb_region_files;
int sb_slice_region_files(sb_store *s, const sb_slice *slices, size_t n, int with_data, int32_t *status,
                          sb_region_files **out);
int sb_region_files_get(const sb_region_files *r, const sb_region_file **files, size_t *n, const uint8_t **data,
                        size_t *data_len);
void sb_region_files_free(sb_region_files *r);

/* ---- duplicateVariantSearch -------------------------------------------------
 * One sb_dedup_job = one duplicateVariantSearch SNS message {"rangeStart",
 * "rangeEnd", "contig", "targetFilepaths", "dataset"} (lambda/
 * duplicateVariantSearch/source/main.cpp:31-43) with its region files named
 * by the VCFs they summarise.  unique = |{ to_string(pos) + ref'_alt' }| over
 * every region-file entry (record x ALT, write_data_to_s3.h:150-228) of those
 * VCFs on `contig` with range_start <= pos <= range_end
 * (duplicateVariantSearch.cpp:31-84, readVcfData.cpp:3-38; see DESIGN.md for
 * the reference's end-of-file range quirk this does not reproduce).  A job
 * over VCFs of several datasets is a cross-dataset union count.  Jobs whose
 * range holds a record the reference's summariseSlice would throw on
 * (compressSeq of an IUPAC code, write_data_to_s3.h:103-134) get
 * status SB_QERR_UNSUPPORTED. */
typedef struct {
    const uint32_t *vcf_ids;
    uint32_t n_vcf;
    uint32_t contig_len;
    const char *contig; /* CHROM text, length-delimited */
    uint64_t range_start, range_end; /* inclusive */
} sb_dedup_job;

typedef struct {
    uint64_t keys;        /* keys gathered and sorted (all jobs) */
    uint64_t collisions;  /* equal 64-bit words holding different strings (recounted on the host) */
    double device_ms;     /* HIP-event time of the device part */
    uint32_t path;        /* SB_DEDUP_WINDOWS (one read per key), SB_DEDUP_BUCKETS, SB_DEDUP_RADIX */
    uint32_t windows;     /* window workgroups launched (window path) */
} sb_dedup_stats;
enum { SB_DEDUP_WINDOWS = 0, SB_DEDUP_BUCKETS = 1, SB_DEDUP_RADIX = 2 };

/* unique[i] / status[i] per job; stats optional */
int sb_dedup_count(sb_store *s, const sb_dedup_job *jobs, size_t n_jobs, uint64_t *unique, int32_t *status,
                   sb_dedup_stats *stats);

/* Reference-exact duplicateVariantSearch over region FILES (the message's
 * targetFilepaths, duplicateVariantSearch/source/main.cpp:31-43): unique[i] =
 * |union over the job's files of ReadVcfData::getVcfData(file, rangeStart,
 * rangeEnd)| (duplicateVariantSearch.cpp:31-84, readVcfData.cpp:3-71): per
 * file, every entry with pos >= rangeStart that the reader reaches -- it
 * keeps reading while the gzip stream has more data, and only in the last
 * decompressed 1 KiB window stops after the first entry past rangeEnd, so
 * entries past rangeEnd are counted as the reference counts them.  A file is
 * named by the summariseSlice message that wrote it (vcf, virtual offsets)
 * and its index among that slice's region files (sb_slice_region_files
 * order); its bytes are the ones sb_slice_region_files(with_data = 2) emits.
 * status[i] = SB_QERR_RUNTIME where the reference's getVcfData throws (an
 * entry skipped below rangeStart straddling a 1 KiB window, a truncated
 * entry), SB_QERR_UNSUPPORTED where that summariseSlice throws. */
typedef struct {
    uint32_t vcf_id;
    uint32_t file;       /* index among the slice's region files */
    uint64_t virtual_start, virtual_end;
} sb_region_ref;

typedef struct {
    const sb_region_ref *files;
    uint32_t n_files;
    uint32_t _pad;
    uint64_t range_start, range_end;
} sb_dedup_file_job;

int sb_dedup_count_files(sb_store *s, const sb_dedup_file_job *jobs, size_t n_jobs, uint64_t *unique, int32_t *status,
                         sb_dedup_stats *stats);

/* ---- CSI / TBI index of a BGZF VCF (host only, no device) -----------------
 * The index summariseVcf reads its chunk boundaries from
 * (lambda/summariseVcf/lambda_function.py:90-104 get_chunk_boundaries,
 * :144-156 get_vcf_index; index_reader.py:4-125 Csi / Tbi), in the place of
 * the one `bcftools index` / `tabix -p vcf` writes next to the VCF: the same
 * binning and chunk boundaries, not byte-identical to htslib's file (linear
 * index fill and bin loff differ; see csrc/index.cpp).
 * min_shift <= 0 -> 14; depth <= 0 -> 5 for TBI, and for CSI the smallest
 * depth >= 5 covering the longest record.  *out = the BGZF-compressed index
 * (release with sb_free).  SB_EINVAL for an unsorted VCF or a position past
 * the index's range. */
enum { SB_INDEX_CSI = 0, SB_INDEX_TBI = 1 };
int sb_index_vcf(const char *path, int fmt, int min_shift, int depth, uint8_t **out, size_t *out_len);
void sb_free(void *p);

/* ---- performQuery at the wire -------------------------------------------
 * The performQuery Lambda (lambda/performQuery/lambda_function.py:23-49) for
 * a batch of events: event i is the JSON text text[offsets[i] ..
 * offsets[i + 1]) -- a PerformQueryPayload (shared_resources/payloads/
 * lambda_payloads.py:46-77) or its SNS envelope (Records[0].Sns.Message).
 * Each event's vcf_location picks the store that holds it; every store's
 * events are answered by one sb_query_batch.  Response i is the JSON text of
 * the handler's return value, json.dumps(response.dump())
 * (lambda_responses.py:14-23; ensure_ascii escapes, ", " / ": "
 * separators), or {"errorMessage", "errorType"} where the reference raises
 * from the query.  status[i] = 1 (no text) marks an event outside the typed
 * fast path -- a field of an unexpected JSON type, a key the payload does not
 * take, a vcf_location no store holds, invalid UTF-8 -- for the caller to
 * answer through the Python handler, which reproduces the reference's
 * behaviour.  flags bit 0: strict variantType (the reference's
 * UnboundLocalError).  Output: JSON lines -- response i is buf[offsets[i] ..
 * offsets[i + 1] - 1), each followed by '\n' (empty for status 1); release it
 * with sb_json_out_free. */
typedef struct sb_json_out sb_json_out;
int sb_perform_query_events(sb_store *const *stores, size_t n_stores, const char *text, const uint64_t *offsets,
                            size_t n, uint32_t flags, sb_json_out **out);
int sb_json_out_get(const sb_json_out *o, const char **buf, size_t *len, const uint64_t **offsets,
                    const uint8_t **status);
void sb_json_out_free(sb_json_out *o);

typedef struct sb_batch sb_batch;

/* One request row: the route-level sums of its slices' performQuery
 * responses (lambda/getGenomicVariants/route_g_variants.py:144-171). */
typedef struct {
    int64_t exists;            /* slices whose response has exists = True */
    int64_t n_variants;        /* variant strings emitted (hits) */
    int64_t call_count;
    int64_t all_alleles_count;
    int64_t errors;            /* slices whose performQuery raised */
} sb_request_partial;

/* ---- split-query requests (the splitQuery fan-out in the library) ---------
 * One sb_request = one SplitQueryPayload (shared_resources/payloads/
 * lambda_payloads.py:8-44) for ONE of its vcf_locations: the VCF and the
 * contig (index into sb_store_contig_name) its chrom maps to.  The library
 * cuts it into splitQuery's 10 kb slices (lambda/splitQuery/
 * lambda_function.py:74-110: [s, min(s + 9999, start_max)] for s =
 * start_min, start_min + 10000, ...) and answers each as performQuery would;
 * include_details = check_all (include_datasets in {HIT, ALL}).  A contig
 * index the VCF lacks, or start_min > start_max, gives a row with no slices.
 * Every request is one ROW (sb_request_partial: the route-level sums of its
 * slices' responses, route_g_variants.py:144-171) with its hit list. */
typedef struct {
    uint32_t vcf_id;
    uint32_t contig;
    int64_t start_min, start_max; /* split_payload.start_min / start_max (inclusive) */
    int64_t end_min, end_max;
    const char *reference_bases; size_t reference_len;
    const char *alternate_bases; size_t alternate_len; /* NULL = None (variantType query) */
    const char *variant_type; size_t variant_type_len; /* NULL = None */
    int64_t variant_min_length, variant_max_length;    /* max < 0 = infinity */
    uint8_t granularity;           /* SB_GRAN_* */
    uint8_t include_details;       /* check_all */
    uint8_t include_samples;       /* passthrough.includeSamples */
    uint8_t selected_samples_only; /* passthrough.selectedSamplesOnly */
    uint8_t strict_variant_type;
    uint8_t _pad[3];
    const char *sample_names; size_t sample_names_len; /* ','-joined passthrough.sampleNames, NULL = ['_'] */
} sb_request;

/* Plan and upload a request batch (sb_batch_free releases it); its
 * sb_batch_get_stats().hits is the output capacity (hits). */
int sb_requests_prepare(sb_store *s, const sb_request *r, size_t n, sb_batch **out);

/* The same requests as columns -- no per-request struct, no per-request
 * string: what a batched caller holds (numpy columns, a parsed event
 * batch).  A numeric / flag column is an array of n values, or NULL to give
 * every request the `*_all` scalar after it.  A string column is a
 * dictionary of distinct values (sb_str, p == NULL = None) and a uint32 code
 * per request into it (codes NULL = every request takes dict[0]); a NULL
 * dictionary = None for every request.  start_min / start_max are required.
 * Replaces the per-SplitQueryPayload fan-out of split_query_sync
 * (lambda/splitQuery/lambda_function.py:74-110) for a whole batch. */
typedef struct {
    const char *p;
    size_t len;
} sb_str;

typedef struct {
    const uint32_t *vcf_id;  uint32_t vcf_id_all;
    const uint32_t *contig;  uint32_t contig_all;
    const int64_t *start_min, *start_max;
    const int64_t *end_min;  int64_t end_min_all;
    const int64_t *end_max;  int64_t end_max_all;
    const int64_t *variant_min_length;  int64_t variant_min_length_all;
    const int64_t *variant_max_length;  int64_t variant_max_length_all;
    const sb_str *reference_dict;    const uint32_t *reference_code;    uint32_t n_reference;
    const sb_str *alternate_dict;    const uint32_t *alternate_code;    uint32_t n_alternate;
    const sb_str *variant_type_dict; const uint32_t *variant_type_code; uint32_t n_variant_type;
    const sb_str *sample_names_dict; const uint32_t *sample_names_code; uint32_t n_sample_names;
    const uint8_t *granularity;           uint8_t granularity_all;
    const uint8_t *include_details;       uint8_t include_details_all;
    const uint8_t *include_samples;       uint8_t include_samples_all;
    const uint8_t *selected_samples_only; uint8_t selected_samples_only_all;
    uint8_t strict_variant_type;
} sb_request_columns;

int sb_requests_prepare_columns(sb_store *s, const sb_request_columns *c, size_t n, sb_batch **out);

/* The same batch straight from the route's query parameters: one row = one
 * /g_variants query against ONE VCF, turned into its SplitQueryPayload as
 * perform_variant_search_sync does (shared_resources/variantutils/
 * search_variants.py:179-197: start / end of one or two elements ->
 * start_min, start_max, end_min, end_max, each + 1), optionally restricted to
 * one shard's core: only the splitQuery slices (lambda/splitQuery/
 * lambda_function.py:74-110) whose (contig, first base) lies in [lo, hi) are
 * answered -- sbeacon.sharding.ShardPlan.slice_runs in the library, fused
 * into the packing pass (no per-request conversion by the caller).  Numeric
 * columns are the caller's int64 arrays as they are. */
typedef struct {
    uint32_t vcf_id;
    const int64_t *contig;         /* request contig code (n values) */
    const uint32_t *contig_map;    /* code -> contig index in the VCF (sb_store_contig_name); NULL = identity; */
    uint32_t n_contig_map;         /* a code past the map or mapped to UINT32_MAX: absent (no slices) */
    const int64_t *start, *start2; /* requestParameters start[0], start[1] (start2 NULL: one-element start) */
    const int64_t *end, *end2;     /* end[0], end[1] (end2 NULL: one-element end) */
    const int64_t *variant_type_code; /* into variant_type_dict (NULL: every row takes dict[0]) */
    const sb_str *variant_type_dict;  /* NULL = None for every row */
    uint32_t n_variant_type;
    const int64_t *variant_min_length; int64_t variant_min_length_all;
    const int64_t *variant_max_length; int64_t variant_max_length_all;
    sb_str reference_bases;        /* p NULL = None */
    sb_str alternate_bases;        /* p NULL = None (a variantType query) */
    uint8_t granularity;           /* SB_GRAN_* */
    uint8_t include_details;       /* includeResultsetResponses in {HIT, ALL} */
} sb_beacon_requests;

/* A shard's core in one VCF: slices whose (contig code, first base) is >=
 * (contig_lo, pos_lo) and < (contig_hi, pos_hi) -- contig codes as the
 * request columns carry them (the VCF's contig order, before contig_map: a
 * shard store may hold only some contigs).  contig_hi == UINT32_MAX: no
 * upper end; contig_lo == UINT32_MAX: an empty core. */
typedef struct {
    uint32_t contig_lo; int64_t pos_lo;
    uint32_t contig_hi; int64_t pos_hi;
} sb_shard_core;

/* core NULL: every slice.  The batch is sb_requests_prepare_columns's. */
int sb_requests_prepare_beacon(sb_store *s, const sb_beacon_requests *q, size_t n, const sb_shard_core *core,
                               sb_batch **out);
/* Enqueue one pass: answer every request, then write dev_rows[n]
 * (sb_request_partial), dev_row_off[n + 1] and the rows' hit lists densely
 * in request order: row w's hits ((record + rec_base) | alt << 32, the
 * reference's variant order) are dev_hits[row_off[w] .. row_off[w + 1]).
 * Device pointers on the store's device; sb_batch_sync waits, and
 * sb_batch_last_timing reports the passes' device time. */
int sb_requests_run(sb_batch *b, void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base);
/* Measurement: with on != 0 every pass also records events around its
 * request_eval_kernel launch (the dominant kernel); sb_batch_last_timing's
 * scan_ms then reports that kernel's average over the passes since the last
 * sync (total_ms stays the whole pass).  Off by default: the markers add
 * stream gaps. */
int sb_requests_time_eval(sb_batch *b, int on);
/* With on != 0 every pass of a device-planned batch (sb_requests_prepare_columns
 * / _beacon when the columns qualify) first re-runs the planning kernels
 * (request_plan_kernel: each chain's candidate range by a batched lower /
 * upper bound in its (segment, kind) index and its staging capacity;
 * request_stage_scan_kernel) from the packed requests the batch keeps in HBM
 * -- the whole device path of a request batch in one pass, with the sizes
 * the prepare already read back.  SB_EINVAL for a host-planned batch.
 * Replaces splitQuery's per-request fan-out (lambda/splitQuery/
 * lambda_function.py:74-110) as a device step. */
int sb_requests_set_replan(sb_batch *b, int on);
/* *fused = 1 when the batch's last pass planned each run inside
 * request_eval_kernel (a re-planning pass of a fixed-stride batch with
 * record staging and no per-slice part: no request_plan_kernel launch, the
 * chain descriptors never leave LDS), else 0.  Measurement: the eval
 * kernel's events then include the planning. */
int sb_requests_plan_fused(sb_batch *b, int *fused);
/* One row of the compact output (sb_requests_set_compact): the
 * sb_request_partial sums as u32 (no error count: compact batches have no
 * per-slice part, whose slices are the only ones that can raise). */
typedef struct {
    uint32_t exists, n_variants, call_count, all_alleles_count;
} sb_request_row32;
/* Output widths of sb_requests_run.  SB_COMPACT_ALL: the narrow form a host
 * copy-back wants -- dev_rows[n] as sb_request_row32 (16 B instead of 40),
 * dev_row_off[n + 1] as uint32, and each hit as uint32 (record + rec_base) |
 * ALT label << 29.  SB_COMPACT_HITS: wide rows and offsets, uint32 hits as
 * above.  Either form holds every answer: a row the compact form cannot hold
 * (a sum past 32 bits, a slice that raised, a count past int64) is written as
 * {UINT32_MAX, n_variants, UINT32_MAX, UINT32_MAX} (SB_ROW32_ESCAPED) with its
 * wide sums kept by the batch (sb_requests_wide_rows); a hit whose ALT index
 * is 7 or more carries the label 7 (SB_HIT32_LABEL_ESCAPE) with its ALT index
 * kept by the batch (sb_requests_hit_labels); sb_requests_escapes says whether
 * the passes since the last sync wrote any.  Errors: SB_EINVAL at run when
 * record numbers reach 2^29; at sb_batch_sync, SB_EINVAL when the hit
 * offsets pass 32 bits (SB_COMPACT_ALL) or a per-slice ALT index passes 65,535.
 * 0: wide. */
#define SB_COMPACT_ALL 1
#define SB_COMPACT_HITS 2
int sb_requests_set_compact(sb_batch *b, int on);
#define SB_ROW32_ESCAPED 0xffffffffu
#define SB_HIT32_LABEL_ESCAPE 7u
/* After sb_batch_sync of compact passes: *rows = 1 when some row was written
 * escaped, *hits = 1 when some hit carries the escape label. */
int sb_requests_escapes(sb_batch *b, int *rows, int *hits);
/* The wide sums (sb_request_partial) of the listed rows of the last
 * SB_COMPACT_ALL pass whose compact row is SB_ROW32_ESCAPED. */
int sb_requests_wide_rows(sb_batch *b, const uint32_t *rows, size_t n, sb_request_partial *out);
/* The ALT index of the listed output hit positions of the last compact pass
 * whose label is SB_HIT32_LABEL_ESCAPE. */
int sb_requests_hit_labels(sb_batch *b, const uint64_t *pos, size_t n, uint32_t *out);
/* After a pass (waits for it): flags[w] = 1 when row w's call_count or
 * all_alleles_count is not exact in int64 -- a slice's count past 64 bits
 * (Python ints, records answered by the general path) or a sum that
 * overflows; the row then holds the low 64 bits of the exact value (the
 * per-slice results, sb_result_view.big_*, carry the exact limbs).
 * Replaces nothing in the reference (its counts are Python ints). */
int sb_requests_inexact_rows(sb_batch *b, uint8_t *flags);

/* ---- g_variants route bodies (the route aggregation in the library) ------
 * GET / POST /g_variants (lambda/getGenomicVariants/route_g_variants.py:
 * 49-208) for a batch of route events whose fan-out -- one request row per
 * (dataset, VCF) pair, perform_variant_search_sync's SplitQueryPayloads
 * (shared_resources/variantutils/search_variants.py:158-244) -- was answered
 * by a request pass (sb_requests_run).  Event e owns the consecutive rows
 * [row_lo, row_hi).  The route's aggregation (:153-171) over them:
 * exists = OR of the rows' exists; with check_all (includeResultsetResponses
 * in {HIT, ALL}) variants = the distinct strings
 * f'{chrom}\t{POS}\t{REF}\t{ALT}\t{VT}' of the rows' hits and one
 * get_variant_entry (shared_resources/apiutils/entries.py:1-24) per distinct
 * f'{assembly}\t{chrom}\t{pos}\t{ref}\t{alt}' (first-seen order); then the
 * body of get_boolean_response / get_counts_response / get_result_sets_response
 * (shared_resources/apiutils/responses.py:160-254) as json.dumps writes it
 * (the `body` of bundle_response, api_response.py:37-46).  status[e]: 0 =
 * body written; 1 = answer this event through the Python route (a row whose
 * slices raised -- the route re-raises --, a VCF with negative AC (the
 * route's completion-order gate on exists then matters), text that is not
 * UTF-8, an escaped compact row or hit); 2 = the route returns None
 * (another requestedGranularity). */
typedef struct {
    uint32_t row_lo, row_hi;  /* the event's request rows */
    uint8_t granularity;      /* SB_GRAN_*; 255 = any other requestedGranularity */
    uint8_t check_all;        /* includeResultsetResponses in {HIT, ALL} */
    uint8_t _pad[2];
    uint32_t assembly;        /* index into assembly_dict (assemblyId; p NULL = None) */
    uint32_t pagination;      /* index into pagination_dict: json.dumps of {'limit': .., 'skip': ..} */
} sb_route_event;

typedef struct {
    const sb_route_event *events;
    size_t n_events;
    /* per request row: its VCF and the contig index in it (NULL = the scalar) */
    const uint32_t *row_vcf;    uint32_t vcf_all;
    const uint32_t *row_contig; uint32_t contig_all;
    /* the pass's outputs in host memory: compact = 0 (sb_request_partial rows,
     * uint64 hits and row offsets) or SB_COMPACT_ALL (sb_request_row32, uint32) */
    int32_t compact;
    uint32_t _pad;
    const void *rows, *hits, *row_off;
    uint64_t rec_base;
    const sb_str *assembly_dict;   uint32_t n_assembly;
    const sb_str *pagination_dict; uint32_t n_pagination;
    sb_str beacon_id, api_version; /* BEACON_ID / BEACON_API_VERSION (the envelope's meta) */
} sb_route_input;

/* *out: JSON lines (sb_json_out_get; status as above), one per event. */
int sb_route_bodies(sb_store *s, const sb_route_input *in, sb_json_out **out);

/* ---- device-resident batch (benchmarks / fused pipelines) ----------------
 * Upload a batch once, then launch the query kernels repeatedly on the
 * store's stream with inputs already resident in HBM. */
int sb_batch_prepare(sb_store *s, const sb_query *q, size_t nq, sb_batch **out);
int sb_batch_run(sb_batch *b);               /* enqueue only (async) */
int sb_batch_sync(sb_batch *b);              /* wait for the store stream */
/* average device time (ms) per sb_batch_run since the previous sync: one
 * hipEvent before the first of those runs and one at the sync, on the launch
 * stream, divided by the run count (back-to-back runs, no marker between
 * them; work enqueued on the store stream in between is included).
 * total_ms = scan_ms = that time; bounds_ms = 0 (bounds are found inside the
 * scan kernels) */
int sb_batch_last_timing(const sb_batch *b, double *total_ms, double *scan_ms, double *bounds_ms);
int sb_batch_get_stats(const sb_batch *b, sb_batch_stats *out);
int sb_batch_fetch(sb_batch *b, sb_result_set **out); /* D2H + host views */

/* ---- per-request reduction (sharded fan-out) -------------------------------
 * The route-level aggregation of lambda/getGenomicVariants/route_g_variants.py
 * :144-171 (exists = OR over the request's performQuery responses; the
 * counts summed) for the slice queries one store (shard) holds, so that a
 * request whose slices live on several GPUs is answered by summing the
 * shards' rows (an RCCL reduce / gather).  owner[i] = row of query i (rows are
 * the caller's requests, 0 <= owner < n_rows, non-decreasing in query order).
 * sb_batch_reduce_requests enqueues, on the store's stream after the
 * preceding sb_batch_run, n_rows sb_request_partial rows into dev_out — a
 * device pointer on the store's device (e.g. a torch tensor's data_ptr);
 * sb_batch_sync waits for it.  Rows without a query are zero. */
int sb_batch_set_owners(sb_batch *b, const uint32_t *owner, size_t nq, uint32_t n_rows);
int sb_batch_reduce_requests(sb_batch *b, void *dev_out);
/* The hit lists that go with the rows (the `variants` of each request's
 * responses, route_g_variants.py:159-171): enqueues, after the preceding run,
 * dev_hits[row_off[w] .. row_off[w+1]) = row w's hits, each
 * (record + rec_base) | alt << 32 (rec_base: the shard's first global record,
 * so rows from several shards name records alike); dev_row_off = n_rows + 1
 * u64.  dev_rows (optional) = this run's sb_batch_reduce_requests output on
 * the same stream.  A row lists its queries' hits query by query, except that
 * when every chain of slices (one request's 10 kb slices answered together)
 * lies in one row the chain's hits come as one block at its first slice --
 * the same multiset; the route treats it as a set (route_g_variants.py:160).
 * Device pointers on the batch's device; dev_hits must hold
 * sb_batch_get_stats().hits (the planned capacity) entries. */
/* sb_batch_reduce_requests + sb_batch_compact_hits(rows = dev_rows) in one
 * call: with every chain in one request row the reduction also leaves each
 * row's n_variants densely, so the offset scan reads 8 B per row. */
int sb_batch_deliver(sb_batch *b, void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base);
/* Per-slice QRes rows of chained slices on (default) or off.  Off: a run
 * leaves only what the request rows and their hit lists need (per-chain
 * partials and dense chain hits; sb_batch_reduce_requests /
 * sb_batch_compact_hits), which requires every chain to lie in one request
 * row (sb_batch_set_owners); sb_batch_fetch then refuses until a run with
 * them on.  Not between a run and its sync. */
int sb_batch_set_slice_results(sb_batch *b, int on);
int sb_batch_compact_hits(sb_batch *b, const void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base);
/* Enqueue this batch's work (run, reduce, compact, and the timing events) on
 * `stream` -- a hipStream_t of the store's device, e.g. the caller's current
 * torch stream -- instead of the store's own stream, so it is ordered with the
 * caller's reads and writes of dev_out / dev_hits and with its collectives;
 * NULL restores the store's stream.  sb_batch_sync then waits for `stream`. */
int sb_batch_set_stream(sb_batch *b, void *stream);
void sb_batch_free(sb_batch *b);

#ifdef __cplusplus
}
#endif
#endif /* SBEACON_H */
