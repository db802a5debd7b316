// store.hpp — host-side columnar variant store and its HBM image.
//
// Built once at ingest from VCF text (what bcftools would have decoded per
// slice, lambda/performQuery/search_variants.py:42-50), then uploaded to one
// device and queried by query_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

// a HIP runtime call that must succeed (sb::Error SB_EHIP otherwise)
#define HIP_OK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            throw ::sb::Error(SB_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

#include "devtypes.hpp"

namespace sb {

struct Segment {  // one (vcf, contig), position-sorted, contiguous records
    std::string contig;
    uint32_t lo = 0, hi = 0;  // record range (vcf-local while building, global in a store)
};

// Columns of one VCF (vcf-local indices while building).
struct VcfCols {
    // record-indexed
    std::vector<RecHot> rec;
    std::vector<RangeHot> rng;
    std::vector<uint32_t> pos, a0_len, x_lo{0};
    std::vector<uint64_t> ref_key, a0_key, ref_off, a0_off;
    std::vector<int64_t> fb_off;
    std::vector<uint16_t> vt;  // VT dictionary id (host-side formatting only)
    // extra-ALT rows (ALT index >= 1)
    std::vector<uint32_t> x_cls, x_len;
    std::vector<int32_t> x_ac;
    std::vector<uint64_t> x_key, x_off;
    // bulk
    std::vector<uint8_t> blob;
    std::vector<uint64_t> planes0;  // [record][words]
    std::vector<uint64_t> planesx;  // [extra row][words]
    std::vector<uint32_t> fb;       // [fallback row][n_samples]
    bool any_negative = false;      // some INFO AC entry < 0
    // summariseSlice columns (record-indexed)
    std::vector<uint64_t> start;    // absolute line start in the VCF text stream
    std::vector<SumHot> sum;
    std::vector<uint32_t> cur, dcount;
    // duplicateVariantSearch keys: one per region-file entry (record x ALT,
    // write_data_to_s3.h:150-228), in record order
    std::vector<uint32_t> dk_pos, dk_lo{0};  // dk_lo: first key of each record (+ end)
    std::vector<uint64_t> dk_hash, dk_tail;   // hash of the key string; tail word (devtypes.hpp)
    std::vector<uint8_t> dk_blob;             // tails longer than 7 bytes
    std::vector<uint32_t> dk_bad;             // records where compressSeq would throw
    // general records (devtypes.hpp GenRec; vcf-local rec / number / token /
    // value indices until upload): numbers are variable-length two's
    // complement limbs here (gnum_off[k] .. gnum_off[k + 1])
    std::vector<GenRec> gen;
    std::vector<uint64_t> gnum_off{0};
    std::vector<uint32_t> gnum;
    std::vector<uint64_t> gtok_off;
    std::vector<uint32_t> gtok;
    std::vector<GenVal> gval;
};

struct BucketIndex {  // coarse POS index of one segment
    uint64_t off = 0;    // into the store's bucket array
    uint32_t base = 0;   // POS of the segment's first record
    uint32_t shift = 0;  // bucket width = 1 << shift bp
    uint32_t n = 0;      // buckets; bucket[off + n] = segment end
};

// a source file of a VCF (sb_builder_add_file): what sb_store_open checks
// to tell whether the persisted store still describes it
struct SourceFile {
    std::string path;
    uint64_t size = 0;
    int64_t mtime_ns = 0;
    uint64_t sample_hash = 0;  // of the first and last 64 KiB
};
SourceFile fingerprint(const std::string &path);  // persist.cpp

struct VcfData {
    std::string location;
    std::vector<SourceFile> sources;  // the files it was read from (none: text)
    // shard builds (sb_builder_set_record_range): keep records [rec_lo, rec_hi) of the file
    uint64_t rec_lo = 0, rec_hi = UINT64_MAX, lines_seen = 0;
    std::vector<std::string> samples;
    // name -> header indices (built at upload; bcftools --samples lookups)
    std::unordered_map<std::string, std::vector<uint32_t>> sample_pos;
    uint32_t words = 0;  // ceil(n_samples / 64)
    bool header_seen = false;
    std::vector<Segment> segments;
    std::unordered_map<std::string, uint32_t> seg_index;
    std::vector<BucketIndex> buckets;  // parallel to segments (set by finish)
    std::vector<std::array<VcIndex, kVtKinds>> vc_index;  // parallel to segments (set by finish)
    uint32_t seg_base = 0;  // store-wide index of segment 0 (DStore::vcx rows)
    VcfCols c;
    std::string carry;  // partial line kept between add_text calls
    uint64_t stream_off = 0;  // text bytes consumed so far (incl. carry)
    // BGZF block table (compressed offset, uncompressed start) incl. the EOF
    // block, for virtual-offset -> stream-offset conversion; empty for text
    std::vector<uint64_t> blk_coff, blk_ustart;
    uint64_t stream_len = 0;
    // global placement (set by finish)
    uint32_t rec_base = 0, x_base = 0;
    uint64_t plane0_base = 0, planex_base = 0;
    bool nonneg = true;
    bool has_planes = false;
    // RangeHot8 usable (>= 98 % of the single-base-ALT records fit it), AN value
    bool range8 = false;
    int32_t an_default = 0;
};

// CHROM / POS of a VCF's records without a store (shard planning)
struct VcfScan {
    struct Contig {
        std::string name;
        uint64_t lo, hi;  // records [lo, hi) in file order
    };
    std::vector<Contig> contigs;
    std::vector<uint32_t> pos;
};

struct Dict {
    std::vector<std::string> items;
    std::unordered_map<std::string, uint32_t> index;
    uint32_t get(const std::string &s) {
        auto it = index.find(s);
        if (it != index.end()) return it->second;
        const uint32_t id = static_cast<uint32_t>(items.size());
        items.push_back(s);
        index.emplace(s, id);
        return id;
    }
};

struct DeviceBuffer {
    void *p = nullptr;
    size_t bytes = 0;
};

}  // namespace sb

struct sb_builder {
    sb_build_opts opts{};
    std::vector<sb::VcfData> vcfs;
    sb::Dict vt;   // id 0 = "N/A" (no VT= tag, search_variants.py:193)
    sb::Dict sym;  // symbolic ALT strings
};

struct sb_store {
    // the open handle + every live batch and result set (sb_store_close
    // defers the teardown until the last of them is freed)
    std::atomic<uint32_t> holders{1};
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;  // serialises batches on this device
    std::shared_ptr<void> dedup_ws;      // dedup scratch (api.cpp DedupWs), reused across calls
    std::shared_ptr<void> win_ws;        // window-dedup scratch (api.cpp WinWs)
    std::shared_ptr<void> summarise_ws;  // summariseSlice scratch (api.cpp SumWs)
    std::shared_ptr<void> req_pool;      // request batches' pinned / device buffers (api.cpp ReqPool)
    std::shared_ptr<void> region_cache;  // strict dedup: slices' region files (api.cpp RegionCache)
    std::once_flag req_pool_once;
    std::shared_ptr<void> var_text;      // wire: escaped variant-string tails (api.cpp VarText)
    std::once_flag var_text_once;
    std::once_flag label7_once;  // request batches: some chain record has 8 ALTs (label 7; requests.cpp)
    bool label7 = false;
    std::vector<sb::VcfData> vcfs;  // metadata (columns are moved to the globals below)
    std::unordered_map<std::string, uint32_t> vcf_by_location;
    sb::Dict vt, sym;
    uint64_t n_records = 0, n_extra = 0;
    uint32_t max_words = 0;
    // host copies needed to plan outputs and format results (global indexing)
    std::vector<uint32_t> h_pos, h_end, h_a0_len, h_x_lo, h_x_len, h_bucket;
    std::vector<uint16_t> h_vt;
    std::vector<uint32_t> h_vt_slow;  // records whose VtHot word is VT_SLOW (sorted; chain planning)
    // per (vcf, segment): POS of its VT_SLOW records, sorted (request batches:
    // a request whose window holds one is answered per slice)
    std::vector<std::vector<std::vector<uint32_t>>> seg_slow_pos;
    std::vector<uint32_t> h_vc_pos, h_vc_bucket;  // candidate POS + coarse candidate index (chain statistics)
    std::vector<uint64_t> h_vc_altpre;  // ALTs of candidates [0, j) (chain hit capacity)
    std::vector<uint64_t> h_ref_off, h_a0_off, h_x_off;
    std::vector<uint8_t> h_blob;
    std::vector<uint64_t> h_start;  // line start in the VCF text stream (summariseSlice planning)
    // the summariseSlice reader walk on the host (region files): rem, cursor,
    // delimiter count and the unsupported flag of every record
    std::vector<uint32_t> h_rem, h_cur, h_dcount;
    std::vector<uint8_t> h_sum_bad;
    // duplicateVariantSearch keys (global indexing): planning + collision fixup
    uint64_t n_keys = 0;
    std::vector<uint32_t> h_dk_pos, h_dk_lo, h_dk_bad;
    std::vector<uint64_t> h_dk_tail;
    std::vector<uint8_t> h_dk_blob;
    // general records (GenRec side table): device image + sizes
    sb::GStore g{};
    // device image
    sb::DStore d{};
    sb::SStore ds{};
    sb::KStore dk{};
    std::vector<sb::DeviceBuffer> bufs;
    uint64_t device_bytes = 0;
    ~sb_store();
};
