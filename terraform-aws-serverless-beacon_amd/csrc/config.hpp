// The library's knobs in one struct (SURVEY.md §5 "config"): every tuning
// parameter, test hook and diagnostic switch, with its default here and its
// SBEACON_* environment override.  sb::config() takes a snapshot of the
// environment (a few getenv calls): entry points read it when they start, so
// a test may switch a knob between two calls of one process.  None of these
// is set by the benches or the product handlers.
#pragma once
#include <cstdlib>
#include <string>

namespace sb {

struct Config {
    // ---- tuning
    double vc_bucket = 1.0;       // SBEACON_VC_BUCKET: variantType candidates per coarse-index bucket (>= 0.25)
    int pack_run = 0;             // SBEACON_PACK_RUN: chains per chain_pack_kernel run (0: the kernel's maximum)
    int slices_per_wave = 0;      // SBEACON_SLICES_PER_WAVE: slices per scan wave (0: by batch size)
    int dedup_win_target = 0;     // SBEACON_DEDUP_WIN_TARGET: keys per dedup window (0: kWinTarget)
    int dedup_bucket_cap = 0;     // SBEACON_DEDUP_BUCKET_CAP: keys per bucket hash set (0: 3/4 of its slots)
    int max_nacc = 16;            // SBEACON_MAX_NACC: sample words OR-ed per register window (16 / 4 / 1)
    // ---- paths (A/B and test coverage of the fallbacks)
    bool no_range8 = false;       // SBEACON_NO_RANGE8=1: every VCF on the 16-byte RangeHot words
    bool no_chains = false;       // SBEACON_NO_CHAINS=1: variantType slices answered one by one
    bool no_rowout = false;       // SBEACON_NO_ROWOUT: per-run row sources instead of static row hit regions
    char dedup_exact = 0;         // SBEACON_DEDUP_EXACT=radix|bucket ('r' / 'b'): the sorted dedup paths
    int dedup_hash_bits = 0;      // SBEACON_DEDUP_HASH_BITS (test hook): key hashes cut to this many bits
    bool strict_check = false;    // SBEACON_STRICT_CHECK: reference-exact dedup entries re-checked by the reader walk
    // ---- diagnostics
    bool prep_trace = false;      // SBEACON_PREP_TRACE: request-batch planning phase times (stderr)
    bool ingest_trace = false;    // SBEACON_INGEST_TRACE: ingest phase times (stderr)
    bool wire_trace = false;      // SBEACON_WIRE_TRACE: wire-path phase times (stderr)
    bool dedup_debug = false;     // SBEACON_DEDUP_DEBUG: dedup call details (stderr)
    int dedup_bucket_dbg = 0;     // SBEACON_DEDUP_BUCKET_DBG: bucket-kernel timing ablations
    int dedup_win_dbg = 0;        // SBEACON_DEDUP_WIN_DBG: window-kernel timing ablations
    int req_inject = 0;           // SBEACON_REQ_INJECT=1/2/3 (tests): one wrong per-chain exists / call-count / AN sum, so the pass's invariants fire
    bool req_index_stage = false; // SBEACON_REQ_INDEX_STAGE=1 (tests): stage candidate indices, as stores past 2^29 records do
    bool req_plan_apart = false;  // SBEACON_REQ_PLAN_APART=1: re-planning passes launch request_plan_kernel (no fused planning)
    bool req_tile_scan = false;   // SBEACON_REQ_TILE_SCAN=1: request_tile_scan_kernel before the delivery (no in-delivery sums)
};

inline Config config() {
    Config c;
    auto str = [](const char *k) -> const char * { return std::getenv(k); };
    auto flag = [&](const char *k) { return str(k) != nullptr; };
    auto one = [&](const char *k) { const char *e = str(k); return e && e[0] == '1'; };
    auto num = [&](const char *k, int d) { const char *e = str(k); return e ? std::atoi(e) : d; };
    if (const char *e = str("SBEACON_VC_BUCKET")) {
        const double x = std::atof(e);
        c.vc_bucket = x < 0.25 ? 0.25 : x;
    }
    c.pack_run = num("SBEACON_PACK_RUN", 0);
    c.slices_per_wave = num("SBEACON_SLICES_PER_WAVE", 0);
    c.dedup_win_target = num("SBEACON_DEDUP_WIN_TARGET", 0);
    c.dedup_bucket_cap = num("SBEACON_DEDUP_BUCKET_CAP", 0);
    c.max_nacc = num("SBEACON_MAX_NACC", 16);
    c.no_range8 = one("SBEACON_NO_RANGE8");
    c.no_chains = one("SBEACON_NO_CHAINS");
    c.no_rowout = flag("SBEACON_NO_ROWOUT");
    if (const char *e = str("SBEACON_DEDUP_EXACT")) c.dedup_exact = (e[0] == 'r' || e[0] == 'b') ? e[0] : 0;
    c.dedup_hash_bits = num("SBEACON_DEDUP_HASH_BITS", 0);
    c.strict_check = flag("SBEACON_STRICT_CHECK");
    c.prep_trace = flag("SBEACON_PREP_TRACE");
    c.ingest_trace = flag("SBEACON_INGEST_TRACE");
    c.wire_trace = flag("SBEACON_WIRE_TRACE");
    c.dedup_debug = flag("SBEACON_DEDUP_DEBUG");
    c.dedup_bucket_dbg = num("SBEACON_DEDUP_BUCKET_DBG", 0);
    c.dedup_win_dbg = num("SBEACON_DEDUP_WIN_DBG", 0);
    c.req_inject = num("SBEACON_REQ_INJECT", 0);
    c.req_index_stage = one("SBEACON_REQ_INDEX_STAGE");
    c.req_plan_apart = one("SBEACON_REQ_PLAN_APART");
    c.req_tile_scan = one("SBEACON_REQ_TILE_SCAN");
    return c;
}

}  // namespace sb
