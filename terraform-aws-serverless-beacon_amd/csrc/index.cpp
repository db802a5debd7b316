// index.cpp — CSI / TBI coordinate index of a BGZF-compressed VCF.
//
// summariseVcf cuts a VCF into summariseSlice slices at the chunk boundaries
// of the file's CSI (or, failing that, TBI) index (lambda/summariseVcf/
// lambda_function.py:90-104,144-156; index_reader.py:4-125 parses it).  The
// reference expects the index to sit next to the VCF, written by
// `bcftools index` / `tabix -p vcf`; the ingest writes one here so a VCF
// arriving without an index still gets the reference's slices.
//
// The file is a valid SAMv1 §5 index that index_reader.py (and htslib)
// parse, with the chunk boundaries summariseVcf reads; it is NOT claimed to
// be byte-identical to what htslib writes (htslib is absent here, so that is
// unpinned): empty linear-index windows take the NEXT window's offset (htslib
// forward-fills from the previous one), a bin's loff is its smallest record
// offset (htslib: the linear-index entry of its bottom bin) and the CSI
// default depth is 5 (bcftools' tbx path uses 6).
//
// Layout: SAMv1 §5 (binning scheme, CSI v1 and tabix formats).  A record
// covers [POS-1, POS-1+len(REF)), or [POS-1, END) when INFO carries END= past
// POS (the tabix VCF preset).  Chunks are built as htslib's hts_idx_push does:
// a chunk grows while consecutive records fall in the same bin and closes at
// the virtual offset where the next record starts; a bin whose chunks all lie
// within one BGZF block's distance moves into its parent bin, and chunks of a
// bin that meet in one block merge (htslib hts.c compress_binning, restated
// from the format description: htslib is not in this image).  Every contig
// carries the pseudo-bin (bin_limit + 1: [first record, past last record],
// [mapped, unmapped]) that get_chunk_boundaries excludes.  Virtual offsets use
// bgzf_tell's spelling: a position at the end of a block is (next block, 0).
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <unordered_set>
#include <vector>

#include "common.hpp"

namespace sb {
namespace {

constexpr uint64_t kNoOff = ~0ull;
constexpr uint64_t kMinMarkerDist = 0x10000;  // one BGZF block's compressed span

struct Chunk {
    uint64_t u, v;
};

struct Bin {
    std::vector<Chunk> list;
    uint64_t loff = kNoOff;
};

struct Ref {
    std::string name;
    std::map<uint32_t, Bin> bins;
    std::vector<uint64_t> lidx;  // TBI linear index: first record offset per 2^min_shift window
    uint64_t off_beg = kNoOff, off_end = 0, n_mapped = 0;
};

// SAMv1 §5.3 reg2bin over [beg, end) at n_lvls levels of 2^min_shift leaves
uint32_t reg2bin(int64_t beg, int64_t end, int min_shift, int n_lvls) {
    --end;
    int s = min_shift;
    int64_t t = ((1ll << (3 * n_lvls)) - 1) / 7;  // first bin of the deepest level
    for (int l = n_lvls; l > 0; --l) {
        if ((beg >> s) == (end >> s)) return static_cast<uint32_t>(t + (beg >> s));
        s += 3;
        t -= 1ll << (3 * (l - 1));
    }
    return 0;
}

inline uint32_t bin_first(int l) { return static_cast<uint32_t>(((1ll << (3 * l)) - 1) / 7); }
inline uint32_t bin_parent(uint32_t b) { return (b - 1) >> 3; }

int bin_level(uint32_t b, int n_lvls) {
    for (int l = n_lvls; l > 0; --l)
        if (b >= bin_first(l)) return l;
    return 0;
}

struct Builder {
    int min_shift, depth;
    std::vector<Ref> refs;
    std::unordered_set<std::string> seen;
    int64_t last_beg = -1;
    uint32_t cur_bin = ~0u;
    uint64_t save_off = 0, last_end_off = 0;

    void close_chunk(uint64_t end_off) {
        if (cur_bin == ~0u) return;
        Bin &b = refs.back().bins[cur_bin];
        b.list.push_back({save_off, end_off});
    }

    void push(const std::string &contig, int64_t beg, int64_t end, uint64_t off0, uint64_t off1) {
        if (refs.empty() || refs.back().name != contig) {
            close_chunk(last_end_off);
            if (!seen.insert(contig).second)
                throw Error(SB_EINVAL, "VCF not sorted: contig " + contig + " appears in two runs");
            refs.push_back(Ref{});
            refs.back().name = contig;
            cur_bin = ~0u;
            last_beg = -1;
        }
        if (beg < last_beg) throw Error(SB_EINVAL, "VCF not sorted by POS in contig " + contig);
        if ((end - 1) >> (min_shift + 3 * depth))
            throw Error(SB_EINVAL, "position beyond the index's coordinate range (raise depth or use CSI)");
        last_beg = beg;
        Ref &r = refs.back();
        const uint32_t bin = reg2bin(beg, end, min_shift, depth);
        if (bin != cur_bin) {
            close_chunk(off0);
            cur_bin = bin;
            save_off = off0;
        }
        Bin &b = r.bins[bin];
        b.loff = std::min(b.loff, off0);
        const uint64_t w0 = static_cast<uint64_t>(beg) >> min_shift, w1 = static_cast<uint64_t>(end - 1) >> min_shift;
        if (r.lidx.size() <= w1) r.lidx.resize(w1 + 1, kNoOff);
        for (uint64_t w = w0; w <= w1; ++w)
            if (r.lidx[w] == kNoOff) r.lidx[w] = off0;
        r.off_beg = std::min(r.off_beg, off0);
        r.off_end = off1;
        ++r.n_mapped;
        last_end_off = off1;
    }

    void finish() {
        close_chunk(last_end_off);
        cur_bin = ~0u;
        for (Ref &r : refs) compress(r);
    }

    // bins spanning less than one block move into their parent (deepest level
    // first), then chunks of a bin that meet in one block merge
    void compress(Ref &r) {
        const uint32_t n_bins = bin_first(depth + 1);
        for (int l = depth; l > 0; --l) {
            std::vector<uint32_t> level;
            for (auto &kv : r.bins)
                if (kv.first < n_bins && bin_level(kv.first, depth) == l) level.push_back(kv.first);
            for (uint32_t id : level) {
                Bin &p = r.bins[id];
                std::sort(p.list.begin(), p.list.end(), [](const Chunk &a, const Chunk &b) { return a.u < b.u; });
                if ((p.list.back().v >> 16) - (p.list.front().u >> 16) >= kMinMarkerDist) continue;
                auto q = r.bins.find(bin_parent(id));
                if (q == r.bins.end()) continue;
                q->second.list.insert(q->second.list.end(), p.list.begin(), p.list.end());
                q->second.loff = std::min(q->second.loff, p.loff);
                r.bins.erase(id);
            }
        }
        for (auto &kv : r.bins) {
            auto &L = kv.second.list;
            std::sort(L.begin(), L.end(), [](const Chunk &a, const Chunk &b) { return a.u < b.u; });
            size_t m = 0;
            for (size_t i = 1; i < L.size(); ++i) {
                if ((L[m].v >> 16) >= (L[i].u >> 16))
                    L[m].v = std::max(L[m].v, L[i].v);
                else
                    L[++m] = L[i];
            }
            if (!L.empty()) L.resize(m + 1);
        }
        // linear index: windows no record starts in take the next window's offset
        for (size_t w = r.lidx.size(); w-- > 0;)
            if (r.lidx[w] == kNoOff) r.lidx[w] = w + 1 < r.lidx.size() ? r.lidx[w + 1] : r.off_end;
    }
};

struct Out {
    std::string s;
    void i32(int32_t x) { s.append(reinterpret_cast<const char *>(&x), 4); }
    void u32(uint32_t x) { s.append(reinterpret_cast<const char *>(&x), 4); }
    void u64(uint64_t x) { s.append(reinterpret_cast<const char *>(&x), 8); }
};

// tabix header fields (the CSI aux block carries the same, index_reader.py:11-30)
void tabix_conf(Out &o, const std::vector<Ref> &refs) {
    std::string names;
    for (const Ref &r : refs) names += r.name + '\0';
    o.i32(2);    // format: VCF
    o.i32(1);    // col_seq
    o.i32(2);    // col_beg
    o.i32(0);    // col_end
    o.i32('#');  // meta
    o.i32(0);    // skip
    o.i32(static_cast<int32_t>(names.size()));
    o.s += names;
}

void write_bins(Out &o, const Ref &r, uint32_t pseudo, bool csi) {
    o.i32(static_cast<int32_t>(r.bins.size() + 1));
    for (const auto &kv : r.bins) {
        o.u32(kv.first);
        if (csi) o.u64(kv.second.loff);
        o.i32(static_cast<int32_t>(kv.second.list.size()));
        for (const Chunk &c : kv.second.list) {
            o.u64(c.u);
            o.u64(c.v);
        }
    }
    o.u32(pseudo);
    if (csi) o.u64(0);
    o.i32(2);
    o.u64(r.off_beg);
    o.u64(r.off_end);
    o.u64(r.n_mapped);
    o.u64(0);
}

// BGZF (SAMv1 §4.1): <= 0xff00-byte blocks, each one gzip member with the BC
// extra field, then the 28-byte EOF block
std::string bgzf(const std::string &data) {
    std::string out;
    std::vector<uint8_t> buf(compressBound(0xff00) + 64);
    for (size_t at = 0; at < data.size() || at == 0; at += 0xff00) {
        const size_t n = std::min<size_t>(0xff00, data.size() - at);
        z_stream z{};
        if (deflateInit2(&z, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) throw Error(SB_EIO, "deflateInit2");
        z.next_in = reinterpret_cast<Bytef *>(const_cast<char *>(data.data() + at));
        z.avail_in = static_cast<uInt>(n);
        z.next_out = buf.data() + 18;
        z.avail_out = static_cast<uInt>(buf.size() - 26);
        const int rc = deflate(&z, Z_FINISH);
        const size_t clen = z.total_out;
        deflateEnd(&z);
        if (rc != Z_STREAM_END) throw Error(SB_EIO, "deflate failed");
        const size_t bsize = 18 + clen + 8;
        const uint8_t hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                                 static_cast<uint8_t>((bsize - 1) & 0xff), static_cast<uint8_t>((bsize - 1) >> 8)};
        std::copy(hdr, hdr + 18, buf.begin());
        const uint32_t crc = static_cast<uint32_t>(crc32(0, reinterpret_cast<const Bytef *>(data.data() + at), static_cast<uInt>(n)));
        const uint32_t isz = static_cast<uint32_t>(n);
        std::copy(reinterpret_cast<const uint8_t *>(&crc), reinterpret_cast<const uint8_t *>(&crc) + 4, buf.begin() + 18 + clen);
        std::copy(reinterpret_cast<const uint8_t *>(&isz), reinterpret_cast<const uint8_t *>(&isz) + 4, buf.begin() + 22 + clen);
        out.append(reinterpret_cast<const char *>(buf.data()), bsize);
        if (data.empty()) break;
    }
    static const uint8_t eof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C',
                                    2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    out.append(reinterpret_cast<const char *>(eof), sizeof eof);
    return out;
}

size_t block_size(const uint8_t *c, size_t avail) {
    if (avail < 18 || c[0] != 0x1f || c[1] != 0x8b || c[2] != 8 || !(c[3] & 4)) return 0;
    const size_t xlen = c[10] | (c[11] << 8);
    for (size_t x = 12; x + 4 <= 12 + xlen && x + 4 <= avail;) {
        const size_t slen = c[x + 2] | (c[x + 3] << 8);
        if (c[x] == 'B' && c[x + 1] == 'C' && slen == 2 && x + 6 <= avail) {
            const size_t bs = (c[x + 4] | (c[x + 5] << 8)) + 1u;
            return bs >= 26 ? bs : 0;
        }
        x += 4 + slen;
    }
    return 0;
}

// the columns tabix reads from one VCF data line: CHROM, POS, REF, INFO/END
void parse_line(const std::string &line, std::string *contig, int64_t *beg, int64_t *end) {
    size_t f[9], nf = 0, at = 0;
    f[nf++] = 0;
    while (nf < 9 && (at = line.find('\t', at)) != std::string::npos) f[nf++] = ++at;
    if (nf < 5) throw Error(SB_EPARSE, "VCF line with fewer than 5 columns: " + line.substr(0, 80));
    *contig = line.substr(0, f[1] - 1);
    int64_t pos = 0;
    size_t p = f[1];
    if (p >= line.size() || line[p] < '0' || line[p] > '9') throw Error(SB_EPARSE, "bad POS: " + line.substr(0, 80));
    for (; p < line.size() && line[p] >= '0' && line[p] <= '9'; ++p) {
        pos = pos * 10 + (line[p] - '0');
        if (pos > (1ll << 40)) throw Error(SB_EPARSE, "POS out of range");
    }
    const size_t ref_len = f[4] - 1 - f[3];
    *beg = pos > 0 ? pos - 1 : 0;
    *end = *beg + static_cast<int64_t>(std::max<size_t>(ref_len, 1));
    if (nf >= 8) {  // INFO
        const size_t i0 = f[7], i1 = nf >= 9 ? f[8] - 1 : line.size();
        for (size_t k = i0; k + 4 <= i1;) {
            if (line.compare(k, 4, "END=") == 0) {
                int64_t e = 0;
                size_t q = k + 4;
                bool any = false;
                for (; q < i1 && line[q] >= '0' && line[q] <= '9' && e < (1ll << 40); ++q, any = true) e = e * 10 + (line[q] - '0');
                if (any && e > *beg) *end = e;
                break;
            }
            const size_t semi = line.find(';', k);
            if (semi == std::string::npos || semi >= i1) break;
            k = semi + 1;
        }
    }
}

std::string index_file(const char *path, bool tbi, int min_shift, int depth) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) throw Error(SB_EIO, std::string("cannot open ") + path);
    std::vector<uint8_t> c;
    {
        uint8_t buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) c.insert(c.end(), buf, buf + n);
        std::fclose(fp);
    }
    // pass 1: the longest record end, to size the binning (CSI auto depth)
    struct Rec {
        uint32_t contig;
        int64_t beg, end;
        uint64_t off0, off1;
    };
    std::vector<Rec> recs;
    std::vector<std::string> contigs;
    std::map<std::string, uint32_t> contig_id;
    std::string line;
    uint64_t line_off = kNoOff;
    std::vector<uint8_t> ub(1 << 16);
    bool header_done = false;
    int64_t max_end = 1;
    for (size_t at = 0; at < c.size();) {
        const size_t bs = block_size(c.data() + at, c.size() - at);
        if (!bs || at + bs > c.size()) throw Error(SB_EIO, std::string("not a BGZF file or corrupt block: ") + path);
        z_stream z{};
        if (inflateInit2(&z, -15) != Z_OK) throw Error(SB_EIO, "inflateInit2");
        const size_t xlen = c[at + 10] | (c[at + 11] << 8);
        z.next_in = c.data() + at + 12 + xlen;
        z.avail_in = static_cast<uInt>(bs - 12 - xlen - 8);
        z.next_out = ub.data();
        z.avail_out = static_cast<uInt>(ub.size());
        const int rc = inflate(&z, Z_FINISH);
        const size_t ulen = z.total_out;
        inflateEnd(&z);
        if (rc != Z_STREAM_END) throw Error(SB_EIO, std::string("BGZF inflate failed in ") + path);
        const uint64_t coff = at, next = at + bs;
        for (size_t i = 0; i < ulen; ++i) {
            if (line_off == kNoOff) line_off = (coff << 16) | i;
            const char ch = static_cast<char>(ub[i]);
            if (ch != '\n') {
                line.push_back(ch);
                continue;
            }
            const uint64_t end_off = i + 1 < ulen ? ((coff << 16) | (i + 1)) : (next << 16);
            if (!line.empty() && line.back() == '\r') line.pop_back();
            if (!line.empty() && line[0] == '#') {
                if (header_done) throw Error(SB_EPARSE, "header line after data lines");
            } else if (!line.empty()) {
                header_done = true;
                std::string ctg;
                int64_t beg, end;
                parse_line(line, &ctg, &beg, &end);
                auto it = contig_id.find(ctg);
                if (it == contig_id.end()) {
                    it = contig_id.emplace(ctg, static_cast<uint32_t>(contigs.size())).first;
                    contigs.push_back(ctg);
                }
                recs.push_back({it->second, beg, end, line_off, end_off});
                max_end = std::max(max_end, end);
            }
            line.clear();
            line_off = kNoOff;
        }
        at = next;
    }
    if (!line.empty()) throw Error(SB_EPARSE, "VCF does not end with a newline");
    if (min_shift <= 0) min_shift = 14;
    if (depth <= 0) {
        depth = 5;
        if (!tbi)
            while ((max_end - 1) >> (min_shift + 3 * depth)) ++depth;
    }
    if (tbi && (min_shift != 14 || depth != 5)) throw Error(SB_EINVAL, "TBI is fixed at min_shift 14, depth 5");
    if (min_shift + 3 * depth > 62 || depth > 9) throw Error(SB_EINVAL, "CSI min_shift/depth out of range");
    Builder b{min_shift, depth, {}, {}, -1, ~0u, 0, 0};
    for (const Rec &r : recs) b.push(contigs[r.contig], r.beg, r.end, r.off0, r.off1);
    b.finish();
    const uint32_t pseudo = bin_first(depth + 1) + 1;
    Out o;
    if (tbi) {
        o.s = "TBI\x01";
        o.i32(static_cast<int32_t>(b.refs.size()));
        tabix_conf(o, b.refs);
        for (const Ref &r : b.refs) {
            write_bins(o, r, pseudo, false);
            o.i32(static_cast<int32_t>(r.lidx.size()));
            for (uint64_t x : r.lidx) o.u64(x);
        }
    } else {
        o.s = "CSI\x01";
        o.i32(min_shift);
        o.i32(depth);
        Out aux;
        tabix_conf(aux, b.refs);
        o.i32(static_cast<int32_t>(aux.s.size()));
        o.s += aux.s;
        o.i32(static_cast<int32_t>(b.refs.size()));
        for (const Ref &r : b.refs) write_bins(o, r, pseudo, true);
    }
    o.u64(0);  // n_no_coor
    return bgzf(o.s);
}

}  // namespace
}  // namespace sb

extern "C" int sb_index_vcf(const char *path, int fmt, int min_shift, int depth, uint8_t **out, size_t *out_len) {
    try {
        if (!path || !out || !out_len || (fmt != SB_INDEX_CSI && fmt != SB_INDEX_TBI))
            throw sb::Error(SB_EINVAL, "sb_index_vcf: bad argument");
        *out = nullptr;
        *out_len = 0;
        const std::string s = sb::index_file(path, fmt == SB_INDEX_TBI, min_shift, depth);
        uint8_t *p = static_cast<uint8_t *>(std::malloc(s.size()));
        if (!p) throw sb::Error(SB_ENOMEM, "sb_index_vcf: out of memory");
        std::copy(s.begin(), s.end(), p);
        *out = p;
        *out_len = s.size();
        return SB_OK;
    } catch (const sb::Error &e) {
        sb::set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        sb::set_last_error("out of memory");
        return SB_ENOMEM;
    } catch (const std::exception &e) {
        sb::set_last_error(e.what());
        return SB_EINVAL;
    }
}

extern "C" void sb_free(void *p) { std::free(p); }
