// results.cpp — result sets (sb_result_*): hit views and the
// reference's variant / sample-name text.
#include "internal.hpp"

extern "C" {

int sb_result_get(const sb_result_set *r, size_t i, sb_result_view *out) {
    if (!r || !out || i >= r->res.size()) return SB_EINVAL;
    std::call_once(r->tmp_once, [r] {  // the record / ALT views of every hit
        const size_t total = r->hit.size();
        r->tmp_rec.resize(total);
        r->tmp_alt.resize(total);
        parallel_for(total, [r](size_t h) {
            r->tmp_rec[h] = static_cast<uint32_t>(r->hit[h]);
            r->tmp_alt[h] = static_cast<uint32_t>(r->hit[h] >> kHitAltShift);
        }, 16, 1 << 16);
    });
    return sb::result_view(r, i, out);
}
}  // extern "C"

namespace sb {
// sb_result_get without the hit views (the wire formatter)
int result_view(const sb_result_set *r, size_t i, sb_result_view *out) {
    if (!r || !out || i >= r->res.size()) return SB_EINVAL;
    const QRes &q = r->res[i];
    out->error = q.error;
    out->exists = q.exists;
    out->call_count = q.call_count;
    out->all_alleles_count = q.all_alleles_count;
    const uint64_t a = r->dense_off[i], b = r->dense_off[i + 1];
    out->n_variants = q.error ? 0 : b - a;
    const bool views = r->tmp_rec.size() == r->hit.size();  // sb_result_get split them
    out->hit_record = views ? r->tmp_rec.data() + a : nullptr;
    out->hit_alt = views ? r->tmp_alt.data() + a : nullptr;
    out->n_sample_indices = r->sidx[i].size();
    out->sample_indices = r->sidx[i].data();
    out->big_limbs = 0;
    out->_pad = 0;
    out->big_call_count = out->big_all_alleles_count = nullptr;
    if (!r->big.empty()) {
        auto it = r->big.find(static_cast<uint32_t>(i));
        if (it != r->big.end() && !q.error) {
            out->big_limbs = r->big_limbs;
            out->big_call_count = it->second.data();
            out->big_all_alleles_count = it->second.data() + r->big_limbs;
        }
    }
    return SB_OK;
}
}  // namespace sb

extern "C" {
int sb_result_get_all(const sb_result_set *r, sb_result_view *out, size_t n) {
    if (!r || (!out && n) || n > r->res.size()) return SB_EINVAL;
    for (size_t i = 0; i < n; ++i) sb_result_get(r, i, out + i);
    return SB_OK;
}

namespace {
// f'{chrom}\t{position}\t{reference}\t{alts[i]}\t{variant_type}' (search_variants.py:210)
void append_variant(std::string &o, const sb_store &s, const std::string &chrom, uint64_t hit) {
    const uint32_t rec = static_cast<uint32_t>(hit);
    const uint32_t k = static_cast<uint32_t>(hit >> kHitAltShift);
    char num[16];
    o += chrom;
    o.push_back('\t');
    {  // decimal POS (no snprintf: millions of variant strings per batch)
        uint32_t v = s.h_pos[rec];
        char *e = num + sizeof num, *q = e;
        do {
            *--q = static_cast<char>('0' + v % 10);
            v /= 10;
        } while (v);
        o.append(q, static_cast<size_t>(e - q));
    }
    o.push_back('\t');
    o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_ref_off[rec]), s.h_end[rec] - s.h_pos[rec] + 1);
    o.push_back('\t');
    if (k == 0) {
        o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_a0_off[rec]), s.h_a0_len[rec]);
    } else {
        const uint32_t x = s.h_x_lo[rec] + k - 1;
        o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_x_off[x]), s.h_x_len[x]);
    }
    o.push_back('\t');
    o += s.vt.items[s.h_vt[rec]];
}
}  // namespace

}  // extern "C"

namespace sb {
// The wire formatter's per-store cache: for every ALT row (record rec's ALT
// 0 = row rec, its extra ALT x = row n_records + x) the JSON-escaped tail of
// its variant string, "\\t" POS "\\t" REF "\\t" ALT "\\t" VT
// (search_variants.py:210), built once on first use (parallel): a response's
// variant list is then its chrom and one copy per hit.  A row whose text is
// not UTF-8 has no entry (bad): its events take the Python handler.
struct VarText {
    std::vector<uint64_t> off;  // rows + 1
    std::vector<char> text;
    std::vector<uint8_t> bad;
};

const VarText &var_text(sb_store &s) {
    std::call_once(s.var_text_once, [&] {
        auto V = std::make_shared<VarText>();
        const size_t nr = s.n_records, rows = nr + s.n_extra;
        std::vector<std::string> vt(s.vt.items.size());
        std::vector<uint8_t> vt_bad(vt.size(), 0);
        for (size_t k = 0; k < vt.size(); ++k)
            if (!json_escape_append(vt[k], s.vt.items[k].data(), s.vt.items[k].size())) vt_bad[k] = 1;
        std::vector<uint32_t> xrec(s.n_extra);  // extra ALT row -> its record
        for (size_t r = 0; r < nr; ++r) {
            const uint32_t nx = (r + 1 < nr ? s.h_x_lo[r + 1] : static_cast<uint32_t>(s.n_extra)) - s.h_x_lo[r];
            for (uint32_t j = 0; j < nx; ++j) xrec[s.h_x_lo[r] + j] = static_cast<uint32_t>(r);
        }
        const char *blob = reinterpret_cast<const char *>(s.h_blob.data());
        auto parts = [&](size_t row, const char *&alt, size_t &al, uint32_t &rec) {
            if (row < nr) {
                rec = static_cast<uint32_t>(row);
                alt = blob + s.h_a0_off[rec];
                al = s.h_a0_len[rec];
            } else {
                const size_t x = row - nr;
                rec = xrec[x];
                alt = blob + s.h_x_off[x];
                al = s.h_x_len[x];
            }
        };
        // pass 1: each row's escaped length (0 + bad mark where not UTF-8)
        std::vector<uint32_t> len(rows, 0);
        V->bad.assign(rows, 0);
        parallel_for(rows, [&](size_t row) {
            const char *alt;
            size_t al;
            uint32_t rec;
            parts(row, alt, al, rec);
            const size_t rl = s.h_end[rec] - s.h_pos[rec] + 1;
            thread_local std::string tmp;
            tmp.clear();
            bool ok = json_escape_append(tmp, blob + s.h_ref_off[rec], rl) && json_escape_append(tmp, alt, al) &&
                      !vt_bad[s.h_vt[rec]];
            uint32_t digits = 1;
            for (uint32_t v = s.h_pos[rec]; v >= 10; v /= 10) ++digits;
            if (!ok) V->bad[row] = 1;
            else len[row] = static_cast<uint32_t>(8 + digits + tmp.size() + vt[s.h_vt[rec]].size());
        });
        V->off.assign(rows + 1, 0);
        for (size_t r = 0; r < rows; ++r) V->off[r + 1] = V->off[r] + len[r];
        V->text.resize(V->off[rows]);
        // pass 2: the text
        parallel_for(rows, [&](size_t row) {
            if (V->bad[row]) return;
            const char *alt;
            size_t al;
            uint32_t rec;
            parts(row, alt, al, rec);
            char *p = V->text.data() + V->off[row];
            *p++ = '\\';
            *p++ = 't';
            char num[16];
            uint32_t v = s.h_pos[rec];
            char *e = num + sizeof num, *q = e;
            do {
                *--q = static_cast<char>('0' + v % 10);
                v /= 10;
            } while (v);
            std::memcpy(p, q, static_cast<size_t>(e - q));
            p += e - q;
            *p++ = '\\';
            *p++ = 't';
            p = json_escape_to(p, blob + s.h_ref_off[rec], s.h_end[rec] - s.h_pos[rec] + 1);
            *p++ = '\\';
            *p++ = 't';
            p = json_escape_to(p, alt, al);
            *p++ = '\\';
            *p++ = 't';
            const std::string &t = vt[s.h_vt[rec]];
            std::memcpy(p, t.data(), t.size());
        });
        s.var_text = V;
    });
    return *static_cast<const VarText *>(s.var_text.get());
}

void result_prepare_json(sb_result_set *r) {
    if (!r->vt_json.empty()) return;
    (void)var_text(*r->s);
    const auto &items = r->s->vt.items;
    r->vt_json.resize(items.size());
    for (size_t k = 0; k < items.size(); ++k)
        if (!json_escape_append(r->vt_json[k], items[k].data(), items[k].size())) r->vt_json[k] = std::string("\x01");
    // sample names: the reference joins the selected names with ',' and the
    // response lists the pieces of splitting that text on ',' -- per name,
    // the pieces of the name split on ','
    r->names_json.assign(r->s->vcfs.size(), {});
    std::vector<uint8_t> need(r->s->vcfs.size(), 0);
    for (size_t i = 0; i < r->res.size(); ++i)
        if (!r->sidx[i].empty()) need[r->vcf_of[i]] = 1;
    for (size_t f = 0; f < need.size(); ++f) {
        if (!need[f]) continue;
        const auto &names = r->s->vcfs[f].samples;
        auto &out = r->names_json[f];
        out.resize(names.size());
        for (size_t h = 0; h < names.size(); ++h) {
            const std::string &nm = names[h];
            std::string &o = out[h];
            size_t a = 0;
            for (size_t k = 0; k <= nm.size(); ++k)
                if (k == nm.size() || nm[k] == ',') {
                    if (a) o += ", ";
                    o.push_back('"');
                    if (!json_escape_append(o, nm.data() + a, k - a)) {
                        o = std::string("\x01");
                        break;
                    }
                    o.push_back('"');
                    a = k + 1;
                }
        }
    }
}

namespace {
// query i's chrom, JSON-escaped (in buf when it fits); false: not UTF-8
struct ChromText {
    char buf[256];
    std::string lng;
    const char *p = nullptr;
    size_t n = 0;
    bool make(const std::string &cs) {
        if (6 * cs.size() <= sizeof buf) {
            char *e = json_escape_to(buf, cs.data(), cs.size());
            if (!e) return false;
            p = buf;
            n = static_cast<size_t>(e - buf);
        } else {
            if (!json_escape_append(lng, cs.data(), cs.size())) return false;
            p = lng.data();
            n = lng.size();
        }
        return true;
    }
};
uint64_t variant_row(const sb_store &s, uint64_t hit) {
    const uint32_t rec = static_cast<uint32_t>(hit);
    const uint32_t k = static_cast<uint32_t>(hit >> kHitAltShift);
    return k == 0 ? rec : s.n_records + s.h_x_lo[rec] + k - 1;
}
}  // namespace

bool result_variants_len(const sb_result_set *r, size_t i, size_t *need) {
    const sb_store &s = *r->s;
    const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
    *need = 0;
    if (b == a) return true;
    const VarText &V = *static_cast<const VarText *>(s.var_text.get());  // result_prepare_json built it
    ChromText c;
    if (!c.make(r->chrom[i])) return false;
    size_t n = 0;
    for (uint64_t h = a; h < b; ++h) {
        const uint64_t row = variant_row(s, r->hit[h]);
        if (V.bad[row]) return false;  // not UTF-8: the Python handler
        n += 4 + c.n + (V.off[row + 1] - V.off[row]);
    }
    *need = n - 2;  // no ", " before the first
    return true;
}

void result_variants_write(const sb_result_set *r, size_t i, char *p) {
    const sb_store &s = *r->s;
    const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
    if (b == a) return;
    const VarText &V = *static_cast<const VarText *>(s.var_text.get());
    ChromText c;
    c.make(r->chrom[i]);  // (result_variants_len accepted it)
    for (uint64_t h = a; h < b; ++h) {
        const uint64_t row = variant_row(s, r->hit[h]);
        if (h > a) {
            *p++ = ',';
            *p++ = ' ';
        }
        *p++ = '"';
        std::memcpy(p, c.p, c.n);
        p += c.n;
        const size_t n = V.off[row + 1] - V.off[row];
        std::memcpy(p, V.text.data() + V.off[row], n);
        p += n;
        *p++ = '"';
    }
}

bool result_variants_json(const sb_result_set *r, size_t i, std::string &o) {
    size_t need;
    if (!result_variants_len(r, i, &need)) return false;
    const size_t o0 = o.size();
    o.resize(o0 + need);
    result_variants_write(r, i, &o[o0]);
    return true;
}

bool result_sample_names_len(const sb_result_set *r, size_t i, size_t *need) {
    const auto &ix = r->sidx[i];
    const auto &nj = r->names_json[r->vcf_of[i]];
    size_t n = ix.empty() ? 0 : 2 * (ix.size() - 1);
    for (size_t j = 0; j < ix.size(); ++j) {
        const std::string &x = nj[r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j]];
        if (x.size() == 1 && x[0] == '\x01') return false;  // not UTF-8
        n += x.size();
    }
    *need = n;
    return true;
}

void result_sample_names_write(const sb_result_set *r, size_t i, char *p) {
    const auto &ix = r->sidx[i];
    const auto &nj = r->names_json[r->vcf_of[i]];
    for (size_t j = 0; j < ix.size(); ++j) {
        const std::string &x = nj[r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j]];
        if (j) {
            *p++ = ',';
            *p++ = ' ';
        }
        std::memcpy(p, x.data(), x.size());
        p += x.size();
    }
}

bool result_sample_names_json(const sb_result_set *r, size_t i, std::string &o) {
    size_t need;
    if (!result_sample_names_len(r, i, &need)) return false;
    const size_t o0 = o.size();
    o.resize(o0 + need);
    result_sample_names_write(r, i, &o[o0]);
    return true;
}
}  // namespace sb

extern "C" {

int sb_result_variants_text(sb_result_set *r, size_t i, const char **p, size_t *len) {
    if (!r || !p || !len || i >= r->res.size()) return SB_EINVAL;
    if (!r->vbuilt[i]) {
        std::string &o = r->vtext[i];
        const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
        for (uint64_t h = a; h < b; ++h) {
            if (h > a) o.push_back('\n');
            append_variant(o, *r->s, r->chrom[i], r->hit[h]);
        }
        r->vbuilt[i] = 1;
    }
    *p = r->vtext[i].data();
    *len = r->vtext[i].size();
    return SB_OK;
}

int sb_result_distinct_variants(sb_result_set *r, const uint32_t *queries, size_t n, const char **p, size_t *len,
                                uint64_t *count) {
    return guard([&] {
        if (!r || !p || !len || !count || (n && !queries)) throw Error(SB_EINVAL, "NULL argument");
        // (chrom string, record, alt) first, then the formatted strings: two
        // records (or two VCFs naming the contig alike) can print the same line
        std::unordered_map<std::string, uint32_t> chrom_id;
        std::unordered_set<uint64_t> seen_hit;
        std::unordered_set<std::string> seen_text;
        std::string &o = r->distinct;
        o.clear();
        uint64_t c = 0;
        std::string line;
        for (size_t j = 0; j < n; ++j) {
            const uint32_t i = queries[j];
            if (i >= r->res.size()) throw Error(SB_EINVAL, "query index out of range");
            if (r->res[i].error) continue;
            const uint32_t cid = chrom_id.emplace(r->chrom[i], static_cast<uint32_t>(chrom_id.size())).first->second;
            for (uint64_t h = r->dense_off[i]; h < r->dense_off[i + 1]; ++h) {
                // hit = rec | alt << kHitAltShift; rec < 2^32, alt < 64: fold the chrom id above both
                const uint64_t key = r->hit[h] ^ (static_cast<uint64_t>(cid) << 40);
                if (!seen_hit.insert(key).second) continue;
                line.clear();
                append_variant(line, *r->s, r->chrom[i], r->hit[h]);
                if (!seen_text.insert(line).second) continue;
                if (c++) o.push_back('\n');
                o += line;
            }
        }
        *p = o.data();
        *len = o.size();
        *count = c;
    });
}

int sb_result_sample_names_text(sb_result_set *r, size_t i, const char **p, size_t *len) {
    if (!r || !p || !len || i >= r->res.size()) return SB_EINVAL;
    if (!r->nbuilt[i]) {
        std::string &o = r->ntext[i];
        const VcfData &v = r->s->vcfs[r->vcf_of[i]];
        const auto &ix = r->sidx[i];
        for (size_t j = 0; j < ix.size(); ++j) {
            const uint32_t h = r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j];
            if (j) o.push_back(',');
            o += v.samples[h];
        }
        r->nbuilt[i] = 1;
    }
    *p = r->ntext[i].data();
    *len = r->ntext[i].size();
    return SB_OK;
}

int sb_result_stats(const sb_result_set *r, sb_batch_stats *out) {
    if (!r || !out) return SB_EINVAL;
    *out = r->stats;
    return SB_OK;
}

void sb_result_free(sb_result_set *r) { delete r; }

}  // extern "C"
