// jsonesc.hpp -- JSON text as Python's json.dumps writes it (ensure_ascii:
// every non-ASCII code point as \\uXXXX, surrogate pairs above the BMP,
// control characters and DEL escaped, '/' kept), shared by the wire path
// (wire.cpp) and the result set's variant writer (api.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>

#include "../../include/sbeacon.h"

namespace sb {

// the escaped body (no quotes) of a str holding UTF-8 bytes s[0 .. n);
// false on invalid UTF-8
inline bool json_escape_append(std::string &o, const char *s, size_t n) {
    static const char kHex[] = "0123456789abcdef";
    auto u4 = [&](uint32_t v) {
        const char e[6] = {'\\', 'u', kHex[(v >> 12) & 15], kHex[(v >> 8) & 15], kHex[(v >> 4) & 15], kHex[v & 15]};
        o.append(e, 6);
    };
    for (size_t i = 0; i < n;) {
        size_t r = i;  // a run of printable ASCII other than '"' and '\\' is copied as is
        while (r < n) {
            const unsigned char x = static_cast<unsigned char>(s[r]);
            if (x < 0x20 || x >= 0x7f || x == '"' || x == '\\') break;
            ++r;
        }
        if (r > i) {
            o.append(s + i, r - i);
            i = r;
            if (i >= n) break;
        }
        const unsigned char c = static_cast<unsigned char>(s[i]);
        if (c < 0x80) {
            switch (c) {
                case '"': o += "\\\""; break;
                case '\\': o += "\\\\"; break;
                case '\n': o += "\\n"; break;
                case '\r': o += "\\r"; break;
                case '\t': o += "\\t"; break;
                case '\b': o += "\\b"; break;
                case '\f': o += "\\f"; break;
                default:
                    if (c < 0x20 || c == 0x7f) u4(c);
                    else o.push_back(static_cast<char>(c));
            }
            ++i;
            continue;
        }
        const int len = (c & 0xe0) == 0xc0 ? 2 : (c & 0xf0) == 0xe0 ? 3 : (c & 0xf8) == 0xf0 ? 4 : 0;
        if (!len || i + len > n) return false;
        uint32_t cp = c & (0x7f >> len);
        for (int k = 1; k < len; ++k) {
            const unsigned char cc = static_cast<unsigned char>(s[i + k]);
            if ((cc & 0xc0) != 0x80) return false;
            cp = (cp << 6) | (cc & 0x3f);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10ffff)) ||
            (cp >= 0xd800 && cp < 0xe000))
            return false;
        if (cp >= 0x10000) {
            const uint32_t v = cp - 0x10000;
            u4(0xd800 + (v >> 10));
            u4(0xdc00 + (v & 0x3ff));
        } else {
            u4(cp);
        }
        i += static_cast<size_t>(len);
    }
    return true;
}

// the same into a raw buffer with room for 6 * n bytes (the worst case:
// every byte a \uXXXX escape); returns the end, nullptr on invalid UTF-8
inline char *json_escape_to(char *p, const char *s, size_t n) {
    static const char kHex[] = "0123456789abcdef";
    auto u4 = [&](uint32_t v) {
        p[0] = '\\';
        p[1] = 'u';
        p[2] = kHex[(v >> 12) & 15];
        p[3] = kHex[(v >> 8) & 15];
        p[4] = kHex[(v >> 4) & 15];
        p[5] = kHex[v & 15];
        p += 6;
    };
    for (size_t i = 0; i < n;) {
        const unsigned char c = static_cast<unsigned char>(s[i]);
        if (c >= 0x20 && c < 0x7f && c != '"' && c != '\\') {
            *p++ = static_cast<char>(c);
            ++i;
            continue;
        }
        if (c < 0x80) {
            switch (c) {
                case '"': *p++ = '\\'; *p++ = '"'; break;
                case '\\': *p++ = '\\'; *p++ = '\\'; break;
                case '\n': *p++ = '\\'; *p++ = 'n'; break;
                case '\r': *p++ = '\\'; *p++ = 'r'; break;
                case '\t': *p++ = '\\'; *p++ = 't'; break;
                case '\b': *p++ = '\\'; *p++ = 'b'; break;
                case '\f': *p++ = '\\'; *p++ = 'f'; break;
                default: u4(c);  // other control characters and DEL
            }
            ++i;
            continue;
        }
        const int len = (c & 0xe0) == 0xc0 ? 2 : (c & 0xf0) == 0xe0 ? 3 : (c & 0xf8) == 0xf0 ? 4 : 0;
        if (!len || i + len > n) return nullptr;
        uint32_t cp = c & (0x7f >> len);
        for (int k = 1; k < len; ++k) {
            const unsigned char cc = static_cast<unsigned char>(s[i + k]);
            if ((cc & 0xc0) != 0x80) return nullptr;
            cp = (cp << 6) | (cc & 0x3f);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10ffff)) ||
            (cp >= 0xd800 && cp < 0xe000))
            return nullptr;
        if (cp >= 0x10000) {
            const uint32_t v = cp - 0x10000;
            u4(0xd800 + (v >> 10));
            u4(0xdc00 + (v & 0x3ff));
        } else {
            u4(cp);
        }
        i += static_cast<size_t>(len);
    }
    return p;
}

// the result set's variant strings of query i as JSON strings joined by ", "
// (f'{chrom}\\t{POS}\\t{REF}\\t{ALT}\\t{VT}', search_variants.py:210), written
// straight from the store's columns; false on text Python could not decode.
// result_prepare_json first (once per result set, single-threaded); then
// result_variants_json may run on many threads for different i.
void result_prepare_json(sb_result_set *r);
int result_view(const sb_result_set *r, size_t i, sb_result_view *out);  // sb_result_get without hit views
void run_tasks(size_t n, const std::function<void(size_t)> &fn);          // on the host worker pool
bool result_variants_json(const sb_result_set *r, size_t i, std::string &o);
// the same text in two steps: its exact length (false: the Python handler),
// then exactly that many bytes written at p (the wire writes in place)
bool result_variants_len(const sb_result_set *r, size_t i, size_t *need);
void result_variants_write(const sb_result_set *r, size_t i, char *p);
bool result_sample_names_len(const sb_result_set *r, size_t i, size_t *need);
void result_sample_names_write(const sb_result_set *r, size_t i, char *p);
// the sample_names list items of query i (false: a name that is not UTF-8)
bool result_sample_names_json(const sb_result_set *r, size_t i, std::string &o);

}  // namespace sb
