// common.hpp — host helpers shared by ingest and the C ABI.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/sbeacon.h"

namespace sb {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

inline uint8_t upc(uint8_t c) { return (c >= 'a' && c <= 'z') ? static_cast<uint8_t>(c - 32) : c; }

// Python int(str) over the ASCII forms a VCF carries (whitespace, sign,
// digits, single '_' between digits) — the parse the reference applies to
// INFO/AC and INFO/AN (search_variants.py:199,206).
inline bool py_int(const char *p, size_t n, int64_t *out) {
    size_t i = 0, j = n;
    auto sp = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; };
    while (i < j && sp(p[i])) ++i;
    while (j > i && sp(p[j - 1])) --j;
    if (i == j) return false;
    bool neg = false;
    if (p[i] == '+' || p[i] == '-') {
        neg = p[i] == '-';
        ++i;
    }
    if (i == j || p[i] < '0' || p[i] > '9') return false;
    int64_t v = 0;
    for (size_t k = i; k < j; ++k) {
        const char c = p[k];
        if (c == '_') {
            if (k + 1 >= j || p[k + 1] < '0' || p[k + 1] > '9' || p[k - 1] < '0' || p[k - 1] > '9') return false;
            continue;
        }
        if (c < '0' || c > '9') return false;
        if (v > (INT64_MAX - 9) / 10) return false;  // beyond int64: not representable in the store
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return true;
}

// 64-bit allele key.  Alleles of <= 8 printable-ASCII bytes are packed
// verbatim (exact, bit 63 clear); anything else is a 63-bit hash with bit 63
// set, and equal keys are confirmed byte-for-byte on the device.
inline uint64_t allele_key(const uint8_t *p, size_t n, bool to_upper, bool *hashed) {
    if (n <= 8) {
        uint64_t k = 0;
        bool ok = true;
        for (size_t i = 0; i < n; ++i) {
            const uint8_t c = to_upper ? upc(p[i]) : p[i];
            if (c == 0 || c >= 0x80) ok = false;
            k |= static_cast<uint64_t>(c) << (8 * i);
        }
        if (ok) {
            *hashed = false;
            return k;
        }
    }
    uint64_t h = 0xcbf29ce484222325ull ^ (static_cast<uint64_t>(n) * 0x9E3779B97F4A7C15ull);
    for (size_t i = 0; i < n; ++i) {
        h ^= to_upper ? upc(p[i]) : p[i];
        h *= 0x100000001b3ull;
    }
    h ^= h >> 31;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 29;
    *hashed = true;
    return h | (1ull << 63);
}

}  // namespace sb
