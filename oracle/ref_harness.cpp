// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" entry points over the parts of the reference C++ that compile
// without the AWS SDK, built from the sources where they lie under
// /root/reference by oracle/Makefile.ref into oracle/_ref/libsbref.so:
//   lambda/shared/gzip/gzip.cpp + gzip.hpp      (zlib writer / streaming reader)
//   lambda/shared/source/generalutils.cpp + .hpp (sequenceToBinary, fast_atoi)
//   lambda/summariseSlice/source/fast_atoi.h     (atoui64)
// Used by tests/test_ref_pinned.py to pin oracle/summarise_oracle.c and the
// engine's region-file / dedup paths to the reference's own code.  Nothing in
// the product (sbeacon/, csrc/) links or loads this.
//
// ref_region_keys restates ReadVcfData::getVcfData / readString /
// checkForAvailableData (lambda/duplicateVariantSearch/source/
// readVcfData.cpp:3-71, which needs the AWS SDK for its S3 download) statement
// by statement, over the REAL reference gzip class reading the file bytes
// from a std::stringstream instead of the S3 body.
#include <cstdint>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "fast_atoi.h"
#include "generalutils.hpp"
#include "gzip.hpp"

namespace {

constexpr size_t kBufferSize = 1024;  // readVcfData.hpp:7 BUFFER_SIZE
constexpr size_t kMinDataSize = sizeof(uint64_t) + sizeof(uint16_t);  // readVcfData.hpp:8

// readVcfData.cpp:56-71
bool check_available(size_t bytes_needed, size_t &buffer_pos, gzip &input, size_t &data_length) {
    if (data_length >= (buffer_pos + bytes_needed)) return true;
    if (!input.hasMoreData()) return false;
    data_length = input.proccesData(static_cast<unsigned int>(buffer_pos), static_cast<unsigned int>(data_length));
    if (data_length > 0) {
        buffer_pos = 0;
        return true;
    }
    return false;
}

// readVcfData.cpp:40-54
std::string read_string(size_t &buffer_pos, gzip &input, size_t &data_length, char *buf) {
    uint16_t len;
    memcpy(reinterpret_cast<char *>(&len), &buf[buffer_pos], sizeof(uint16_t));
    buffer_pos += sizeof(uint16_t);
    if (!check_available(len, buffer_pos, input, data_length)) throw std::runtime_error("Invalid File Read - readString()");
    std::string ret(&buf[buffer_pos], len);
    buffer_pos += len;
    return ret;
}

}  // namespace

extern "C" {

// generalutils.hpp:19-36 sequenceToBinary.at(c); -1 where .at throws
int ref_seq_code(int c) {
    try {
        return generalutils::sequenceToBinary.at(static_cast<char>(c));
    } catch (const std::out_of_range &) {
        return -1;
    }
}

// fast_atoi.h:54-80 atoui64(str, len)
uint64_t ref_atoui64_len(const char *s, uint8_t len) { return atoui64(s, len); }

// generalutils.hpp:38-45 fast_atoi<uint64_t>
uint64_t ref_fast_atoi_u64(const char *s, size_t len) { return generalutils::fast_atoi<uint64_t>(s, len); }

// gzip.cpp:19-59 deflateFile(level) of one buffer (one gzip member, as
// write_data_to_s3.h:51-52 writes per <= 50 MB buffer); returns the bytes
// written to out (or -1 if cap is too small / -2 on a zlib error)
int64_t ref_gzip_deflate(const char *buf, uint32_t n, int level, char *out, int64_t cap) {
    try {
        std::stringstream ss(std::stringstream::in | std::stringstream::out | std::stringstream::binary);
        std::vector<char> b(buf, buf + n);
        gzip gz(ss, 0, b.data(), n);
        if (gz.deflateFile(level) != Z_OK) return -2;
        const std::string s = ss.str();
        if (static_cast<int64_t>(s.size()) > cap) return -1;
        memcpy(out, s.data(), s.size());
        return static_cast<int64_t>(s.size());
    } catch (const std::exception &) {
        return -2;
    }
}

// ReadVcfData::getVcfData (readVcfData.cpp:3-38) over one region file's
// bytes: the key strings to_string(pos) + ref'_alt' it returns, written to
// out as [u32 length][bytes] records.  Returns the number of keys, -1 when
// the reference throws (*what = 1: getVcfData's "Invalid File Read", 2:
// readString's, 3: a gzip error), -2 when out is too small.
int64_t ref_region_keys(const char *file, uint64_t n, uint64_t range_start, uint64_t range_end, char *out, int64_t cap,
                        int64_t *out_len, int *what) {
    *what = 0;
    int64_t nk = 0, ol = 0;
    try {
        size_t buffer_pos = 0, data_length = 0;
        char stream_buffer[kBufferSize];
        generalutils::vcfData vcf;
        std::stringstream ss(std::string(file, n), std::stringstream::in | std::stringstream::binary);
        gzip input = gzip(ss, static_cast<long long>(n), stream_buffer, sizeof(stream_buffer));
        input.inflateFile();
        do {
            if (check_available(kMinDataSize, buffer_pos, input, data_length)) {
                memcpy(reinterpret_cast<unsigned char *>(&vcf.pos), &stream_buffer[buffer_pos], sizeof(vcf.pos));
                buffer_pos += sizeof(vcf.pos);
                if (range_start <= vcf.pos) {
                    const std::string key = std::to_string(vcf.pos) + read_string(buffer_pos, input, data_length,
                                                                                  stream_buffer);
                    const uint32_t kl = static_cast<uint32_t>(key.size());
                    if (ol + 4 + static_cast<int64_t>(kl) > cap) return -2;
                    memcpy(out + ol, &kl, 4);
                    memcpy(out + ol + 4, key.data(), kl);
                    ol += 4 + kl;
                    ++nk;
                } else {
                    uint16_t len;  // skip the rest of the entry (no availability check, as in :27-30)
                    memcpy(reinterpret_cast<char *>(&len), &stream_buffer[buffer_pos], sizeof(uint16_t));
                    buffer_pos += len + sizeof(uint16_t);
                }
            } else {
                *what = 1;
                return -1;
            }
        } while ((data_length != buffer_pos && vcf.pos <= range_end) || input.hasMoreData());
    } catch (const std::runtime_error &e) {
        *what = std::strstr(e.what(), "readString") ? 2 : 3;
        return -1;
    }
    *out_len = ol;
    return nk;
}

}  // extern "C"
