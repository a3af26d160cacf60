// audio_file.hpp -- WAVE / AIFF / AIFF-C container handling for the lowcut
// tool.
//
// The reference opens the file through c_lib's AudioFile/AudioFormat
// (ProcessFile.cp:32-35), reads every sample into a deinterleaved buffer
// (:40-41), and writes the output as "copy every chunk of the input, then
// write the filtered samples" (:103-117), so all metadata survives.  Here the
// output file is the input file's bytes with only the sample payload
// rewritten in place (same format, same size): every chunk, its order and
// its padding are preserved byte for byte.
//
// Supported sample encodings (the ones lcfir_decode/encode_pcm_dev handle):
//   WAVE  PCM 16/24/32-bit LE, IEEE float32 LE, WAVE_FORMAT_EXTENSIBLE of those
//   AIFF  PCM 16/24/32-bit BE
//   AIFC  NONE (BE PCM), sowt (LE PCM), fl32/FL32 (BE float32)
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "lcfir.h"

namespace lcfir_host {

struct AudioFile {
    enum class Kind { Wave, Aiff } kind = Kind::Wave;
    std::shared_ptr<uint8_t> storage; // the whole file (vector- or pinned-backed)
    uint8_t *data = nullptr;
    size_t size = 0;
    int channels = 0;
    int64_t frames = 0;
    double sample_rate = 0.0;
    int bits = 0;
    int pcm_format = 0;        // lcfir_pcm_format
    size_t data_offset = 0;    // first sample byte
    size_t data_bytes = 0;     // frames * channels * bytes per sample
    std::vector<std::string> chunk_ids;

    const char *format_name() const {
        switch (pcm_format) {
        case LCFIR_PCM_S16LE: return "s16le";
        case LCFIR_PCM_S24LE: return "s24le";
        case LCFIR_PCM_S32LE: return "s32le";
        case LCFIR_PCM_F32LE: return "f32le";
        case LCFIR_PCM_S16BE: return "s16be";
        case LCFIR_PCM_S24BE: return "s24be";
        case LCFIR_PCM_S32BE: return "s32be";
        case LCFIR_PCM_F32BE: return "f32be";
        default: return "?";
        }
    }
};

class FormatError : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

// Where read_audio_file puts the file: a plain heap buffer, or (the lowcut
// pipeline) pinned host memory so H2D/D2H run asynchronously.
using Allocator = std::function<std::shared_ptr<uint8_t>(size_t)>;

inline std::shared_ptr<uint8_t> heap_alloc(size_t n) {
    return std::shared_ptr<uint8_t>(new uint8_t[n ? n : 1], std::default_delete<uint8_t[]>());
}

namespace detail {
struct ByteView {
    const uint8_t *p;
    size_t n;
    size_t size() const { return n; }
    const uint8_t &operator[](size_t i) const { return p[i]; }
};

inline uint32_t le32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }
inline uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }
inline uint16_t be16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }

// IEEE 754 80-bit extended (AIFF COMM sampleRate), big-endian
inline double be_extended(const uint8_t *p) {
    const int sign = p[0] >> 7;
    const int exp = ((p[0] & 0x7f) << 8) | p[1];
    uint64_t mant = 0;
    for (int i = 0; i < 8; ++i) mant = (mant << 8) | p[2 + i];
    if (exp == 0 && mant == 0) return 0.0;
    const double v = std::ldexp((double)mant, exp - 16383 - 63);
    return sign ? -v : v;
}

inline int pcm_int_format(int bits, bool be) {
    switch (bits) {
    case 16: return be ? LCFIR_PCM_S16BE : LCFIR_PCM_S16LE;
    case 24: return be ? LCFIR_PCM_S24BE : LCFIR_PCM_S24LE;
    case 32: return be ? LCFIR_PCM_S32BE : LCFIR_PCM_S32LE;
    default: throw FormatError("unsupported PCM bit depth " + std::to_string(bits));
    }
}

inline void parse_wave(AudioFile &f) {
    const ByteView b{f.data, f.size};
    size_t pos = 12;
    bool have_fmt = false, have_data = false;
    int tag = 0, bits = 0;
    while (pos + 8 <= b.size()) {
        const std::string id(reinterpret_cast<const char *>(&b[pos]), 4);
        const uint32_t size = le32(&b[pos + 4]);
        const size_t body = pos + 8;
        if (body + size > b.size() && id != "data") throw FormatError("truncated chunk " + id);
        f.chunk_ids.push_back(id);
        if (id == "fmt ") {
            if (size < 16) throw FormatError("short fmt chunk");
            tag = le16(&b[body]);
            f.channels = le16(&b[body + 2]);
            f.sample_rate = le32(&b[body + 4]);
            bits = le16(&b[body + 14]);
            if (tag == 0xFFFE && size >= 40) tag = le16(&b[body + 24]); // SubFormat GUID
            have_fmt = true;
        } else if (id == "data") {
            f.data_offset = body;
            f.data_bytes = std::min<size_t>(size, b.size() - body);
            have_data = true;
        }
        pos = body + size + (size & 1);
    }
    if (!have_fmt || !have_data) throw FormatError("WAVE file without fmt or data chunk");
    f.bits = bits;
    if (tag == 1) f.pcm_format = pcm_int_format(bits, false);
    else if (tag == 3 && bits == 32) f.pcm_format = LCFIR_PCM_F32LE;
    else throw FormatError("unsupported WAVE format tag " + std::to_string(tag));
}

inline void parse_aiff(AudioFile &f, bool aifc) {
    const ByteView b{f.data, f.size};
    size_t pos = 12;
    bool have_comm = false, have_ssnd = false;
    int bits = 0;
    std::string comp = "NONE";
    int64_t frames = 0;
    while (pos + 8 <= b.size()) {
        const std::string id(reinterpret_cast<const char *>(&b[pos]), 4);
        const uint32_t size = be32(&b[pos + 4]);
        const size_t body = pos + 8;
        if (body + size > b.size() && id != "SSND") throw FormatError("truncated chunk " + id);
        f.chunk_ids.push_back(id);
        if (id == "COMM") {
            if (size < 18) throw FormatError("short COMM chunk");
            f.channels = be16(&b[body]);
            frames = be32(&b[body + 2]);
            bits = be16(&b[body + 6]);
            f.sample_rate = be_extended(&b[body + 8]);
            if (aifc && size >= 22) comp.assign(reinterpret_cast<const char *>(&b[body + 18]), 4);
            have_comm = true;
        } else if (id == "SSND") {
            // offset + blockSize precede the samples; the chunk may run past
            // EOF (exempt above) but those 8 bytes must be there
            if (size < 8 || body + 8 > b.size()) throw FormatError("truncated SSND chunk");
            const uint32_t offset = be32(&b[body]);
            f.data_offset = body + 8 + offset;
            have_ssnd = true;
        }
        pos = body + size + (size & 1);
    }
    if (!have_comm || !have_ssnd) throw FormatError("AIFF file without COMM or SSND chunk");
    f.bits = bits;
    if (comp == "NONE" || comp == "twos") f.pcm_format = pcm_int_format(bits, true);
    else if (comp == "sowt") f.pcm_format = pcm_int_format(bits, false);
    else if ((comp == "fl32" || comp == "FL32") && bits == 32) f.pcm_format = LCFIR_PCM_F32BE;
    else throw FormatError("unsupported AIFF-C compression '" + comp + "'");
    f.frames = frames;
    f.data_bytes = (size_t)frames * (size_t)f.channels * (size_t)(bits / 8);
    if (f.data_offset + f.data_bytes > b.size()) throw FormatError("SSND shorter than COMM says");
}
} // namespace detail

inline AudioFile read_audio_file(const std::string &path, const Allocator &alloc = heap_alloc) {
    std::ifstream in(path, std::ios::binary | std::ios::ate);
    if (!in) throw std::runtime_error("cannot open " + path);
    AudioFile f;
    f.size = (size_t)in.tellg();
    f.storage = alloc(f.size);
    f.data = f.storage.get();
    in.seekg(0);
    if (f.size && !in.read(reinterpret_cast<char *>(f.data), (std::streamsize)f.size))
        throw std::runtime_error("read failed: " + path);
    const detail::ByteView b{f.data, f.size};
    if (b.size() < 12) throw FormatError("file too short: " + path);
    const std::string riff(reinterpret_cast<const char *>(&b[0]), 4);
    const std::string kind(reinterpret_cast<const char *>(&b[8]), 4);
    if (riff == "RIFF" && kind == "WAVE") {
        f.kind = AudioFile::Kind::Wave;
        detail::parse_wave(f);
    } else if (riff == "FORM" && (kind == "AIFF" || kind == "AIFC")) {
        f.kind = AudioFile::Kind::Aiff;
        detail::parse_aiff(f, kind == "AIFC");
    } else {
        throw FormatError("not a WAVE or AIFF file: " + path);
    }
    if (f.channels < 1) throw FormatError("no channels");
    const int bps = lcfir_pcm_bytes(f.pcm_format);
    if (f.kind == AudioFile::Kind::Wave) {
        f.frames = (int64_t)(f.data_bytes / ((size_t)bps * (size_t)f.channels));
        f.data_bytes = (size_t)f.frames * (size_t)bps * (size_t)f.channels;
    }
    return f;
}

inline void write_bytes(const std::string &path, const uint8_t *data, size_t size) {
    std::ofstream out(path, std::ios::binary | std::ios::trunc);
    if (!out) throw std::runtime_error("cannot create " + path);
    out.write(reinterpret_cast<const char *>(data), (std::streamsize)size);
    if (!out) throw std::runtime_error("write failed: " + path);
}

} // namespace lcfir_host
