// RIFF/WAVE header parser shared by libmsdsp's reader (ingest.hip) and the CPU sanitizer harness
// (host_check.cpp): plain C++, no HIP.  It restates what scipy.io.wavfile.read (scipy 1.15,
// scipy/io/wavfile.py:568-733 read(), _read_fmt_chunk, _read_data_chunk, _skip_unknown_chunk)
// accepts and how it sizes the data, for little-endian RIFF (the reference reads its files with it,
// dsp/src/main.py:249):
//   * the chunk walk runs while the position is inside the RIFF size + 8 (read()'s file_size);
//   * "fmt ": size < 16 is an error; WAVE_FORMAT_EXTENSIBLE with size >= 18 needs cbSize >= 22 and
//     the standard GUID tail, whose first 4 bytes are then the format; only PCM and IEEE float are
//     known; PCM needs nAvgBytesPerSec == nSamplesPerSec * nBlockAlign; the chunk is skipped by
//     max(size, bytes read) and its pad byte;
//   * "data": the container size is nBlockAlign / nChannels (integer division), the sample count
//     size // container, capped at the complete containers the file holds (numpy.fromfile reads
//     what is there); several channels must divide it (scipy's reshape);
//   * any other chunk is skipped by its size and its pad byte.
// Differences, all refusals of files scipy reads: RIFX / RF64, containers of 5..8 bytes and
// 64-bit PCM, and the walk stops at the first "data" chunk (scipy keeps walking: a later chunk can
// still raise, a later "data" chunk replaces the first).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

namespace msd {
namespace wav {

// dtype codes as include/msdsp.h (MSD_U8 .. MSD_F64)
enum : int { D_U8 = 1, D_I16 = 2, D_I32 = 3, D_F32 = 4, D_F64 = 5 };
// result codes as include/msdsp.h
enum : int { OK = 0, E_INVALID = -1, E_UNSUPPORTED = -3 };

struct Header {
    int rate = 0, channels = 0, bits = 0, format = 0, dtype = 0;
    int container = 0;          // bytes per sample in the file (nBlockAlign / nChannels)
    int64_t frames = 0;         // complete frames of the data chunk that the file holds
    int64_t data_offset = 0, data_bytes = 0;
};

inline uint16_t le16(const unsigned char *b) { return (uint16_t)(b[0] | (b[1] << 8)); }
inline uint32_t le32(const unsigned char *b) {
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

// rd(dst, n, off) reads exactly n bytes at off or returns false; fsize = file size in bytes.
// Returns OK or an error code with msg set.
template <typename Read>
int parse(Read &&rd, int64_t fsize, Header &h, std::string &msg) {
    auto err = [&](int code, const std::string &m) {
        msg = m;
        return code;
    };
    unsigned char head[12];
    if (fsize < 12 || !rd(head, 12, 0)) return err(E_INVALID, "wav: File format not understood (short file)");
    if (std::memcmp(head, "RIFX", 4) == 0) return err(E_UNSUPPORTED, "wav: big-endian RIFX files are not supported");
    if (std::memcmp(head, "RF64", 4) == 0) return err(E_UNSUPPORTED, "wav: RF64 files are not supported");
    if (std::memcmp(head, "RIFF", 4) != 0 || std::memcmp(head + 8, "WAVE", 4) != 0)
        return err(E_INVALID, "wav: File format not understood. Only 'RIFF' WAV files are supported.");
    const int64_t file_size = (int64_t)le32(head + 4) + 8;
    int64_t pos = 12;
    bool have_fmt = false;
    int tag = 0, channels = 0, bits = 0, block_align = 0;
    uint32_t rate = 0, byte_rate = 0;
    while (pos < file_size) {
        if (pos >= fsize) return err(E_INVALID, "wav: Unexpected end of file.");
        if (pos + 4 > fsize) return err(E_INVALID, "wav: Incomplete chunk ID");
        unsigned char c[8];
        if (pos + 8 > fsize || !rd(c, 8, pos)) return err(E_INVALID, "wav: Unexpected end of file: truncated chunk header");
        const uint32_t size = le32(c + 4);
        if (std::memcmp(c, "fmt ", 4) == 0) {
            if (size < 16) return err(E_INVALID, "wav: Binary structure of wave file is not compliant (fmt size < 16)");
            unsigned char f[40] = {};
            if (!rd(f, 16, pos + 8)) return err(E_INVALID, "wav: Unexpected end of file in the fmt chunk");
            int64_t got = 16;
            tag = le16(f);
            channels = le16(f + 2);
            rate = le32(f + 4);
            byte_rate = le32(f + 8);
            block_align = le16(f + 12);
            bits = le16(f + 14);
            if (tag == 0xFFFE && size >= 18) {  // WAVE_FORMAT_EXTENSIBLE
                if (!rd(f + 16, 2, pos + 8 + 16)) return err(E_INVALID, "wav: Unexpected end of file in the fmt chunk");
                got += 2;
                if (le16(f + 16) < 22)
                    return err(E_INVALID, "wav: Binary structure of wave file is not compliant (cbSize < 22)");
                if (!rd(f + 18, 22, pos + 8 + 18)) return err(E_INVALID, "wav: Unexpected end of file in the fmt chunk");
                got += 22;
                static const unsigned char tail[12] = {0x00, 0x00, 0x10, 0x00, 0x80, 0x00,
                                                       0x00, 0xAA, 0x00, 0x38, 0x9B, 0x71};
                if (std::memcmp(f + 24 + 4, tail, 12) == 0) tag = (int)le32(f + 24);
            }
            if (tag != 1 && tag != 3)
                return err(E_UNSUPPORTED, "wav: Unknown wave file format. Supported formats: PCM, IEEE_FLOAT");
            if (tag == 1 && (uint64_t)byte_rate != (uint64_t)rate * (uint64_t)block_align)
                return err(E_INVALID, "wav: WAV header is invalid: nAvgBytesPerSec must equal product of "
                                      "nSamplesPerSec and nBlockAlign");
            have_fmt = true;
            pos += 8 + ((int64_t)size > got ? (int64_t)size : got) + (size & 1);
        } else if (std::memcmp(c, "data", 4) == 0) {
            if (!have_fmt) return err(E_INVALID, "wav: No fmt chunk before data");
            if (channels <= 0) return err(E_INVALID, "wav: zero channels (integer division by zero in scipy)");
            const int cont = block_align / channels;
            if (cont <= 0) return err(E_INVALID, "wav: zero-byte sample container (nBlockAlign < nChannels)");
            int dtype = 0;
            if (tag == 1) {
                if (bits >= 1 && bits <= 8) dtype = cont == 1 ? D_U8 : 0;
                else if (bits > 64) return err(E_INVALID, "wav: Unsupported bit depth for integer data");
                else dtype = cont == 2 ? D_I16 : (cont == 3 || cont == 4) ? D_I32 : 0;
                if (!dtype) return err(E_UNSUPPORTED, "wav: unsupported integer sample container");
            } else {
                if (bits != 32 && bits != 64) return err(E_UNSUPPORTED, "wav: Unsupported bit depth for floating-point data");
                dtype = cont == 4 ? D_F32 : cont == 8 ? D_F64 : 0;
                if (!dtype) return err(E_UNSUPPORTED, "wav: unsupported floating-point sample container");
            }
            const int64_t start = pos + 8;
            const int64_t have = fsize > start ? fsize - start : 0;
            int64_t n = (int64_t)size / cont;           // n_samples
            if (have / cont < n) n = have / cont;       // numpy.fromfile: what the file holds
            if (channels > 1 && n % channels) return err(E_INVALID, "wav: cannot reshape the data into whole frames");
            h.rate = (int)rate;
            h.channels = channels;
            h.bits = bits;
            h.format = tag;
            h.dtype = dtype;
            h.container = cont;
            h.frames = n / channels;
            h.data_offset = start;
            h.data_bytes = n * cont;
            return OK;
        } else {
            pos += 8 + (int64_t)size + (size & 1);
        }
    }
    return err(E_INVALID, "wav: Unexpected end of file: no data chunk inside the RIFF size");
}

// frames [frame0, frame0 + nframes) of channel `channel` (-1: all, interleaved) decoded into dst
// (dst_bytes): the container's bytes as they are, 3-byte containers widened into the top 3 bytes of
// an int32 (scipy's layout).  stage: scratch for the gathering reads (grown as needed).
template <typename Read, typename Vec>
int read_frames(Read &&rd, const Header &h, int channel, int64_t frame0, int64_t nframes, void *dst, int64_t dst_bytes,
                Vec &stage, std::string &msg) {
    auto err = [&](int code, const std::string &m) {
        msg = m;
        return code;
    };
    if (frame0 < 0 || nframes < 0 || frame0 > h.frames || nframes > h.frames - frame0)
        return err(E_INVALID, "msd_wav_read: frame range outside the data chunk");
    if (channel < -1 || channel >= h.channels) return err(E_INVALID, "msd_wav_read: no such channel");
    if (nframes == 0) return OK;
    const int in_b = h.container;
    const bool w24 = in_b == 3;
    const int out_b = w24 ? 4 : in_b;
    const int nch = channel < 0 ? h.channels : 1;
    if (!dst || dst_bytes / out_b / nch < nframes) return err(-5, "msd_wav_read: destination too small");
    const int64_t frame_b = (int64_t)in_b * h.channels;
    const int64_t off = h.data_offset + frame0 * frame_b;
    char *out = static_cast<char *>(dst);
    if (!w24 && (channel < 0 || h.channels == 1)) {  // the common case: one read
        if (!rd(out, (size_t)(nframes * frame_b), off)) return err(E_INVALID, "wav: short read");
        return OK;
    }
    const int64_t chunk = 1 << 16;  // frames per staging read
    if ((int64_t)stage.size() < chunk * frame_b) stage.resize((size_t)(chunk * frame_b));
    for (int64_t f0 = 0; f0 < nframes; f0 += chunk) {
        const int64_t m = nframes - f0 < chunk ? nframes - f0 : chunk;
        if (!rd(stage.data(), (size_t)(m * frame_b), off + f0 * frame_b)) return err(E_INVALID, "wav: short read");
        for (int64_t i = 0; i < m; ++i) {
            for (int c = 0; c < nch; ++c) {
                const int ch = channel < 0 ? c : channel;
                const unsigned char *src = stage.data() + i * frame_b + (int64_t)ch * in_b;
                char *d = out + ((f0 + i) * nch + c) * out_b;
                if (w24) {
                    const uint32_t v = ((uint32_t)src[0] << 8) | ((uint32_t)src[1] << 16) | ((uint32_t)src[2] << 24);
                    std::memcpy(d, &v, 4);
                } else {
                    std::memcpy(d, src, (size_t)in_b);
                }
            }
        }
    }
    return OK;
}

}  // namespace wav
}  // namespace msd
