// WAV ingest straight into (pinned) host memory and the copy stream that moves it to HBM —
// SURVEY §8(f) row 1.  The parse follows what scipy.io.wavfile.read accepts and returns for
// the reference's files (dsp/src/main.py:249; scipy/io/wavfile.py:568-733): RIFF little-endian,
// chunks walked to "fmt " and "data", PCM 8 (uint8) / 16 (int16) / 24 (int32 with the sample
// in the top 3 bytes) / 32 (int32), IEEE float 32 / 64, WAVE_FORMAT_EXTENSIBLE's sub-format.
// Samples are read with pread directly into the caller's buffer (one channel is gathered from
// interleaved frames through a bounded staging buffer).
#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <vector>

#include "msd_internal.h"

namespace msd {
namespace {

struct Fd {
    int fd = -1;
    explicit Fd(const char *path) { fd = ::open(path, O_RDONLY | O_CLOEXEC); }
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

bool pread_all(int fd, void *dst, size_t n, int64_t off) {
    char *p = static_cast<char *>(dst);
    while (n > 0) {
        const ssize_t r = ::pread(fd, p, n, (off_t)off);
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
        off += r;
    }
    return true;
}

uint16_t le16(const unsigned char *b) { return (uint16_t)(b[0] | (b[1] << 8)); }
uint32_t le32(const unsigned char *b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24); }

int probe_fd(int fd, const char *path, msd_wav_info *info) {
    unsigned char h[12];
    if (!pread_all(fd, h, 12, 0)) return fail(MSD_ERR_INVALID, std::string("wav: short file: ") + path);
    if (std::memcmp(h, "RIFX", 4) == 0) return fail(MSD_ERR_UNSUPPORTED, "wav: big-endian RIFX files are not supported");
    if (std::memcmp(h, "RIFF", 4) != 0 || std::memcmp(h + 8, "WAVE", 4) != 0)
        return fail(MSD_ERR_INVALID, "wav: File format not understood. Only 'RIFF' WAV files are supported.");
    const off_t fsize = ::lseek(fd, 0, SEEK_END);
    int64_t pos = 12;
    bool have_fmt = false;
    int tag = 0, channels = 0, rate = 0, bits = 0;
    while (true) {
        unsigned char c[8];
        if (pos + 8 > fsize || !pread_all(fd, c, 8, pos)) return fail(MSD_ERR_INVALID, "wav: Unexpected end of file: no data chunk");
        const uint32_t size = le32(c + 4);
        if (std::memcmp(c, "fmt ", 4) == 0) {
            unsigned char f[40] = {};
            const uint32_t want = size < 40 ? size : 40;
            if (want < 16 || !pread_all(fd, f, want, pos + 8)) return fail(MSD_ERR_INVALID, "wav: bad fmt chunk");
            tag = le16(f);
            channels = le16(f + 2);
            rate = (int)le32(f + 4);
            bits = le16(f + 14);
            if (tag == 0xFFFE && want >= 26) tag = le16(f + 24);  // WAVE_FORMAT_EXTENSIBLE sub-format
            have_fmt = true;
        } else if (std::memcmp(c, "data", 4) == 0) {
            if (!have_fmt) return fail(MSD_ERR_INVALID, "wav: No fmt chunk before data");
            const int64_t start = pos + 8;
            int64_t bytes = size;
            if (start + bytes > fsize) bytes = fsize - start;
            int dtype = 0;
            if (tag == 1) {
                dtype = bits == 8 ? MSD_U8 : bits == 16 ? MSD_I16 : (bits == 24 || bits == 32) ? MSD_I32 : 0;
                if (!dtype) return fail(MSD_ERR_UNSUPPORTED, "wav: Unsupported bit depth for integer data");
            } else if (tag == 3) {
                dtype = bits == 32 ? MSD_F32 : bits == 64 ? MSD_F64 : 0;
                if (!dtype) return fail(MSD_ERR_UNSUPPORTED, "wav: Unsupported bit depth for floating-point data");
            } else {
                return fail(MSD_ERR_UNSUPPORTED, "wav: Unknown wave file format. Supported formats: PCM, IEEE_FLOAT");
            }
            if (channels <= 0) return fail(MSD_ERR_INVALID, "wav: zero channels");
            info->rate = rate;
            info->channels = channels;
            info->bits = bits;
            info->format = tag;
            info->dtype = dtype;
            info->reserved = 0;
            info->frames = bytes / ((bits / 8) * (int64_t)channels);
            info->data_offset = start;
            info->data_bytes = bytes;
            return MSD_OK;
        }
        pos += 8 + (int64_t)size + (size & 1);
    }
}

}  // namespace
}  // namespace msd

using namespace msd;

extern "C" {

int msd_wav_probe(const char *path, msd_wav_info *info) {
    if (!path || !info) return fail(MSD_ERR_INVALID, "msd_wav_probe: null");
    Fd f(path);
    if (f.fd < 0) return fail(MSD_ERR_INVALID, std::string("wav: cannot open ") + path);
    return probe_fd(f.fd, path, info);
}

int msd_wav_read(const char *path, int32_t channel, int64_t frame0, int64_t nframes, void *dst, int64_t dst_bytes,
                 msd_wav_info *info) {
    if (!path || !info || (!dst && nframes > 0)) return fail(MSD_ERR_INVALID, "msd_wav_read: null");
    Fd f(path);
    if (f.fd < 0) return fail(MSD_ERR_INVALID, std::string("wav: cannot open ") + path);
    int rc = probe_fd(f.fd, path, info);
    if (rc) return rc;
    if (frame0 < 0 || nframes < 0 || frame0 + nframes > info->frames)
        return fail(MSD_ERR_INVALID, "msd_wav_read: frame range outside the data chunk");
    if (channel < -1 || channel >= info->channels) return fail(MSD_ERR_INVALID, "msd_wav_read: no such channel");
    const int in_b = info->bits / 8;
    const int out_b = info->bits == 24 ? 4 : in_b;
    const int nch = channel < 0 ? info->channels : 1;
    if (dst_bytes < nframes * nch * out_b) return fail(MSD_ERR_CAPACITY, "msd_wav_read: destination too small");
    const int64_t frame_b = (int64_t)in_b * info->channels;
    const int64_t off = info->data_offset + frame0 * frame_b;
    char *out = static_cast<char *>(dst);
    if (info->bits != 24 && (channel < 0 || info->channels == 1)) {  // the common case: one pread
        if (!pread_all(f.fd, out, (size_t)(nframes * frame_b), off)) return fail(MSD_ERR_INVALID, "wav: short read");
        return MSD_OK;
    }
    // staged: gather one channel and / or widen 24-bit samples
    const int64_t chunk = 1 << 16;  // frames per staging read
    std::vector<unsigned char> st((size_t)(chunk * frame_b));
    for (int64_t f0 = 0; f0 < nframes; f0 += chunk) {
        const int64_t m = nframes - f0 < chunk ? nframes - f0 : chunk;
        if (!pread_all(f.fd, st.data(), (size_t)(m * frame_b), off + f0 * frame_b))
            return fail(MSD_ERR_INVALID, "wav: short read");
        for (int64_t i = 0; i < m; ++i) {
            for (int c = 0; c < nch; ++c) {
                const int ch = channel < 0 ? c : channel;
                const unsigned char *s = st.data() + i * frame_b + (int64_t)ch * in_b;
                char *d = out + ((f0 + i) * nch + c) * out_b;
                if (info->bits == 24) {  // scipy: the 3 bytes in the top of an int32
                    const uint32_t v = ((uint32_t)s[0] << 8) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 24);
                    std::memcpy(d, &v, 4);
                } else {
                    std::memcpy(d, s, in_b);
                }
            }
        }
    }
    return MSD_OK;
}

int msd_host_alloc(msd_ctx *ctx, size_t bytes, void **ptr) {
    if (!ctx || !ptr) return fail(MSD_ERR_INVALID, "msd_host_alloc: null");
    DeviceGuard g(ctx->device);
    *ptr = nullptr;
    MSD_HIP(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault));
    return MSD_OK;
}

int msd_host_free(msd_ctx *ctx, void *ptr) {
    if (!ctx) return fail(MSD_ERR_INVALID, "msd_host_free: null ctx");
    if (!ptr) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipHostFree(ptr));
    return MSD_OK;
}

static int copy_stream(msd_ctx *ctx) {
    if (!ctx->copy_stream) MSD_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    if (!ctx->fence_ev) MSD_HIP(hipEventCreateWithFlags(&ctx->fence_ev, hipEventDisableTiming));
    return MSD_OK;
}

int msd_memcpy_h2d_async(msd_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return fail(MSD_ERR_INVALID, "msd_memcpy_h2d_async: null");
    DeviceGuard g(ctx->device);
    int rc = copy_stream(ctx);
    if (rc) return rc;
    if (bytes) MSD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->copy_stream));
    return MSD_OK;
}

int msd_fence(msd_ctx *ctx, int direction) {
    if (!ctx || (direction != 0 && direction != 1)) return fail(MSD_ERR_INVALID, "msd_fence: bad args");
    DeviceGuard g(ctx->device);
    int rc = copy_stream(ctx);
    if (rc) return rc;
    hipStream_t from = direction == 0 ? ctx->copy_stream : ctx->stream;
    hipStream_t to = direction == 0 ? ctx->stream : ctx->copy_stream;
    MSD_HIP(hipEventRecord(ctx->fence_ev, from));
    MSD_HIP(hipStreamWaitEvent(to, ctx->fence_ev, 0));
    return MSD_OK;
}

int msd_stream_wait(msd_ctx *waiter, msd_ctx *signaler) {
    if (!waiter || !signaler || waiter == signaler) return fail(MSD_ERR_INVALID, "msd_stream_wait: bad args");
    if (waiter->device != signaler->device) return fail(MSD_ERR_INVALID, "msd_stream_wait: contexts on different devices");
    DeviceGuard g(signaler->device);
    if (!signaler->join_ev) MSD_HIP(hipEventCreateWithFlags(&signaler->join_ev, hipEventDisableTiming));
    MSD_HIP(hipEventRecord(signaler->join_ev, signaler->stream));
    MSD_HIP(hipStreamWaitEvent(waiter->stream, signaler->join_ev, 0));
    return MSD_OK;
}

int msd_copy_synchronize(msd_ctx *ctx) {
    if (!ctx) return fail(MSD_ERR_INVALID, "msd_copy_synchronize: null");
    if (!ctx->copy_stream) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipStreamSynchronize(ctx->copy_stream));
    return MSD_OK;
}

}  // extern "C"
