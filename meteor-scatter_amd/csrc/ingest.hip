// WAV ingest straight into (pinned) host memory and the copy stream that moves it to HBM —
// SURVEY §8(f) row 1.  The parse (wav_parse.h) follows what scipy.io.wavfile.read accepts and
// returns for the reference's files (dsp/src/main.py:249; scipy/io/wavfile.py:568-733): RIFF
// little-endian, chunks walked to "fmt " and "data", PCM 8 (uint8) / 16 (int16) / 24 (int32 with
// the sample in the top 3 bytes) / 32 (int32), IEEE float 32 / 64, WAVE_FORMAT_EXTENSIBLE.
// Samples are read with pread directly into the caller's buffer (one channel is gathered from
// interleaved frames through a bounded staging buffer).
#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <vector>

#include "msd_internal.h"
#include "wav_parse.h"

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

// the header through wav_parse.h (scipy.io.wavfile.read's rules, shared with the CPU sanitizer
// harness); the container size rides in msd_wav_info.reserved
int probe_fd(int fd, const char *path, msd_wav_info *info, wav::Header *hout = nullptr) {
    const off_t fsize = ::lseek(fd, 0, SEEK_END);
    if (fsize < 0) return fail(MSD_ERR_INVALID, std::string("wav: cannot seek ") + path);
    wav::Header h;
    std::string msg;
    auto rd = [&](void *dst, size_t n, int64_t off) { return pread_all(fd, dst, n, off); };
    const int rc = wav::parse(rd, (int64_t)fsize, h, msg);
    if (rc) return fail(rc, msg + " (" + path + ")");
    info->rate = h.rate;
    info->channels = h.channels;
    info->bits = h.bits;
    info->format = h.format;
    info->dtype = h.dtype;
    info->reserved = h.container;
    info->frames = h.frames;
    info->data_offset = h.data_offset;
    info->data_bytes = h.data_bytes;
    if (hout) *hout = h;
    return MSD_OK;
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
    wav::Header h;
    int rc = probe_fd(f.fd, path, info, &h);
    if (rc) return rc;
    std::vector<unsigned char> stage;
    std::string msg;
    auto rd = [&](void *d, size_t n, int64_t off) { return pread_all(f.fd, d, n, off); };
    rc = wav::read_frames(rd, h, channel, frame0, nframes, dst, dst_bytes, stage, msg);
    return rc ? fail(rc, msg) : MSD_OK;
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
