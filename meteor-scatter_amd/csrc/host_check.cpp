// CPU-only sanitizer harness for libmsdsp's host C++ that parses untrusted input or plans device
// work (SURVEY §5 "race detection / sanitizers"): built with g++ -fsanitize=address,undefined by
// `make -C meteor-scatter_amd/csrc sanitize` (no HIP; the same headers ingest.hip, stream.hip and
// refine.hip compile), driven by tests/test_sanitize.py.
//   host_check wav FILE            parse + decode FILE (wav_parse.h) with pread, as msd_wav_probe /
//                                  msd_wav_read do: "ok rate channels bits format dtype container
//                                  frames data_offset data_bytes fnv1a64" or "err CODE MESSAGE";
//                                  every channel is also gathered alone and checked against the
//                                  interleaved read
//   host_check program N           np_program.h's leaf records for an N-element np.sum: checks
//                                  they tile [0, N) in <= 128-element leaves with numpy's chunking
//   host_check refine N HOP BLO BHI NLO NHI NSAMP [A B]...
//                                  refine_plan.h for frame ranges [A, B): checks the block mapping
//   host_check fuzz SEED ITERS     mutated / truncated WAV images parsed and decoded in memory,
//                                  random programs and refinement plans
#include <fcntl.h>
#include <unistd.h>

#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "np_program.h"
#include "refine_plan.h"
#include "wav_parse.h"

namespace {

using msd::wav::Header;

uint64_t fnv1a(const unsigned char *p, size_t n, uint64_t h = 1469598103934665603ull) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

int out_bytes(const Header &h) { return h.container == 3 ? 4 : h.container; }

// decode everything (interleaved), then every channel alone and compare
template <typename Read>
int decode_all(Read &rd, const Header &h, std::vector<unsigned char> &buf, std::string &msg) {
    std::vector<unsigned char> stage;
    const int ob = out_bytes(h);
    buf.assign((size_t)(h.frames * h.channels * ob), 0);
    int rc = msd::wav::read_frames(rd, h, -1, 0, h.frames, buf.data(), (int64_t)buf.size(), stage, msg);
    if (rc) return rc;
    std::vector<unsigned char> one((size_t)(h.frames * ob) + 1);
    for (int c = 0; c < h.channels && c < 8; ++c) {
        rc = msd::wav::read_frames(rd, h, c, 0, h.frames, one.data(), (int64_t)(h.frames * ob), stage, msg);
        if (rc) return rc;
        for (int64_t i = 0; i < h.frames; ++i)
            if (std::memcmp(one.data() + i * ob, buf.data() + (i * h.channels + c) * ob, (size_t)ob)) {
                msg = "channel gather differs from the interleaved read";
                return -100;
            }
    }
    // a sub-range and the bounds checks
    if (h.frames > 2) {
        rc = msd::wav::read_frames(rd, h, -1, 1, h.frames - 2, one.data(), 0, stage, msg);
        if (rc != -5) {
            msg = "a zero-byte destination was accepted";
            return -100;
        }
    }
    if (msd::wav::read_frames(rd, h, -1, h.frames, 1, buf.data(), (int64_t)buf.size(), stage, msg) == 0) {
        msg = "a range past the data was accepted";
        return -100;
    }
    msg.clear();
    return 0;
}

int cmd_wav(const char *path) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) {
        std::printf("err -1 cannot open\n");
        return 0;
    }
    const off_t fsize = ::lseek(fd, 0, SEEK_END);
    auto rd = [&](void *dst, size_t n, int64_t off) {
        char *p = static_cast<char *>(dst);
        while (n > 0) {
            const ssize_t r = ::pread(fd, p, n, (off_t)off);
            if (r <= 0) return false;
            p += r;
            n -= (size_t)r;
            off += r;
        }
        return true;
    };
    Header h;
    std::string msg;
    int rc = msd::wav::parse(rd, (int64_t)fsize, h, msg);
    std::vector<unsigned char> buf;
    if (!rc) rc = decode_all(rd, h, buf, msg);
    ::close(fd);
    if (rc) {
        std::printf("err %d %s\n", rc, msg.c_str());
        return rc == -100 ? 1 : 0;
    }
    std::printf("ok %d %d %d %d %d %d %" PRId64 " %" PRId64 " %" PRId64 " %016" PRIx64 "\n", h.rate, h.channels, h.bits,
                h.format, h.dtype, h.container, h.frames, h.data_offset, h.data_bytes, fnv1a(buf.data(), buf.size()));
    return 0;
}

bool check_program(int64_t n, std::string &why) {
    std::vector<msd::LeafRec> r;
    msd::build_program(n, r);
    int64_t pos = 0, chunks = 0, depth = 0;
    for (size_t i = 0; i < r.size(); ++i) {
        const auto &l = r[i];
        if (l.off != pos || l.len <= 0 || l.len > 128 || l.adds < 0) {
            why = "leaf " + std::to_string(i) + " does not continue the tiling";
            return false;
        }
        pos += l.len;
        depth += 1 - l.adds;  // a leaf pushes one partial sum, each add pops one
        if (depth < 1) {
            why = "an add with fewer than two partial sums";
            return false;
        }
        if (l.chunk_end) {
            if (depth != 1 || (pos % msd::NP_CHUNK && pos != n)) {
                why = "a chunk ends with " + std::to_string(depth) + " partial sums at " + std::to_string(pos);
                return false;
            }
            depth = 0;
            ++chunks;
        }
    }
    if (pos != n || chunks != (n + msd::NP_CHUNK - 1) / msd::NP_CHUNK || depth != 0) {
        why = "the records cover " + std::to_string(pos) + " of " + std::to_string(n);
        return false;
    }
    return true;
}

bool check_plan(const msd::RefinePlan &P, const std::vector<int64_t> &ranges, int64_t nsamp, std::string &why) {
    const auto &G = P.G;
    const auto &K = P.K;
    if (G.D <= 0 || G.N % G.D || G.hop % G.D || G.R * G.D != G.N) {
        why = "block geometry";
        return false;
    }
    // block_kernel's assumptions (refine.hip): 16 lanes x D/16 samples loaded as aligned quads, so
    // the row path needs D % 64 == 0; any other D must take the one-lane path
    if (G.rows != (G.D % 64 == 0 ? 1 : 0) || (G.rows && (G.L * 16 != G.D || G.L % 4)) || (!G.rows && G.L != G.D)) {
        why = "kernel path";
        return false;
    }
    if (K.nk < 0 || K.nk > msd::RF_MAXK || K.nb > msd::RF_MAXK / 2 || K.nn > msd::RF_MAXK / 2) {
        why = "bin counts";
        return false;
    }
    for (int q = 0; q < K.nb + K.nn; ++q)
        for (int t = 0; t < 3; ++t) {
            const int v = q < K.nb ? K.bidx[q][t] : K.nidx[q - K.nb][t];
            if (v < 0 || v >= K.nk) {
                why = "tap index";
                return false;
            }
        }
    const int64_t nr = (int64_t)ranges.size() / 2;
    for (int64_t r = 0; r < nr; ++r) {
        const int64_t a = ranges[2 * r], b = ranges[2 * r + 1];
        if (P.fcs[r + 1] - P.fcs[r] != b - a || P.fstart[r] != a) {
            why = "frame mapping";
            return false;
        }
        // every frame's R blocks inside its range's compact block range, and inside the samples
        const int64_t nb = P.bcs[r + 1] - P.bcs[r];
        for (int64_t t : {a, b - 1}) {
            const int64_t m0 = t * G.hop / G.D - P.bstart[r];
            if (m0 < 0 || m0 + G.R > nb || (t * G.hop / G.D + G.R) * G.D > nsamp) {
                why = "block mapping";
                return false;
            }
        }
    }
    if (P.nblocks != P.bcs[nr] || P.nframes != P.fcs[nr] || !(G.chain > 0) || !(G.scale > 0)) {
        why = "totals";
        return false;
    }
    return true;
}

int cmd_program(int64_t n) {
    std::string why;
    if (!check_program(n, why)) {
        std::printf("bad %s\n", why.c_str());
        return 1;
    }
    std::vector<msd::LeafRec> r;
    msd::build_program(n, r);
    std::printf("ok %zu\n", r.size());
    return 0;
}

int cmd_refine(int argc, char **argv) {
    const int N = std::atoi(argv[0]);
    const int64_t hop = std::atoll(argv[1]);
    const int blo = std::atoi(argv[2]), bhi = std::atoi(argv[3]), nlo = std::atoi(argv[4]), nhi = std::atoi(argv[5]);
    const int64_t nsamp = std::atoll(argv[6]);
    std::vector<int64_t> ranges;
    for (int i = 7; i < argc; ++i) ranges.push_back(std::atoll(argv[i]));
    msd::RefinePlan P;
    std::string msg;
    const int rc = msd::plan_refine(N, hop, 192000.0, blo, bhi, nlo, nhi, ranges.data(), (int64_t)ranges.size() / 2,
                                    nsamp, P, msg);
    if (rc) {
        std::printf("err %d %s\n", rc, msg.c_str());
        return 0;
    }
    std::string why;
    if (!check_plan(P, ranges, nsamp, why)) {
        std::printf("bad %s\n", why.c_str());
        return 1;
    }
    std::printf("ok %d %d %d %" PRId64 " %" PRId64 " %d\n", P.K.nk, P.G.D, P.G.R, P.nblocks, P.nframes, P.G.rows);
    return 0;
}

// a valid little-endian WAV image
std::vector<unsigned char> make_wav(std::mt19937_64 &g, int &channels) {
    auto put16 = [](std::vector<unsigned char> &v, int x) {
        v.push_back((unsigned char)(x & 255));
        v.push_back((unsigned char)((x >> 8) & 255));
    };
    auto put32 = [](std::vector<unsigned char> &v, uint32_t x) {
        for (int i = 0; i < 4; ++i) v.push_back((unsigned char)((x >> (8 * i)) & 255));
    };
    static const int conts[] = {1, 2, 3, 4, 4, 8};
    static const int tags[] = {1, 1, 1, 1, 3, 3};
    const int pick = (int)(g() % 6);
    const int cont = conts[pick], tag = tags[pick], bits = cont * 8;
    channels = 1 + (int)(g() % 3);
    const int frames = (int)(g() % 300);
    const bool ext = g() % 3 == 0;
    std::vector<unsigned char> fmt;
    put16(fmt, ext ? 0xFFFE : tag);
    put16(fmt, channels);
    put32(fmt, 48000);
    put32(fmt, 48000u * (uint32_t)(cont * channels));
    put16(fmt, cont * channels);
    put16(fmt, bits);
    if (ext) {
        put16(fmt, 22);
        put16(fmt, bits);
        put32(fmt, 0);
        static const unsigned char tail[12] = {0x00, 0x00, 0x10, 0x00, 0x80, 0x00, 0x00, 0xAA, 0x00, 0x38, 0x9B, 0x71};
        put32(fmt, (uint32_t)tag);
        fmt.insert(fmt.end(), tail, tail + 12);
    }
    std::vector<unsigned char> w = {'R', 'I', 'F', 'F', 0, 0, 0, 0, 'W', 'A', 'V', 'E'};
    if (g() % 2) {  // an odd-sized chunk before fmt
        const char *id = "LIST";
        w.insert(w.end(), id, id + 4);
        put32(w, 5);
        for (int i = 0; i < 6; ++i) w.push_back((unsigned char)g());
    }
    const char *f = "fmt ";
    w.insert(w.end(), f, f + 4);
    put32(w, (uint32_t)fmt.size());
    w.insert(w.end(), fmt.begin(), fmt.end());
    const char *d = "data";
    w.insert(w.end(), d, d + 4);
    const uint32_t nbytes = (uint32_t)(frames * channels * cont);
    put32(w, nbytes);
    for (uint32_t i = 0; i < nbytes; ++i) w.push_back((unsigned char)g());
    if (nbytes & 1) w.push_back(0);
    const uint32_t riff = (uint32_t)(w.size() - 8);
    std::memcpy(w.data() + 4, &riff, 4);
    return w;
}

int cmd_fuzz(uint64_t seed, int64_t iters) {
    std::mt19937_64 g(seed);
    int64_t parsed = 0, rejected = 0;
    for (int64_t it = 0; it < iters; ++it) {
        int ch = 1;
        std::vector<unsigned char> w = make_wav(g, ch);
        const int kind = (int)(g() % 6);
        if (kind == 1 && !w.empty()) w.resize(g() % w.size());  // truncated anywhere
        if (kind >= 2) {                                       // 1-8 random bytes / fields
            const int k = 1 + (int)(g() % 8);
            for (int i = 0; i < k && !w.empty(); ++i) w[g() % w.size()] = (unsigned char)g();
        }
        if (kind == 5 && w.size() > 44) {  // a size field set to an extreme value
            static const uint32_t ext[] = {0xFFFFFFFFu, 0x7FFFFFFFu, 0u, 1u, 15u, 17u};
            const uint32_t v = ext[g() % 6];
            std::memcpy(w.data() + 4 + 4 * (g() % 8), &v, 4);
        }
        // exact-size copy: ASan catches any read past the image
        std::vector<unsigned char> img(w);
        auto rd = [&](void *dst, size_t n, int64_t off) {
            if (off < 0 || (uint64_t)off > img.size() || n > img.size() - (size_t)off) return false;
            std::memcpy(dst, img.data() + off, n);
            return true;
        };
        Header h;
        std::string msg;
        if (msd::wav::parse(rd, (int64_t)img.size(), h, msg)) {
            ++rejected;
            continue;
        }
        if (h.data_offset + h.data_bytes > (int64_t)img.size() || h.frames * h.channels * h.container != h.data_bytes) {
            std::printf("bad header sizes past the image (iter %" PRId64 ")\n", it);
            return 1;
        }
        std::vector<unsigned char> buf;
        const int rc = decode_all(rd, h, buf, msg);
        if (rc) {
            std::printf("bad decode %d %s (iter %" PRId64 ")\n", rc, msg.c_str(), it);
            return 1;
        }
        ++parsed;
    }
    for (int64_t it = 0; it < iters / 8 + 1; ++it) {
        const int64_t n = (int64_t)(g() % 70000);
        std::string why;
        if (!check_program(n, why)) {
            std::printf("bad program %" PRId64 ": %s\n", n, why.c_str());
            return 1;
        }
    }
    int64_t plans = 0;
    for (int64_t it = 0; it < iters / 4 + 1; ++it) {
        static const int Ns[] = {16, 256, 1024, 4096, 8192};
        const int N = Ns[g() % 5];
        const int64_t hop = 1 + (int64_t)(g() % (uint64_t)N);
        const int h = N / 2;
        auto rb = [&]() { return (int)(g() % (uint64_t)N) - h - 2; };
        int blo = rb(), bhi = blo + (int)(g() % 8) - 1, nlo = rb(), nhi = nlo + (int)(g() % 8) - 1;
        const int64_t nsamp = N + (int64_t)(g() % 20000);
        std::vector<int64_t> ranges;
        int64_t a = (int64_t)(g() % 50);
        const int nr = (int)(g() % 6);
        for (int r = 0; r < nr; ++r) {
            const int64_t b = a + 1 + (int64_t)(g() % 40);
            ranges.push_back(a);
            ranges.push_back(b);
            a = b + (int64_t)(g() % 30);
        }
        msd::RefinePlan P;
        std::string msg;
        if (msd::plan_refine(N, hop, 48000.0, blo, bhi, nlo, nhi, ranges.data(), (int64_t)ranges.size() / 2, nsamp, P,
                             msg))
            continue;
        std::string why;
        if (!check_plan(P, ranges, nsamp, why)) {
            std::printf("bad plan N %d hop %" PRId64 ": %s\n", N, hop, why.c_str());
            return 1;
        }
        // the density scale from a fresh window sum (the planner keeps its sum per frame length;
        // N changes between the plans here)
        double sw = 0.0;
        for (int n = 0; n < N; ++n) {
            const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * (double)n / (double)N);
            sw += w * w;
        }
        if (P.G.scale != 1.0 / (48000.0 * sw)) {
            std::printf("bad plan N %d: density scale\n", N);
            return 1;
        }
        ++plans;
    }
    std::printf("ok %" PRId64 " parsed %" PRId64 " rejected %" PRId64 " plans\n", parsed, rejected, plans);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc >= 3 && !std::strcmp(argv[1], "wav")) return cmd_wav(argv[2]);
    if (argc >= 3 && !std::strcmp(argv[1], "program")) return cmd_program(std::atoll(argv[2]));
    if (argc >= 9 && !std::strcmp(argv[1], "refine")) return cmd_refine(argc - 2, argv + 2);
    if (argc >= 4 && !std::strcmp(argv[1], "fuzz")) return cmd_fuzz(std::strtoull(argv[2], nullptr, 10), std::atoll(argv[3]));
    std::fprintf(stderr, "usage: host_check wav FILE | program N | refine N HOP BLO BHI NLO NHI NSAMP [A B]... | "
                         "fuzz SEED ITERS\n");
    return 2;
}
