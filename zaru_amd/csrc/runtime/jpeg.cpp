// jpeg.cpp -- the host half of the JPEG frame source: marker parsing and
// baseline Huffman entropy decoding (ITU T.81 F.2.2) into quantised coefficients, which the
// device half (kernels/jpeg.hip) turns into RGBA8 frames in HBM.  Entropy decoding is bit-serial
// within a scan, so it stays on a CPU core, as in every GPU JPEG pipeline; the pixel work
// (IDCT, upsampling, colour conversion: ~all of libjpeg-turbo's decode time) runs on the GPU.
// Streams with restart intervals (DRI) are entropy-decoded on the GPU too, one thread per
// interval (kernels/jpeg_huff.hip): only the scan bytes cross PCIe then.
// Supported: baseline sequential DCT (SOF0/SOF1), 8-bit samples, 1 or 3 components with luma
// sampling 1x1 / 2x1 / 2x2 over 1x1 chroma, one interleaved scan, restart intervals.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/zaru_hip.h"
#include "zr_jpeg.h"

namespace zr_internal {
int set_error(int code, const std::string &msg);
}

namespace {

constexpr uint8_t ZIGZAG[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    // canonical decoding (T.81 F.2.2.3): per code length the largest code and symbol offset
    int32_t maxcode[18];
    int32_t valoff[17];
    uint8_t vals[256];
    // 9-bit lookahead: (length << 8) | symbol, 0 = longer code
    uint16_t look[512];
    // AC only: code + magnitude bits within the 9-bit lookahead decoded in one step:
    // (value << 8) | (run << 4) | total bits, 0 = take the slow path
    int16_t fast_ac[512];
};

struct Comp {
    int id, h, v, tq, td, ta;
};

struct Header {
    int W = 0, H = 0, ncomp = 0;
    Comp comp[3];
    uint16_t q[4][64];  // natural order
    bool qpresent[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    int restart = 0;
    size_t scan_begin = 0;  // entropy-coded data
};

struct JpegError {
    int code;
    std::string msg;
};

[[noreturn]] void fail(const std::string &m) { throw JpegError{ZR_ERR_INVALID_ARGUMENT, "jpeg: " + m}; }

void build_huff(Huff &h, const uint8_t *counts, const uint8_t *vals, int nvals) {
    h.present = true;
    std::memcpy(h.vals, vals, nvals);
    int code = 0, k = 0;
    std::memset(h.look, 0, sizeof h.look);
    for (int len = 1; len <= 16; len++) {
        h.valoff[len] = k - code;
        for (int i = 0; i < counts[len - 1]; i++) {
            if (len <= 9) {  // fill every 9-bit lookahead slot this code prefixes
                const int shift = 9 - len;
                for (int f = 0; f < (1 << shift); f++) h.look[(code << shift) | f] = (uint16_t)((len << 8) | vals[k]);
            }
            code++;
            k++;
        }
        h.maxcode[len] = counts[len - 1] ? code - 1 : -1;
        if (code > (1 << len)) fail("bad Huffman table");
        code <<= 1;
    }
    h.maxcode[17] = 0x7fffffff;
    for (int i = 0; i < 512; i++) {  // stb_image-style fast AC entries (values fit int8 here)
        h.fast_ac[i] = 0;
        const uint16_t e = h.look[i];
        if (!e) continue;
        const int len = e >> 8, rs = e & 0xFF, run = rs >> 4, size = rs & 15;
        if (size == 0 || len + size > 9 || size > 7) continue;
        const int bits = (i >> (9 - len - size)) & ((1 << size) - 1);
        const int v = bits < (1 << (size - 1)) ? bits - (1 << size) + 1 : bits;
        h.fast_ac[i] = (int16_t)((v * 256) | (run << 4) | (len + size));
    }
}

void parse(const uint8_t *d, size_t n, Header &hd) {
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) fail("missing SOI");
    size_t p = 2;
    bool sof = false;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) fail("marker expected");
        const uint8_t m = d[p + 1];
        if (m == 0xFF) {
            p++;
            continue;
        }
        p += 2;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) fail("no scan");
        const size_t len = ((size_t)d[p] << 8) | d[p + 1];
        if (len < 2 || p + len > n) fail("truncated segment");
        const uint8_t *s = d + p + 2;
        const size_t sl = len - 2;
        if (m == 0xDB) {  // DQT
            size_t i = 0;
            while (i < sl) {
                const int pq = s[i] >> 4, tq = s[i] & 15;
                if (tq > 3 || pq > 1 || i + 1 + 64 * (pq + 1) > sl) fail("bad DQT");
                for (int k = 0; k < 64; k++)
                    hd.q[tq][ZIGZAG[k]] = pq ? (uint16_t)((s[i + 1 + 2 * k] << 8) | s[i + 2 + 2 * k]) : s[i + 1 + k];
                hd.qpresent[tq] = true;
                i += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xC4) {  // DHT
            size_t i = 0;
            while (i < sl) {
                if (i + 17 > sl) fail("bad DHT");
                const int tc = s[i] >> 4, th = s[i] & 15;
                int tot = 0;
                for (int k = 0; k < 16; k++) tot += s[i + 1 + k];
                if (tc > 1 || th > 3 || tot > 256 || i + 17 + tot > sl) fail("bad DHT");
                build_huff(tc ? hd.ac[th] : hd.dc[th], s + i + 1, s + i + 17, tot);
                i += 17 + tot;
            }
        } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1 (baseline / extended Huffman)
            if (sl < 6 || s[0] != 8) fail("only 8-bit baseline frames are supported");
            hd.H = (s[1] << 8) | s[2];
            hd.W = (s[3] << 8) | s[4];
            hd.ncomp = s[5];
            if (hd.W <= 0 || hd.H <= 0 || hd.W > 16384 || hd.H > 16384) fail("bad frame size");
            if ((hd.ncomp != 1 && hd.ncomp != 3) || sl < 6 + 3 * (size_t)hd.ncomp) fail("1 or 3 components only");
            for (int c = 0; c < hd.ncomp; c++) {
                hd.comp[c].id = s[6 + 3 * c];
                hd.comp[c].h = s[7 + 3 * c] >> 4;
                hd.comp[c].v = s[7 + 3 * c] & 15;
                hd.comp[c].tq = s[8 + 3 * c];
                if (hd.comp[c].tq > 3) fail("bad quant table selector");
            }
            if (hd.ncomp == 1) hd.comp[0].h = hd.comp[0].v = 1;
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            fail("progressive / lossless / arithmetic JPEG is not supported");
        } else if (m == 0xDD) {  // DRI
            if (sl < 2) fail("bad DRI");
            hd.restart = (s[0] << 8) | s[1];
        } else if (m == 0xDA) {  // SOS
            if (!sof) fail("SOS before SOF");
            const int ns = s[0];
            if (ns != hd.ncomp || sl < 1 + 2 * (size_t)ns + 3) fail("only one interleaved scan of all components");
            for (int k = 0; k < ns; k++) {
                const int id = s[1 + 2 * k], t = s[2 + 2 * k];
                int c = -1;
                for (int j = 0; j < hd.ncomp; j++)
                    if (hd.comp[j].id == id) c = j;
                if (c != k) fail("scan component order");
                hd.comp[c].td = t >> 4;
                hd.comp[c].ta = t & 15;
                if (hd.comp[c].td > 3 || hd.comp[c].ta > 3 || !hd.dc[hd.comp[c].td].present ||
                    !hd.ac[hd.comp[c].ta].present || !hd.qpresent[hd.comp[c].tq])
                    fail("missing tables");
            }
            hd.scan_begin = p + len;
            return;
        }
        p += len;
    }
    fail("truncated stream");
}

struct Bits {
    const uint8_t *d;
    size_t n, p;
    uint64_t acc = 0;
    int cnt = 0;
    bool marker = false;  // a marker was reached: feed zeros (T.81 F.2.2.5 leaves this to us)
    void fill() {
        // bulk path: 4 bytes at once while none of them is 0xFF (no stuffing, no marker)
        while (cnt <= 32 && !marker && p + 4 <= n) {
            const uint32_t x = ((uint32_t)d[p] << 24) | ((uint32_t)d[p + 1] << 16) | ((uint32_t)d[p + 2] << 8) | d[p + 3];
            const uint32_t t = ~x;
            if ((t - 0x01010101u) & ~t & 0x80808080u) break;  // some byte is 0xFF
            acc |= (uint64_t)x << (32 - cnt);
            cnt += 32;
            p += 4;
        }
        while (cnt <= 56) {
            uint32_t b = 0;
            if (!marker && p < n) {
                b = d[p];
                if (b == 0xFF) {
                    const uint8_t nx = p + 1 < n ? d[p + 1] : 0xD9;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        marker = true;
                        b = 0;
                    }
                } else {
                    p++;
                }
            }
            acc |= (uint64_t)b << (56 - cnt);
            cnt += 8;
        }
    }
    uint32_t peek(int k) {
        if (cnt < k) fill();
        return (uint32_t)(acc >> (64 - k));
    }
    void skip(int k) {
        acc <<= k;
        cnt -= k;
    }
    int get(int k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return (int)v;
    }
    void restart() {  // drop the padding bits, consume the RSTn marker (T.81 F.2.2.5)
        acc = 0;
        cnt = 0;
        marker = false;
        while (p + 1 < n && !(d[p] == 0xFF && d[p + 1] >= 0xD0 && d[p + 1] <= 0xD7)) p++;
        if (p + 1 < n) p += 2;
    }
};

inline int decode(Bits &b, const Huff &h) {
    const uint32_t l = b.peek(9);
    const uint16_t e = h.look[l];
    if (e) {
        b.skip(e >> 8);
        return e & 0xFF;
    }
    uint32_t code = b.peek(16);
    for (int len = 10; len <= 16; len++) {
        const int32_t c = (int32_t)(code >> (16 - len));
        if (c <= h.maxcode[len]) {
            b.skip(len);
            return h.vals[c + h.valoff[len]];
        }
    }
    fail("bad Huffman code");
}

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

}  // namespace

struct zr_jpeg_decoder {
    int device = 0;
    std::mutex mu;
    int16_t *h_coef = nullptr, *d_coef = nullptr;
    size_t coef_cap = 0;  // blocks
    uint8_t *d_planes = nullptr;
    size_t planes_cap = 0;
    // device entropy decoding (streams with restart intervals): tables + interval offsets + scan
    // bytes staged in pinned memory and copied once per frame
    uint8_t *h_stage = nullptr, *d_stage = nullptr;
    size_t stage_cap = 0;
    // self-synchronising device decoding (streams without restart intervals): per-segment states
    uint8_t *d_sync = nullptr;
    size_t sync_cap = 0;
    uint8_t *d_hwords = nullptr;  // restart-interval frames' scans as big-endian dwords
    size_t hwords_cap = 0;
    int *d_err = nullptr;         // [4096] per frame of the last call: set by jpeg_huff_kernel on a corrupt interval
    size_t n_last = 0;            // frames of the last call
    uint64_t n_gpu = 0, n_host = 0;
    hipEvent_t staged = nullptr;  // the last H2D copy out of h_coef / h_stage has completed
    hipEvent_t done = nullptr;    // the last decode's kernels (readers of d_coef / d_planes) completed
};

namespace {
// every ZR_ERR_DEVICE here is a failed HIP call: its last-error slot is consumed with the
// return, so the failure is reported once (session.cpp's HIP_TRY does the same)
int err(int code, const std::string &m) {
    if (code == ZR_ERR_DEVICE) (void)hipGetLastError();
    return zr_internal::set_error(code, m);
}


// Frame layout + entropy decoding shared by the device decode and the host coefficient dump.
void layout_of(const Header &hd, zr::JpegParams &P) {
    int hmax = 1, vmax = 1;
    for (int c = 0; c < hd.ncomp; c++) {
        hmax = std::max(hmax, hd.comp[c].h);
        vmax = std::max(vmax, hd.comp[c].v);
    }
    if (hd.ncomp == 3) {
        const bool luma_ok = (hd.comp[0].h == 1 && hd.comp[0].v == 1) || (hd.comp[0].h == 2 && hd.comp[0].v == 1) ||
                             (hd.comp[0].h == 2 && hd.comp[0].v == 2);
        if (!luma_ok || hd.comp[1].h != 1 || hd.comp[1].v != 1 || hd.comp[2].h != 1 || hd.comp[2].v != 1)
            fail("sampling must be 4:4:4, 4:2:2 or 4:2:0");
    }
    const int mcux = (hd.W + 8 * hmax - 1) / (8 * hmax), mcuy = (hd.H + 8 * vmax - 1) / (8 * vmax);
    P = zr::JpegParams{};
    P.ncomp = hd.ncomp;
    int64_t blocks = 0, pbytes = 0;
    for (int c = 0; c < hd.ncomp; c++) {
        P.bw[c] = mcux * hd.comp[c].h;
        P.bh[c] = mcuy * hd.comp[c].v;
        P.coef_off[c] = blocks;
        P.plane_off[c] = pbytes;
        P.qsel[c] = hd.comp[c].tq;
        blocks += (int64_t)P.bw[c] * P.bh[c];
        pbytes += (int64_t)P.bw[c] * P.bh[c] * 64;
    }
    std::memcpy(P.q, hd.q, sizeof P.q);
    P.total_blocks = (int)blocks;
    P.W = hd.W;
    P.H = hd.H;
    P.hs = hd.ncomp == 3 ? hd.comp[0].h : 1;
    P.vs = hd.ncomp == 3 ? hd.comp[0].v : 1;
    P.cw = hd.ncomp == 3 ? (hd.W + P.hs - 1) / P.hs : 0;  // downsampled_width (jdinput.c)
    P.ch = hd.ncomp == 3 ? (hd.H + P.vs - 1) / P.vs : 0;
}

// T.81 F.2.2: MCU by MCU, components in scan order, h x v blocks each; every block written
// whole (zeroed, then its nonzero coefficients), so `coef` needs no clearing beforehand.
void entropy_decode(const Header &hd, const zr::JpegParams &P, const uint8_t *jpeg, size_t len, int16_t *coef) {
    Bits bits{jpeg, len, hd.scan_begin};
    int pred[3] = {0, 0, 0};
    const int mcux = P.bw[0] / hd.comp[0].h, mcuy = P.bh[0] / hd.comp[0].v;
    const int nmcu = mcux * mcuy;
    for (int m = 0; m < nmcu; m++) {
        if (hd.restart && m > 0 && m % hd.restart == 0) {
            bits.restart();
            pred[0] = pred[1] = pred[2] = 0;
        }
        const int my = m / mcux, mx = m - my * mcux;
        for (int c = 0; c < hd.ncomp; c++) {
            const Comp &cp = hd.comp[c];
            const Huff &dc = hd.dc[cp.td], &ac = hd.ac[cp.ta];
            for (int v = 0; v < cp.v; v++)
                for (int h = 0; h < cp.h; h++) {
                    const int by = my * cp.v + v, bx = mx * cp.h + h;
                    int16_t *blk = coef + (P.coef_off[c] + (int64_t)by * P.bw[c] + bx) * 64;
                    std::memset(blk, 0, 128);
                    const int s = decode(bits, dc);
                    if (s > 11) fail("bad DC category");
                    pred[c] += s ? extend(bits.get(s), s) : 0;
                    blk[0] = (int16_t)pred[c];
                    for (int k = 1; k < 64;) {
                        const int fa = ac.fast_ac[bits.peek(9)];
                        if (fa) {  // run, size and magnitude in one lookup
                            k += (fa >> 4) & 15;
                            bits.skip(fa & 15);
                            if (k > 63) fail("AC index out of range");
                            blk[ZIGZAG[k]] = (int16_t)(fa >> 8);
                            k++;
                            continue;
                        }
                        const int rs = decode(bits, ac);
                        const int r = rs >> 4, sz = rs & 15;
                        if (sz) {
                            k += r;
                            if (k > 63) fail("AC index out of range");
                            blk[ZIGZAG[k]] = (int16_t)extend(bits.get(sz), sz);
                            k++;
                        } else {
                            if (r != 15) break;
                            k += 16;
                        }
                    }
                }
        }
    }
}

void dev_table(const Huff &h, zr::JpegHuffTable &t) {
    std::memset(&t, 0, sizeof t);
    if (!h.present) return;
    for (int i = 0; i < 512; i++) t.lk[i] = ((uint32_t)(uint16_t)h.fast_ac[i] << 16) | h.look[i];
    // code >> (16 - l) <= maxcode[l]  <=>  code < (maxcode[l] + 1) << (16 - l): decode()'s test
    for (int l = 10; l <= 16; l++) {
        t.lim[l - 10] = (uint32_t)(h.maxcode[l] + 1) << (16 - l);
        t.off[l - 10] = h.valoff[l];
    }
    std::memcpy(t.vals, h.vals, sizeof t.vals);
}

// The scan's restart intervals, unstuffed and back to back in `out` (which has room for the scan):
// interval i is out[off[i], off[i+1]).  Each interval is cut at its first marker -- a 0xFF not
// followed by 0x00, so a fill byte or the RSTn itself -- since the host reader (Bits) feeds zeros
// from there; its next interval starts after the next RSTn, where Bits::restart() resumes.  False
// when the stream does not have exactly one interval per `restart` MCUs (the caller then decodes
// on the host, which reports the errors).
bool unstuff_intervals(const uint8_t *d, size_t n, size_t begin, int n_iv, uint8_t *out, std::vector<int32_t> &off) {
    off.clear();
    off.push_back(0);
    size_t p = begin, o = 0;
    bool open = true;  // the current interval still takes bytes
    while (p < n) {
        const uint8_t *f = static_cast<const uint8_t *>(std::memchr(d + p, 0xFF, n - p));
        const size_t q = f ? (size_t)(f - d) : n;
        if (open) {
            std::memcpy(out + o, d + p, q - p);
            o += q - p;
        }
        if (q + 1 >= n) {  // no marker left (a trailing 0xFF reads as one: Bits' 0xD9 rule)
            p = n;
            break;
        }
        const uint8_t nx = d[q + 1];
        if (nx == 0x00) {  // stuffed 0xFF
            if (open) out[o++] = 0xFF;
            p = q + 2;
        } else if (nx == 0xFF) {  // fill byte: Bits stops here, restart() looks for the RSTn
            open = false;
            p = q + 1;
        } else if (nx >= 0xD0 && nx <= 0xD7) {
            if (o >= ((size_t)1 << 31)) return false;
            off.push_back((int32_t)o);
            open = true;
            p = q + 2;
        } else {
            break;  // EOI or another marker ends the scan
        }
    }
    if (o >= ((size_t)1 << 31)) return false;
    off.push_back((int32_t)o);
    return (int)off.size() == n_iv + 1;
}

bool sync_entropy_enabled() {  // ZARU_JPEG_SYNC=0: streams without DRI decode on the host (A/B)
    static const bool on = [] {
        const char *e = std::getenv("ZARU_JPEG_SYNC");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool gpu_entropy_enabled() {  // ZARU_JPEG_HOST_ENTROPY=1 keeps every decode on the host (A/B)
    static const bool on = [] {
        const char *e = std::getenv("ZARU_JPEG_HOST_ENTROPY");
        return !(e && e[0] == '1');
    }();
    return on;
}

}  // namespace

extern "C" {

int zr_jpeg_decoder_create(int device, zr_jpeg_decoder **out) {
    try {
        if (!out) return err(ZR_ERR_INVALID_ARGUMENT, "null out");
        *out = nullptr;
        if (hipSetDevice(device) != hipSuccess) return err(ZR_ERR_DEVICE, "hipSetDevice failed");
        auto *d = new zr_jpeg_decoder();
        d->device = device;
        if (hipEventCreateWithFlags(&d->staged, hipEventDisableTiming) != hipSuccess) {
            delete d;
            return err(ZR_ERR_DEVICE, "hipEventCreate failed");
        }
        if (hipEventCreateWithFlags(&d->done, hipEventDisableTiming) != hipSuccess) {
            (void)hipEventDestroy(d->staged);
            delete d;
            return err(ZR_ERR_DEVICE, "hipEventCreate failed");
        }
        if (hipMalloc((void **)&d->d_err, 4096 * sizeof(int)) != hipSuccess ||
            hipMemset(d->d_err, 0, 4096 * sizeof(int)) != hipSuccess) {
            (void)hipEventDestroy(d->staged);
            (void)hipEventDestroy(d->done);
            delete d;
            return err(ZR_ERR_DEVICE, "hipMalloc failed");
        }
        *out = d;
        return ZR_OK;
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg decoder creation failed");
    }
}

void zr_jpeg_decoder_destroy(zr_jpeg_decoder *d) {
    if (!d) return;
    (void)hipEventSynchronize(d->staged);
    (void)hipEventSynchronize(d->done);
    (void)hipEventDestroy(d->staged);
    (void)hipEventDestroy(d->done);
    (void)hipHostFree(d->h_coef);
    (void)hipFree(d->d_coef);
    (void)hipFree(d->d_planes);
    (void)hipHostFree(d->h_stage);
    (void)hipFree(d->d_stage);
    (void)hipFree(d->d_sync);
    (void)hipFree(d->d_hwords);
    (void)hipFree(d->d_err);
    delete d;
}

int zr_jpeg_decoder_status(zr_jpeg_decoder *d, uint64_t *gpu_entropy, uint64_t *host_entropy, int *corrupt) {
    try {
        if (!d) return err(ZR_ERR_INVALID_ARGUMENT, "null decoder");
        std::lock_guard<std::mutex> g(d->mu);
        if (gpu_entropy) *gpu_entropy = d->n_gpu;
        if (host_entropy) *host_entropy = d->n_host;
        if (corrupt) {
            int e[4096];
            const size_t n = d->n_last;
            if (hipSetDevice(d->device) != hipSuccess || hipEventSynchronize(d->done) != hipSuccess ||
                (n && hipMemcpy(e, d->d_err, n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess))
                return err(ZR_ERR_DEVICE, "jpeg: status read failed");
            *corrupt = 0;
            for (size_t f = 0; f < n; f++) *corrupt |= e[f] ? 1 : 0;
        }
        return ZR_OK;
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg: internal error");
    }
}

int zr_jpeg_frame_errors(zr_jpeg_decoder *d, int32_t *flags, size_t cap, size_t *n) {
    try {
        if (!d || !n) return err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        std::lock_guard<std::mutex> g(d->mu);
        *n = d->n_last;
        if (!flags) return ZR_OK;
        if (cap < d->n_last) return err(ZR_ERR_INVALID_ARGUMENT, "jpeg: flag buffer smaller than the last call");
        if (hipSetDevice(d->device) != hipSuccess || hipEventSynchronize(d->done) != hipSuccess ||
            (d->n_last && hipMemcpy(flags, d->d_err, d->n_last * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess))
            return err(ZR_ERR_DEVICE, "jpeg: status read failed");
        return ZR_OK;
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg: internal error");
    }
}

int zr_jpeg_info(const uint8_t *jpeg, size_t len, uint32_t *width, uint32_t *height) {
    try {
        if (!jpeg || !width || !height) return err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        Header hd;
        parse(jpeg, len, hd);
        *width = (uint32_t)hd.W;
        *height = (uint32_t)hd.H;
        return ZR_OK;
    } catch (const JpegError &e) {
        return err(e.code, e.msg);
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg: internal error");
    }
}

int zr_jpeg_coefficients(const uint8_t *jpeg, size_t len, int16_t *coef, size_t cap_blocks,
                         zr_jpeg_layout *layout) {
    try {
        if (!jpeg || !layout) return err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        Header hd;
        parse(jpeg, len, hd);
        zr::JpegParams P;
        layout_of(hd, P);
        std::memset(layout, 0, sizeof *layout);
        layout->width = (uint32_t)hd.W;
        layout->height = (uint32_t)hd.H;
        layout->ncomp = (uint32_t)hd.ncomp;
        layout->h_samp = (uint32_t)P.hs;
        layout->v_samp = (uint32_t)P.vs;
        layout->total_blocks = (uint32_t)P.total_blocks;
        for (int c = 0; c < hd.ncomp; c++) {
            layout->bw[c] = (uint32_t)P.bw[c];
            layout->bh[c] = (uint32_t)P.bh[c];
            layout->qsel[c] = (uint32_t)P.qsel[c];
        }
        std::memcpy(layout->quant, P.q, sizeof layout->quant);
        if (!coef) return ZR_OK;  // layout only
        if (cap_blocks < (size_t)P.total_blocks) return err(ZR_ERR_INVALID_ARGUMENT, "coefficient buffer too small");
        entropy_decode(hd, P, jpeg, len, coef);
        return ZR_OK;
    } catch (const JpegError &e) {
        return err(e.code, e.msg);
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg: internal error");
    }
}

int zr_jpeg_decode_async(zr_jpeg_decoder *dec, const uint8_t *jpeg, size_t len, uint8_t *d_rgba,
                         size_t row_stride, void *hip_stream) {
    return zr_jpeg_decode_batch_async(dec, 1, &jpeg, &len, &d_rgba, &row_stride, hip_stream);
}

int zr_jpeg_decode_batch_async(zr_jpeg_decoder *dec, size_t n, const uint8_t *const *jpegs, const size_t *lens,
                               uint8_t *const *d_rgba, const size_t *row_strides, void *hip_stream) {
    try {
        if (!dec || !jpegs || !lens || !d_rgba || !row_strides) return err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0) return ZR_OK;
        if (n > 4096) return err(ZR_ERR_INVALID_ARGUMENT, "jpeg: batch larger than 4096 frames");
        std::lock_guard<std::mutex> g(dec->mu);
        // every frame parsed and checked before anything is enqueued
        std::vector<Header> hd(n);
        std::vector<zr::JpegParams> P(n);
        std::vector<int64_t> cofs(n);  // block offset of each frame's coefficients in d_coef
        int64_t blocks = 0, pbytes = 0;
        for (size_t f = 0; f < n; f++) {
            if (!jpegs[f] || !d_rgba[f]) return err(ZR_ERR_INVALID_ARGUMENT, "null argument");
            try {
                parse(jpegs[f], lens[f], hd[f]);
                layout_of(hd[f], P[f]);
            } catch (const JpegError &e) {
                return err(e.code, n > 1 ? e.msg + " (frame " + std::to_string(f) + ")" : e.msg);
            }
            if (row_strides[f] < (size_t)hd[f].W * 4) return err(ZR_ERR_INVALID_ARGUMENT, "row_stride < 4*width");
            cofs[f] = blocks;
            blocks += P[f].total_blocks;
            pbytes = std::max(pbytes, (int64_t)P[f].total_blocks * 64);
        }
        // the previous decode's copies out of the staging buffers must be done
        if (hipSetDevice(dec->device) != hipSuccess) return err(ZR_ERR_DEVICE, "hipSetDevice failed");
        if (hipEventSynchronize(dec->staged) != hipSuccess) return err(ZR_ERR_DEVICE, "event sync failed");
        // which frames decode their entropy on the device, and the staging they need at most:
        // [frames][wg list][per frame: 8 tables, interval offsets, unstuffed intervals + look-ahead]
        const size_t tb = 8 * sizeof(zr::JpegHuffTable);
        std::vector<int> n_iv(n, 0), mcux(n, 0), nmcu(n, 0);
        std::vector<size_t> ob(n, 0), fofs(n, 0);
        size_t groups = 0, stage = 0;
        for (size_t f = 0; f < n; f++) {
            mcux[f] = P[f].bw[0] / hd[f].comp[0].h;
            nmcu[f] = mcux[f] * (P[f].bh[0] / hd[f].comp[0].v);
            n_iv[f] = hd[f].restart > 0 ? (nmcu[f] + hd[f].restart - 1) / hd[f].restart : 0;
            if (!gpu_entropy_enabled() || n_iv[f] < 8) n_iv[f] = 0;
            if (!n_iv[f]) continue;
            ob[f] = ((size_t)(n_iv[f] + 1) * 4 + 15) / 16 * 16;
            groups += (size_t)(n_iv[f] + zr::JH_LANES - 1) / zr::JH_LANES;
        }
        // streams without restart intervals: self-synchronising decoding (jpeg_sync.hip), its
        // staged scan padded to whole 64-segment workgroup ranges + the overrun margin
        std::vector<char> sync(n, 0);
        std::vector<size_t> sofs(n, 0), spad(n, 0);
        size_t nsync = 0, sgroups = 0;
        for (size_t f = 0; f < n; f++) {
            if (!gpu_entropy_enabled() || !sync_entropy_enabled() || hd[f].restart != 0) continue;
            const size_t bound = lens[f] - hd[f].scan_begin;
            const size_t nseg = (bound * 8 + zr::JS_SEG - 1) / zr::JS_SEG;
            if (nseg == 0 || bound * 8 >= ((size_t)1 << 30)) continue;
            // scans of > JS_MAX_BITS_PER_BLOCK bits per block on average (near-lossless noise) fall
            // into step too slowly for the sync passes (measured: q100 noise, ~700 bits per block,
            // still had chains after 32 passes): the host decodes them
            int bpm_f = 0;
            for (int c = 0; c < hd[f].ncomp; c++) bpm_f += hd[f].comp[c].h * hd[f].comp[c].v;
            if ((int64_t)bound * 8 > (int64_t)zr::JS_MAX_BITS_PER_BLOCK * nmcu[f] * bpm_f) continue;
            sync[f] = 1;
            nsync++;
            sgroups += (nseg + zr::JS_LANES - 1) / zr::JS_LANES;
            spad[f] = (nseg + zr::JS_LANES - 1) / zr::JS_LANES * zr::JS_LANES * (zr::JS_SEG / 8) + zr::JS_MARGIN +
                      zr::JS_WARM_MAX / 8 + 16;  // (the first workgroup stages its warm-up's worth past the rest)
        }
        const size_t fb = (n * sizeof(zr::JpegHuffFrame) + 15) / 16 * 16, wb = (groups * 8 + 15) / 16 * 16;
        const size_t sfb = (nsync * sizeof(zr::JpegSyncFrame) + 15) / 16 * 16, swb = (sgroups * 8 + 15) / 16 * 16;
        stage = fb + wb + sfb + swb;
        for (size_t f = 0; f < n; f++)
            if (n_iv[f]) {
                fofs[f] = stage;
                stage += tb + ob[f] + ((lens[f] - hd[f].scan_begin) + 48 + 15) / 16 * 16;
            } else if (sync[f]) {
                sofs[f] = stage;
                stage += tb + spad[f];
            }
        // growing frees device buffers: the previous decode's kernels must be done with them
        // the restart-interval frames' big-endian copies (bounded by their scans' sizes)
        size_t hw_bytes = 0;
        for (size_t f = 0; f < n; f++)
            if (n_iv[f]) hw_bytes += ((lens[f] - hd[f].scan_begin) + 48 + 15) / 16 * 16;
        // per-segment device states of the sync frames (ck, exits x2, start, base, pred) + err_block
        size_t sync_bytes = 0;
        for (size_t f = 0; f < n; f++)
            if (sync[f]) {
                const size_t nseg = (spad[f] - zr::JS_MARGIN - zr::JS_WARM_MAX / 8 - 16) / (zr::JS_SEG / 8);
                sync_bytes += nseg * (zr::JS_CK * sizeof(zr::JpegSyncState) + sizeof(zr::JpegSyncState) + 8 + 4 + 12) + 16 +
                              (spad[f] + 15) / 16 * 16;  // (+ the big-endian copy of the scan)
            }
        if (sync_bytes) sync_bytes += 256;  // the per-pass change counters
        const bool grow = (size_t)blocks > dec->coef_cap || (size_t)pbytes > dec->planes_cap ||
                          ((groups || nsync) && stage > dec->stage_cap) || sync_bytes > dec->sync_cap ||
                          hw_bytes > dec->hwords_cap;
        if (grow && hipEventSynchronize(dec->done) != hipSuccess) return err(ZR_ERR_DEVICE, "event sync failed");
        if ((size_t)blocks > dec->coef_cap) {
            (void)hipHostFree(dec->h_coef);
            (void)hipFree(dec->d_coef);
            dec->h_coef = nullptr;
            dec->d_coef = nullptr;
            dec->coef_cap = 0;
            const size_t cap = (size_t)blocks + (size_t)blocks / 4;
            if (hipHostMalloc((void **)&dec->h_coef, cap * 128) != hipSuccess ||
                hipMalloc((void **)&dec->d_coef, cap * 128) != hipSuccess)
                return err(ZR_ERR_DEVICE, "jpeg: out of memory");
            dec->coef_cap = cap;
        }
        if ((size_t)pbytes > dec->planes_cap) {
            (void)hipFree(dec->d_planes);
            dec->d_planes = nullptr;
            dec->planes_cap = 0;
            const size_t cap = (size_t)pbytes + (size_t)pbytes / 4;
            if (hipMalloc((void **)&dec->d_planes, cap) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: out of memory");
            dec->planes_cap = cap;
        }
        if (hw_bytes > dec->hwords_cap) {
            (void)hipFree(dec->d_hwords);
            dec->d_hwords = nullptr;
            dec->hwords_cap = 0;
            const size_t cap = hw_bytes + hw_bytes / 4;
            if (hipMalloc((void **)&dec->d_hwords, cap) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: out of memory");
            dec->hwords_cap = cap;
        }
        if (sync_bytes > dec->sync_cap) {
            (void)hipFree(dec->d_sync);
            dec->d_sync = nullptr;
            dec->sync_cap = 0;
            const size_t cap = sync_bytes + sync_bytes / 4;
            if (hipMalloc((void **)&dec->d_sync, cap) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: out of memory");
            dec->sync_cap = cap;
        }
        if ((groups || nsync) && stage > dec->stage_cap) {
            (void)hipHostFree(dec->h_stage);
            (void)hipFree(dec->d_stage);
            dec->h_stage = nullptr;
            dec->d_stage = nullptr;
            dec->stage_cap = 0;
            const size_t cap = stage + stage / 4;
            if (hipHostMalloc((void **)&dec->h_stage, cap) != hipSuccess ||
                hipMalloc((void **)&dec->d_stage, cap) != hipSuccess)
                return err(ZR_ERR_DEVICE, "jpeg: out of memory");
            dec->stage_cap = cap;
        }
        // unstuff the device frames' scans; a frame whose intervals do not match its DRI, or whose
        // 64-interval ranges exceed a workgroup's LDS, goes to the host path
        std::vector<int32_t> ivo;
        auto *fr = reinterpret_cast<zr::JpegHuffFrame *>(dec->h_stage);
        auto *wg = reinterpret_cast<int32_t *>(dec->h_stage + fb);
        size_t n_wg = 0, used = fb + wb + sfb + swb, hw = 0;
        if (groups)
            for (size_t f = 0; f < n; f++) fr[f] = zr::JpegHuffFrame{};  // (nwords = 0: not a device frame)
        for (size_t f = 0; f < n; f++) {
            if (!n_iv[f]) continue;
            uint8_t *const base = dec->h_stage + fofs[f];
            if (!unstuff_intervals(jpegs[f], lens[f], hd[f].scan_begin, n_iv[f], base + tb + ob[f], ivo)) {
                n_iv[f] = 0;
                continue;
            }
            const size_t db = (size_t)ivo.back();
            auto *tabs = reinterpret_cast<zr::JpegHuffTable *>(base);
            for (int t = 0; t < 4; t++) {
                dev_table(hd[f].dc[t], tabs[t]);
                dev_table(hd[f].ac[t], tabs[4 + t]);
            }
            std::memcpy(base + tb, ivo.data(), (size_t)(n_iv[f] + 1) * 4);
            std::memset(base + tb + ob[f] + db, 0, 48);
            uint8_t *const dbase = dec->d_stage + fofs[f];
            zr::JpegHuffFrame &F = fr[f];
            F = zr::JpegHuffFrame{};
            F.tables = reinterpret_cast<const zr::JpegHuffTable *>(dbase);
            F.iv_off = reinterpret_cast<const int32_t *>(dbase + tb);
            F.data = dbase + tb + ob[f];
            F.words = reinterpret_cast<uint32_t *>(dec->d_hwords + hw);
            F.nwords = (int)((db + 48 + 15) / 16 * 4);
            hw += (size_t)F.nwords * 4;
            F.coef = dec->d_coef + cofs[f] * 64;
            F.n_iv = n_iv[f];
            F.restart = hd[f].restart;
            F.nmcu = nmcu[f];
            F.mcux = mcux[f];
            F.ncomp = hd[f].ncomp;
            for (int c = 0; c < hd[f].ncomp; c++) {
                F.ch[c] = hd[f].comp[c].h;
                F.cv[c] = hd[f].comp[c].v;
                F.td[c] = hd[f].comp[c].td;
                F.ta[c] = hd[f].comp[c].ta;
                F.coef_off[c] = P[f].coef_off[c];
                F.bw[c] = P[f].bw[c];
            }
            for (int g0 = 0; g0 < n_iv[f]; g0 += zr::JH_LANES) {
                wg[2 * n_wg] = (int32_t)f;
                wg[2 * n_wg + 1] = g0;
                n_wg++;
            }
            used = std::max(used, fofs[f] + tb + ob[f] + (db + 48 + 15) / 16 * 16);
        }
        // the sync frames: unstuffed scans, tables, per-segment state arrays, workgroup list
        auto *sfr = reinterpret_cast<zr::JpegSyncFrame *>(dec->h_stage + fb + wb);
        auto *swg = reinterpret_cast<int32_t *>(dec->h_stage + fb + wb + sfb);
        size_t ns = 0, n_swg = 0, sy = 256;  // [0, 256): the change counters
        for (size_t f = 0; f < n; f++) {
            if (!sync[f]) continue;
            uint8_t *const base = dec->h_stage + sofs[f];
            std::vector<int32_t> one;
            if (!unstuff_intervals(jpegs[f], lens[f], hd[f].scan_begin, 1, base + tb, one)) {
                sync[f] = 0;  // markers inside the scan: the host decoder reports what they are
                continue;
            }
            const size_t nbytes = (size_t)one.back();
            const int nseg = std::max(1, (int)((nbytes * 8 + zr::JS_SEG - 1) / zr::JS_SEG));
            std::memset(base + tb + nbytes, 0, spad[f] - nbytes);
            auto *tabs = reinterpret_cast<zr::JpegHuffTable *>(base);
            for (int t = 0; t < 4; t++) {
                dev_table(hd[f].dc[t], tabs[t]);
                dev_table(hd[f].ac[t], tabs[4 + t]);
            }
            uint8_t *const dbase = dec->d_stage + sofs[f];
            zr::JpegSyncFrame &F = sfr[ns];
            F = zr::JpegSyncFrame{};
            F.tables = reinterpret_cast<const zr::JpegHuffTable *>(dbase);
            F.data = dbase + tb;
            F.nbytes = (int)nbytes;
            F.nbits = (int)nbytes * 8;
            F.nseg = nseg;
            F.mcux = mcux[f];
            F.ncomp = hd[f].ncomp;
            int u = 0;
            for (int c = 0; c < hd[f].ncomp; c++) {
                F.ch[c] = hd[f].comp[c].h;
                F.cv[c] = hd[f].comp[c].v;
                F.td[c] = hd[f].comp[c].td;
                F.ta[c] = hd[f].comp[c].ta;
                F.coef_off[c] = P[f].coef_off[c];
                F.bw[c] = P[f].bw[c];
                for (int v = 0; v < F.cv[c]; v++)
                    for (int h = 0; h < F.ch[c]; h++) {
                        F.ucomp[u] = c;
                        F.uby[u] = v;
                        F.ubx[u] = h;
                        u++;
                    }
            }
            F.bpm = u;
            F.nblocks = nmcu[f] * u;
            // warm-up: ~12 average blocks (high-rate scans fall into step over more bits)
            const int64_t bpb = (int64_t)F.nbits / std::max(1, F.nblocks);
            static const int warm_blocks = [] {  // ZARU_JPEG_SYNC_WARM: warm-up in average blocks (A/B)
                const char *e = std::getenv("ZARU_JPEG_SYNC_WARM");
                const long v = e ? std::strtol(e, nullptr, 10) : 0;
                return v > 0 ? (int)v : 12;
            }();
            F.warm = (int)std::min<int64_t>(zr::JS_WARM_MAX,
                                            std::max<int64_t>(zr::JS_WARM_MIN, (warm_blocks * bpb + 127) / 128 * 128));
            F.coef = dec->d_coef + cofs[f] * 64;
            F.frame = (int)f;
            uint8_t *sp = dec->d_sync + sy;
            F.ck = reinterpret_cast<zr::JpegSyncState *>(sp);
            sp += (size_t)nseg * zr::JS_CK * sizeof(zr::JpegSyncState);
            F.x = reinterpret_cast<zr::JpegSyncState *>(sp);
            sp += (size_t)nseg * sizeof(zr::JpegSyncState);
            F.start = reinterpret_cast<int2 *>(sp);
            sp += (size_t)nseg * 8;
            F.base = reinterpret_cast<int32_t *>(sp);
            sp += (size_t)nseg * 4;
            F.pred = reinterpret_cast<int32_t *>(sp);
            sp += (size_t)nseg * 12;
            F.err_block = reinterpret_cast<int32_t *>(sp);
            sp += 16;
            F.words = reinterpret_cast<uint32_t *>(sp);
            F.nwords = (int)(spad[f] / 16 * 4);
            sp += (spad[f] + 15) / 16 * 16;
            sy = (size_t)(sp - dec->d_sync);
            for (int g0 = 0; g0 < nseg; g0 += zr::JS_LANES) {
                swg[2 * n_swg] = (int32_t)ns;
                swg[2 * n_swg + 1] = g0;
                n_swg++;
            }
            used = std::max(used, sofs[f] + tb + spad[f]);
            ns++;
        }
        // host entropy decoding for the rest, into their slots of the pinned coefficient staging
        for (size_t f = 0; f < n; f++)
            if (!n_iv[f] && !sync[f]) {
                try {
                    entropy_decode(hd[f], P[f], jpegs[f], lens[f], dec->h_coef + cofs[f] * 64);
                } catch (const JpegError &e) {
                    return err(e.code, n > 1 ? e.msg + " (frame " + std::to_string(f) + ")" : e.msg);
                }
            }
        // d_coef / d_planes / d_stage are reused: on another stream the previous decode's kernels
        // may still read them, so this stream waits for them first
        hipStream_t st = (hipStream_t)hip_stream;
        if (hipStreamWaitEvent(st, dec->done, 0) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: stream wait failed");
        for (size_t f = 0; f < n; f++)
            if (!n_iv[f] && !sync[f] && hipMemcpyAsync(dec->d_coef + cofs[f] * 64, dec->h_coef + cofs[f] * 64,
                                           (size_t)P[f].total_blocks * 128, hipMemcpyHostToDevice, st) != hipSuccess)
                return err(ZR_ERR_DEVICE, "jpeg: coefficient upload failed");
        if ((n_wg || ns) && hipMemcpyAsync(dec->d_stage, dec->h_stage, used, hipMemcpyHostToDevice, st) != hipSuccess)
            return err(ZR_ERR_DEVICE, "jpeg: scan upload failed");
        if (hipEventRecord(dec->staged, st) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: event record failed");
        // this call's per-frame error flags (the device decode reports corruption asynchronously)
        if (hipMemsetAsync(dec->d_err, 0, n * sizeof(int), st) != hipSuccess)
            return err(ZR_ERR_DEVICE, "jpeg: flag reset failed");
        dec->n_last = n;
        if (n_wg) {
            zr::JpegHuffParams hp{};
            hp.frames = reinterpret_cast<const zr::JpegHuffFrame *>(dec->d_stage);
            hp.wg = reinterpret_cast<const int32_t *>(dec->d_stage + fb);
            hp.n_wg = (int)n_wg;
            hp.error = dec->d_err;
            hp.nframes = (int)n;
            zr::launch_jpeg_huff(hp, st);
        }
        if (ns) {
            zr::JpegSyncParams sp{};
            sp.frames = reinterpret_cast<const zr::JpegSyncFrame *>(dec->d_stage + fb + wb);
            sp.wg = reinterpret_cast<const int32_t *>(dec->d_stage + fb + wb + sfb);
            sp.n_wg = (int)n_swg;
            sp.nframes = (int)ns;
            sp.error = dec->d_err;
            sp.changed = reinterpret_cast<int *>(dec->d_sync);
            static_assert((zr::JS_PASSES + 1) * sizeof(int) <= 256, "change counters");
            if (hipMemsetAsync(dec->d_sync, 0, 256, st) != hipSuccess) return err(ZR_ERR_DEVICE, "jpeg: counter reset failed");
            // ZARU_JPEG_SYNC_PASSES (0..JS_PASSES, read once per process): fewer sync passes, so
            // the tests can send frames through the serial finish
            static const int passes = [] {
                const char *pe = std::getenv("ZARU_JPEG_SYNC_PASSES");
                return pe ? std::max(0, std::min(zr::JS_PASSES, (int)std::strtol(pe, nullptr, 10))) : zr::JS_PASSES;
            }();
            for (int pass = 0; pass <= passes; pass++) zr::launch_jpeg_sync_scan(sp, pass, st);
            zr::launch_jpeg_sync_finish(sp, st);
            static const char *const dump_path = std::getenv("ZARU_JPEG_SYNC_DUMP");  // read once
            if (const char *dump = dump_path) {  // diagnostics: the first sync frame's states
                const zr::JpegSyncFrame &F0 = sfr[0];
                std::vector<int> cnt(64);
                std::vector<zr::JpegSyncState> xs(F0.nseg);
                std::vector<int2> starts(F0.nseg);
                std::vector<int32_t> bases(F0.nseg);
                int eb = 0;
                (void)hipStreamSynchronize(st);
                (void)hipMemcpy(cnt.data(), dec->d_sync, 256, hipMemcpyDeviceToHost);
                (void)hipMemcpy(xs.data(), F0.x, xs.size() * sizeof(zr::JpegSyncState), hipMemcpyDeviceToHost);
                (void)hipMemcpy(starts.data(), F0.start, starts.size() * 8, hipMemcpyDeviceToHost);
                (void)hipMemcpy(bases.data(), F0.base, bases.size() * 4, hipMemcpyDeviceToHost);
                (void)hipMemcpy(&eb, F0.err_block, 4, hipMemcpyDeviceToHost);
                if (FILE *fp = std::fopen(dump, "w")) {
                    std::fprintf(fp, "nseg %d nblocks %d warm %d err_block %d\nchanged", F0.nseg, F0.nblocks, F0.warm, eb);
                    for (int i = 0; i <= zr::JS_PASSES; i++) std::fprintf(fp, " %d", cnt[i]);
                    std::fprintf(fp, "\n");
                    for (int i = 0; i < F0.nseg; i++)
                        std::fprintf(fp, "%d start %d %d exit %d %d nblk %d err %d base %d\n", i, starts[i].x, starts[i].y,
                                     xs[i].pos, xs[i].u, xs[i].nblk, xs[i].err, bases[i]);
                    std::fclose(fp);
                }
            }
        }
        for (size_t f = 0; f < n; f++) {
            P[f].coef = dec->d_coef + cofs[f] * 64;
            P[f].planes = dec->d_planes;
            P[f].out = d_rgba[f];
            P[f].out_stride = (int64_t)row_strides[f];
            zr::launch_jpeg(P[f], st);
            if (n_iv[f] || sync[f])
                dec->n_gpu++;
            else
                dec->n_host++;
        }
        if (hipGetLastError() != hipSuccess || hipEventRecord(dec->done, st) != hipSuccess)
            return err(ZR_ERR_DEVICE, "jpeg: kernel launch failed");
        return ZR_OK;
    } catch (const JpegError &e) {
        return err(e.code, e.msg);
    } catch (const std::bad_alloc &) {
        return err(ZR_ERR_INTERNAL, "jpeg: out of host memory");
    } catch (...) {
        return err(ZR_ERR_INTERNAL, "jpeg: internal error");
    }
}

}  // extern "C"
