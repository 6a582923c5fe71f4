// jpeg_huff.hip -- baseline JPEG Huffman entropy decoding on the device for
// streams with restart intervals: one lane per interval (T.81 F.2.2.5: every RSTn resets the
// DC predictions and byte-aligns the bit stream, so intervals decode independently -- the
// parallelism the reference's decoders never use, crates/zaru-image/src/jpeg.rs:107-205 and
// TODO.txt:9-12).  The decode is runtime/jpeg.cpp's entropy_decode restated (same tables, same
// lookahead fast paths, same byte stuffing / marker rule), so the coefficients are identical and
// the IDCT / colour stages downstream produce the same bytes as the host path.
#include "../runtime/zr_jpeg.h"
#include "jpeg_bits.h"

namespace zr {
namespace {

using namespace jpegbits;


// Every coefficient goes to the lane's block in LDS (natural order through an LDS zig-zag table)
// and the finished block leaves in eight 16-B stores.  The interval bits are read from global
// memory (the call's big-endian copy; the window's look-ahead load is off the symbol chain): a
// workgroup of 256 lanes then needs 19 KB of tables + 32 KB of blocks in LDS, 3 workgroups per
// CU, where staging each 64-interval range in LDS held the kernel to about one wave per CU.
__global__ __launch_bounds__(JH_LANES) void jpeg_huff_kernel(const JpegHuffParams P) {
    __shared__ JpegHuffTable T[8];
    __shared__ uint8_t zz[64];
    __shared__ int4 sblk[JH_LANES][8];  // one 64-coefficient int16 block per lane
    const JpegHuffFrame &F = P.frames[P.wg[2 * blockIdx.x]];
    const int iv0 = P.wg[2 * blockIdx.x + 1], iv1 = min(iv0 + JH_LANES, F.n_iv);
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(F.tables);
        uint4 *dst = reinterpret_cast<uint4 *>(T);
        constexpr int n16 = (int)(8 * sizeof(JpegHuffTable) / 16);
        for (int i = threadIdx.x; i < n16; i += JH_LANES) dst[i] = src[i];
        if (threadIdx.x < 64) zz[threadIdx.x] = kZigzag[threadIdx.x];
    }
    __syncthreads();
    const int iv = iv0 + threadIdx.x;
    if (iv >= iv1) return;
    int bp = F.iv_off[iv] * 8;
    Window win;
    win.init(F.words, F.nwords - 1, bp, F.iv_off[iv + 1] * 8);
    int4 *const mine = sblk[threadIdx.x];
    int16_t *const co = reinterpret_cast<int16_t *>(mine);
    int pred[3] = {0, 0, 0};
    bool bad = false;
    const int m0 = iv * F.restart, m1 = min(m0 + F.restart, F.nmcu);
    // Every block of the interval is written, also after a corrupt symbol: the block holding the
    // first bad code and the rest of the interval are all-zero blocks (libjpeg's insufficient-data
    // rule: jdhuff.c zeroes the MCU and skips decoding; the sync decoder's rule per frame), so no
    // block keeps a partial decode or a previous frame's coefficients from the reused buffer.  The
    // frame's error flag reports it.
    for (int m = m0; m < m1; m++) {
        const int my = m / F.mcux, mx = m - my * F.mcux;
        for (int c = 0; c < F.ncomp; c++) {
            const JpegHuffTable &dc = T[F.td[c]], &ac = T[4 + F.ta[c]];
            LongCodes dcl, acl;
            dcl.load(dc);
            acl.load(ac);
            for (int v = 0; v < F.cv[c]; v++)
                for (int h = 0; h < F.ch[c]; h++) {
                    const int by = my * F.cv[c] + v, bx = mx * F.ch[c] + h;
                    int4 *const b4 = reinterpret_cast<int4 *>(
                        F.coef + (F.coef_off[c] + (int64_t)by * F.bw[c] + bx) * 64);
#pragma unroll
                    for (int z = 0; z < 8; z++) mine[z] = make_int4(0, 0, 0, 0);
                    const bool was_bad = bad;
                    {  // DC: category, then that many magnitude bits
                        const uint32_t w = win.at(bp);
                        const uint32_t e = dc.lk[w >> 23] & 0xFFFFu;
                        int ll;
                        const int slow = dcl.decode(w, dc, ll);
                        const int len = e ? (int)(e >> 8) : ll;
                        const int sc = e ? (int)(e & 0xFF) : slow;
                        const bool ok = len && sc <= 11;
                        bad |= !ok;
                        pred[c] += ok && sc ? extend(bits_after(w, len, sc), sc) : 0;
                        bp += len + (ok ? sc : 0);
                        co[0] = was_bad ? (int16_t)0 : (int16_t)pred[c];
                    }
                    // AC, branch-free per symbol (lanes decode different data, so every branch
                    // would be taken by some lane): the fast entry and the long-code search are
                    // both evaluated and selected
                    for (int k = bad ? 64 : 1; k < 64;) {
                        const uint32_t w = win.at(bp);
                        const uint32_t e = ac.lk[w >> 23];
                        int ll;
                        const int slow = acl.decode(w, ac, ll);
                        const int fa = (int32_t)e >> 16;
                        const bool f = fa != 0, look = (e & 0xFFFFu) != 0;
                        const int len = look ? (int)((e >> 8) & 0xFF) : ll;
                        const int rs = look ? (int)(e & 0xFF) : slow;
                        const int r = rs >> 4, sz = rs & 15;
                        const bool coef = f || sz;  // writes a coefficient (else EOB / ZRL)
                        const int kn = k + (f ? (fa >> 4) & 15 : r);
                        const bool bad_now = (!f && !len) || (coef && kn > 63);
                        const int val = f ? fa >> 8 : sz ? extend(bits_after(w, len, sz), sz) : 0;
                        if (coef && !bad_now) co[zz[kn & 63]] = (int16_t)val;
                        bp += f ? fa & 15 : len + sz;
                        k = bad_now ? 64 : coef ? kn + 1 : r == 15 ? k + 16 : 64;
                        bad |= bad_now;
                    }
                    const int4 zero4 = make_int4(0, 0, 0, 0);
#pragma unroll
                    for (int z = 0; z < 8; z++) b4[z] = bad ? zero4 : mine[z];  // (the bad block too)
                }
        }
    }
    if (bad) P.error[P.wg[2 * blockIdx.x]] = 1;  // per frame of the call
}

// The call's interval bytes as big-endian dwords (what the bit window reads), per frame.
__global__ __launch_bounds__(256) void jpeg_huff_bswap_kernel(const JpegHuffParams P) {
    const JpegHuffFrame &F = P.frames[blockIdx.y];
    if (F.nwords == 0) return;
    const uint4 *src = reinterpret_cast<const uint4 *>(F.data);
    uint4 *dst = reinterpret_cast<uint4 *>(F.words);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < F.nwords / 4; i += gridDim.x * 256) {
        const uint4 v = src[i];
        dst[i] = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
    }
}

}  // namespace

const char *launch_jpeg_huff(const JpegHuffParams &p, hipStream_t s) {
    hipLaunchKernelGGL(jpeg_huff_bswap_kernel, dim3(64, p.nframes), dim3(256), 0, s, p);
    hipLaunchKernelGGL(jpeg_huff_kernel, dim3(p.n_wg), dim3(JH_LANES), 0, s, p);
    return "jpeg_huff_kernel";
}

}  // namespace zr
