// jpeg_bits.h -- the device Huffman decoder's building blocks, shared by the restart-interval
// kernel (jpeg_huff.hip) and the self-synchronising one (jpeg_sync.hip): the LDS bit window, the
// long-code search and the magnitude helpers, runtime/jpeg.cpp's decode restated.
#pragma once
#include "../runtime/zr_jpeg.h"

namespace zr {
namespace jpegbits {

constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// The host unstuffs the scan while it copies it (0xFF00 -> 0xFF, each interval cut at its first
// marker: runtime/jpeg.cpp unstuff_intervals), so an interval's bits are a plain byte range,
// followed by zeros (the host reader's rule after a marker).  A workgroup (64 intervals, one per
// lane) stages its contiguous range in LDS as big-endian dwords; a lane's 32-bit window at bit
// `bp` is then a funnel shift of two register-cached dwords, and one window covers a whole
// symbol (code <= 16 bits + magnitude <= 15 bits).  No refill loop, no per-byte branches: the earlier
// byte-reader form of this kernel ran ~350 wave instructions per symbol.
struct Window {
    const uint32_t *w;  // the workgroup's staged dwords (big-endian)
    int last;           // last dword index the reader may touch
    int ebp;            // end of the lane's interval (bits)
    int i;              // dword of the current bit position: hi = w[i], lo = w[i + 1], nx = w[i + 2]
    uint32_t hi, lo, nx;
    __device__ __forceinline__ void init(const uint32_t *words, int last_word, int bp, int end) {
        w = words;
        last = last_word;
        ebp = end;
        i = bp >> 5;
        hi = w[min(i, last)];
        lo = w[min(i + 1, last)];
        nx = w[min(i + 2, last)];
    }
    // A symbol consumes at most 31 bits, so the position moves at most one dword per call.  `nx`
    // is reloaded every call (no branch) and first read a call later: the LDS latency is off the
    // per-symbol dependency chain, which is then one table lookup.
    __device__ __forceinline__ uint32_t at(int bp) {
        const bool sh = (bp >> 5) != i;
        hi = sh ? lo : hi;
        lo = sh ? nx : lo;
        i += sh;
        nx = w[min(i + 2, last)];
        const int rem = ebp - bp, s = bp & 31;
        const uint32_t v = s ? __builtin_amdgcn_alignbit(hi, lo, 32 - s) : hi;
        return rem >= 32 ? v : rem <= 0 ? 0u : v & (~0u << (32 - rem));
    }
};

// A table's long-code limits in registers (uniform per block): the 10..16-bit search is seven
// compares, not seven dependent LDS reads as in the host decoder's loop (runtime/jpeg.cpp decode).
struct LongCodes {
    uint32_t lim[7];
    int32_t off[7];
    __device__ __forceinline__ void load(const JpegHuffTable &t) {
#pragma unroll
        for (int j = 0; j < 7; j++) {
            lim[j] = t.lim[j];
            off[j] = t.off[j];
        }
    }
    // symbol of the >= 10-bit code at the top of `win`; len = 0: no such code
    __device__ __forceinline__ int decode(uint32_t win, const JpegHuffTable &t, int &len) const {
        const uint32_t code = win >> 16;
        int l = 0, o = 0;
#pragma unroll
        for (int j = 6; j >= 0; j--)
            if (code < lim[j]) {
                l = j + 10;
                o = off[j];
            }
        len = l;
        return l ? t.vals[((int)(code >> (16 - l)) + o) & 255] : 0;
    }
};

// `s` bits of `win` after the first `len` (s >= 1, len + s <= 32)
__device__ __forceinline__ int bits_after(uint32_t win, int len, int s) { return (int)((win << len) >> (32 - s)); }

__device__ __forceinline__ int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

}  // namespace jpegbits
}  // namespace zr
