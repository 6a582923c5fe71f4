// zr_jpeg.h -- the device half of the JPEG frame source: dequantisation +
// inverse DCT per 8x8 block, then upsampling + YCbCr -> RGBA per output pixel, restating the
// reference's libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:164-182: turbojpeg 0.5.3 /
// turbojpeg-sys 0.2.3, default flags: accurate integer IDCT "islow", fancy upsampling).  The
// entropy decoding runs on the device for streams with restart intervals (one lane per
// interval, jpeg_huff.hip) and on the host otherwise (runtime/jpeg.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zr {

struct JpegParams {
    const int16_t *coef;   // per component: [bh][bw][64] quantised coefficients, natural order
    uint8_t *planes;       // per component: [bh*8][bw*8] samples
    int ncomp;
    int64_t coef_off[3];   // block offsets (in blocks) of each component
    int64_t plane_off[3];  // byte offsets of each component plane
    int bw[3], bh[3];      // block grid of each component
    int qsel[3];           // quantisation table of each component
    uint16_t q[4][64];     // natural order
    int total_blocks;
    // colour stage
    int W, H;              // image size
    int hs, vs;            // luma sampling factors relative to chroma (1 or 2)
    int cw, ch;            // chroma downsampled width / height (ceil(W*hc/hmax) ...)
    uint8_t *out;          // RGBA8
    int64_t out_stride;    // bytes per row
};

const char *launch_jpeg(const JpegParams &p, hipStream_t s);

// Baseline Huffman entropy decoding on the device (jpeg_huff.hip) for streams with restart
// intervals (DRI): the intervals decode independently (T.81 F.2.2: the DC predictions reset and
// the bit stream is byte-aligned at every RSTn), so one thread decodes one interval.  Tables in
// the host decoder's form (runtime/jpeg.cpp Huff), copied with the scan data.
struct JpegHuffTable {
    uint32_t lk[512];  // 9-bit lookahead: (fast_ac << 16) | look -- look = (length << 8) | symbol,
                       // 0 = longer code; fast_ac = (value << 8) | (run << 4) | total bits, 0 = none
    uint32_t lim[8];   // codes of 10..16 bits: [l - 10] = (maxcode[l] + 1) << (16 - l), 0 = none
    int32_t off[8];    // [l - 10] = valoff[l]
    uint8_t vals[256];
};
static_assert(sizeof(JpegHuffTable) % 16 == 0, "JpegHuffTable is copied as 16-byte slots");

struct JpegHuffFrame {
    const JpegHuffTable *tables;  // [8]: DC 0..3, AC 0..3
    const int32_t *iv_off;        // [n_iv + 1] byte offsets of the intervals in `data` (+ end)
    const uint8_t *data;          // the intervals' unstuffed bytes, back to back (16-B aligned)
    uint32_t *words;              // the same as big-endian dwords (jpeg_huff_bswap_kernel; 0: not a device frame)
    int nwords;                   // a multiple of 4, with >= 32 B of zero slack past the data
    int16_t *coef;                // as JpegParams::coef
    int64_t coef_off[3];
    int n_iv, restart, nmcu, mcux, ncomp;
    int ch[3], cv[3], td[3], ta[3];
    int bw[3];
};

// One launch decodes a batch of frames: workgroup w takes frame wg[2w]'s JH_LANES intervals from
// wg[2w + 1] on.
constexpr int JH_LANES = 256;
struct JpegHuffParams {
    const JpegHuffFrame *frames;
    const int32_t *wg;            // [n_wg][2]
    int n_wg;
    int *error;                   // [frame of the call] set to 1 on a corrupt interval (bad code / AC index)
    int nframes;                  // frames[] entries (the call's frames; nwords = 0: not on this path)
};
const char *launch_jpeg_huff(const JpegHuffParams &p, hipStream_t s);

// Self-synchronising entropy decoding (jpeg_sync.hip) for streams without restart intervals:
// the unstuffed scan is cut into JS_SEG-bit segments, one lane each.  A lane first decodes its
// segment from a guessed state (its first bit, first block of an MCU); Huffman decoders that
// start out of step fall into step with the true one within a few symbols, so the exit state a
// lane reaches (the first block boundary past its segment) is, almost always, the true state of
// the next lane's start.  Sync passes re-decode each lane from its predecessor's exit until the
// lane meets a checkpoint of its earlier decode (same bit, same block of the MCU: the same state,
// so the rest is unchanged); then a scan over the lanes gives each one its first block index and
// DC predictors, and a final pass writes the coefficients.
constexpr int JS_SEG = 4096;  // bits per segment (a multiple of 128)
constexpr int JS_CK = 8;      // checkpoints per segment: the first block boundary at or past each
                              // JS_SEG / JS_CK-bit mark; the last one is the lane's exit
constexpr int JS_LANES = 256;  // segments per workgroup (a lane each)
constexpr int JS_MARGIN = 4096;  // bytes staged past a workgroup's last segment (blocks that run over)
// bits a lane's guessed decode runs before its segment, to fall into step (per frame: about a
// dozen blocks' worth of the frame's average, a multiple of 128)
constexpr int JS_WARM_MIN = 2048, JS_WARM_MAX = 32768;
struct JpegSyncState {
    int32_t pos, u, nblk;       // bit, block of the MCU, blocks since the lane's start
    int32_t err;                // first block since the start with a bad code / AC index, + 1 (0: none)
    int32_t dc[3], pad;         // DC differences since the lane's start, per component
};
struct JpegSyncFrame {
    const JpegHuffTable *tables;  // [8]
    const uint8_t *data;          // the scan, unstuffed (16-B aligned, zero slack past the end)
    uint32_t *words;              // the same as big-endian dwords (jpeg_sync_bswap_kernel)
    int nwords;                   // dwords of `data` incl. the slack (a multiple of 4)
    int nbytes, nbits, nseg, nblocks, bpm, mcux, ncomp, warm;
    int ucomp[10], uby[10], ubx[10];  // block u of an MCU: component, block row / column offset
    int td[3], ta[3], ch[3], cv[3], bw[3];
    int16_t *coef;
    int64_t coef_off[3];
    JpegSyncState *ck;            // [nseg][JS_CK]
    JpegSyncState *x;             // [nseg] exit states
    int2 *start;                  // [nseg] the (pos, u) the lane's checkpoints were decoded from
    int32_t *base;                // [nseg] first block index (-1: nothing to write)
    int32_t *pred;                // [nseg][3] DC predictors at the lane's start
    int32_t *err_block;           // [4]: [0] blocks from here on are zero (nblocks: none);
                                  // [1] first lane out of step after the sync passes (-1: none),
                                  // [2] its first block: the serial kernel decodes from there
    int frame;                    // index into the call's error flags
};
struct JpegSyncParams {
    const JpegSyncFrame *frames;
    const int32_t *wg;            // [n_wg][2]: frame, first segment
    int n_wg, nframes;
    int *error;                   // [frame of the call]
    int *changed;                 // [JS_PASSES + 1] exits changed per pass (zeroed per call)
};
constexpr int JS_PASSES = 32;     // sync passes launched per call at most (each returns at once
                                  // once a pass changed nothing)
constexpr int JS_MAX_BITS_PER_BLOCK = 600;  // denser scans decode on the host
// pass 0: the guessed decode, 1..passes (<= JS_PASSES): sync passes; then prefix, write, the serial
// decode of a frame whose sync passes ran out, and the zero fill
const char *launch_jpeg_sync_scan(const JpegSyncParams &p, int pass, hipStream_t s);
const char *launch_jpeg_sync_finish(const JpegSyncParams &p, hipStream_t s);

}  // namespace zr
