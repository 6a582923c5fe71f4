// zr_jpeg.h -- the device half of the JPEG frame source: dequantisation +
// inverse DCT per 8x8 block, then upsampling + YCbCr -> RGBA per output pixel, restating the
// reference's libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:164-182: turbojpeg 0.5.3 /
// turbojpeg-sys 0.2.3, default flags: accurate integer IDCT "islow", fancy upsampling).  The
// entropy decoding (inherently sequential) runs on the host in runtime/jpeg.cpp.
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

}  // namespace zr
