// jpeg_sync.hip -- baseline JPEG Huffman decoding on the device for streams WITHOUT restart
// intervals (the reference decodes them serially on the CPU,
// crates/zaru-image/src/jpeg.rs:107-205).  Self-synchronising decoding (zr_jpeg.h): a lane per
// JS_SEG-bit segment of the unstuffed scan, a guessed start, sync passes until every lane's start
// is its predecessor's exit, a prefix over the lanes (first block index, DC predictors), and a
// write pass.  The per-block decode is jpeg_huff.hip's (runtime/jpeg.cpp entropy_decode
// restated: same tables, fast paths and end-of-data rule), so a synchronised frame's
// coefficients are the host decoder's, and the IDCT / colour stages make the same bytes.
#include "../runtime/zr_jpeg.h"
#include "jpeg_bits.h"

namespace zr {
namespace {

using namespace jpegbits;

constexpr int JS_CKB = JS_SEG / JS_CK;  // bits between checkpoint marks

// One block at bit `bp`: the DC difference, the AC coefficients
// into `co` (natural order, WRITE only), false on a bad code / AC index (T.81 F.2.2: the block is
// not decoded further).
template <bool WRITE>
__device__ __forceinline__ bool decode_block(Window &win, int &bp, const JpegHuffTable &dc, const JpegHuffTable &ac,
                                             const LongCodes &dcl, const LongCodes &acl, int &diff, int16_t *co,
                                             const uint8_t *zz) {
    {
        const uint32_t w = win.at(bp);
        const uint32_t e = dc.lk[w >> 23] & 0xFFFFu;
        int ll;
        const int slow = dcl.decode(w, dc, ll);
        const int len = e ? (int)(e >> 8) : ll;
        const int sc = e ? (int)(e & 0xFF) : slow;
        if (!len || sc > 11) return false;
        diff = sc ? extend(bits_after(w, len, sc), sc) : 0;
        bp += len + sc;
    }
    for (int k = 1; k < 64;) {
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
        if ((!f && !len) || (coef && kn > 63)) return false;
        if (WRITE && coef) co[zz[kn]] = (int16_t)(f ? fa >> 8 : extend(bits_after(w, len, sz), sz));
        bp += f ? fa & 15 : len + sz;
        k = coef ? kn + 1 : r == 15 ? k + 16 : 64;
    }
    return true;
}

// a lane's new exit; a changed one keeps the sync passes going
__device__ __forceinline__ void publish(const JpegSyncParams &P, int pass, JpegSyncState *x, const JpegSyncState &e) {
    const JpegSyncState o = *x;
    if (pass == 0 || o.pos != e.pos || o.u != e.u || o.nblk != e.nblk || o.err != e.err || o.dc[0] != e.dc[0] ||
        o.dc[1] != e.dc[1] || o.dc[2] != e.dc[2]) {
        *x = e;
        if (pass > 0) atomicAdd(&P.changed[pass], 1);
    }
}

// The frame's 8 tables into the workgroup's LDS.  The scan itself is read from global memory
// (L1 / L2; a lane's window loads the dword two ahead of its position, so the load is off the
// symbol chain): staging a workgroup's bit range in LDS held the kernel to one 64-lane workgroup
// (< 1 wave per SIMD) per 56 KB, and these lanes are latency-bound -- occupancy is what pays.
__device__ __forceinline__ void stage_tables(const JpegSyncFrame &F, JpegHuffTable *T) {
    const uint4 *src = reinterpret_cast<const uint4 *>(F.tables);
    uint4 *dst = reinterpret_cast<uint4 *>(T);
    constexpr int n16 = (int)(8 * sizeof(JpegHuffTable) / 16);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
}

// The unstuffed scan as big-endian dwords (what the bit window reads), per frame.
__global__ __launch_bounds__(256) void jpeg_sync_bswap_kernel(const JpegSyncParams P) {
    const JpegSyncFrame &F = P.frames[blockIdx.y];
    const uint4 *src = reinterpret_cast<const uint4 *>(F.data);
    uint4 *dst = reinterpret_cast<uint4 *>(F.words);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < F.nwords / 4; i += gridDim.x * 256) {
        const uint4 v = src[i];
        dst[i] = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
    }
}

// Pass 0 decodes every lane from its guess and records its checkpoints and exit; pass p >= 1
// re-decodes the lanes whose predecessor's exit differs from the start they were decoded from,
// until they meet one of their checkpoints (same bit, same block of the MCU).  The exits live in
// one array that a pass reads and writes at once: a lane that sees its predecessor's new exit
// (or a half-written one) only gets ahead (or is redone next pass); a pass runs only while the
// previous one changed an exit, and the prefix pass checks every start against its predecessor's
// final exit.
__global__ __launch_bounds__(256) void jpeg_sync_scan_kernel(const JpegSyncParams P, int pass) {
    __shared__ JpegHuffTable T[8];
    if (pass > 0 && __atomic_load_n(&P.changed[pass - 1], __ATOMIC_RELAXED) == 0) return;  // converged
    if (pass == 0 && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&P.changed[0], 1);
    const JpegSyncFrame &F = P.frames[P.wg[2 * blockIdx.x]];
    const int s0 = P.wg[2 * blockIdx.x + 1];
    const int s = s0 + (int)threadIdx.x;
    // a lane with nothing to decode this pass leaves before the staging (no barrier after it)
    JpegSyncState st{};
    JpegSyncState *const xs = F.x;
    bool work = s < F.nseg;
    if (work && pass > 0) {
        if (s == 0) {
            work = false;
        } else {
            const JpegSyncState S = xs[s - 1];
            const int2 old = F.start[s];
            if (S.pos == old.x && S.u == old.y) {
                work = false;
            } else {
                F.start[s] = make_int2(S.pos, S.u);
                st.pos = S.pos;
                st.u = S.u;
            }
        }
    } else if (work) {
        // the guess: the first block of an MCU, JS_WARM bits before the segment (lane 0: the
        // scan's true start); the lane's own start is its first block boundary in its segment
        st.pos = max(0, s * JS_SEG - F.warm);
        F.start[s] = make_int2(-1, -1);  // (set when the decode reaches the segment)
    }
    if (!__syncthreads_or(work)) return;
    stage_tables(F, T);
    __syncthreads();
    if (!work) return;

    const int a0b = 0;  // (bit positions are the scan's own)
    Window win;
    win.init(F.words, F.nwords - 1, st.pos, F.nbits);
    const int lim = F.nwords * 32 - 64;  // positions past the padded scan: an error
    const int seg_lo = s * JS_SEG;
    JpegSyncState *const ck = F.ck + (size_t)s * JS_CK;
    int bp = st.pos - a0b;
    int mark = 0;
    bool warm = pass == 0;  // pass 0: decoding the warm-up (nothing counted or recorded yet)
    for (;;) {
        if (warm && st.pos >= seg_lo) {
            warm = false;
            F.start[s] = make_int2(st.pos, st.u);
            st.nblk = 0;
            st.err = 0;
            st.dc[0] = st.dc[1] = st.dc[2] = 0;
        }
        // the marks this block boundary passes: record (pass 0) or compare (sync passes)
        while (!warm && mark < JS_CK && st.pos >= seg_lo + (mark + 1) * JS_CKB) {
            if (pass > 0) {
                const JpegSyncState c = ck[mark];
                if (!c.err && c.pos == st.pos && c.u == st.u) {
                    // in step with the earlier decode from here on: its later states hold, with the
                    // counts rebased on this start
                    const int dn = st.nblk - c.nblk, d0 = st.dc[0] - c.dc[0], d1 = st.dc[1] - c.dc[1],
                              d2 = st.dc[2] - c.dc[2];
                    JpegSyncState e{};
                    for (int m = mark; m < JS_CK; ++m) {
                        e = ck[m];
                        e.nblk += dn;
                        e.dc[0] += d0;
                        e.dc[1] += d1;
                        e.dc[2] += d2;
                        e.err = st.err ? st.err : e.err ? e.err + dn : 0;  // the first bad block of this trajectory
                        ck[m] = e;
                    }
                    publish(P, pass, xs + s, e);
                    return;
                }
            }
            ck[mark++] = st;
        }
        if (mark == JS_CK) break;  // the exit: the first block boundary at or past the segment's end
        const int u = st.u, c = F.ucomp[u];
        const JpegHuffTable &dc = T[F.td[c]], &ac = T[4 + F.ta[c]];
        LongCodes dcl, acl;
        dcl.load(dc);
        acl.load(ac);
        int diff = 0;
        if (!decode_block<false>(win, bp, dc, ac, dcl, acl, diff, nullptr, nullptr)) {
            // a bad code / AC index: fatal on the true trajectory (the prefix pass zero-fills from
            // this block on), routine on a guessed one -- which goes on a bit further so that it
            // can still fall into step
            if (!st.err) st.err = st.nblk + 1;
            diff = 0;
            bp += 1;
        }
        if (bp + a0b > lim) {  // ran past the staged range (not a JPEG any decoder finishes)
            if (!st.err) st.err = st.nblk + 1;
            while (mark < JS_CK) ck[mark++] = st;  // never matched again
            break;
        }
        st.pos = bp + a0b;
        st.dc[c] += diff;
        st.nblk++;
        st.u = u + 1 == F.bpm ? 0 : u + 1;
    }
    publish(P, pass, xs + s, ck[JS_CK - 1]);
}

// Per frame: the lanes' first block indices and DC predictors (an exclusive scan of their block
// counts and DC sums), in chunks of 256 lanes.  The first lane that fails ends the lanes' part:
//   * a bad code on the true trajectory (corrupt data): err_block = that block, the frame's error
//     flag is set, and the zero pass clears every block from it on;
//   * a start that is not its predecessor's exit (the sync passes ran out before that lane fell
//     into step -- a valid scan): no flag; err_block[1] = the lane, err_block[2] = its first block,
//     and jpeg_sync_serial_kernel decodes the rest of the frame from its predecessor's exit.
__global__ __launch_bounds__(256) void jpeg_sync_prefix_kernel(const JpegSyncParams P) {
    const JpegSyncFrame &F = P.frames[blockIdx.x];
    const JpegSyncState *x = F.x;
    __shared__ int sc[4][256];
    __shared__ int s_fail;
    int carry[4] = {0, 0, 0, 0};
    bool dead = false;
    int err_block = F.nblocks;
    __shared__ int s_sync_lane, s_sync_blk;  // the first out-of-step lane (-1: none) and its block
    if (threadIdx.x == 0) s_sync_lane = -1;
    for (int c0 = 0; c0 < F.nseg; c0 += 256) {  // (after a failure: every later lane base = -1)
        const int t = threadIdx.x, s = c0 + t;
        int v[4] = {0, 0, 0, 0};
        bool bad_start = false, bad_end = false;
        int e_err = 0;
        if (s < F.nseg) {
            const JpegSyncState e = x[s];
            const int2 st = F.start[s];
            if (s > 0) {
                const JpegSyncState p = x[s - 1];
                bad_start = st.x != p.pos || st.y != p.u;  // the sync passes ran out
            }
            bad_end = e.err != 0;
            e_err = e.err;
            v[0] = e.nblk;
            v[1] = e.dc[0];
            v[2] = e.dc[1];
            v[3] = e.dc[2];
        }
        // inclusive scan (Hillis-Steele) of the four sums
        for (int k = 0; k < 4; ++k) sc[k][t] = v[k];
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            int a[4];
            for (int k = 0; k < 4; ++k) a[k] = t >= o ? sc[k][t - o] : 0;
            __syncthreads();
            for (int k = 0; k < 4; ++k) sc[k][t] += a[k];
            __syncthreads();
        }
        int ex[4];
        for (int k = 0; k < 4; ++k) ex[k] = carry[k] + sc[k][t] - v[k];
        // the first lane (in scan order) that fails before the frame's last block
        if (t == 0) s_fail = 1 << 30;
        __syncthreads();
        int fail_at = -1;  // block index where this lane's failure starts the zero fill
        if (s < F.nseg && ex[0] < F.nblocks) {
            if (bad_start) fail_at = ex[0];
            else if (bad_end && ex[0] + e_err - 1 < F.nblocks) fail_at = ex[0] + e_err - 1;
        }
        if (fail_at >= 0) atomicMin(&s_fail, s);
        __syncthreads();
        const int fs = s_fail;
        if (s < F.nseg) {
            const bool live = !dead && !(s > fs || (s == fs && bad_start)) && ex[0] < F.nblocks;
            F.base[s] = live ? ex[0] : -1;
            F.pred[3 * s] = ex[1];
            F.pred[3 * s + 1] = ex[2];
            F.pred[3 * s + 2] = ex[3];
            if (s == fs) {  // (only lane fs's thread holds it)
                if (bad_start) {
                    s_sync_lane = s;
                    s_sync_blk = fail_at;
                } else {
                    err_block = fail_at;
                }
            }
        }
        for (int k = 0; k < 4; ++k) carry[k] += sc[k][255];
        dead = dead || fs < (1 << 30);
        __syncthreads();
    }
    // the frame ran out before its last block (a truncated scan): the rest is not decoded
    if (!dead && threadIdx.x == 0 && carry[0] < F.nblocks) {
        err_block = carry[0];
        dead = true;
    }
    __shared__ int s_err;
    if (threadIdx.x == 0) s_err = F.nblocks;
    __syncthreads();
    if (err_block < F.nblocks) atomicMin(&s_err, err_block);
    __syncthreads();
    if (threadIdx.x == 0) {
        F.err_block[0] = s_err;
        F.err_block[1] = s_sync_lane;
        F.err_block[2] = s_sync_blk;
        if (s_err < F.nblocks) P.error[F.frame] = 1;
    }
}

// The rest of a frame whose sync passes ran out (err_block[1] = the first lane out of step):
// decoded serially by one lane from the predecessor's exit -- the true state there, since every
// earlier lane is in step -- with the predictors and block index the prefix gave that lane.  Only
// a bad code here is corrupt data (err_block[0] and the flag, then the zero pass).  This is the
// rare path (a long chain of out-of-step lanes in a dense scan): correct, one symbol chain long.
__global__ __launch_bounds__(64) void jpeg_sync_serial_kernel(const JpegSyncParams P) {
    __shared__ JpegHuffTable T[8];
    __shared__ uint8_t zz[64];
    __shared__ int4 blk[8];
    const JpegSyncFrame &F = P.frames[blockIdx.x];
    const int fs = F.err_block[1];
    if (fs <= 0) return;  // in step throughout (lane 0 starts at the scan's start: never out of step)
    stage_tables(F, T);
    zz[threadIdx.x] = kZigzag[threadIdx.x];
    __syncthreads();
    if (threadIdx.x != 0) return;
    const JpegSyncState p = F.x[fs - 1];
    Window win;
    win.init(F.words, F.nwords - 1, p.pos, F.nbits);
    const int lim = F.nwords * 32 - 64;
    int bp = p.pos, u = p.u;
    int pred[3] = {F.pred[3 * fs], F.pred[3 * fs + 1], F.pred[3 * fs + 2]};
    int16_t *const co = reinterpret_cast<int16_t *>(blk);
    for (int b = F.err_block[2]; b < F.nblocks; ++b) {
        const int m = b / F.bpm, c = F.ucomp[u];
        const int my = m / F.mcux, mx = m - my * F.mcux;
        const int by = my * F.cv[c] + F.uby[u], bx = mx * F.ch[c] + F.ubx[u];
        const JpegHuffTable &dc = T[F.td[c]], &ac = T[4 + F.ta[c]];
        LongCodes dcl, acl;
        dcl.load(dc);
        acl.load(ac);
#pragma unroll
        for (int z = 0; z < 8; z++) blk[z] = make_int4(0, 0, 0, 0);
        int diff = 0;
        if (!decode_block<true>(win, bp, dc, ac, dcl, acl, diff, co, zz) || bp > lim) {
            F.err_block[0] = b;  // corrupt (or truncated) from this block on: the zero pass
            P.error[F.frame] = 1;
            break;
        }
        pred[c] += diff;
        co[0] = (int16_t)pred[c];
        int4 *const b4 = reinterpret_cast<int4 *>(F.coef + (F.coef_off[c] + (int64_t)by * F.bw[c] + bx) * 64);
#pragma unroll
        for (int z = 0; z < 8; z++) b4[z] = blk[z];
        u = u + 1 == F.bpm ? 0 : u + 1;
    }
}

// The write pass: every live lane decodes its blocks from its start into the coefficient array.
__global__ __launch_bounds__(256) void jpeg_sync_write_kernel(const JpegSyncParams P) {
    __shared__ JpegHuffTable T[8];
    __shared__ uint8_t zz[64];
    __shared__ int4 sblk[256][8];
    const JpegSyncFrame &F = P.frames[P.wg[2 * blockIdx.x]];
    const int s0 = P.wg[2 * blockIdx.x + 1];
    const int s = s0 + (int)threadIdx.x;
    const int base = s < F.nseg ? F.base[s] : -1;
    if (!__syncthreads_or(base >= 0)) return;
    stage_tables(F, T);
    if (threadIdx.x < 64) zz[threadIdx.x] = kZigzag[threadIdx.x];
    __syncthreads();
    if (base < 0) return;
    const JpegSyncState e = F.x[s];
    const int2 st = F.start[s];
    const int end = min(base + e.nblk, F.err_block[0]);
    Window win;
    win.init(F.words, F.nwords - 1, st.x, F.nbits);
    int bp = st.x;
    int pred[3] = {F.pred[3 * s], F.pred[3 * s + 1], F.pred[3 * s + 2]};
    int4 *const mine = sblk[threadIdx.x];
    int16_t *const co = reinterpret_cast<int16_t *>(mine);
    int u = st.y;
    for (int b = base; b < end; ++b) {
        const int m = b / F.bpm, c = F.ucomp[u];
        const int my = m / F.mcux, mx = m - my * F.mcux;
        const int by = my * F.cv[c] + F.uby[u], bx = mx * F.ch[c] + F.ubx[u];
        const JpegHuffTable &dc = T[F.td[c]], &ac = T[4 + F.ta[c]];
        LongCodes dcl, acl;
        dcl.load(dc);
        acl.load(ac);
#pragma unroll
        for (int z = 0; z < 8; z++) mine[z] = make_int4(0, 0, 0, 0);
        int diff = 0;
        if (!decode_block<true>(win, bp, dc, ac, dcl, acl, diff, co, zz)) break;  // (err_block covers it)
        pred[c] += diff;
        co[0] = (int16_t)pred[c];
        int4 *const b4 = reinterpret_cast<int4 *>(F.coef + (F.coef_off[c] + (int64_t)by * F.bw[c] + bx) * 64);
#pragma unroll
        for (int z = 0; z < 8; z++) b4[z] = mine[z];
        u = u + 1 == F.bpm ? 0 : u + 1;
    }
}

// Blocks from a frame's err_block on are zero: the block holding the bad code and every later one
// (libjpeg's rule after corrupt data; the restart-interval kernel applies the same rule per
// interval).
__global__ __launch_bounds__(256) void jpeg_sync_zero_kernel(const JpegSyncParams P) {
    const JpegSyncFrame &F = P.frames[blockIdx.x];
    const int b0 = F.err_block[0];
    for (int i = b0 * 8 + (int)threadIdx.x; i < F.nblocks * 8; i += 256) {
        const int b = i >> 3, z = i & 7;
        const int m = b / F.bpm, u = b - m * F.bpm, c = F.ucomp[u];
        const int my = m / F.mcux, mx = m - my * F.mcux;
        const int by = my * F.cv[c] + F.uby[u], bx = mx * F.ch[c] + F.ubx[u];
        reinterpret_cast<int4 *>(F.coef + (F.coef_off[c] + (int64_t)by * F.bw[c] + bx) * 64)[z] = make_int4(0, 0, 0, 0);
    }
}

}  // namespace

const char *launch_jpeg_sync_scan(const JpegSyncParams &p, int pass, hipStream_t s) {
    if (pass == 0) hipLaunchKernelGGL(jpeg_sync_bswap_kernel, dim3(64, p.nframes), dim3(256), 0, s, p);
    hipLaunchKernelGGL(jpeg_sync_scan_kernel, dim3(p.n_wg), dim3(JS_LANES), 0, s, p, pass);
    return "jpeg_sync_scan_kernel";
}

const char *launch_jpeg_sync_finish(const JpegSyncParams &p, hipStream_t s) {
    hipLaunchKernelGGL(jpeg_sync_prefix_kernel, dim3(p.nframes), dim3(256), 0, s, p);
    hipLaunchKernelGGL(jpeg_sync_write_kernel, dim3(p.n_wg), dim3(JS_LANES), 0, s, p);
    hipLaunchKernelGGL(jpeg_sync_serial_kernel, dim3(p.nframes), dim3(64), 0, s, p);
    hipLaunchKernelGGL(jpeg_sync_zero_kernel, dim3(p.nframes), dim3(256), 0, s, p);
    return "jpeg_sync_write_kernel";
}

}  // namespace zr
