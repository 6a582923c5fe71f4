// dwpw_mfma.hip -- layout choice and launch of the MFMA dwpw forms (dwpw_mfma.h), and the grouped
// launches of sibling layers.  Reference: the Conv nodes of the four ONNX graphs that ORT/tract
// execute at crates/zaru/src/nn/mod.rs:483-533 (the BlazeBlocks).
#include <array>
#include <map>
#include <mutex>
#include <vector>

#include "dwpw_mfma.h"

namespace zr {

// Layout choice for the MFMA forms: no M split unless Mpad > 256, at most 1/3 padded rows;
// among those, the widest column tile that still gives >= 4 workgroups per CU (else the most
// workgroups).
static const DwPwLayout *choose_layout(const DwPwParams &p) {
    // workgroups one launch should reach (ZARU_HIP_MINWGS overrides it for layout sweeps)
    static const int64_t min_wgs = [] {
        const char *e = std::getenv("ZARU_HIP_MINWGS");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int64_t)(v > 0 ? v : 1024);
    }();
    const DwPwLayout *best = nullptr;
    int64_t best_wgs = 0;
    for (const DwPwLayout &l : kLayouts) {
        const int mb = (p.g.Mpad + l.bm() - 1) / l.bm();
        if (mb > 1 && l.bm() < 256) continue;
        if ((int64_t)mb * l.bm() * 3 > (int64_t)p.g.Mpad * 4 && p.g.Mpad <= 256) continue;
        const int64_t wgs = (int64_t)((p.g.ncols + l.bn() - 1) / l.bn()) * mb;
        bool better;
        if (!best) better = true;
        else if ((wgs >= min_wgs) != (best_wgs >= min_wgs)) better = wgs >= min_wgs;
        else if (wgs >= min_wgs) better = l.bn() > best->bn() || (l.bn() == best->bn() && l.bm() < best->bm());
        else better = wgs > best_wgs || (wgs == best_wgs && l.bm() < best->bm());
        if (better) {
            best = &l;
            best_wgs = wgs;
        }
    }
    if (!best) {
        // no tile height wastes <= 1/3 of its rows without an M split (e.g. Mpad = 160, the
        // 144-channel blocks of BlazeFace full range): the unsplit tile with the fewest padded
        // rows, else the tallest split one
        int waste = 1 << 30;
        for (const DwPwLayout &l : kLayouts) {
            const int mb = (p.g.Mpad + l.bm() - 1) / l.bm();
            if (mb > 1 && l.bm() < 256) continue;
            const int w = mb * l.bm() - p.g.Mpad;
            if (w < waste) {
                waste = w;
                best = &l;
            }
        }
    }
    return best;
}

static const char *launch_layout(const DwPwParams &p, const DwPwLayout &l, hipStream_t s) {
    if (p.k == 3) return p.stride == 1 ? dwpw_layout_k3s1(p, l, s) : dwpw_layout_k3s2(p, l, s);
    return p.stride == 1 ? dwpw_layout_k5s1(p, l, s) : dwpw_layout_k5s2(p, l, s);
}

// Layout tuning (ZARU_HIP_TUNE=1): the layouts compute the same arithmetic in the same order
// (tests/test_gpu_forms.py), so which one runs is only a question of time.  The first launch of
// a layer shape (kernel, stride, planes, channels, batch columns) times every admissible layout
// on the launch's own stream (best of 3), and later launches of that shape take the fastest.
static bool tune_on() {
    static const bool v = [] {
        const char *e = std::getenv("ZARU_HIP_TUNE");
        return e && *e == '1';
    }();
    return v;
}

static const DwPwLayout *tuned_layout(const DwPwParams &p, hipStream_t s) {
    typedef std::array<int64_t, 10> Key;
    static std::mutex mu;
    static std::map<Key, int> cache;
    const Key key{p.k, p.stride, p.in.H, p.in.W, p.OW, p.g.K, p.g.M, p.g.Mpad, p.g.ncols, p.g.res_mode};
    {
        std::lock_guard<std::mutex> g(mu);
        const auto it = cache.find(key);
        if (it != cache.end()) return &kLayouts[it->second];
    }
    std::vector<int> cand;
    for (int i = 0; i < (int)(sizeof(kLayouts) / sizeof(kLayouts[0])); ++i) {
        const DwPwLayout &l = kLayouts[i];
        const int mb = (p.g.Mpad + l.bm() - 1) / l.bm();
        if (mb > 1 && l.bm() < 256) continue;
        if ((int64_t)mb * l.bm() * 3 > (int64_t)p.g.Mpad * 4 && p.g.Mpad <= 256) continue;
        cand.push_back(i);
    }
    const DwPwLayout *h = choose_layout(p);
    int best = (int)(h - kLayouts);
    if (cand.size() > 1) {
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) != hipSuccess) return h;
        if (hipEventCreate(&e1) != hipSuccess) {
            (void)hipEventDestroy(e0);
            return h;
        }
        float tbest = 1e30f;
        for (int rep = 0; rep < 3; ++rep)
            for (int i : cand) {
                if (hipEventRecord(e0, s) != hipSuccess) continue;
                launch_layout(p, kLayouts[i], s);
                if (hipEventRecord(e1, s) != hipSuccess) continue;
                float ms = 0.f;
                if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
                if (ms < tbest) {
                    tbest = ms;
                    best = i;
                }
            }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    std::lock_guard<std::mutex> g(mu);
    cache.emplace(key, best);
    return &kLayouts[best];
}

const char *launch_dwpw_mfma(const DwPwParams &p, hipStream_t s) {
    if (const char *k = launch_dwpw_ws(p, s, true)) return k;
    const DwPwLayout *best = tune_on() ? tuned_layout(p, s) : choose_layout(p);
    return launch_layout(p, *best, s);
}

namespace {

template <int K, int S, int WM, int MTW, int DFKC>
const char *dma_group(const DwPwParams *p, int n, hipStream_t s) {
    constexpr int BN = (4 / WM) * 32, BM = WM * MTW * 32, RH = rt_hi(K, MTW, DFKC * BN / 256);
    // one row-task width for every part (the parts are siblings of one shape)
    const int rt = rt_for<K, S>(p[0], BN, RH);
    for (int i = 1; i < n; ++i)
        if (rt_for<K, S>(p[i], BN, RH) != rt) return nullptr;
    LaunchGroup<DwPwParams> G{};
    G.n = n;
    size_t lds = 0;
    int total = 0;
    for (int i = 0; i < n; ++i) {
        int runmax = 0, bufsz = 0;
        const size_t l = dma_plan<K, S, WM, MTW, DFKC>(p[i], &runmax, &bufsz);
        if (!l) return nullptr;
        lds = std::max(lds, l);
        const int nct = (p[i].g.ncols + BN - 1) / BN, mb = (p[i].g.Mpad + BM - 1) / BM;
        G.p[i] = p[i];
        G.a0[i] = nct, G.a1[i] = runmax, G.a2[i] = bufsz;
        G.gx[i] = (nct + 7) / 8 * 8;
        G.start[i] = total;
        total += G.gx[i] * mb;
    }
    for (int i = n; i <= ZR_GROUP_MAX; ++i) G.start[i] = total;
    if (rt == RH) {
        hipLaunchKernelGGL((dwpw_dma_group_kernel<K, S, WM, MTW, DFKC, RH>), dim3(total), dim3(256), lds, s, G);
        return kernel_name("dwpw_dma_group_kernel<%d,%d,%d,%d,%d,%d>", K, S, WM, MTW, DFKC, RH);
    }
    if constexpr (RH >= 4)
        if (rt == RH / 2) {
            hipLaunchKernelGGL((dwpw_dma_group_kernel<K, S, WM, MTW, DFKC, RH / 2>), dim3(total), dim3(256), lds, s, G);
            return kernel_name("dwpw_dma_group_kernel<%d,%d,%d,%d,%d,%d>", K, S, WM, MTW, DFKC, RH / 2);
        }
    hipLaunchKernelGGL((dwpw_dma_group_kernel<K, S, WM, MTW, DFKC, 0>), dim3(total), dim3(256), lds, s, G);
    return kernel_name("dwpw_dma_group_kernel<%d,%d,%d,%d,%d,0>", K, S, WM, MTW, DFKC);
}

template <int K, int S, int DFKC>
const char *dma_group_layout(const DwPwParams *p, int n, const DwPwLayout &l, hipStream_t s) {
    switch (l.wm * 10 + l.mtw) {  // the layouts of the 6^2 / 3^2 sibling blocks (FaceMesh heads)
    case 11: return dma_group<K, S, 1, 1, DFKC>(p, n, s);
    case 21: return dma_group<K, S, 2, 1, DFKC>(p, n, s);
    case 41: return dma_group<K, S, 4, 1, DFKC>(p, n, s);
    default: return nullptr;
    }
}

}  // namespace

// Sibling MFMA dwpw layers in one launch when every part takes the LDS-DMA form with the same
// kernel, layout and 16-channel chunks; nullptr otherwise (the caller launches them one by one).
const char *launch_dwpw_mfma_group(const DwPwParams *p, int n, hipStream_t s) {
    if (n < 2 || n > ZR_GROUP_MAX) return nullptr;
    const DwPwLayout *l0 = nullptr;
    for (int i = 0; i < n; ++i) {
        if (p[i].k != p[0].k || p[i].stride != p[0].stride || launch_dwpw_ws(p[i], s, false)) return nullptr;
        const DwPwLayout *l = choose_layout(p[i]);
        if (l0 && (l->wm != l0->wm || l->mtw != l0->mtw)) return nullptr;
        l0 = l;
    }
    if (p[0].k != 3 || l0->mtw != 1) return nullptr;
    // the chunk each part would use alone (the rule on the whole group's workgroups: at most
    // twice one part's, so the group keeps the parts' chunk unless that crosses the threshold)
    const int bn = (4 / l0->wm) * 32;
    int wgs = 0;
    for (int i = 0; i < n; ++i) wgs = std::max(wgs, (p[i].g.ncols + bn - 1) / bn);
    const int dk = dfkc_for(wgs, p[0].g.K);
    if (dk == 32) return p[0].stride == 1 ? dma_group_layout<3, 1, 32>(p, n, *l0, s) : dma_group_layout<3, 2, 32>(p, n, *l0, s);
    if (dk == 16) return p[0].stride == 1 ? dma_group_layout<3, 1, 16>(p, n, *l0, s) : dma_group_layout<3, 2, 16>(p, n, *l0, s);
    return nullptr;
}


}  // namespace zr

