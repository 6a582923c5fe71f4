/*
 * nnexec_impl.h -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * A deliberately naive ONNX interpreter: NCHW, batch 1, every operator evaluated
 * straight from its ONNX definition (onnx.ai/onnx/operators) in REAL precision.
 * It stands in for ONNX Runtime 1.14.8 / tract 0.20.7, which execute these graphs
 * for the reference (crates/zaru/src/nn/mod.rs:483-533) and are absent here.
 * Included twice by nnexec.c with REAL = double and REAL = float.
 */

typedef struct {
    char *name;
    int ndim;
    int64_t dims[6];
    REAL *f;      /* float data (NULL for int tensors) */
    int64_t *i64; /* int64 data */
    size_t n;
} NN(tensor);

typedef struct {
    char *op;
    int nin, nout;
    char **in, **out;
    pb_slice attrs[16];
    int nattr;
} NN(node);

struct NN(net_s) {
    NN(tensor) **vals; /* initializers + computed values; each individually allocated, so a
                        * tensor pointer stays valid while later values are pushed */
    size_t nvals, cap;
    NN(node) *nodes;
    size_t nnodes;
    char *input_name;
    int64_t input_dims[4];
    char *outputs[8];
    size_t noutputs;
    size_t nstatic; /* number of initializer entries (kept across runs) */
};

static NN(tensor) *NN(find)(struct NN(net_s) *n, const char *name) {
    for (size_t i = n->nvals; i-- > 0;)
        if (strcmp(n->vals[i]->name, name) == 0) return n->vals[i];
    return NULL;
}

static NN(tensor) *NN(push)(struct NN(net_s) *n, const char *name) {
    if (n->nvals == n->cap) {
        n->cap = n->cap ? n->cap * 2 : 256;
        n->vals = (NN(tensor) **)realloc(n->vals, n->cap * sizeof(NN(tensor) *));
    }
    NN(tensor) *t = (NN(tensor) *)calloc(1, sizeof(NN(tensor)));
    n->vals[n->nvals++] = t;
    t->name = strdup(name);
    return t;
}

static size_t NN(numel)(const int64_t *d, int nd) {
    size_t s = 1;
    for (int i = 0; i < nd; i++) s *= (size_t)d[i];
    return s;
}

static NN(tensor) *NN(new_out)(struct NN(net_s) *n, const char *name, int nd, const int64_t *d) {
    NN(tensor) *t = NN(push)(n, name);
    t->ndim = nd;
    memcpy(t->dims, d, sizeof(int64_t) * nd);
    t->n = NN(numel)(d, nd);
    t->f = (REAL *)calloc(t->n ? t->n : 1, sizeof(REAL));
    return t;
}

/* ---- attributes ---- */
static int NN(attr)(const NN(node) *nd, const char *name, pb_attr *a) {
    for (int i = 0; i < nd->nattr; i++) {
        pb_attr_parse(nd->attrs[i], a);
        if (a->name_len == strlen(name) && memcmp(a->name, name, a->name_len) == 0) return 1;
    }
    return 0;
}
static int64_t NN(attr_i)(const NN(node) *nd, const char *name, int64_t dflt) {
    pb_attr a;
    return NN(attr)(nd, name, &a) ? a.i : dflt;
}
static float NN(attr_f)(const NN(node) *nd, const char *name, float dflt) {
    pb_attr a;
    return NN(attr)(nd, name, &a) ? a.f : dflt;
}
static int NN(attr_ints)(const NN(node) *nd, const char *name, int64_t *out, int cap) {
    pb_attr a;
    if (!NN(attr)(nd, name, &a)) return -1;
    return pb_attr_ints(&a, out, cap);
}
static int NN(attr_s)(const NN(node) *nd, const char *name, const char *want) {
    pb_attr a;
    if (!NN(attr)(nd, name, &a)) return 0;
    return a.s_len == strlen(want) && memcmp(a.s, want, a.s_len) == 0;
}

/* ---- operators ---- */
#define FAIL(msg)                                                                            \
    do {                                                                                     \
        snprintf(g_err, sizeof(g_err), "%s (%s)", msg, nd->op);                               \
        return -1;                                                                           \
    } while (0)

static int NN(op_conv)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]), *w = NN(find)(n, nd->in[1]);
    NN(tensor) *b = nd->nin > 2 ? NN(find)(n, nd->in[2]) : NULL;
    if (!x || !w) FAIL("missing input");
    int64_t st[2] = {1, 1}, pads[4] = {0, 0, 0, 0}, dil[2] = {1, 1};
    NN(attr_ints)(nd, "strides", st, 2);
    NN(attr_ints)(nd, "pads", pads, 4);
    NN(attr_ints)(nd, "dilations", dil, 2);
    int64_t g = NN(attr_i)(nd, "group", 1);
    int64_t C = x->dims[1], H = x->dims[2], W = x->dims[3];
    int64_t M = w->dims[0], CG = w->dims[1], KH = w->dims[2], KW = w->dims[3];
    int64_t OH = (H + pads[0] + pads[2] - dil[0] * (KH - 1) - 1) / st[0] + 1;
    int64_t OW = (W + pads[1] + pads[3] - dil[1] * (KW - 1) - 1) / st[1] + 1;
    if (CG * g != C) FAIL("group mismatch");
    int64_t od[4] = {1, M, OH, OW};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    int64_t mg = M / g;
    /* Every output starts at its bias and accumulates w * x over (c, ky, kx) in ascending
     * order, skipping taps outside the input -- the ONNX Conv definition evaluated term by
     * term.  The loops run tap-major with the output row innermost (vectorisable), which
     * keeps exactly that per-output summation order. */
    for (int64_t m = 0; m < M; m++) {
        REAL *ym = y->f + m * OH * OW;
        const REAL bm = b ? b->f[m] : (REAL)0;
        for (int64_t p = 0; p < OH * OW; p++) ym[p] = bm;
        int64_t grp = m / mg;
        if (KH == 1 && KW == 1 && st[0] == 1 && st[1] == 1 && !pads[0] && !pads[1] && !pads[2] &&
            !pads[3]) { /* 1x1: one contiguous axpy per input channel */
            for (int64_t c = 0; c < CG; c++) {
                const REAL wv = w->f[m * CG + c], *xc = x->f + (grp * CG + c) * H * W;
                for (int64_t p = 0; p < OH * OW; p++) ym[p] += wv * xc[p];
            }
            continue;
        }
        for (int64_t c = 0; c < CG; c++) {
            int64_t ic = grp * CG + c;
            const REAL *xc = x->f + ic * H * W;
            for (int64_t ky = 0; ky < KH; ky++) {
                /* oy with 0 <= oy*st0 - pad0 + ky*dil0 < H */
                int64_t a = pads[0] - ky * dil[0];
                int64_t oy0 = a <= 0 ? 0 : (a + st[0] - 1) / st[0];
                int64_t oy1 = H - 1 + a < 0 ? -1 : (H - 1 + a) / st[0];
                if (oy1 > OH - 1) oy1 = OH - 1;
                for (int64_t kx = 0; kx < KW; kx++) {
                    const REAL wv = w->f[((m * CG + c) * KH + ky) * KW + kx];
                    int64_t bx = pads[1] - kx * dil[1];
                    int64_t ox0 = bx <= 0 ? 0 : (bx + st[1] - 1) / st[1];
                    int64_t ox1 = W - 1 + bx < 0 ? -1 : (W - 1 + bx) / st[1];
                    if (ox1 > OW - 1) ox1 = OW - 1;
                    for (int64_t oy = oy0; oy <= oy1; oy++) {
                        const REAL *xr = xc + (oy * st[0] - a) * W - bx;
                        REAL *yr = ym + oy * OW;
                        if (st[1] == 1)
                            for (int64_t ox = ox0; ox <= ox1; ox++) yr[ox] += wv * xr[ox];
                        else
                            for (int64_t ox = ox0; ox <= ox1; ox++) yr[ox] += wv * xr[ox * st[1]];
                    }
                }
            }
        }
    }
    return 0;
}

static int NN(op_unary)(struct NN(net_s) *n, const NN(node) *nd, int kind) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    NN(tensor) *y = NN(new_out)(n, nd->out[0], x->ndim, x->dims);
    REAL lo = 0, hi = 0;
    if (kind == 2) { /* Clip: attributes (opset < 11) or inputs */
        lo = (REAL)NN(attr_f)(nd, "min", -3.4e38f);
        hi = (REAL)NN(attr_f)(nd, "max", 3.4e38f);
        if (nd->nin > 1 && nd->in[1][0]) lo = NN(find)(n, nd->in[1])->f[0];
        if (nd->nin > 2 && nd->in[2][0]) hi = NN(find)(n, nd->in[2])->f[0];
    }
    for (size_t i = 0; i < x->n; i++) {
        REAL v = x->f[i];
        if (kind == 0) v = v > 0 ? v : 0;                       /* Relu */
        else if (kind == 1) v = (REAL)1 / ((REAL)1 + exp(-(double)v)); /* Sigmoid */
        else if (kind == 2) v = v < lo ? lo : (v > hi ? hi : v);
        y->f[i] = v;
    }
    return 0;
}

static int NN(op_prelu)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]), *s = NN(find)(n, nd->in[1]);
    if (!x || !s) FAIL("missing input");
    NN(tensor) *y = NN(new_out)(n, nd->out[0], x->ndim, x->dims);
    size_t C = (size_t)x->dims[1], plane = x->n / C;
    if (s->n != C && s->n != 1) FAIL("unsupported slope shape");
    for (size_t c = 0; c < C; c++) {
        REAL sl = s->f[s->n == 1 ? 0 : c];
        for (size_t p = 0; p < plane; p++) {
            REAL v = x->f[c * plane + p];
            y->f[c * plane + p] = v < 0 ? v * sl : v;
        }
    }
    return 0;
}

static int NN(op_add)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *a = NN(find)(n, nd->in[0]), *b = NN(find)(n, nd->in[1]);
    if (!a || !b) FAIL("missing input");
    if (a->n != b->n) FAIL("broadcasting add unsupported");
    NN(tensor) *y = NN(new_out)(n, nd->out[0], a->ndim, a->dims);
    for (size_t i = 0; i < a->n; i++) y->f[i] = a->f[i] + b->f[i];
    return 0;
}

static int NN(op_pad)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t pads[8] = {0};
    if (nd->nin > 1) {
        NN(tensor) *p = NN(find)(n, nd->in[1]);
        for (int i = 0; i < 8 && i < (int)p->n; i++) pads[i] = p->i64[i];
    } else {
        NN(attr_ints)(nd, "pads", pads, 8);
    }
    REAL cval = 0;
    if (nd->nin > 2 && nd->in[2][0]) cval = NN(find)(n, nd->in[2])->f[0];
    if (x->ndim != 4) FAIL("rank");
    int64_t od[4];
    for (int i = 0; i < 4; i++) {
        if (pads[i] < 0 || pads[i + 4] < 0) FAIL("negative pad");
        od[i] = x->dims[i] + pads[i] + pads[i + 4];
    }
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    for (size_t i = 0; i < y->n; i++) y->f[i] = cval;
    for (int64_t a0 = 0; a0 < x->dims[0]; a0++)
        for (int64_t a1 = 0; a1 < x->dims[1]; a1++)
            for (int64_t a2 = 0; a2 < x->dims[2]; a2++)
                for (int64_t a3 = 0; a3 < x->dims[3]; a3++) {
                    int64_t o = (((a0 + pads[0]) * od[1] + a1 + pads[1]) * od[2] + a2 + pads[2]) *
                                    od[3] + a3 + pads[3];
                    y->f[o] = x->f[((a0 * x->dims[1] + a1) * x->dims[2] + a2) * x->dims[3] + a3];
                }
    return 0;
}

static int NN(op_maxpool)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t k[2] = {1, 1}, st[2] = {1, 1}, pads[4] = {0, 0, 0, 0};
    NN(attr_ints)(nd, "kernel_shape", k, 2);
    NN(attr_ints)(nd, "strides", st, 2);
    NN(attr_ints)(nd, "pads", pads, 4);
    int64_t C = x->dims[1], H = x->dims[2], W = x->dims[3];
    int64_t OH = (H + pads[0] + pads[2] - k[0]) / st[0] + 1;
    int64_t OW = (W + pads[1] + pads[3] - k[1]) / st[1] + 1;
    int64_t od[4] = {1, C, OH, OW};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    for (int64_t c = 0; c < C; c++)
        for (int64_t oy = 0; oy < OH; oy++)
            for (int64_t ox = 0; ox < OW; ox++) {
                REAL m = -INFINITY;
                for (int64_t ky = 0; ky < k[0]; ky++)
                    for (int64_t kx = 0; kx < k[1]; kx++) {
                        int64_t iy = oy * st[0] - pads[0] + ky, ix = ox * st[1] - pads[1] + kx;
                        if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
                        REAL v = x->f[(c * H + iy) * W + ix];
                        if (v > m) m = v;
                    }
                y->f[(c * OH + oy) * OW + ox] = m;
            }
    return 0;
}

/* Resize, mode=linear, coordinate_transformation_mode=half_pixel: separable, edge-clamped */
static int NN(op_resize)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    if (!NN(attr_s)(nd, "mode", "linear") ||
        !NN(attr_s)(nd, "coordinate_transformation_mode", "half_pixel"))
        FAIL("only linear/half_pixel resize supported");
    int64_t C = x->dims[1], H = x->dims[2], W = x->dims[3], OH, OW;
    NN(tensor) *sizes = nd->nin > 3 && nd->in[3][0] ? NN(find)(n, nd->in[3]) : NULL;
    NN(tensor) *scales = nd->nin > 2 && nd->in[2][0] ? NN(find)(n, nd->in[2]) : NULL;
    double sy, sx;
    if (sizes && sizes->n == 4) {
        OH = sizes->i64[2];
        OW = sizes->i64[3];
        sy = (double)OH / H;
        sx = (double)OW / W;
    } else if (scales && scales->n == 4) {
        sy = scales->f[2];
        sx = scales->f[3];
        OH = (int64_t)floor(H * sy);
        OW = (int64_t)floor(W * sx);
    } else
        FAIL("resize needs sizes or scales");
    int64_t od[4] = {1, C, OH, OW};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    for (int64_t c = 0; c < C; c++)
        for (int64_t oy = 0; oy < OH; oy++) {
            double fy = (oy + 0.5) / sy - 0.5;
            double y0f = floor(fy);
            double ry = fy - y0f;
            int64_t y0 = (int64_t)y0f, y1 = y0 + 1;
            y0 = y0 < 0 ? 0 : (y0 >= H ? H - 1 : y0);
            y1 = y1 < 0 ? 0 : (y1 >= H ? H - 1 : y1);
            for (int64_t ox = 0; ox < OW; ox++) {
                double fx = (ox + 0.5) / sx - 0.5;
                double x0f = floor(fx);
                double rx = fx - x0f;
                int64_t x0 = (int64_t)x0f, x1 = x0 + 1;
                x0 = x0 < 0 ? 0 : (x0 >= W ? W - 1 : x0);
                x1 = x1 < 0 ? 0 : (x1 >= W ? W - 1 : x1);
                const REAL *p = x->f + c * H * W;
                REAL top = (REAL)((1 - rx) * p[y0 * W + x0] + rx * p[y0 * W + x1]);
                REAL bot = (REAL)((1 - rx) * p[y1 * W + x0] + rx * p[y1 * W + x1]);
                y->f[(c * OH + oy) * OW + ox] = (REAL)((1 - ry) * top + ry * bot);
            }
        }
    return 0;
}

static int NN(op_transpose)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t perm[6];
    int np = NN(attr_ints)(nd, "perm", perm, 6);
    if (np != x->ndim) FAIL("perm");
    int64_t od[6], ist[6], s = 1;
    for (int i = x->ndim - 1; i >= 0; i--) {
        ist[i] = s;
        s *= x->dims[i];
    }
    for (int i = 0; i < np; i++) od[i] = x->dims[perm[i]];
    NN(tensor) *y = NN(new_out)(n, nd->out[0], np, od);
    int64_t idx[6] = {0};
    for (size_t o = 0; o < y->n; o++) {
        int64_t src = 0;
        for (int i = 0; i < np; i++) src += idx[i] * ist[perm[i]];
        y->f[o] = x->f[src];
        for (int i = np - 1; i >= 0; i--) {
            if (++idx[i] < od[i]) break;
            idx[i] = 0;
        }
    }
    return 0;
}

static int NN(op_reshape)(struct NN(net_s) *n, const NN(node) *nd, int squeeze) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t od[6];
    int nd_out = 0;
    if (squeeze) {
        int64_t axes[6];
        int na = NN(attr_ints)(nd, "axes", axes, 6);
        for (int i = 0; i < x->ndim; i++) {
            int drop = 0;
            for (int j = 0; j < na; j++)
                if (axes[j] == i || axes[j] + x->ndim == i) drop = 1;
            if (na < 0 && x->dims[i] == 1) drop = 1;
            if (!drop) od[nd_out++] = x->dims[i];
        }
    } else {
        NN(tensor) *s = NN(find)(n, nd->in[1]);
        if (!s || !s->i64) FAIL("shape");
        int64_t known = 1;
        int neg = -1;
        for (size_t i = 0; i < s->n; i++) {
            od[i] = s->i64[i] == 0 ? x->dims[i] : s->i64[i];
            if (od[i] == -1) neg = (int)i;
            else known *= od[i];
        }
        nd_out = (int)s->n;
        if (neg >= 0) od[neg] = (int64_t)x->n / known;
    }
    NN(tensor) *y = NN(new_out)(n, nd->out[0], nd_out, od);
    if (y->n != x->n) FAIL("reshape size");
    memcpy(y->f, x->f, sizeof(REAL) * x->n);
    return 0;
}

static int NN(op_concat)(struct NN(net_s) *n, const NN(node) *nd) {
    int64_t axis = NN(attr_i)(nd, "axis", 0);
    NN(tensor) *x0 = NN(find)(n, nd->in[0]);
    if (!x0) FAIL("missing input");
    if (axis < 0) axis += x0->ndim;
    int64_t od[6];
    memcpy(od, x0->dims, sizeof(od));
    od[axis] = 0;
    for (int i = 0; i < nd->nin; i++) od[axis] += NN(find)(n, nd->in[i])->dims[axis];
    NN(tensor) *y = NN(new_out)(n, nd->out[0], x0->ndim, od);
    size_t outer = 1, inner = 1;
    for (int i = 0; i < axis; i++) outer *= (size_t)od[i];
    for (int i = (int)axis + 1; i < x0->ndim; i++) inner *= (size_t)od[i];
    size_t off = 0;
    for (int i = 0; i < nd->nin; i++) {
        NN(tensor) *x = NN(find)(n, nd->in[i]);
        size_t chunk = (size_t)x->dims[axis] * inner;
        for (size_t o = 0; o < outer; o++)
            memcpy(y->f + o * od[axis] * inner + off, x->f + o * chunk, sizeof(REAL) * chunk);
        off += chunk;
    }
    return 0;
}

static int NN(op_gap)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t C = x->dims[1], P = x->dims[2] * x->dims[3];
    int64_t od[4] = {1, C, 1, 1};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    for (int64_t c = 0; c < C; c++) {
        REAL s = 0;
        for (int64_t p = 0; p < P; p++) s += x->f[c * P + p];
        y->f[c] = s / (REAL)P;
    }
    return 0;
}

/* AveragePool (count_include_pad = 0, no ceil_mode): the mean of the in-bounds window */
static int NN(op_avgpool)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t k[2] = {1, 1}, st[2] = {1, 1}, pads[4] = {0, 0, 0, 0};
    NN(attr_ints)(nd, "kernel_shape", k, 2);
    NN(attr_ints)(nd, "strides", st, 2);
    NN(attr_ints)(nd, "pads", pads, 4);
    if (NN(attr_i)(nd, "ceil_mode", 0)) FAIL("AveragePool ceil_mode unsupported");
    int64_t C = x->dims[1], H = x->dims[2], W = x->dims[3];
    int64_t OH = (H + pads[0] + pads[2] - k[0]) / st[0] + 1;
    int64_t OW = (W + pads[1] + pads[3] - k[1]) / st[1] + 1;
    int64_t od[4] = {1, C, OH, OW};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 4, od);
    for (int64_t c = 0; c < C; c++)
        for (int64_t oy = 0; oy < OH; oy++)
            for (int64_t ox = 0; ox < OW; ox++) {
                REAL s = 0;
                int64_t cnt = 0;
                for (int64_t ky = 0; ky < k[0]; ky++)
                    for (int64_t kx = 0; kx < k[1]; kx++) {
                        int64_t iy = oy * st[0] - pads[0] + ky, ix = ox * st[1] - pads[1] + kx;
                        if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
                        s += x->f[(c * H + iy) * W + ix];
                        cnt++;
                    }
                y->f[(c * OH + oy) * OW + ox] = s / (REAL)cnt;
            }
    return 0;
}

/* ReduceMean over a set of trailing axes (opset <= 17: axes attribute) */
static int NN(op_reducemean)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *x = NN(find)(n, nd->in[0]);
    if (!x) FAIL("missing input");
    int64_t axes[6];
    int na = NN(attr_ints)(nd, "axes", axes, 6);
    if (na <= 0) FAIL("ReduceMean needs axes");
    int keep = (int)NN(attr_i)(nd, "keepdims", 1);
    int red[6] = {0};
    for (int i = 0; i < na; i++) red[axes[i] < 0 ? axes[i] + x->ndim : axes[i]] = 1;
    /* outer = dims before the first reduced axis (reduced axes must be trailing) */
    int first = x->ndim;
    for (int i = 0; i < x->ndim; i++)
        if (red[i]) { first = i; break; }
    for (int i = first; i < x->ndim; i++)
        if (!red[i]) FAIL("ReduceMean over non-trailing axes unsupported");
    int64_t outer = 1, inner = 1, od[6];
    int nd_out = 0;
    for (int i = 0; i < x->ndim; i++) {
        if (i < first) { outer *= x->dims[i]; od[nd_out++] = x->dims[i]; }
        else { inner *= x->dims[i]; if (keep) od[nd_out++] = 1; }
    }
    NN(tensor) *y = NN(new_out)(n, nd->out[0], nd_out, od);
    for (int64_t o = 0; o < outer; o++) {
        REAL s = 0;
        for (int64_t i = 0; i < inner; i++) s += x->f[o * inner + i];
        y->f[o] = s / (REAL)inner;
    }
    return 0;
}

static int NN(op_gemm)(struct NN(net_s) *n, const NN(node) *nd) {
    NN(tensor) *a = NN(find)(n, nd->in[0]), *b = NN(find)(n, nd->in[1]);
    NN(tensor) *c = nd->nin > 2 ? NN(find)(n, nd->in[2]) : NULL;
    if (!a || !b) FAIL("missing input");
    int64_t ta = NN(attr_i)(nd, "transA", 0), tb = NN(attr_i)(nd, "transB", 0);
    REAL alpha = NN(attr_f)(nd, "alpha", 1.0f), beta = NN(attr_f)(nd, "beta", 1.0f);
    int64_t M = ta ? a->dims[1] : a->dims[0], K = ta ? a->dims[0] : a->dims[1];
    int64_t N = tb ? b->dims[0] : b->dims[1];
    int64_t od[2] = {M, N};
    NN(tensor) *y = NN(new_out)(n, nd->out[0], 2, od);
    for (int64_t i = 0; i < M; i++)
        for (int64_t j = 0; j < N; j++) {
            REAL s = 0;
            for (int64_t k = 0; k < K; k++) {
                REAL av = ta ? a->f[k * M + i] : a->f[i * K + k];
                REAL bv = tb ? b->f[j * K + k] : b->f[k * N + j];
                s += av * bv;
            }
            REAL cv = c ? c->f[c->n == (size_t)N ? j : (c->n == 1 ? 0 : i * N + j)] : 0;
            y->f[i * N + j] = alpha * s + beta * cv;
        }
    return 0;
}

static int NN(exec_node)(struct NN(net_s) *n, const NN(node) *nd) {
    const char *op = nd->op;
    if (!strcmp(op, "Conv")) return NN(op_conv)(n, nd);
    if (!strcmp(op, "Relu")) return NN(op_unary)(n, nd, 0);
    if (!strcmp(op, "Sigmoid")) return NN(op_unary)(n, nd, 1);
    if (!strcmp(op, "Clip")) return NN(op_unary)(n, nd, 2);
    if (!strcmp(op, "PRelu")) return NN(op_prelu)(n, nd);
    if (!strcmp(op, "Add")) return NN(op_add)(n, nd);
    if (!strcmp(op, "Pad")) return NN(op_pad)(n, nd);
    if (!strcmp(op, "MaxPool")) return NN(op_maxpool)(n, nd);
    if (!strcmp(op, "Resize")) return NN(op_resize)(n, nd);
    if (!strcmp(op, "Transpose")) return NN(op_transpose)(n, nd);
    if (!strcmp(op, "Reshape")) return NN(op_reshape)(n, nd, 0);
    if (!strcmp(op, "Squeeze")) return NN(op_reshape)(n, nd, 1);
    if (!strcmp(op, "Concat")) return NN(op_concat)(n, nd);
    if (!strcmp(op, "GlobalAveragePool")) return NN(op_gap)(n, nd);
    if (!strcmp(op, "Gemm")) return NN(op_gemm)(n, nd);
    if (!strcmp(op, "AveragePool")) return NN(op_avgpool)(n, nd);
    if (!strcmp(op, "ReduceMean")) return NN(op_reducemean)(n, nd);
    snprintf(g_err, sizeof(g_err), "unsupported op %s", op);
    return -1;
}

static void NN(clear_dynamic)(struct NN(net_s) *n) {
    while (n->nvals > n->nstatic) {
        NN(tensor) *t = n->vals[--n->nvals];
        free(t->name);
        free(t->f);
        free(t->i64);
        free(t);
    }
}

static int NN(run)(struct NN(net_s) *n, const float *input) {
    NN(clear_dynamic)(n);
    NN(tensor) *x = NN(new_out)(n, n->input_name, 4, n->input_dims);
    for (size_t i = 0; i < x->n; i++) x->f[i] = (REAL)input[i];
    for (size_t i = 0; i < n->nnodes; i++)
        if (NN(exec_node)(n, &n->nodes[i])) return -1;
    return 0;
}
#undef FAIL
