/*
 * nnexec.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Minimal protobuf wire-format reader for ONNX ModelProto (onnx/onnx.proto field
 * numbers) plus the f64 / f32 instantiations of the naive interpreter in nnexec_impl.h.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char g_err[512];
const char *zo_net_error(void) { return g_err; }

typedef struct {
    const uint8_t *p;
    size_t n;
} pb_slice;

typedef struct {
    uint32_t field, wire;
    uint64_t v;      /* varint / fixed value */
    pb_slice bytes;  /* length-delimited payload */
} pb_field;

static int pb_varint(const uint8_t **p, const uint8_t *end, uint64_t *out) {
    uint64_t r = 0;
    int s = 0;
    while (*p < end && s < 64) {
        uint8_t c = *(*p)++;
        r |= (uint64_t)(c & 0x7F) << s;
        if (!(c & 0x80)) {
            *out = r;
            return 1;
        }
        s += 7;
    }
    return 0;
}

/* iterate: returns 1 and fills f while fields remain */
static int pb_next(pb_slice *s, pb_field *f) {
    if (s->n == 0) return 0;
    const uint8_t *p = s->p, *end = s->p + s->n;
    uint64_t key;
    if (!pb_varint(&p, end, &key)) return 0;
    f->field = (uint32_t)(key >> 3);
    f->wire = (uint32_t)(key & 7);
    f->bytes.p = NULL;
    f->bytes.n = 0;
    switch (f->wire) {
    case 0:
        if (!pb_varint(&p, end, &f->v)) return 0;
        break;
    case 1:
        if (end - p < 8) return 0;
        memcpy(&f->v, p, 8);
        p += 8;
        break;
    case 5: {
        if (end - p < 4) return 0;
        uint32_t t;
        memcpy(&t, p, 4);
        f->v = t;
        p += 4;
        break;
    }
    case 2: {
        uint64_t len;
        if (!pb_varint(&p, end, &len) || (uint64_t)(end - p) < len) return 0;
        f->bytes.p = p;
        f->bytes.n = (size_t)len;
        p += len;
        break;
    }
    default:
        return 0;
    }
    s->n -= (size_t)(p - s->p);
    s->p = p;
    return 1;
}

static char *pb_str(pb_slice b) {
    char *s = (char *)malloc(b.n + 1);
    memcpy(s, b.p, b.n);
    s[b.n] = 0;
    return s;
}

/* AttributeProto: 1 name, 2 f, 3 i, 4 s, 7 floats, 8 ints */
typedef struct {
    const char *name;
    size_t name_len;
    float f;
    int64_t i;
    const char *s;
    size_t s_len;
    pb_slice ints_packed;
    pb_slice raw;
} pb_attr;

static void pb_attr_parse(pb_slice b, pb_attr *a) {
    memset(a, 0, sizeof(*a));
    a->raw = b;
    pb_field f = {0};
    while (pb_next(&b, &f)) {
        if (f.field == 1 && f.wire == 2) {
            a->name = (const char *)f.bytes.p;
            a->name_len = f.bytes.n;
        } else if (f.field == 2 && f.wire == 5) {
            uint32_t t = (uint32_t)f.v;
            memcpy(&a->f, &t, 4);
        } else if (f.field == 3 && f.wire == 0) {
            a->i = (int64_t)f.v;
        } else if (f.field == 4 && f.wire == 2) {
            a->s = (const char *)f.bytes.p;
            a->s_len = f.bytes.n;
        }
    }
}

static int pb_attr_ints(const pb_attr *a, int64_t *out, int cap) {
    pb_slice b = a->raw;
    pb_field f = {0};
    int n = 0;
    while (pb_next(&b, &f)) {
        if (f.field != 8) continue;
        if (f.wire == 0) {
            if (n < cap) out[n] = (int64_t)f.v;
            n++;
        } else if (f.wire == 2) {
            const uint8_t *p = f.bytes.p, *end = p + f.bytes.n;
            uint64_t v;
            while (p < end && pb_varint(&p, end, &v)) {
                if (n < cap) out[n] = (int64_t)v;
                n++;
            }
        }
    }
    return n;
}

/* ---------------------------------------------------------------- f64 / f32 */
#define REAL double
#define NN(x) x##_f64
#include "nnexec_impl.h"
#undef REAL
#undef NN
#define REAL float
#define NN(x) x##_f32
#include "nnexec_impl.h"
#undef REAL
#undef NN

/* TensorProto: 1 dims, 2 data_type, 4 float_data, 5 int32_data, 7 int64_data, 8 name,
 * 9 raw_data */
typedef struct {
    char *name;
    int ndim;
    int64_t dims[6];
    int dtype;
    pb_slice raw, floats, ints, i32s;
} raw_tensor;

/* IEEE 754 binary16 -> binary64, exact (every half is representable in float and double).
 * FaceMesh V2 (face_landmarks_detector.onnx) stores its weights as FLOAT16 initializers;
 * ONNX Runtime upcasts them exactly before the f32 convolutions. */
static double half_to_double(uint16_t h) {
    int e = (h >> 10) & 0x1f, m = h & 0x3ff;
    double v;
    if (e == 0) v = ldexp((double)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = ldexp((double)(m | 0x400), e - 25);
    return (h & 0x8000) ? -v : v;
}

static void parse_tensor(pb_slice b, raw_tensor *t) {
    memset(t, 0, sizeof(*t));
    pb_field f = {0};
    while (pb_next(&b, &f)) {
        if (f.field == 1) {
            if (f.wire == 0) t->dims[t->ndim++] = (int64_t)f.v;
            else {
                const uint8_t *p = f.bytes.p, *end = p + f.bytes.n;
                uint64_t v;
                while (p < end && pb_varint(&p, end, &v)) t->dims[t->ndim++] = (int64_t)v;
            }
        } else if (f.field == 2) t->dtype = (int)f.v;
        else if (f.field == 4) t->floats = f.bytes;
        else if (f.field == 5) t->i32s = f.bytes;
        else if (f.field == 7) t->ints = f.bytes;
        else if (f.field == 8) t->name = pb_str(f.bytes);
        else if (f.field == 9) t->raw = f.bytes;
    }
}

struct zo_net {
    int f64;
    struct net_s_f64 *d;
    struct net_s_f32 *s;
};

#define LOAD_IMPL(SUF, REALT)                                                                   \
    static struct net_s_##SUF *load_##SUF(const uint8_t *bytes, size_t len) {                   \
        struct net_s_##SUF *n = (struct net_s_##SUF *)calloc(1, sizeof(*n));                    \
        pb_slice m = {bytes, len}, g = {NULL, 0};                                               \
        pb_field f = {0};                                                                             \
        while (pb_next(&m, &f))                                                                 \
            if (f.field == 7 && f.wire == 2) g = f.bytes;                                       \
        if (!g.p) {                                                                             \
            snprintf(g_err, sizeof(g_err), "no graph");                                         \
            return NULL;                                                                        \
        }                                                                                       \
        pb_slice gg = g;                                                                        \
        size_t nn = 0;                                                                          \
        while (pb_next(&gg, &f))                                                                \
            if (f.field == 1) nn++;                                                             \
        n->nodes = (node_##SUF *)calloc(nn ? nn : 1, sizeof(node_##SUF));                        \
        gg = g;                                                                                 \
        while (pb_next(&gg, &f)) {                                                              \
            if (f.field == 1) {                                                                 \
                node_##SUF *nd = &n->nodes[n->nnodes++];                                         \
                nd->in = (char **)calloc(16, sizeof(char *));                                   \
                nd->out = (char **)calloc(8, sizeof(char *));                                   \
                pb_slice ns = f.bytes;                                                          \
                pb_field g2 = {0};                                                                    \
                while (pb_next(&ns, &g2)) {                                                     \
                    if (g2.field == 1) nd->in[nd->nin++] = pb_str(g2.bytes);                    \
                    else if (g2.field == 2) nd->out[nd->nout++] = pb_str(g2.bytes);             \
                    else if (g2.field == 4) nd->op = pb_str(g2.bytes);                          \
                    else if (g2.field == 5 && nd->nattr < 16) nd->attrs[nd->nattr++] = g2.bytes; \
                }                                                                               \
            } else if (f.field == 5) {                                                          \
                raw_tensor rt;                                                                  \
                parse_tensor(f.bytes, &rt);                                                     \
                tensor_##SUF *t = push_##SUF(n, rt.name);                                        \
                t->ndim = rt.ndim;                                                              \
                memcpy(t->dims, rt.dims, sizeof(t->dims));                                      \
                t->n = numel_##SUF(rt.dims, rt.ndim);                                           \
                if (rt.dtype == 1) {                                                            \
                    t->f = (REALT *)calloc(t->n ? t->n : 1, sizeof(REALT));                     \
                    for (size_t i = 0; i < t->n; i++) {                                         \
                        float v;                                                                \
                        if (rt.raw.p) memcpy(&v, rt.raw.p + 4 * i, 4);                          \
                        else memcpy(&v, rt.floats.p + 4 * i, 4);                                \
                        t->f[i] = (REALT)v;                                                     \
                    }                                                                           \
                } else if (rt.dtype == 7) {                                                     \
                    t->i64 = (int64_t *)calloc(t->n ? t->n : 1, sizeof(int64_t));               \
                    if (rt.raw.p) memcpy(t->i64, rt.raw.p, 8 * t->n);                           \
                    else {                                                                      \
                        const uint8_t *p = rt.ints.p, *end = p + rt.ints.n;                     \
                        uint64_t v;                                                             \
                        size_t k = 0;                                                           \
                        while (p < end && k < t->n && pb_varint(&p, end, &v))                   \
                            t->i64[k++] = (int64_t)v;                                           \
                    }                                                                           \
                } else if (rt.dtype == 10) { /* FLOAT16: raw bytes or one varint per value */  \
                    t->f = (REALT *)calloc(t->n ? t->n : 1, sizeof(REALT));                     \
                    if (rt.raw.p) {                                                             \
                        if (rt.raw.n != 2 * t->n) {                                             \
                            snprintf(g_err, sizeof(g_err), "fp16 raw_data size mismatch");      \
                            return NULL;                                                        \
                        }                                                                       \
                        for (size_t i = 0; i < t->n; i++) {                                     \
                            uint16_t h;                                                         \
                            memcpy(&h, rt.raw.p + 2 * i, 2);                                    \
                            t->f[i] = (REALT)half_to_double(h);                                 \
                        }                                                                       \
                    } else {                                                                    \
                        const uint8_t *p = rt.i32s.p, *end = p + rt.i32s.n;                     \
                        uint64_t v;                                                             \
                        size_t k = 0;                                                           \
                        while (p < end && k < t->n && pb_varint(&p, end, &v))                   \
                            t->f[k++] = (REALT)half_to_double((uint16_t)v);                     \
                        if (k != t->n) {                                                        \
                            snprintf(g_err, sizeof(g_err), "fp16 int32_data size mismatch");    \
                            return NULL;                                                        \
                        }                                                                       \
                    }                                                                           \
                }                                                                               \
                free(rt.name);                                                                  \
            } else if (f.field == 11 && !n->input_name) {                                       \
                pb_slice vi = f.bytes;                                                          \
                pb_field g2 = {0};                                                                    \
                while (pb_next(&vi, &g2)) {                                                     \
                    if (g2.field == 1) n->input_name = pb_str(g2.bytes);                        \
                    else if (g2.field == 2) { /* TypeProto.tensor_type.shape.dim */             \
                        pb_slice tp = g2.bytes;                                                 \
                        pb_field g3 = {0};                                                            \
                        while (pb_next(&tp, &g3)) {                                             \
                            if (g3.field != 1) continue;                                        \
                            pb_slice tt = g3.bytes;                                             \
                            pb_field g4 = {0};                                                        \
                            while (pb_next(&tt, &g4)) {                                         \
                                if (g4.field != 2) continue;                                    \
                                pb_slice sh = g4.bytes;                                         \
                                pb_field g5 = {0};                                                    \
                                int d = 0;                                                      \
                                while (pb_next(&sh, &g5)) {                                     \
                                    pb_slice dm = g5.bytes;                                     \
                                    pb_field g6 = {0};                                                \
                                    while (pb_next(&dm, &g6))                                   \
                                        if (g6.field == 1 && d < 4)                             \
                                            n->input_dims[d] = (int64_t)g6.v;                   \
                                    d++;                                                        \
                                }                                                               \
                            }                                                                   \
                        }                                                                       \
                    }                                                                           \
                }                                                                               \
            } else if (f.field == 12 && n->noutputs < 8) {                                      \
                pb_slice vi = f.bytes;                                                          \
                pb_field g2 = {0};                                                                    \
                while (pb_next(&vi, &g2))                                                       \
                    if (g2.field == 1) n->outputs[n->noutputs++] = pb_str(g2.bytes);            \
            }                                                                                   \
        }                                                                                       \
        n->input_dims[0] = 1;                                                                   \
        n->nstatic = n->nvals;                                                                  \
        return n;                                                                               \
    }

LOAD_IMPL(f64, double)
LOAD_IMPL(f32, float)

zo_net *zo_net_load(const uint8_t *bytes, size_t len, int f64) {
    zo_net *n = (zo_net *)calloc(1, sizeof(zo_net));
    n->f64 = f64;
    if (f64) n->d = load_f64(bytes, len);
    else n->s = load_f32(bytes, len);
    if (!n->d && !n->s) {
        free(n);
        return NULL;
    }
    return n;
}

void zo_net_free(zo_net *n) {
    if (!n) return;
    /* process-lifetime test helper: leak the graph rather than track every string */
    free(n);
}

size_t zo_net_num_outputs(const zo_net *n) { return n->f64 ? n->d->noutputs : n->s->noutputs; }

size_t zo_net_output_shape(const zo_net *n, size_t idx, int64_t *shape) {
    if (n->f64) {
        tensor_f64 *t = find_f64(n->d, n->d->outputs[idx]);
        if (!t) return 0;
        memcpy(shape, t->dims, sizeof(int64_t) * t->ndim);
        return (size_t)t->ndim;
    }
    tensor_f32 *t = find_f32(n->s, n->s->outputs[idx]);
    if (!t) return 0;
    memcpy(shape, t->dims, sizeof(int64_t) * t->ndim);
    return (size_t)t->ndim;
}

int zo_net_run(zo_net *n, const float *input, float *const *outputs) {
    if (n->f64) {
        if (run_f64(n->d, input)) return -1;
        for (size_t o = 0; o < n->d->noutputs; o++) {
            tensor_f64 *t = find_f64(n->d, n->d->outputs[o]);
            if (!t) return -1;
            if (outputs[o])
                for (size_t i = 0; i < t->n; i++) outputs[o][i] = (float)t->f[i];
        }
        return 0;
    }
    if (run_f32(n->s, input)) return -1;
    for (size_t o = 0; o < n->s->noutputs; o++) {
        tensor_f32 *t = find_f32(n->s, n->s->outputs[o]);
        if (!t) return -1;
        if (outputs[o]) memcpy(outputs[o], t->f, sizeof(float) * t->n);
    }
    return 0;
}

/* f64 variant that keeps full precision for the golden generator */
int zo_net_run_f64out(zo_net *n, const float *input, double *const *outputs) {
    if (!n->f64 || run_f64(n->d, input)) return -1;
    for (size_t o = 0; o < n->d->noutputs; o++) {
        tensor_f64 *t = find_f64(n->d, n->d->outputs[o]);
        if (!t) return -1;
        if (outputs[o]) memcpy(outputs[o], t->f, sizeof(double) * t->n);
    }
    return 0;
}

/* Debug/bisection helper: any tensor of the last run of an f64 net by name (copies at most
 * `cap` values; returns the element count, 0 when absent) and its shape. */
size_t zo_net_tensor(const zo_net *n, const char *name, double *out, size_t cap, int64_t *shape,
                     size_t *rank) {
    if (!n->f64) return 0;
    tensor_f64 *t = find_f64(n->d, name);
    if (!t || !t->f) return 0;
    if (out) memcpy(out, t->f, sizeof(double) * (t->n < cap ? t->n : cap));
    if (shape) memcpy(shape, t->dims, sizeof(int64_t) * t->ndim);
    if (rank) *rank = (size_t)t->ndim;
    return t->n;
}
