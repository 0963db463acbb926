/* ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
 *
 * Plain-C restatement of the reference renderer's hot path.  Every function
 * cites the reference file:line it follows (reference = /root/reference, the
 * lutfullaherkaya/raytracer-ceng477-graphics-hw-1 tree).  Floating-point
 * expressions keep the reference's exact association, precision (float, with
 * the three double-precision islands) and std::min/std::max select semantics;
 * compile with -ffp-contract=off (the reference's x86-64 SSE2 build has no FMA).
 *
 * Parity status: pinned bit-exact against the compiled reference
 * (oracle/_ref/ref_harness) through tests/golden/ (see tests/test_oracle.py).
 */
#define _GNU_SOURCE
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Vec3f (parser.h:18-105)                                                    */
/* ------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;

static inline v3 v_add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }  /* :22 */
static inline v3 v_sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }  /* :34 */
static inline v3 v_mul(v3 a, float f) { v3 r = {a.x * f, a.y * f, a.z * f}; return r; }     /* :26 */
static inline v3 v_div(v3 a, float f) { v3 r = {a.x / f, a.y / f, a.z / f}; return r; }     /* :68 */
static inline v3 v_neg(v3 a) { v3 r = {-a.x, -a.y, -a.z}; return r; }                       /* :38 */
static inline float v_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }         /* :30 */
static inline v3 v_had(v3 a, v3 b) { v3 r = {a.x * b.x, a.y * b.y, a.z * b.z}; return r; }  /* :46 dotWithoutSum */
static inline v3 v_cross(v3 a, v3 b) {                                                        /* :42 */
    v3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static inline float v_len(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }       /* :77-79 */
static inline v3 v_norm(v3 a) { float l = v_len(a); v3 r = {a.x / l, a.y / l, a.z / l}; return r; } /* :72-75 */
static inline float v_get(v3 a, int i) { return i == 1 ? a.y : (i == 2 ? a.z : a.x); }     /* :55-66 */
static inline void v_set(v3* a, int i, float f) { if (i == 1) a->y = f; else if (i == 2) a->z = f; else a->x = f; }

/* std::min / std::max as libstdc++ defines them: (b < a) ? b : a, (a < b) ? b : a */
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }

static inline v3 v_clamp(v3 a, float lo, float hi) {                                        /* parser.h:81-86 */
    v3 r = {smax(lo, smin(a.x, hi)), smax(lo, smin(a.y, hi)), smax(lo, smin(a.z, hi))};
    return r;
}
static inline float clamp_float(float x, float lo, float hi) { return smax(lo, smin(hi, x)); } /* raytracer.cpp:21-23 */

static inline void to_pixel(v3 c, uint8_t* px) {                                            /* parser.h:88-93 */
    v3 k = v_clamp(c, 0.0f, 255.0f);
    px[0] = (uint8_t)roundf(k.x);
    px[1] = (uint8_t)roundf(k.y);
    px[2] = (uint8_t)roundf(k.z);
}

/* ------------------------------------------------------------------------- */
/* Scene model (parser.h:170-323)                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 position, gaze, up;
    float near_plane[4];
    float near_distance;
    int width, height;
    char name[256];
} ro_camera;

typedef struct { v3 position, intensity; } ro_light;
typedef struct { int is_mirror; v3 ambient, diffuse, specular, mirror; float phong; } ro_material;
typedef struct { int material_id; int v0, v1, v2; v3 normal, center; } ro_tri;
typedef struct { int material_id; int center_id; float radius; } ro_sphere;

typedef struct {
    v3 bmin, bmax;
    int axis;
    int right;       /* rightIndex (bvh.h:42)                            */
    int leaf;        /* isLeaf() (bvh.h:107-109)                          */
    int tri_begin, tri_count;   /* into leaf_tris (leaf triangle copies, bvh.h:43) */
    int sph_begin, sph_count;   /* into leaf_sph                               */
} ro_node;

struct ro_scene {
    int bg[3];
    float eps;
    int max_depth;
    int ncam; ro_camera* cams;
    v3 ambient;
    int nlights; ro_light* lights;
    int nmat; ro_material* mats;
    int nvert; v3* verts;
    int ntri; ro_tri* tris;       /* scene.triangles then mesh faces (raytracer.cpp:336-341) */
    int nsph; ro_sphere* sph;
    int nnodes; ro_node* nodes;
    int* leaf_tris; int n_leaf_tris;
    int* leaf_sph; int n_leaf_sph;
};

/* ------------------------------------------------------------------------- */
/* Minimal XML reader: element tree with first text segment + raw attributes. */
/* Replaces tinyxml2 (no arithmetic on the path); numbers are then parsed with */
/* strtof / strtol, i.e. the semantics of std::istream >> float / int.        */
/* ------------------------------------------------------------------------- */
typedef struct {
    const char* name; int name_len;
    const char* attrs; int attrs_len;
    const char* text; int text_len;
    int parent, first_child, last_child, next;
} xnode;

typedef struct { xnode* n; int count, cap; } xdoc;

static int x_add(xdoc* d) {
    if (d->count == d->cap) {
        d->cap = d->cap ? d->cap * 2 : 256;
        d->n = (xnode*)realloc(d->n, sizeof(xnode) * d->cap);
    }
    memset(&d->n[d->count], 0, sizeof(xnode));
    d->n[d->count].parent = d->n[d->count].first_child = d->n[d->count].last_child = d->n[d->count].next = -1;
    return d->count++;
}

static int x_parse(xdoc* d, const char* s, size_t len) {
    const char* p = s; const char* e = s + len;
    int root = x_add(d); /* document node */
    int cur = root;
    while (p < e) {
        if (*p == '<') {
            if (p + 4 <= e && !strncmp(p, "<!--", 4)) {
                const char* q = strstr(p + 4, "-->"); if (!q) return -1; p = q + 3; continue;
            }
            if (p[1] == '?' || p[1] == '!') { const char* q = memchr(p, '>', e - p); if (!q) return -1; p = q + 1; continue; }
            if (p[1] == '/') {  /* closing tag */
                const char* q = memchr(p, '>', e - p); if (!q) return -1;
                cur = d->n[cur].parent; if (cur < 0) return -1;
                p = q + 1; continue;
            }
            const char* q = p + 1;
            while (q < e && *q != ' ' && *q != '\t' && *q != '\n' && *q != '\r' && *q != '>' && *q != '/') q++;
            int id = x_add(d);
            xnode* nd = &d->n[id];
            nd->name = p + 1; nd->name_len = (int)(q - p - 1);
            const char* a = q;
            while (q < e && *q != '>') { if (*q == '"') { q = memchr(q + 1, '"', e - q - 1); if (!q) return -1; } q++; }
            if (q >= e) return -1;
            int selfclose = (q[-1] == '/');
            nd->attrs = a; nd->attrs_len = (int)(q - a);
            nd->parent = cur;
            if (d->n[cur].last_child >= 0) d->n[d->n[cur].last_child].next = id; else d->n[cur].first_child = id;
            d->n[cur].last_child = id;
            if (!selfclose) cur = id;
            p = q + 1;
        } else {
            const char* q = memchr(p, '<', e - p); if (!q) q = e;
            if (cur >= 0 && !d->n[cur].text && d->n[cur].first_child < 0) { d->n[cur].text = p; d->n[cur].text_len = (int)(q - p); }
            p = q;
        }
    }
    return 0;
}

static int x_child(const xdoc* d, int parent, const char* name) {
    if (parent < 0) return -1;
    size_t L = strlen(name);
    for (int c = d->n[parent].first_child; c >= 0; c = d->n[c].next)
        if ((size_t)d->n[c].name_len == L && !strncmp(d->n[c].name, name, L)) return c;
    return -1;
}
static int x_next(const xdoc* d, int node, const char* name) {
    size_t L = strlen(name);
    for (int c = d->n[node].next; c >= 0; c = d->n[c].next)
        if ((size_t)d->n[c].name_len == L && !strncmp(d->n[c].name, name, L)) return c;
    return -1;
}

/* token cursor over an element's text */
typedef struct { char* buf; char* p; } tcur;
static tcur t_open(const xdoc* d, int node) {
    tcur t; int L = node >= 0 ? d->n[node].text_len : 0;
    t.buf = (char*)malloc(L + 1);
    if (L) memcpy(t.buf, d->n[node].text, L);
    t.buf[L] = 0; t.p = t.buf; return t;
}
static int t_float(tcur* t, float* f) { char* e; float v = strtof(t->p, &e); if (e == t->p) return 0; *f = v; t->p = e; return 1; }
static int t_int(tcur* t, int* i) { char* e; long v = strtol(t->p, &e, 10); if (e == t->p) return 0; *i = (int)v; t->p = e; return 1; }
static int t_word(tcur* t, char* out, int n) {
    while (*t->p == ' ' || *t->p == '\t' || *t->p == '\n' || *t->p == '\r') t->p++;
    int k = 0; while (*t->p && *t->p != ' ' && *t->p != '\t' && *t->p != '\n' && *t->p != '\r') { if (k < n - 1) out[k++] = *t->p; t->p++; }
    out[k] = 0; return k > 0;
}
static void t_close(tcur* t) { free(t->buf); }
static int t_v3(tcur* t, v3* v) { return t_float(t, &v->x) && t_float(t, &v->y) && t_float(t, &v->z); }

/* ------------------------------------------------------------------------- */
/* Bounding boxes and BVH build: bvh.h:48-163, parser.h:227-235, 272-317      */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 bmin, bmax; int axis;
    int left, right;            /* temp-tree children, -1 = nullptr */
    int* tris; int ntris;       /* leaf copies in stored order       */
    int* sph; int nsph;
} tnode;

typedef struct { tnode* n; int count, cap; } ttree;

static int tt_add(ttree* t) {
    if (t->count == t->cap) { t->cap = t->cap ? t->cap * 2 : 1024; t->n = (tnode*)realloc(t->n, sizeof(tnode) * t->cap); }
    memset(&t->n[t->count], 0, sizeof(tnode)); t->n[t->count].left = t->n[t->count].right = -1;
    return t->count++;
}

/* Scene::getBoundingBox + extendBoundingBox (parser.h:272-317) */
static void bbox(const ro_scene* s, const int* tris, int nt, const int* sph, int ns, v3* mn, v3* mx) {
    v3 a = {FLT_MAX, FLT_MAX, FLT_MAX}, b = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = 0; i < nt; ++i) {
        const ro_tri* tr = &s->tris[tris[i]];
        int ids[3] = {tr->v0, tr->v1, tr->v2};
        for (int k = 0; k < 3; ++k) {
            v3 v = s->verts[ids[k] - 1];
            if (v.x < a.x) a.x = v.x;
            if (v.y < a.y) a.y = v.y;
            if (v.z < a.z) a.z = v.z;
            if (v.x > b.x) b.x = v.x;
            if (v.y > b.y) b.y = v.y;
            if (v.z > b.z) b.z = v.z;
        }
    }
    for (int i = 0; i < ns; ++i) {
        const ro_sphere* sp = &s->sph[sph[i]];
        v3 c = s->verts[sp->center_id - 1];
        for (int ax = 0; ax < 3; ++ax) {
            if (v_get(c, ax) - sp->radius < v_get(a, ax)) v_set(&a, ax, v_get(c, ax) - sp->radius);
            if (v_get(c, ax) + sp->radius > v_get(b, ax)) v_set(&b, ax, v_get(c, ax) + sp->radius);
        }
    }
    *mn = a; *mx = b;
}

static int widest_axis(v3 mn, v3 mx) {  /* Box::getWidestAxis parser.h:227-235 */
    int w = 0;
    for (int ax = 1; ax < 3; ++ax)
        if (v_get(mx, ax) - v_get(mn, ax) > v_get(mx, w) - v_get(mn, w)) w = ax;
    return w;
}

#define RO_MAX_DEPTH 19 /* bvh.h:18 */

/* BVHNode::build (bvh.h:48-79) with BVHNode::partition (bvh.h:111-163) inlined. */
static int build_rec(const ro_scene* s, ttree* t, int* tris, int nt, int* sph, int ns, int depth) {
    if (nt == 0 && ns == 0) { free(tris); free(sph); return -1; }
    int id = tt_add(t);
    v3 mn, mx; bbox(s, tris, nt, sph, ns, &mn, &mx);
    t->n[id].bmin = mn; t->n[id].bmax = mx;
    if (nt + ns <= 1 || depth >= RO_MAX_DEPTH) {
        t->n[id].tris = tris; t->n[id].ntris = nt; t->n[id].sph = sph; t->n[id].nsph = ns;
        return id;
    }
    int axis = widest_axis(mn, mx);
    t->n[id].axis = axis;
    /* partition (bvh.h:111-163) */
    float start = v_get(mn, axis), end = v_get(mx, axis);
    float mid = (start + end) / 2;
    int tries = 19, lc = 0, rc = 0;
    int *lt = NULL, *rt = NULL, *ls = NULL, *rs = NULL; int nlt = 0, nrt = 0, nls = 0, nrs = 0;
    while (tries-- && (lc == 0 || rc == 0)) {
        lc = rc = 0;
        for (int i = 0; i < nt; ++i) { if (v_get(s->tris[tris[i]].center, axis) < mid) lc++; else rc++; }
        for (int i = 0; i < ns; ++i) { if (v_get(s->verts[s->sph[sph[i]].center_id - 1], axis) < mid) lc++; else rc++; }
        if (lc == 0) { start = mid; mid = (start + end) / 2; }
        else if (rc == 0) { end = mid; mid = (start + end) / 2; }
        else {
            lt = (int*)malloc(sizeof(int) * (nt + 1)); rt = (int*)malloc(sizeof(int) * (nt + 1));
            ls = (int*)malloc(sizeof(int) * (ns + 1)); rs = (int*)malloc(sizeof(int) * (ns + 1));
            for (int i = 0; i < nt; ++i) { if (v_get(s->tris[tris[i]].center, axis) < mid) lt[nlt++] = tris[i]; else rt[nrt++] = tris[i]; }
            for (int i = 0; i < ns; ++i) { if (v_get(s->verts[s->sph[sph[i]].center_id - 1], axis) < mid) ls[nls++] = sph[i]; else rs[nrs++] = sph[i]; }
        }
    }
    if ((nlt == 0 && nls == 0) || (nrt == 0 && nrs == 0)) {
        free(lt); free(rt); free(ls); free(rs);
        t->n[id].tris = tris; t->n[id].ntris = nt; t->n[id].sph = sph; t->n[id].nsph = ns;
        return id;
    }
    free(tris); free(sph);
    int r = build_rec(s, t, rt, nrt, rs, nrs, depth + 1);   /* right first, as bvh.h:69-70 */
    int l = build_rec(s, t, lt, nlt, ls, nls, depth + 1);
    t->n[id].right = r; t->n[id].left = l;
    return id;
}

/* BVHNode::vectorize (bvh.h:81-105): pre-order, left child at index + 1. */
static int flatten(ro_scene* s, const ttree* t, int tn, int* next) {
    int idx = (*next)++;
    const tnode* n = &t->n[tn];
    ro_node* o = &s->nodes[idx];
    o->bmin = n->bmin; o->bmax = n->bmax; o->axis = n->axis;
    o->leaf = (n->left < 0 && n->right < 0);
    o->right = 0;
    o->tri_begin = s->n_leaf_tris; o->tri_count = o->leaf ? n->ntris : 0;
    o->sph_begin = s->n_leaf_sph; o->sph_count = o->leaf ? n->nsph : 0;
    if (o->leaf) {
        for (int i = 0; i < n->ntris; ++i) s->leaf_tris[s->n_leaf_tris++] = n->tris[i];
        for (int i = 0; i < n->nsph; ++i) s->leaf_sph[s->n_leaf_sph++] = n->sph[i];
    }
    if (n->left >= 0) flatten(s, t, n->left, next);
    if (n->right >= 0) { int r = flatten(s, t, n->right, next); s->nodes[idx].right = r; }
    return idx;
}

static void build_bvh(ro_scene* s) {
    ttree t = {0};
    int* tris = (int*)malloc(sizeof(int) * (s->ntri + 1));
    int* sph = (int*)malloc(sizeof(int) * (s->nsph + 1));
    for (int i = 0; i < s->ntri; ++i) tris[i] = i;
    for (int i = 0; i < s->nsph; ++i) sph[i] = i;
    int root = build_rec(s, &t, tris, s->ntri, sph, s->nsph, 0);
    s->nnodes = t.count;
    s->nodes = (ro_node*)calloc(t.count + 1, sizeof(ro_node));
    s->leaf_tris = (int*)malloc(sizeof(int) * (s->ntri + 1));
    s->leaf_sph = (int*)malloc(sizeof(int) * (s->nsph + 1));
    s->n_leaf_tris = s->n_leaf_sph = 0;
    if (root >= 0) { int next = 0; flatten(s, &t, root, &next); }
    for (int i = 0; i < t.count; ++i) { free(t.n[i].tris); free(t.n[i].sph); }
    free(t.n);
}

/* ------------------------------------------------------------------------- */
/* Scene::loadFromXml (parser.cpp:6-218) + RayTracer ctor (raytracer.cpp:335-350) */
/* ------------------------------------------------------------------------- */
ro_scene* ro_load(const char* path, char* err, int errlen) {
    FILE* f = fopen(path, "rb");
    if (!f) { snprintf(err, errlen, "Error: The xml file cannot be loaded."); return NULL; }
    fseek(f, 0, SEEK_END); long L = ftell(f); fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc(L + 1);
    if (fread(buf, 1, L, f) != (size_t)L) { fclose(f); free(buf); snprintf(err, errlen, "read failed"); return NULL; }
    buf[L] = 0; fclose(f);
    xdoc d = {0};
    if (x_parse(&d, buf, L) != 0) { free(buf); free(d.n); snprintf(err, errlen, "Error: The xml file cannot be loaded."); return NULL; }
    int root = d.n[0].first_child;
    if (root < 0) { free(buf); free(d.n); snprintf(err, errlen, "Error: Root is not found."); return NULL; }
    ro_scene* s = (ro_scene*)calloc(1, sizeof(ro_scene));
    tcur t; int e;
    /* :24-33 */ e = x_child(&d, root, "BackgroundColor");
    if (e >= 0) { t = t_open(&d, e); t_int(&t, &s->bg[0]); t_int(&t, &s->bg[1]); t_int(&t, &s->bg[2]); t_close(&t); }
    /* :36-45 */ s->eps = 0.001f; e = x_child(&d, root, "ShadowRayEpsilon");
    if (e >= 0) { t = t_open(&d, e); t_float(&t, &s->eps); t_close(&t); }
    /* :48-57 */ s->max_depth = 0; e = x_child(&d, root, "MaxRecursionDepth");
    if (e >= 0) { t = t_open(&d, e); t_int(&t, &s->max_depth); t_close(&t); }
    /* :60-90 cameras */
    int cams = x_child(&d, root, "Cameras");
    for (int c = x_child(&d, cams, "Camera"); c >= 0; c = x_next(&d, c, "Camera")) {
        s->cams = (ro_camera*)realloc(s->cams, sizeof(ro_camera) * (s->ncam + 1));
        ro_camera* cm = &s->cams[s->ncam++];
        memset(cm, 0, sizeof(*cm));
        t = t_open(&d, x_child(&d, c, "Position")); t_v3(&t, &cm->position); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Gaze")); t_v3(&t, &cm->gaze); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Up")); t_v3(&t, &cm->up); t_close(&t);
        t = t_open(&d, x_child(&d, c, "NearPlane"));
        for (int k = 0; k < 4; ++k) t_float(&t, &cm->near_plane[k]);
        t_close(&t);
        t = t_open(&d, x_child(&d, c, "NearDistance")); t_float(&t, &cm->near_distance); t_close(&t);
        t = t_open(&d, x_child(&d, c, "ImageResolution")); t_int(&t, &cm->width); t_int(&t, &cm->height); t_close(&t);
        t = t_open(&d, x_child(&d, c, "ImageName")); t_word(&t, cm->name, sizeof(cm->name)); t_close(&t);
    }
    /* :93-111 lights */
    int lights = x_child(&d, root, "Lights");
    t = t_open(&d, x_child(&d, lights, "AmbientLight")); t_v3(&t, &s->ambient); t_close(&t);
    for (int c = x_child(&d, lights, "PointLight"); c >= 0; c = x_next(&d, c, "PointLight")) {
        s->lights = (ro_light*)realloc(s->lights, sizeof(ro_light) * (s->nlights + 1));
        ro_light* l = &s->lights[s->nlights++];
        t = t_open(&d, x_child(&d, c, "Position")); t_v3(&t, &l->position); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Intensity")); t_v3(&t, &l->intensity); t_close(&t);
    }
    /* :114-140 materials */
    int mats = x_child(&d, root, "Materials");
    for (int c = x_child(&d, mats, "Material"); c >= 0; c = x_next(&d, c, "Material")) {
        s->mats = (ro_material*)realloc(s->mats, sizeof(ro_material) * (s->nmat + 1));
        ro_material* m = &s->mats[s->nmat++];
        memset(m, 0, sizeof(*m));
        /* Attribute("type", "mirror") (parser.cpp:119) */
        char ab[512]; int al = d.n[c].attrs_len < 511 ? d.n[c].attrs_len : 511;
        memcpy(ab, d.n[c].attrs, al); ab[al] = 0;
        m->is_mirror = strstr(ab, "type=\"mirror\"") != NULL;
        t = t_open(&d, x_child(&d, c, "AmbientReflectance")); t_v3(&t, &m->ambient); t_close(&t);
        t = t_open(&d, x_child(&d, c, "DiffuseReflectance")); t_v3(&t, &m->diffuse); t_close(&t);
        t = t_open(&d, x_child(&d, c, "SpecularReflectance")); t_v3(&t, &m->specular); t_close(&t);
        t = t_open(&d, x_child(&d, c, "MirrorReflectance")); t_v3(&t, &m->mirror); t_close(&t);
        t = t_open(&d, x_child(&d, c, "PhongExponent")); t_float(&t, &m->phong); t_close(&t);
    }
    /* :143-151 vertices */
    t = t_open(&d, x_child(&d, root, "VertexData"));
    { int cap = 0; v3 v;
      while (t_v3(&t, &v)) {
          if (s->nvert == cap) { cap = cap ? cap * 2 : 1024; s->verts = (v3*)realloc(s->verts, sizeof(v3) * cap); }
          s->verts[s->nvert++] = v;
      } }
    t_close(&t);
    /* :154-195 meshes and triangles; flattening order of raytracer.cpp:336-341:
       standalone <Triangle>s first, then every mesh's faces in file order. */
    int objs = x_child(&d, root, "Objects");
    int tcap = 0;
#define PUSH_TRI(mat, a, b, c_) do { \
        if (s->ntri == tcap) { tcap = tcap ? tcap * 2 : 1024; s->tris = (ro_tri*)realloc(s->tris, sizeof(ro_tri) * tcap); } \
        ro_tri* tr_ = &s->tris[s->ntri++]; memset(tr_, 0, sizeof(*tr_)); \
        tr_->material_id = (mat); tr_->v0 = (a); tr_->v1 = (b); tr_->v2 = (c_); } while (0)
    for (int c = x_child(&d, objs, "Triangle"); c >= 0; c = x_next(&d, c, "Triangle")) {
        int mat = 0, a = 0, b = 0, cc = 0;
        t = t_open(&d, x_child(&d, c, "Material")); t_int(&t, &mat); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Indices")); t_int(&t, &a); t_int(&t, &b); t_int(&t, &cc); t_close(&t);
        PUSH_TRI(mat, a, b, cc);
    }
    for (int c = x_child(&d, objs, "Mesh"); c >= 0; c = x_next(&d, c, "Mesh")) {
        int mat = 0, a, b, cc;
        t = t_open(&d, x_child(&d, c, "Material")); t_int(&t, &mat); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Faces"));
        while (t_int(&t, &a) && t_int(&t, &b) && t_int(&t, &cc)) PUSH_TRI(mat, a, b, cc);
        t_close(&t);
    }
#undef PUSH_TRI
    /* :198-217 spheres */
    for (int c = x_child(&d, objs, "Sphere"); c >= 0; c = x_next(&d, c, "Sphere")) {
        s->sph = (ro_sphere*)realloc(s->sph, sizeof(ro_sphere) * (s->nsph + 1));
        ro_sphere* sp = &s->sph[s->nsph++];
        t = t_open(&d, x_child(&d, c, "Material")); t_int(&t, &sp->material_id); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Center")); t_int(&t, &sp->center_id); t_close(&t);
        t = t_open(&d, x_child(&d, c, "Radius")); t_float(&t, &sp->radius); t_close(&t);
    }
    free(d.n); free(buf);
    /* raytracer.cpp:342-348: per-triangle normal and centre */
    for (int i = 0; i < s->ntri; ++i) {
        ro_tri* tr = &s->tris[i];
        v3 a = s->verts[tr->v0 - 1], b = s->verts[tr->v1 - 1], c = s->verts[tr->v2 - 1];
        tr->normal = v_norm(v_cross(v_sub(b, a), v_sub(c, a)));
        tr->center = v_div(v_add(v_add(a, b), c), 3);
    }
    build_bvh(s);
    return s;
}

void ro_free(ro_scene* s) {
    if (!s) return;
    free(s->cams); free(s->lights); free(s->mats); free(s->verts); free(s->tris); free(s->sph);
    free(s->nodes); free(s->leaf_tris); free(s->leaf_sph); free(s);
}

int ro_num_cameras(const ro_scene* s) { return s->ncam; }

int ro_camera_info(const ro_scene* s, int cam, int* w, int* h, char* name, int namelen) {
    if (cam < 0 || cam >= s->ncam) return -1;
    if (w) *w = s->cams[cam].width;
    if (h) *h = s->cams[cam].height;
    if (name && namelen > 0) snprintf(name, namelen, "%s", s->cams[cam].name);
    return 0;
}

int ro_bvh_info(const ro_scene* s, int* nodes, int* leaves, int* max_leaf, int* ntris, int* nspheres) {
    int lv = 0, ml = 0;
    for (int i = 0; i < s->nnodes; ++i)
        if (s->nodes[i].leaf) { lv++; int c = s->nodes[i].tri_count + s->nodes[i].sph_count; if (c > ml) ml = c; }
    if (nodes) *nodes = s->nnodes;
    if (leaves) *leaves = lv;
    if (max_leaf) *max_leaf = ml;
    if (ntris) *ntris = s->ntri;
    if (nspheres) *nspheres = s->nsph;
    return 0;
}

int ro_export_nodes(const ro_scene* s, void* out, int capacity) {
    if (out) {
        int n = s->nnodes < capacity ? s->nnodes : capacity;
        for (int i = 0; i < n; ++i) {
            const ro_node* nd = &s->nodes[i];
            float* f = (float*)out + 8 * i;
            int32_t* w = (int32_t*)f;
            f[0] = nd->bmin.x; f[1] = nd->bmin.y; f[2] = nd->bmin.z;
            f[4] = nd->bmax.x; f[5] = nd->bmax.y; f[6] = nd->bmax.z;
            if (nd->leaf) {
                w[3] = nd->tri_begin + nd->sph_begin;  /* slot = tris before + spheres before */
                w[7] = (int32_t)(0x80000000u | ((uint32_t)nd->sph_count << 20) | (uint32_t)nd->tri_count);
            } else {
                w[3] = nd->right;
                w[7] = nd->axis;
            }
        }
    }
    return s->nnodes;
}

/* ------------------------------------------------------------------------- */
/* Ray (raytracer.cpp:47-282)                                                 */
/* ------------------------------------------------------------------------- */
typedef struct { v3 o, d, inv; } ray_t;
typedef struct { float t; v3 n; int mat; int exists; } hit_t;
typedef struct { uint64_t node, tri, sph, node_closest; } work_t;
/* diagnostics: ro_work_map counts closest-hit visits only when set */
int ro_debug_work_closest_only;

/* Ray::Ray (:61-67).  NOTE: the ctor body's `direction = direction.normalize();`
 * assigns to the *parameter* (it shadows the member), so the member direction
 * stays the UN-normalised argument.  Every test, getPoint and the child-order
 * sign therefore use the raw direction; only the explicit .normalize() calls
 * in rayTrace (:413, :414, :431-432) normalise. */
static inline ray_t make_ray(v3 o, v3 dir) {
    ray_t r; r.o = o;
    r.inv.x = 1 / dir.x; r.inv.y = 1 / dir.y; r.inv.z = 1 / dir.z;
    r.d = dir;
    return r;
}

static inline int box_test(const ray_t* r, const ro_node* n, float* tout) {  /* :101-126 */
    float tx1 = (n->bmin.x - r->o.x) * r->inv.x;
    float tx2 = (n->bmax.x - r->o.x) * r->inv.x;
    float tmin = smin(tx1, tx2);
    float tmax = smax(tx1, tx2);
    float ty1 = (n->bmin.y - r->o.y) * r->inv.y;
    float ty2 = (n->bmax.y - r->o.y) * r->inv.y;
    tmin = smax(tmin, smin(ty1, ty2));
    tmax = smin(tmax, smax(ty1, ty2));
    float tz1 = (n->bmin.z - r->o.z) * r->inv.z;
    float tz2 = (n->bmax.z - r->o.z) * r->inv.z;
    tmin = smax(tmin, smin(tz1, tz2));
    tmax = smin(tmax, smax(tz1, tz2));
    if (tmax >= smax(0.0f, tmin)) { *tout = tmin; return 1; }
    *tout = -1; return 0;
}

static inline float det3(float m00, float m01, float m02, float m10, float m11, float m12,
                         float m20, float m21, float m22) {   /* det :15-19 */
    return m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20) + m02 * (m10 * m21 - m11 * m20);
}

static inline int tri_test(const ro_scene* s, const ray_t* r, const ro_tri* tr, float* tout) { /* :129-175 */
    v3 a = s->verts[tr->v0 - 1], b = s->verts[tr->v1 - 1], c = s->verts[tr->v2 - 1];
    v3 o = r->o, d = r->d;
    float detA = det3(a.x - b.x, a.x - c.x, d.x, a.y - b.y, a.y - c.y, d.y, a.z - b.z, a.z - c.z, d.z);
    float beta = det3(a.x - o.x, a.x - c.x, d.x, a.y - o.y, a.y - c.y, d.y, a.z - o.z, a.z - c.z, d.z) / detA;
    float gamma = det3(a.x - b.x, a.x - o.x, d.x, a.y - b.y, a.y - o.y, d.y, a.z - b.z, a.z - o.z, d.z) / detA;
    float t = det3(a.x - b.x, a.x - c.x, a.x - o.x, a.y - b.y, a.y - c.y, a.y - o.y, a.z - b.z, a.z - c.z, a.z - o.z) / detA;
    float alpha = 1 - beta - gamma;
    if (alpha >= 0 && beta >= 0 && gamma >= 0 && t >= 0) { *tout = t; return 1; }
    return 0;
}

static inline int sphere_test(const ro_scene* s, const ray_t* r, const ro_sphere* sp, float* tout, v3* nout) { /* :70-96 */
    v3 c = s->verts[sp->center_id - 1];
    float rad = sp->radius;
    v3 d = r->d, o = r->o;
    v3 oc = v_sub(o, c);
    float B = 2 * v_dot(d, oc);
    float A = v_dot(d, d);
    float C = v_dot(oc, oc) - rad * rad;
    float disc = B * B - 4 * A * C;
    if (disc >= 0) {
        float t1 = (float)(((double)(-B) - sqrt((double)disc)) / (double)(2 * A));
        float t2 = (float)(((double)(-B) + sqrt((double)disc)) / (double)(2 * A));
        if (t1 < 0 && t2 < 0) return 0;
        *tout = t1;
        v3 p = v_add(o, v_mul(d, t1));             /* getPoint :49-51 */
        *nout = v_norm(v_div(v_sub(p, c), rad));
        return 1;
    }
    return 0;
}

#define RO_STACK 64

/* diagnostics: per-node visit histogram [0]=closest-hit [1]=any-hit (NULL = off) */
uint64_t* ro_debug_node_hist[2];
/* diagnostics (single-threaded callers only): mark visited nodes in a byte map */
static uint8_t* g_visit_mark;
#define NOTE_NODE(k, ni) do { if (ro_debug_node_hist[k]) __atomic_fetch_add(&ro_debug_node_hist[k][ni], 1, __ATOMIC_RELAXED); if (g_visit_mark) g_visit_mark[ni] = 1; } while (0)

/* Ray::getFirstIntersection (:177-225) */
static hit_t closest_hit(const ro_scene* s, const ray_t* r, work_t* w) {
    hit_t best; best.t = -1; best.exists = 0; best.mat = -1; best.n.x = best.n.y = best.n.z = -1;
    int stack[RO_STACK]; int sp = 0;
    if (s->nnodes > 0) stack[sp++] = 0;
    float tMax = FLT_MAX;
    while (sp > 0) {
        int ni = stack[--sp];
        const ro_node* n = &s->nodes[ni];
        float bt; int ex = box_test(r, n, &bt);
        w->node++; w->node_closest++; NOTE_NODE(0, ni);
        if (ex && bt <= tMax) {
            if (!n->leaf) {
                if (v_get(r->d, n->axis) > 0) { stack[sp++] = n->right; stack[sp++] = ni + 1; }
                else { stack[sp++] = ni + 1; stack[sp++] = n->right; }
            } else {
                for (int i = 0; i < n->tri_count; ++i) {
                    const ro_tri* tr = &s->tris[s->leaf_tris[n->tri_begin + i]];
                    float t; w->tri++;
                    if (tri_test(s, r, tr, &t)) {
                        if (t < best.t || best.t == -1) {
                            best.t = t; best.n = tr->normal; best.mat = tr->material_id; best.exists = 1;
                            tMax = best.t;
                        }
                    }
                }
                for (int i = 0; i < n->sph_count; ++i) {
                    const ro_sphere* spp = &s->sph[s->leaf_sph[n->sph_begin + i]];
                    float t; v3 nn; w->sph++;
                    if (sphere_test(s, r, spp, &t, &nn)) {
                        if (t < best.t || best.t == -1) {
                            best.t = t; best.n = nn; best.mat = spp->material_id; best.exists = 1;
                            tMax = best.t;
                        }
                    }
                }
            }
        }
    }
    return best;
}

/* Ray::getAnyIntersectionUntilT (:227-253) with traverse (:264-280) */
static int any_hit(const ro_scene* s, const ray_t* r, float tlim, work_t* w) {
    int stack[RO_STACK]; int sp = 0;
    if (s->nnodes > 0) stack[sp++] = 0;
    while (sp > 0) {
        int ni = stack[--sp];
        const ro_node* n = &s->nodes[ni];
        float bt; w->node++; NOTE_NODE(1, ni);
        if (!box_test(r, n, &bt)) continue;
        if (!n->leaf) {
            if (v_get(r->d, n->axis) > 0) { stack[sp++] = n->right; stack[sp++] = ni + 1; }
            else { stack[sp++] = ni + 1; stack[sp++] = n->right; }
            continue;
        }
        for (int i = 0; i < n->tri_count; ++i) {
            float t; w->tri++;
            if (tri_test(s, r, &s->tris[s->leaf_tris[n->tri_begin + i]], &t) && t < tlim) return 1;
        }
        for (int i = 0; i < n->sph_count; ++i) {
            float t; v3 nn; w->sph++;
            if (sphere_test(s, r, &s->sph[s->leaf_sph[n->sph_begin + i]], &t, &nn) && t < tlim) return 1;
        }
    }
    return 0;
}

typedef struct {
    const ro_scene* s;
    int max_depth;
    ro_counters c;
    work_t w;
} ctx_t;

/* RayTracer::rayTrace (:385-452) — recursive, as the reference. */
/* diagnostics: max node visits of a single traversal, [0]=closest [1]=shadow, by depth */
uint32_t ro_debug_maxvisits[2][64];

static void note_visits(int kind, int depth, uint64_t before, uint64_t after) {
    uint32_t v = (uint32_t)(after - before);
    if (depth < 64 && v > ro_debug_maxvisits[kind][depth]) ro_debug_maxvisits[kind][depth] = v; /* racy max: diagnostics only */
}

static v3 ray_trace(ctx_t* x, ray_t* ray, int depth) {
    const ro_scene* s = x->s;
    v3 color = {0, 0, 0};
    if (depth > x->max_depth) return color;                          /* :387-389 */
    if (depth > 0) x->c.reflection_rays++;
    uint64_t nb = x->w.node;
    hit_t h = closest_hit(s, ray, &x->w);                            /* :390 */
    note_visits(0, depth, nb, x->w.node);
    if (!h.exists) {                                                 /* :442-449 */
        if (depth > 0) return color;
        v3 bg = {(float)s->bg[0], (float)s->bg[1], (float)s->bg[2]};
        return bg;
    }
    const ro_material* m = &s->mats[h.mat - 1];
    color = v_add(color, v_had(m->ambient, s->ambient));            /* :394-395 */
    v3 hitp = v_add(ray->o, v_mul(ray->d, h.t));                     /* getPoint */
    v3 p = v_add(hitp, v_mul(h.n, s->eps));                          /* :397 */
    for (int li = 0; li < s->nlights; ++li) {                        /* :399-427 */
        const ro_light* L = &s->lights[li];
        float dist = v_len(v_sub(L->position, p));
        v3 ldir = v_norm(v_sub(L->position, p));
        v3 ldir_real = v_norm(v_sub(L->position, v_add(ray->o, v_mul(ray->d, h.t))));
        ray_t lray = make_ray(p, ldir);
        x->c.shadow_rays++;
        uint64_t sb = x->w.node;
        int occl = any_hit(s, &lray, dist, &x->w);
        note_visits(1, depth, sb, x->w.node);
        if (!occl) {
            float cos_t = v_dot(ldir_real, h.n);
            v3 E = v_div(L->intensity, dist * dist);
            float theta = (float)(acos((double)cos_t) * 180 / 3.1415);
            if ((double)theta <= 90.01) {
                v3 hh = v_norm(v_add(lray.d, v_neg(v_norm(ray->d))));
                float ca = (float)pow((double)smax(0.0f, v_dot(v_norm(h.n), hh)), (double)m->phong);
                color = v_add(color, v_had(v_mul(m->specular, ca), E));
            }
            color = v_add(color, v_had(v_mul(m->diffuse, clamp_float(cos_t, 0, 1)), E));
        }
    }
    if (m->is_mirror) {                                              /* :430-439 */
        ray->d = v_norm(ray->d);
        v3 n = v_norm(h.n);
        float rc = v_dot(v_neg(ray->d), n);
        ray_t rr = make_ray(p, v_add(ray->d, v_mul(v_mul(n, 2), rc)));
        v3 rec = ray_trace(x, &rr, depth + 1);
        color = v_add(color, v_had(rec, m->mirror));
    }
    return v_clamp(color, 0, FLT_MAX);                               /* :451 */
}

/* EyeRayGenerator (:284-325) */
typedef struct { v3 q, u, v, e; float su, sv; } eye_t;

static eye_t eye_init(const ro_camera* cam, int nx, int ny) {         /* :292-314 */
    eye_t g;
    g.e = cam->position;
    v3 w = v_neg(cam->gaze);
    float dist = cam->near_distance;
    float l = cam->near_plane[0], r = cam->near_plane[1], b = cam->near_plane[2], t = cam->near_plane[3];
    g.v = cam->up;
    g.u = v_cross(g.v, w);
    v3 m = v_add(g.e, v_mul(v_neg(w), dist));
    g.q = v_add(v_add(m, v_mul(g.u, l)), v_mul(g.v, t));
    g.su = (r - l) / (float)nx;
    g.sv = (t - b) / (float)ny;
    return g;
}

static ray_t eye_gen(const eye_t* g, int row, int col) {             /* :319-324 */
    float su = (float)((col + 0.5) * (double)g->su);
    float sv = (float)((row + 0.5) * (double)g->sv);
    v3 s = v_sub(v_add(g->q, v_mul(g->u, su)), v_mul(g->v, sv));
    return make_ray(g->e, v_sub(s, g->e));
}

/* ------------------------------------------------------------------------- */
/* Render: thread fan-out (:352-383) + downSample (:459-484)                  */
/* ------------------------------------------------------------------------- */
typedef struct {
    const ro_scene* s; const ro_camera* cam; eye_t eye;
    int aa, W, row_begin, row_end, tid, T, max_depth;
    uint8_t* out;
    uint32_t* work;   /* optional: node visits per output pixel (diagnostics) */
    ro_counters c;
} job_t;

static void* render_worker(void* arg) {
    job_t* j = (job_t*)arg;
    ctx_t x; memset(&x, 0, sizeof(x)); x.s = j->s; x.max_depth = j->max_depth;
    int F = j->aa, W = j->W;
    uint8_t* samp = (uint8_t*)malloc((size_t)F * F * 3);
    for (int orow = j->row_begin + j->tid; orow < j->row_end; orow += j->T) {
        for (int ocol = 0; ocol < W; ++ocol) {
            int sum[3] = {0, 0, 0};
            const uint64_t nodes_before = ro_debug_work_closest_only ? x.w.node_closest : x.w.node;
            for (int k = 0; k < F; ++k)
                for (int l = 0; l < F; ++l) {
                    ray_t r = eye_gen(&j->eye, orow * F + k, ocol * F + l);
                    x.c.primary_rays++;
                    v3 c = ray_trace(&x, &r, 0);
                    uint8_t px[3]; to_pixel(c, px);
                    sum[0] += px[0]; sum[1] += px[1]; sum[2] += px[2];
                }
            uint8_t* o = j->out + ((size_t)(orow - j->row_begin) * W + ocol) * 3;
            o[0] = (uint8_t)(sum[0] / (F * F)); o[1] = (uint8_t)(sum[1] / (F * F)); o[2] = (uint8_t)(sum[2] / (F * F));
            if (j->work) j->work[(size_t)(orow - j->row_begin) * W + ocol] = (uint32_t)((ro_debug_work_closest_only ? x.w.node_closest : x.w.node) - nodes_before);
        }
    }
    free(samp);
    j->c = x.c;
    j->c.node_visits = x.w.node; j->c.tri_tests = x.w.tri; j->c.sphere_tests = x.w.sph;
    return NULL;
}

static int render_impl(const ro_scene* s, int cam, int aa, int threads, int row_begin, int row_end,
                       int max_depth_override, uint8_t* out, ro_counters* counters, uint32_t* work);

int ro_render(const ro_scene* s, int cam, int aa, int threads, int row_begin, int row_end,
              int max_depth_override, uint8_t* out, ro_counters* counters) {
    return render_impl(s, cam, aa, threads, row_begin, row_end, max_depth_override, out, counters, NULL);
}

int ro_work_map(const ro_scene* s, int cam, int aa, int threads, uint8_t* out, uint32_t* work) {
    return render_impl(s, cam, aa, threads, 0, -1, -1000, out, NULL, work);
}

static int render_impl(const ro_scene* s, int cam, int aa, int threads, int row_begin, int row_end,
                       int max_depth_override, uint8_t* out, ro_counters* counters, uint32_t* work) {
    if (!s || cam < 0 || cam >= s->ncam || aa < 1 || !out) return -1;
    const ro_camera* c = &s->cams[cam];
    if (row_begin < 0) row_begin = 0;
    if (row_end < 0 || row_end > c->height) row_end = c->height;
    if (threads < 1) threads = 1;
    eye_t eye = eye_init(c, c->width * aa, c->height * aa);
    job_t* jobs = (job_t*)calloc(threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
    for (int i = 0; i < threads; ++i) {
        job_t* j = &jobs[i];
        j->s = s; j->cam = c; j->eye = eye; j->aa = aa; j->W = c->width;
        j->row_begin = row_begin; j->row_end = row_end; j->tid = i; j->T = threads;
        j->max_depth = max_depth_override < -999 ? s->max_depth : max_depth_override;
        j->out = out;
        j->work = work;
        if (threads == 1) render_worker(j); else pthread_create(&th[i], NULL, render_worker, j);
    }
    ro_counters tot; memset(&tot, 0, sizeof(tot));
    for (int i = 0; i < threads; ++i) {
        if (threads > 1) pthread_join(th[i], NULL);
        tot.primary_rays += jobs[i].c.primary_rays; tot.shadow_rays += jobs[i].c.shadow_rays;
        tot.reflection_rays += jobs[i].c.reflection_rays; tot.node_visits += jobs[i].c.node_visits;
        tot.tri_tests += jobs[i].c.tri_tests; tot.sphere_tests += jobs[i].c.sphere_tests;
    }
    if (counters) *counters = tot;
    free(jobs); free(th);
    return 0;
}

/* Diagnostics: packet coherence of primary rays.  For every 8x8 tile:
 * union of BVH nodes its 64 closest-hit walks visit, the sum and the max of
 * per-ray visits, and whether all rays agree on every interior node's
 * near/far order (sign of d[axis]).  out[0..3] = sums over tiles of union,
 * per-ray sum, per-tile max, tiles with disagreeing signs. */
int ro_debug_tile_mode;
int ro_debug_tile_stats(const ro_scene* s, int cam, double* out) {
    if (!s || cam < 0 || cam >= s->ncam) return -1;
    const ro_camera* c = &s->cams[cam];
    int W = c->width, H = c->height;
    eye_t eye = eye_init(c, W, H);
    work_t w = {0, 0, 0};
    uint8_t* mark = (uint8_t*)calloc((size_t)s->nnodes + 1, 1);
    out[0] = out[1] = out[2] = out[3] = 0;
    for (int ty = 0; ty < H; ty += 8)
        for (int tx = 0; tx < W; tx += 8) {
            memset(mark, 0, (size_t)s->nnodes);
            g_visit_mark = mark;
            double mx = 0; int sgn[3] = {0, 0, 0}; int first = 1, dis = 0;
            for (int y = ty; y < ty + 8 && y < H; ++y)
                for (int x = tx; x < tx + 8 && x < W; ++x) {
                    ray_t r = eye_gen(&eye, y, x);
                    int sg[3] = {r.d.x > 0, r.d.y > 0, r.d.z > 0};
                    if (first) { sgn[0] = sg[0]; sgn[1] = sg[1]; sgn[2] = sg[2]; first = 0; }
                    else if (sg[0] != sgn[0] || sg[1] != sgn[1] || sg[2] != sgn[2]) dis = 1;
                    uint64_t n0 = w.node;
                    hit_t h = closest_hit(s, &r, &w);
                    double v = (double)(w.node - n0);
                    if (ro_debug_tile_mode == 1) {          /* shadow ray to light 0 instead */
                        if (!h.exists || s->nlights < 1) continue;
                        g_visit_mark = NULL;
                        v3 hp = v_add(r.o, v_mul(r.d, h.t));
                        v3 p = v_add(hp, v_mul(h.n, s->eps));
                        v3 lp = s->lights[0].position;
                        float dist = v_len(v_sub(lp, p));
                        ray_t sr = make_ray(p, v_norm(v_sub(lp, p)));
                        g_visit_mark = mark;
                        n0 = w.node;
                        (void)any_hit(s, &sr, dist, &w);
                        v = (double)(w.node - n0);
                    }
                    out[1] += v;
                    if (v > mx) mx = v;
                }
            g_visit_mark = NULL;
            size_t u = 0;
            for (int i = 0; i < s->nnodes; ++i) u += mark[i];
            out[0] += (double)u; out[2] += mx; out[3] += dis;
        }
    free(mark);
    return 0;
}

int ro_primary_hits(const ro_scene* s, int cam, int aa, float* tout, int32_t* mout) {
    if (!s || cam < 0 || cam >= s->ncam || aa < 1) return -1;
    const ro_camera* c = &s->cams[cam];
    int W = c->width * aa, H = c->height * aa;
    eye_t eye = eye_init(c, W, H);
    work_t w = {0, 0, 0};
    for (int row = 0; row < H; ++row)
        for (int col = 0; col < W; ++col) {
            ray_t r = eye_gen(&eye, row, col);
            hit_t h = closest_hit(s, &r, &w);
            if (tout) tout[(size_t)row * W + col] = h.t;
            if (mout) mout[(size_t)row * W + col] = h.exists ? h.mat : 0;
        }
    return 0;
}

/* write_ppm (ppm.cpp:4-39) */
int ro_write_ppm(const char* path, const uint8_t* data, int width, int height) {
    FILE* f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "P3\n%d %d\n255\n", width, height);
    size_t idx = 0;
    for (int j = 0; j < height; ++j) {
        for (int i = 0; i < width; ++i)
            for (int c = 0; c < 3; ++c, ++idx) {
                if (i == width - 1 && c == 2) fprintf(f, "%d", data[idx]);
                else fprintf(f, "%d ", data[idx]);
            }
        fprintf(f, "\n");
    }
    fclose(f);
    return 0;
}
