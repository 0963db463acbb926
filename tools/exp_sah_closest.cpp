// Experiment (CPU, diagnostics only): closest-hit over the SAH occlusion
// hierarchy (spairs: SAH boxes above the reference's leaves) with t-pruning,
// versus the reference's ordered DFS over its own tree (pairs).
//
// For every closest-hit walk of a frame (eye rays + mirror chains) it reports
// box tests of both walks, the per-pixel chain totals (the frame's critical
// path is its heaviest chain), how often the SAH result cannot be certified
// (leaf-entry check, ties across leaves, negative t) and whether any certified
// SAH result differs from the reference walk's result.
//
//   g++ -O2 -std=c++17 -ffp-contract=off -Iinclude -Iraytracer-ceng477-graphics-hw-1_amd/csrc \
//       tools/exp_sah_closest.cpp raytracer-ceng477-graphics-hw-1_amd/csrc/host_scene.cpp -o /tmp/exp_sah
//   /tmp/exp_sah scene.xml [slack_rel]
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <functional>
#include <array>

#include "host_scene.hpp"

using namespace rtx;

namespace {

struct Vf { float x, y, z; };
Vf add(Vf a, Vf b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
Vf sub(Vf a, Vf b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
Vf mul(Vf a, float f) { return {a.x * f, a.y * f, a.z * f}; }
Vf neg(Vf a) { return {-a.x, -a.y, -a.z}; }
float dot(Vf a, Vf b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
float len(Vf a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
Vf nrm(Vf a) { float l = len(a); return {a.x / l, a.y / l, a.z / l}; }
float comp(Vf a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
float smin(float a, float b) { return (b < a) ? b : a; }
float smax(float a, float b) { return (a < b) ? b : a; }

struct Ray { Vf o, d, inv; };
Ray make_ray(Vf o, Vf d) { return {o, d, {1.0f / d.x, 1.0f / d.y, 1.0f / d.z}}; }

bool box_hit(const Ray& r, const float* lo, const float* hi, float* t) {
    float tx1 = (lo[0] - r.o.x) * r.inv.x, tx2 = (hi[0] - r.o.x) * r.inv.x;
    float tmin = smin(tx1, tx2), tmax = smax(tx1, tx2);
    float ty1 = (lo[1] - r.o.y) * r.inv.y, ty2 = (hi[1] - r.o.y) * r.inv.y;
    tmin = smax(tmin, smin(ty1, ty2)); tmax = smin(tmax, smax(ty1, ty2));
    float tz1 = (lo[2] - r.o.z) * r.inv.z, tz2 = (hi[2] - r.o.z) * r.inv.z;
    tmin = smax(tmin, smin(tz1, tz2)); tmax = smin(tmax, smax(tz1, tz2));
    *t = tmin;
    return tmax >= smax(0.0f, tmin);
}
float det3(float m00, float m01, float m02, float m10, float m11, float m12, float m20, float m21, float m22) {
    return m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20) + m02 * (m10 * m21 - m11 * m20);
}
bool tri_hit(const Ray& r, const dl::Prim& p, float* tout) {
    Vf d = r.d;
    float aox = p.p0x - r.o.x, aoy = p.p0y - r.o.y, aoz = p.p0z - r.o.z;
    float detA = det3(p.p1x, p.p2x, d.x, p.p1y, p.p2y, d.y, p.p1z, p.p2z, d.z);
    float beta = det3(aox, p.p2x, d.x, aoy, p.p2y, d.y, aoz, p.p2z, d.z) / detA;
    float gamma = det3(p.p1x, aox, d.x, p.p1y, aoy, d.y, p.p1z, aoz, d.z) / detA;
    float t = det3(p.p1x, p.p2x, aox, p.p1y, p.p2y, aoy, p.p1z, p.p2z, aoz) / detA;
    float alpha = 1.0f - beta - gamma;
    *tout = t;
    return alpha >= 0 && beta >= 0 && gamma >= 0 && t >= 0.0f;
}
bool sphere_hit(const Ray& r, const dl::Prim& p, float* tout) {
    Vf oc{r.o.x - p.p0x, r.o.y - p.p0y, r.o.z - p.p0z};
    float B = 2.0f * dot(r.d, oc), A = dot(r.d, r.d), C = dot(oc, oc) - p.p1y;
    float disc = B * B - 4.0f * A * C;
    if (!(disc >= 0)) return false;
    double sq = sqrt((double)disc), den = (double)(2.0f * A);
    float t1 = (float)(((double)(-B) - sq) / den), t2 = (float)(((double)(-B) + sq) / den);
    *tout = t1;
    return !(t1 < 0 && t2 < 0);
}
bool prim_hit(const Ray& r, const dl::Prim& p, float* t) { return p.id >= 0 ? tri_hit(r, p, t) : sphere_hit(r, p, t); }

const FlatBVH* B;
std::vector<int> leaf_of_prim;            // prim slot -> index into leaf_boxes
std::vector<std::array<float, 6>> leaf_boxes;

void leaf_range(int32_t info, int* a, int* c) {
    int cnt = (info >> dl::kLeafCountShift) & dl::kLeafMaxCount;
    int st = info & dl::kLeafStartMask;
    if (cnt) { *a = st; *c = cnt; } else { *a = B->leaf_big[st].start; *c = B->leaf_big[st].count; }
}

struct Hit { float t; int prim; long visits; };
double g_slack = 0.0;
long g_late = 0;
double g_anom_max = 0; long g_anom_n[4];
long g_rfetch = 0, g_rleaf = 0;

// reference ordered DFS over the child-pair tree (raytracer.cpp:177-225)
Hit closest_ref(const Ray& r) {
    Hit h{-1.0f, -1, 0};
    float tmax = FLT_MAX, bt;
    h.visits++;
    if (!(box_hit(r, B->root_lo, B->root_hi, &bt) && bt <= tmax)) return h;
    struct E { int32_t info; float t; } st[64];
    int sp = 0;
    int32_t cur = B->root_info;
    while (true) {
        if (cur >= 0) {
            const dl::Pair& P = B->pairs[cur];
            g_rfetch++;
            float lo0[3] = {P.l_minx, P.l_miny, P.l_minz}, hi0[3] = {P.l_maxx, P.l_maxy, P.l_maxz};
            float lo1[3] = {P.r_minx, P.r_miny, P.r_minz}, hi1[3] = {P.r_maxx, P.r_maxy, P.r_maxz};
            float tl, tr;
            bool hl = box_hit(r, lo0, hi0, &tl), hr = box_hit(r, lo1, hi1, &tr);
            h.visits += 2;
            bool lf = comp(r.d, P.axis) > 0;
            bool hn = lf ? hl : hr, hf = lf ? hr : hl;
            float tn = lf ? tl : tr, tf = lf ? tr : tl;
            int32_t in_ = lf ? P.l_info : P.r_info, if_ = lf ? P.r_info : P.l_info;
            if (hf) st[sp++] = {if_, tf};
            if (hn && tn <= tmax) { cur = in_; continue; }
        } else {
            int a, c;
            leaf_range(cur, &a, &c);
            g_rleaf++;
            for (int i = a; i < a + c; ++i) {
                float t;
                if (prim_hit(r, B->prims[i], &t)) {
                    const auto& lb = leaf_boxes[leaf_of_prim[i]];
                    float lt;
                    if (box_hit(r, lb.data(), lb.data() + 3, &lt) && lt > t && t > 0) {
                        double rel = ((double)lt - t) / t;
                        g_anom_max = std::max(g_anom_max, rel);
                        for (int k = 0; k < 4; ++k) if (rel > pow(10.0, -7 + k)) g_anom_n[k]++;
                    }
                }
                if (prim_hit(r, B->prims[i], &t) && (t < h.t || h.t == -1.0f)) { h.t = t; h.prim = i; tmax = t; }
            }
        }
        bool found = false;
        while (sp > 0) { --sp; if (st[sp].t <= tmax) { cur = st[sp].info; found = true; break; } }
        if (!found) break;
    }
    return h;
}

// closest hit over the SAH hierarchy above the same leaves.  Front-to-back
// by child entry t; a subtree is skipped once its entry t exceeds
// tbest * (1 + slack).  Returns status: 0 certified, 1 fallback needed.
int closest_sah(const Ray& r, Hit* out) {
    Hit h{-1.0f, -1, 0};
    int status = 0;
    bool tie = false;
    int tie_leaf = -1, best_leaf = -1;
    float bt;
    auto lim = [&](float tb) { return tb < 0 ? FLT_MAX : (float)(tb * (1.0 + g_slack)); };
    h.visits++;
    if (!box_hit(r, B->sroot_lo, B->sroot_hi, &bt)) { *out = h; return 0; }
    struct E { int32_t info; float t; } st[64];
    int sp = 0;
    int32_t cur = B->sroot_info;
    float tb = FLT_MAX;   // best t, FLT_MAX before any hit
    float t2 = FLT_MAX;   // smallest t among the other hits
    int leafno = 0;
    while (true) {
        if (cur >= 0) {
            const dl::Pair& P = B->spairs[cur];
            float lo0[3] = {P.l_minx, P.l_miny, P.l_minz}, hi0[3] = {P.l_maxx, P.l_maxy, P.l_maxz};
            float lo1[3] = {P.r_minx, P.r_miny, P.r_minz}, hi1[3] = {P.r_maxx, P.r_maxy, P.r_maxz};
            float tl, tr;
            bool hl = box_hit(r, lo0, hi0, &tl), hr = box_hit(r, lo1, hi1, &tr);
            h.visits += 2;
            hl = hl && tl <= lim(tb);
            hr = hr && tr <= lim(tb);
            bool lf = hl && (!hr || tl <= tr);
            bool hn = lf ? hl : hr, hf = lf ? hr : hl;
            float tf = lf ? tr : tl;
            int32_t in_ = lf ? P.l_info : P.r_info, if_ = lf ? P.r_info : P.l_info;
            if (hn && hf) st[sp++] = {if_, tf};
            if (hn) { cur = in_; continue; }
            if (hf) { cur = if_; continue; }
        } else {
            ++leafno;
            int a, c;
            leaf_range(cur, &a, &c);
            for (int i = a; i < a + c; ++i) {
                float t;
                if (!prim_hit(r, B->prims[i], &t)) continue;
                if (t < 0 || t == -1.0f || std::isnan(t)) status = 1;
                if (h.prim < 0 || t < h.t) {
                    if (h.prim >= 0) t2 = std::min(t2, h.t);
                    h.t = t; h.prim = i; tb = t; tie = false; best_leaf = leafno;
                } else {
                    t2 = std::min(t2, t);
                    if (t == h.t && leafno != best_leaf) { tie = true; tie_leaf = leafno; }
                }
            }
        }
        bool found = false;
        while (sp > 0) { --sp; if (st[sp].t <= lim(tb)) { cur = st[sp].info; found = true; break; } }
        if (!found) break;
    }
    (void)tie_leaf;
    if (tie) status = 1;
    if (h.prim >= 0 && status == 0) {   // the reference reaches the winner: its leaf entry <= t
        const auto& lb = leaf_boxes[leaf_of_prim[h.prim]];
        float lt;
        if (!box_hit(r, lb.data(), lb.data() + 3, &lt)) status = 1;
        else if (lt > h.t) {            // winner hit before its leaf's entry t (rounding)
            g_late++;
            if (t2 < lt) status = 1;     // another hit could lower tMax below the entry first
        }
    }
    *out = h;
    return status;
}


// The production trees (bvh.wnodes: reference-order closest hit; bvh.swnodes:
// occlusion), walked exactly as traverse2.hpp's wide_closest_step /
// wide_any_step decode and test them, counting dependent fetch rounds: wide
// nodes and leaf records (exact box + prims in one round).
long g_qfetch = 0, g_lfetch = 0;
float pow2f(int e) { uint32_t b = (uint32_t)e << 23; float f; memcpy(&f, &b, 4); return f; }
int g_slab_fma = 1;   // EXP_SLAB_FMA=0: the exact decode
float h16f(uint16_t b) {
    const int ex = (b >> 10) & 31, man = b & 1023;
    return ex == 0 ? ldexpf((float)man, -24) : ldexpf((float)(1024 + man), ex - 25);
}
// entry/exit t of slot c (device arithmetic: fma decode, near plane by the sign of inv)
void wide_slab(const dl::Wide& w, int c, const Ray& r, float* tmn, float* tmx) {
    const float sc[3] = {pow2f(w.exps & 255u), pow2f((w.exps >> 8) & 255u), pow2f((w.exps >> 16) & 255u)};
    const float o[3] = {w.ox, w.oy, w.oz}, ro[3] = {r.o.x, r.o.y, r.o.z}, ri[3] = {r.inv.x, r.inv.y, r.inv.z};
    for (int a = 0; a < 3; ++a) {
        const uint32_t lw = w.h[a * 3 + c / 2], hw = w.h[9 + a * 3 + c / 2];
        const uint16_t hl = (uint16_t)((c & 1) ? lw >> 16 : lw & 0xffff), hh = (uint16_t)((c & 1) ? hw >> 16 : hw & 0xffff);
        const bool neg = std::signbit(ri[a]);
        float tn, tf;
        if (g_slab_fma) {                     // traverse2.hpp wide_slabs, RT_SLAB_FMA
            const float si = sc[a] * ri[a], z = o[a] - ro[a], oi = z * ri[a];
            const float c = fmaf(sc[a], 0x1p-5f, fabsf(o[a]) * 0x1p-23f);
            const float m = fmaf(fabsf(z), 6.0f * 0x1p-23f, c);
            const float M = fmaf(m, fabsf(ri[a]), 0x1p-126f);
            tn = fmaf(h16f(neg ? hh : hl), si, oi - M);
            tf = fmaf(h16f(neg ? hl : hh), si, oi + M);
        } else {
            const float pl = fmaf(h16f(hl), sc[a], o[a]), ph = fmaf(h16f(hh), sc[a], o[a]);
            tn = ((neg ? ph : pl) - ro[a]) * ri[a];
            tf = ((neg ? pl : ph) - ro[a]) * ri[a];
        }
        *tmn = a == 0 ? tn : fmaxf(*tmn, tn);
        *tmx = a == 0 ? tf : fminf(*tmx, tf);
    }
}
Hit closest_prod(const Ray& r) {
    Hit h{-1.0f, -1, 0};
    float tmax = FLT_MAX;
    struct E { int32_t code; float t; } st[128];
    int sp = 0;
    int32_t cur = B->wroot;
    const int sgn = (r.d.x > 0) | (r.d.y > 0) << 1 | (r.d.z > 0) << 2;
    while (true) {
        if (cur >= 0) {
            g_qfetch++;
            const dl::Wide& w = B->wnodes[cur];
            const uint32_t mask = w.exps >> 24;
            uint32_t rw = w.rank[(sgn & 4) ? (sgn ^ 7) : sgn];
            if (sgn & 4) rw = (uint32_t)(__builtin_popcount(mask) - 1) * 0111111u - rw;
            E v[8]; int rank_of[8]; uint32_t vm = 0;
            for (int c = 0; c < dl::kWideSlots; ++c) {
                float tn, tf;
                wide_slab(w, c, r, &tn, &tf);
                const bool ok = ((mask >> c) & 1u) && tf >= fmaxf(0.0f, tn) && tn <= tmax;
                rank_of[c] = (rw >> (3 * c)) & 7;
                if (ok) { v[rank_of[c]] = {w.child[c], tn}; vm |= 1u << rank_of[c]; }
            }
            if (vm) {
                int first = __builtin_ctz(vm);
                for (int k = 7; k > first; --k) if ((vm >> k) & 1u) st[sp++] = v[k];
                cur = v[first].code;
                continue;
            }
        } else {
            g_lfetch++;
            const dl::LeafHead& L = *reinterpret_cast<const dl::LeafHead*>(&B->lrec[cur & ~dl::kLeafBit]);
            float lo[3] = {L.minx, L.miny, L.minz}, hi[3] = {L.maxx, L.maxy, L.maxz}, lt;
            if (box_hit(r, lo, hi, &lt) && lt <= tmax)
                for (int i = L.slot0; i < L.slot0 + L.count; ++i) {
                    float t;
                    if (prim_hit(r, B->prims[i], &t) && (t < h.t || h.t == -1.0f)) { h.t = t; h.prim = i; tmax = t; }
                }
        }
        bool found = false;
        while (sp > 0) { --sp; if (st[sp].t <= tmax) { cur = st[sp].code; found = true; break; } }
        if (!found) break;
    }
    return h;
}
int closest_quad(const Ray& r, Hit* out) { *out = closest_prod(r); return 0; }

// Reference-order 4-wide walk (collapse of the reference tree: a quad = node N's
// children, interior ones replaced by their own children), visiting children in
// the reference's DFS order (near child first by the sign of d[axis] at N and
// at each child), child boxes pruned at push and at pop against tMax, the
// leaf's exact box tested against tMax before its primitives.  Exact by
// construction for NaN-free rays (nested boxes: a leaf passing its test at its
// pop implies every ancestor passed at its earlier pop).
long g_rqfetch = 0, g_rqleaf = 0;
Hit closest_rquad(const Ray& r) {
    Hit h{-1.0f, -1, 0};
    float tmax = FLT_MAX, bt;
    if (!(box_hit(r, B->root_lo, B->root_hi, &bt) && bt <= tmax)) return h;
    struct E { int32_t info; float t; } st[128];
    int sp = 0;
    int32_t cur = B->root_info;
    auto box_of = [](const dl::Pair& P, bool left, float* lo, float* hi) {
        if (left) { lo[0] = P.l_minx; lo[1] = P.l_miny; lo[2] = P.l_minz; hi[0] = P.l_maxx; hi[1] = P.l_maxy; hi[2] = P.l_maxz; }
        else { lo[0] = P.r_minx; lo[1] = P.r_miny; lo[2] = P.r_minz; hi[0] = P.r_maxx; hi[1] = P.r_maxy; hi[2] = P.r_maxz; }
    };
    while (true) {
        if (cur >= 0) {
            g_rqfetch++;
            const dl::Pair& P = B->pairs[cur];
            int32_t ch[4];
            float lo[4][3], hi[4][3];
            int n = 0;
            const bool lf = comp(r.d, P.axis) > 0;
            for (int side = 0; side < 2; ++side) {
                const bool left = (side == 0) == lf;
                const int32_t info = left ? P.l_info : P.r_info;
                if (info < 0) {
                    ch[n] = info;
                    box_of(P, left, lo[n], hi[n]);
                    n++;
                } else {
                    const dl::Pair& Q = B->pairs[info];
                    const bool lf2 = comp(r.d, Q.axis) > 0;
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const bool l2 = (s2 == 0) == lf2;
                        ch[n] = l2 ? Q.l_info : Q.r_info;
                        box_of(Q, l2, lo[n], hi[n]);
                        n++;
                    }
                }
            }
            E v[4];
            int nv = 0;
            for (int c = 0; c < n; ++c) {
                float t;
                if (box_hit(r, lo[c], hi[c], &t) && t <= tmax) v[nv++] = {ch[c], t};
            }
            for (int j = nv - 1; j >= 1; --j) st[sp++] = v[j];
            if (nv) { cur = v[0].info; continue; }
        } else {
            int a, c;
            leaf_range(cur, &a, &c);
            g_rqleaf++;
            const auto& lb = leaf_boxes[leaf_of_prim[a]];
            float lt;
            if (box_hit(r, lb.data(), lb.data() + 3, &lt) && lt <= tmax)
                for (int i = a; i < a + c; ++i) {
                    float t;
                    if (prim_hit(r, B->prims[i], &t) && (t < h.t || h.t == -1.0f)) { h.t = t; h.prim = i; tmax = t; }
                }
        }
        bool found = false;
        while (sp > 0) { --sp; if (st[sp].t <= tmax) { cur = st[sp].info; found = true; break; } }
        if (!found) break;
    }
    return h;
}

// Greedy-filled reference-order quads: a quad's slots are a frontier of up to
// 4 nodes below an interior node, grown by expanding the interior slot of the
// largest box area; the slots keep pre-order and each octant of the ray
// direction has its own slot permutation (the DFS order below every expanded
// node depends only on the sign of d[axis]).
// EXP_QUANT: slot boxes of the greedy wide nodes as the device would decode them
// (outward-rounded, every decoded box contains the exact one): 0 exact floats,
// 1 8-bit offsets on a power-of-two grid (the current dl::Quad / dl::Wide),
// 2 8-bit offsets on a free float scale, 3 fp16 offsets (power-of-two scale,
// 11 significant bits), 4 16-bit fixed offsets on a free float scale.
int g_quant = 0;
float round_down_bits(float x, int bits) {            // x >= 0, keep `bits` significant bits (toward 0)
    if (!(x > 0)) return 0.0f;
    int e; const double m = frexp((double)x, &e);
    return (float)ldexp(floor(ldexp(m, bits)), e - bits);
}
float round_up_bits(float x, int bits) {
    if (!(x > 0)) return 0.0f;
    int e; const double m = frexp((double)x, &e);
    return (float)ldexp(ceil(ldexp(m, bits)), e - bits);
}
void quantize_node(int n, float (*lo)[3], float (*hi)[3]) {
    if (g_quant == 0 || n == 0) return;
    for (int a = 0; a < 3; ++a) {
        float o = FLT_MAX, top = -FLT_MAX;
        for (int i = 0; i < n; ++i) { o = std::min(o, lo[i][a]); top = std::max(top, hi[i][a]); }
        const double ext = (double)top - o;
        for (int i = 0; i < n; ++i) {
            float l = lo[i][a], h = hi[i][a];
            if (!(ext > 0)) continue;
            if (g_quant == 1 || g_quant == 2 || g_quant == 4) {
                const int steps = g_quant == 4 ? 65535 : 255;
                float sc;
                if (g_quant == 1) sc = (float)ldexp(1.0, (int)ceil(log2(ext / steps)));
                else sc = (float)(ext / steps) * (1.0f + 1e-6f);
                while (fmaf((float)steps, sc, o) < top) sc = nextafterf(sc, FLT_MAX);
                int ql = std::max(0, std::min(steps, (int)floor(((double)l - o) / sc)));
                while (ql > 0 && fmaf((float)ql, sc, o) > l) --ql;
                int qh = std::max(0, std::min(steps, (int)ceil(((double)h - o) / sc)));
                while (qh < steps && fmaf((float)qh, sc, o) < h) ++qh;
                l = fmaf((float)ql, sc, o);
                h = fmaf((float)qh, sc, o);
            } else {                                                   // fp16 offsets
                const float sc = (float)ldexp(1.0, (int)ceil(log2(ext)) - 15);
                float hl = round_down_bits((float)(((double)l - o) / sc), 11);
                float hh = round_up_bits((float)(((double)h - o) / sc), 11);
                while (fmaf(hl, sc, o) > l) hl = round_down_bits(nextafterf(hl, 0.0f), 11);
                while (fmaf(hh, sc, o) < h) hh = round_up_bits(nextafterf(hh, FLT_MAX), 11);
                l = fmaf(hl, sc, o);
                h = fmaf(hh, sc, o);
            }
            lo[i][a] = l;
            hi[i][a] = h;
        }
    }
}
int g_width = 4;    // EXP_WIDTH: slots per node
struct GQuad { int32_t info[8]; float lo[8][3], hi[8][3]; int n; uint8_t perm[8][8]; };
std::vector<GQuad> g_gq;
std::vector<int32_t> g_gq_of_pair;
long g_gqfetch = 0, g_gqleaf = 0;
struct Item { int32_t info; float lo[3], hi[3]; };
double box_area(const float* lo, const float* hi) {
    double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}
int32_t build_gq(int32_t pair) {
    // expansion tree: node k of the frontier is a leaf of the expansion; expanded
    // nodes record (axis, first slot of right part)
    struct Exp { int axis; int lo, mid, hi; };
    std::vector<Item> fr;
    std::vector<Exp> ex;
    auto kids = [&](int32_t p, Item* a, Item* b) {
        const dl::Pair& P = B->pairs[p];
        a->info = P.l_info; a->lo[0] = P.l_minx; a->lo[1] = P.l_miny; a->lo[2] = P.l_minz;
        a->hi[0] = P.l_maxx; a->hi[1] = P.l_maxy; a->hi[2] = P.l_maxz;
        b->info = P.r_info; b->lo[0] = P.r_minx; b->lo[1] = P.r_miny; b->lo[2] = P.r_minz;
        b->hi[0] = P.r_maxx; b->hi[1] = P.r_maxy; b->hi[2] = P.r_maxz;
        return P.axis;
    };
    Item a, b;
    int ax = kids(pair, &a, &b);
    fr = {a, b};
    ex.push_back({ax, 0, 1, 2});
    while ((int)fr.size() < g_width) {
        int best = -1;
        double ba = -1;
        for (size_t i = 0; i < fr.size(); ++i)
            if (fr[i].info >= 0 && box_area(fr[i].lo, fr[i].hi) > ba) { ba = box_area(fr[i].lo, fr[i].hi); best = (int)i; }
        if (best < 0) break;
        Item c, d;
        ax = kids(fr[best].info, &c, &d);
        fr[best] = c;
        fr.insert(fr.begin() + best + 1, d);
        for (auto& e : ex) { if (e.mid > best) e.mid++; if (e.hi > best) e.hi++; }   // ranges after the split slot shift
        for (auto& e : ex) { if (e.lo > best) e.lo++; }
        ex.push_back({ax, best, best + 1, best + 2});
    }
    GQuad q{};
    q.n = (int)fr.size();
    for (int i = 0; i < q.n; ++i) { q.info[i] = fr[i].info; memcpy(q.lo[i], fr[i].lo, 12); memcpy(q.hi[i], fr[i].hi, 12); }
    quantize_node(q.n, q.lo, q.hi);
    for (int oct = 0; oct < 8; ++oct) {
        // visit order: recursive over the expansion tree (ex[0] is the root)
        std::vector<int> order;
        std::function<void(int, int)> rec = [&](int lo, int hi) {
            if (hi - lo == 1) { order.push_back(lo); return; }
            for (const auto& e : ex)
                if (e.lo == lo && e.hi == hi) {
                    bool lf = (oct >> e.axis) & 1;
                    if (lf) { rec(e.lo, e.mid); rec(e.mid, e.hi); } else { rec(e.mid, e.hi); rec(e.lo, e.mid); }
                    return;
                }
            abort();
        };
        rec(0, q.n);
        for (int i = 0; i < q.n; ++i) q.perm[oct][i] = (uint8_t)order[i];
    }
    const int me = (int)g_gq.size();
    g_gq.push_back(q);
    for (int i = 0; i < q.n; ++i)
        if (q.info[i] >= 0) {
            const int32_t c = build_gq(q.info[i]);
            g_gq[me].info[i] = c;   // child quad index (>= 0), leaves keep their info (< 0)
        }
    return me;
}
Hit closest_gquad(const Ray& r) {
    Hit h{-1.0f, -1, 0};
    float tmax = FLT_MAX;
    if (B->root_info >= 0 && g_gq.empty()) build_gq(B->root_info);
    const int oct = (r.d.x > 0) | (r.d.y > 0) << 1 | (r.d.z > 0) << 2;
    struct E { int32_t info; float t; } st[128];
    int sp = 0;
    int32_t cur = B->root_info >= 0 ? 0 : B->root_info;
    while (true) {
        if (cur >= 0) {
            g_gqfetch++;
            const GQuad& q = g_gq[cur];
            E v[8];
            int nv = 0;
            for (int j = 0; j < q.n; ++j) {
                const int c = q.perm[oct][j];
                float t;
                if (box_hit(r, q.lo[c], q.hi[c], &t) && t <= tmax) v[nv++] = {q.info[c], t};
            }
            for (int j = nv - 1; j >= 1; --j) st[sp++] = v[j];
            if (nv) { cur = v[0].info; continue; }
        } else {
            int a, c;
            leaf_range(cur, &a, &c);
            g_gqleaf++;
            const auto& lb = leaf_boxes[leaf_of_prim[a]];
            float lt;
            if (box_hit(r, lb.data(), lb.data() + 3, &lt) && lt <= tmax)
                for (int i = a; i < a + c; ++i) {
                    float t;
                    if (prim_hit(r, B->prims[i], &t) && (t < h.t || h.t == -1.0f)) { h.t = t; h.prim = i; tmax = t; }
                }
        }
        bool found = false;
        while (sp > 0) { --sp; if (st[sp].t <= tmax) { cur = st[sp].info; found = true; break; } }
        if (!found) break;
    }
    return h;
}

// Any-hit over the SAH tree (spairs) collapsed greedily to g_width slots per node
// (largest-area interior slot expanded first): fetch rounds only.
struct SNode { int32_t info[8]; float lo[8][3], hi[8][3]; int n; };
std::vector<SNode> g_sn;
int32_t build_sn(int32_t pair) {
    struct It { int32_t info; float lo[3], hi[3]; };
    auto kids = [&](int32_t p, It* a, It* b) {
        const dl::Pair& P = B->spairs[p];
        *a = It{P.l_info, {P.l_minx, P.l_miny, P.l_minz}, {P.l_maxx, P.l_maxy, P.l_maxz}};
        *b = It{P.r_info, {P.r_minx, P.r_miny, P.r_minz}, {P.r_maxx, P.r_maxy, P.r_maxz}};
    };
    std::vector<It> fr(2);
    kids(pair, &fr[0], &fr[1]);
    while ((int)fr.size() < g_width) {
        int best = -1;
        double ba = -1;
        for (size_t i = 0; i < fr.size(); ++i)
            if (fr[i].info >= 0 && box_area(fr[i].lo, fr[i].hi) > ba) { ba = box_area(fr[i].lo, fr[i].hi); best = (int)i; }
        if (best < 0) break;
        It c, d;
        kids(fr[best].info, &c, &d);
        fr[best] = c;
        fr.insert(fr.begin() + best + 1, d);
    }
    SNode q{};
    q.n = (int)fr.size();
    for (int i = 0; i < q.n; ++i) { q.info[i] = fr[i].info; memcpy(q.lo[i], fr[i].lo, 12); memcpy(q.hi[i], fr[i].hi, 12); }
    quantize_node(q.n, q.lo, q.hi);
    const int me = (int)g_sn.size();
    g_sn.push_back(q);
    for (int i = 0; i < q.n; ++i)
        if (q.info[i] >= 0) g_sn[me].info[i] = build_sn(q.info[i]);
    return me;
}
long g_snf = 0, g_snl = 0;
bool any_wide(const Ray& r, float tlim) {
    if (g_sn.empty()) build_sn(B->sroot_info);
    int32_t st[256];
    int sp = 0;
    int32_t cur = 0;
    while (true) {
        if (cur >= 0) {
            g_snf++;
            const SNode& q = g_sn[cur];
            bool have = false;
            int32_t next = 0;
            for (int c = 0; c < q.n; ++c) {
                float t;
                if (box_hit(r, q.lo[c], q.hi[c], &t)) { if (!have) { next = q.info[c]; have = true; } else st[sp++] = q.info[c]; }
            }
            if (have) { cur = next; continue; }
        } else {
            g_snl++;
            int a, c;
            leaf_range(cur, &a, &c);
            const auto& lb = leaf_boxes[leaf_of_prim[a]];
            float lt;
            if (box_hit(r, lb.data(), lb.data() + 3, &lt))
                for (int i = a; i < a + c; ++i) { float t; if (prim_hit(r, B->prims[i], &t) && t < tlim) return true; }
        }
        if (sp == 0) return false;
        cur = st[--sp];
    }
}

bool any_quad(const Ray& r, float tlim, long* qf, long* lf) {     // the production occlusion walk
    int32_t st[128]; int sp = 0; int32_t cur = B->swroot;
    while (true) {
        if (cur >= 0) {
            (*qf)++;
            const dl::Wide& w = B->swnodes[cur];
            const uint32_t mask = w.exps >> 24;
            static const int order_mode = getenv("EXP_ANY_ORDER") ? atoi(getenv("EXP_ANY_ORDER")) : 0;
            struct V { int32_t code; float t; } v[8]; int nv = 0;
            for (int c = 0; c < dl::kWideSlots; ++c) {
                float tn, tf;
                wide_slab(w, c, r, &tn, &tf);
                if (((mask >> c) & 1u) && tf >= fmaxf(0.0f, tn)) v[nv++] = {w.child[c], order_mode == 2 ? -tn : tn};
            }
            if (order_mode)        // 1: nearest entry first, 2: farthest first
                for (int i = 1; i < nv; ++i) for (int j = i; j > 0 && v[j].t < v[j - 1].t; --j) std::swap(v[j], v[j - 1]);
            if (nv) {
                for (int j = nv - 1; j >= 1; --j) st[sp++] = v[j].code;
                cur = v[0].code;
                continue;
            }
        } else {
            (*lf)++;
            const dl::LeafHead& L = *reinterpret_cast<const dl::LeafHead*>(&B->lrec[cur & ~dl::kLeafBit]);
            float lo[3] = {L.minx, L.miny, L.minz}, hi[3] = {L.maxx, L.maxy, L.maxz}, lt;
            if (box_hit(r, lo, hi, &lt)) {
                int a = L.slot0, c = L.count;
                for (int i = a; i < a + c; ++i) { float t; if (prim_hit(r, B->prims[i], &t) && t < tlim) return true; }
            }
        }
        if (sp == 0) return false;
        cur = st[--sp];
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s scene.xml [slack]\n", argv[0]); return 2; }
    if (argc > 2) g_slack = atof(argv[2]);
    if (getenv("EXP_WIDTH")) g_width = atoi(getenv("EXP_WIDTH"));
    if (getenv("EXP_QUANT")) g_quant = atoi(getenv("EXP_QUANT"));
    if (getenv("EXP_SLAB_FMA")) g_slab_fma = atoi(getenv("EXP_SLAB_FMA"));
    int dump_row = -1, dump_col = -1;          // --dump ROW COL: print the pixel's chain rays (o, d) as hex floats
    if (argc > 5 && !strcmp(argv[3], "--dump")) { dump_row = atoi(argv[4]); dump_col = atoi(argv[5]); }
    HostScene sc;
    std::string err = load_xml(argv[1], sc);
    if (!err.empty()) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    prepare_triangles(sc);
    FlatBVH bvh;
    err = build_bvh(sc, bvh);
    if (!err.empty()) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    B = &bvh;
    leaf_of_prim.assign(bvh.prims.size(), -1);
    auto reg = [&](int32_t info, const float* lo, const float* hi) {
        int a, c;
        leaf_range(info, &a, &c);
        leaf_boxes.push_back({lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
        for (int i = a; i < a + c; ++i) leaf_of_prim[i] = (int)leaf_boxes.size() - 1;
    };
    for (const auto& P : bvh.pairs) {
        float lo0[3] = {P.l_minx, P.l_miny, P.l_minz}, hi0[3] = {P.l_maxx, P.l_maxy, P.l_maxz};
        float lo1[3] = {P.r_minx, P.r_miny, P.r_minz}, hi1[3] = {P.r_maxx, P.r_maxy, P.r_maxz};
        if (P.l_info < 0) reg(P.l_info, lo0, hi0);
        if (P.r_info < 0) reg(P.r_info, lo1, hi1);
    }
    const CameraRec& c = sc.cameras[0];
    const int nx = c.width, ny = c.height;
    Vf e{c.position.x, c.position.y, c.position.z}, w{-c.gaze.x, -c.gaze.y, -c.gaze.z};
    Vf v{c.up.x, c.up.y, c.up.z};
    Vf u{v.y * w.z - v.z * w.y, v.z * w.x - v.x * w.z, v.x * w.y - v.y * w.x};
    Vf m = add(e, mul(neg(w), c.near_distance));
    Vf q = add(add(m, mul(u, c.near_plane[0])), mul(v, c.near_plane[3]));
    float su_m = (c.near_plane[1] - c.near_plane[0]) / (float)nx, sv_m = (c.near_plane[3] - c.near_plane[2]) / (float)ny;

    long ref_total = 0, sah_total = 0, walks = 0, fallback = 0, mismatch = 0, cert_mismatch = 0;
    std::vector<long> chain_qb;
    long best_qb = -1; int best_rc[2] = {0, 0};
    long max_cqa = 0, max_walk_q = 0, walks_b = 0;
    long qfall = 0, qmis = 0, sq_f = 0, sl_f = 0, nshadow = 0;
    long rq_mis = 0, max_crb = 0, gq_mis = 0, max_cgb = 0, aw_mis = 0;
    long max_chain_ref = 0, max_chain_sah = 0, max_chain_mixed = 0;
    std::vector<long> chain_ref, chain_mixed;
    chain_ref.reserve((size_t)nx * ny);
    for (int row = 0; row < ny; ++row)
        for (int col = 0; col < nx; ++col) {
            float su = ((float)col + 0.5f) * su_m, sv = ((float)row + 0.5f) * sv_m;
            Vf sp = sub(add(q, mul(u, su)), mul(v, sv));
            Ray r = make_ray(e, sub(sp, e));
            long cr = 0, cs = 0, cm = 0, cq_a = 0, cq_b = 0, cr_b = 0, cg_b = 0;
            for (int k = 0; k <= sc.max_depth; ++k) {
                if (row == dump_row && col == dump_col)
                    printf("RAY %a %a %a %a %a %a\n", r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z);
                Hit hr = closest_ref(r), hs, hq;
                {
                    const long f0 = g_rqfetch + g_rqleaf;
                    const Hit hx = closest_rquad(r);
                    const long fr = g_rqfetch + g_rqleaf - f0;
                    if (k >= 2) cr_b += fr;
                    if (hx.prim != hr.prim || (hr.prim >= 0 && hx.t != hr.t)) rq_mis++;
                    const long g0 = g_gqfetch + g_gqleaf;
                    const Hit hg = closest_gquad(r);
                    if (k >= 2) cg_b += g_gqfetch + g_gqleaf - g0;
                    if (hg.prim != hr.prim || (hr.prim >= 0 && hg.t != hr.t)) gq_mis++;
                }
                int stt = closest_sah(r, &hs);
                const long qf0 = g_qfetch + g_lfetch;
                int qst = closest_quad(r, &hq);
                const long qrounds = g_qfetch + g_lfetch - qf0;
                if (k >= 2) cq_b += qrounds; else cq_a += qrounds;
                if (k >= 2) { walks_b++; }
                max_walk_q = std::max(max_walk_q, qrounds);
                if (qst) qfall++;
                if (!qst && (hq.prim != hr.prim || (hr.prim >= 0 && hq.t != hr.t))) qmis++;
                walks++;
                ref_total += hr.visits;
                sah_total += hs.visits;
                cr += hr.visits;
                cs += hs.visits;
                cm += stt ? hs.visits + hr.visits : hs.visits;
                if (stt) fallback++;
                if (hr.prim != hs.prim || (hr.prim >= 0 && hr.t != hs.t)) {
                    mismatch++;
                    if (!stt) cert_mismatch++;
                }
                if (hr.prim < 0) break;
                const dl::Prim& P = bvh.prims[hr.prim];
                int mat;
                Vf n;
                Vf hp = add(r.o, mul(r.d, hr.t));
                if (P.id >= 0) {
                    const dl::TriShade& ts = bvh.tri_shade[P.id];
                    n = {ts.nx, ts.ny, ts.nz};
                    mat = ts.material;
                } else {
                    Vf cc{P.p0x, P.p0y, P.p0z};
                    Vf dd = sub(hp, cc);
                    n = nrm(Vf{dd.x / P.p1x, dd.y / P.p1x, dd.z / P.p1x});
                    mat = P.p2w;
                }
                Vf pnt = add(hp, mul(n, sc.eps));
                for (const auto& L : sc.lights) {
                    Vf lp{L.position.x, L.position.y, L.position.z};
                    float tl = len(sub(lp, pnt));
                    Ray sr = make_ray(pnt, nrm(sub(lp, pnt)));
                    const bool o1 = any_quad(sr, tl, &sq_f, &sl_f);
                    if (o1 != any_wide(sr, tl)) aw_mis++;
                    nshadow++;
                }
                if (!sc.materials[mat - 1].is_mirror) break;
                Vf d2 = nrm(r.d), n2 = nrm(n);
                float rc = dot(neg(d2), n2);
                r = make_ray(pnt, add(d2, mul(mul(n2, 2.0f), rc)));
            }
            chain_ref.push_back(cr);
            chain_qb.push_back(cq_b);
            max_crb = std::max(max_crb, cr_b);
            max_cgb = std::max(max_cgb, cg_b);
            if (cq_b > best_qb) { best_qb = cq_b; best_rc[0] = row; best_rc[1] = col; }
            max_cqa = std::max(max_cqa, cq_a);
            chain_mixed.push_back(cm);
            max_chain_ref = std::max(max_chain_ref, cr);
            max_chain_sah = std::max(max_chain_sah, cs);
            max_chain_mixed = std::max(max_chain_mixed, cm);
        }
    auto pct = [](const std::vector<long>& v, double p) { return v[(size_t)((v.size() - 1) * p)]; };
    std::sort(chain_ref.begin(), chain_ref.end());
    std::sort(chain_mixed.begin(), chain_mixed.end());
    printf("slack %g walks %ld: box tests ref %.2f/walk sah %.2f/walk (ratio %.2f)\n", g_slack, walks,
           (double)ref_total / walks, (double)sah_total / walks, (double)ref_total / sah_total);
    printf("fallback %ld (%.4f%%) mismatch %ld certified-mismatch %ld\n", fallback, 100.0 * fallback / walks, mismatch,
           cert_mismatch);
    printf("production closest: fallback %ld mismatch %ld; per walk: ref pair fetches %.2f leaves %.2f | wide fetches %.2f leaves %.2f\n",
           qfall, qmis, (double)g_rfetch / walks, (double)g_rleaf / walks, (double)g_qfetch / walks, (double)g_lfetch / walks);
    printf("shadow rays %ld (production wide tree): node fetches %.2f leaves %.2f per ray\n", nshadow, (double)sq_f / nshadow, (double)sl_f / nshadow);
    printf("shadow rays, SAH collapsed to %d slots: node fetches %.2f leaves %.2f per ray, mismatch %ld\n", g_width,
           (double)g_snf / nshadow, (double)g_snl / nshadow, aw_mis);
    printf("ref-order quad: mismatch %ld; per walk quad fetches %.2f leaves %.2f; phase-B chain max rounds %ld\n",
           rq_mis, (double)g_rqfetch / walks, (double)g_rqleaf / walks, max_crb);
    printf("greedy ref-order quad: mismatch %ld; per walk quad fetches %.2f leaves %.2f; phase-B chain max rounds %ld; quads %zu\n",
           gq_mis, (double)g_gqfetch / walks, (double)g_gqleaf / walks, max_cgb, g_gq.size());
    std::sort(chain_qb.begin(), chain_qb.end());
    printf("quad fetch rounds: phase-A chain max %ld, phase-B chain max %ld p99.99 %ld p99.9 %ld, max single walk %ld, phase-B walks %ld\n",
           max_cqa, chain_qb.back(), pct(chain_qb, 0.9999), pct(chain_qb, 0.999), max_walk_q, walks_b);
    printf("heaviest phase-B chain at row %d col %d\n", best_rc[0], best_rc[1]);
    printf("late winners %ld; anomaly max rel %.3g, >1e-7 %ld >1e-6 %ld >1e-5 %ld >1e-4 %ld\n", g_late, g_anom_max,
           g_anom_n[0], g_anom_n[1], g_anom_n[2], g_anom_n[3]);
    printf("chain visits max: ref %ld sah %ld sah+fallback %ld\n", max_chain_ref, max_chain_sah, max_chain_mixed);
    printf("chain p99 / p99.9 / p99.99: ref %ld %ld %ld  mixed %ld %ld %ld\n", pct(chain_ref, 0.99),
           pct(chain_ref, 0.999), pct(chain_ref, 0.9999), pct(chain_mixed, 0.99), pct(chain_mixed, 0.999),
           pct(chain_mixed, 0.9999));
    return 0;
}
