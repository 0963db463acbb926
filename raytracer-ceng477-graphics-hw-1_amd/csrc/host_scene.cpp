// XML scene loader, triangle preparation and bit-exact BVH builder (host).
#include "host_scene.hpp"

#include <atomic>
#include <cfloat>
#include <algorithm>
#include <chrono>
#include <new>
#include <functional>
#include <future>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string_view>
#include <type_traits>

namespace rtx {

// ---------------------------------------------------------------------------
// XML: a small DOM over the file buffer (elements, attributes, the first text
// run as an offset range, no copies).  tinyxml2 4.0.1 is used by the reference
// only to hand element text to a std::stringstream (parser.cpp:9-217); numbers
// therefore follow istream >> float / >> int, i.e. strtof / strtol on
// whitespace-separated tokens.  Element text always ends at the next '<' and
// the buffer is NUL-terminated, so strtof/strtol never read past it.
// Large number lists (VertexData, Faces) are split at whitespace into chunks
// parsed by concurrent threads; every token is parsed by the same call as in
// the serial reading, so the values are identical.
// ---------------------------------------------------------------------------
namespace {

struct Elem {
    std::string name;
    size_t attr_off = 0, attr_len = 0;
    size_t text_off = 0, text_len = 0;
    bool has_text = false;
    std::vector<int> kids;
};

class Dom {
  public:
    std::vector<Elem> el;
    const std::string* src = nullptr;

    bool parse(const std::string& s, std::string& err) {
        src = &s;
        el.clear();
        el.reserve(1024);
        el.push_back(Elem{"#document"});
        std::vector<int> open{0};
        const char* base = s.data();
        size_t i = 0, n = s.size();
        while (i < n) {
            if (s[i] != '<') {
                const void* lt = std::memchr(base + i, '<', n - i);
                const size_t j = lt ? (size_t)(static_cast<const char*>(lt) - base) : n;
                Elem& cur = el[open.back()];
                if (cur.kids.empty() && !cur.has_text) {
                    cur.text_off = i;
                    cur.text_len = j - i;
                    cur.has_text = j > i;
                }
                i = j;
                continue;
            }
            if (s.compare(i, 4, "<!--") == 0) {
                size_t j = s.find("-->", i + 4);
                if (j == std::string::npos) { err = "unterminated comment"; return false; }
                i = j + 3;
                continue;
            }
            if (i + 1 < n && (s[i + 1] == '?' || s[i + 1] == '!')) {
                size_t j = s.find('>', i);
                if (j == std::string::npos) { err = "unterminated declaration"; return false; }
                i = j + 1;
                continue;
            }
            if (i + 1 < n && s[i + 1] == '/') {
                size_t j = s.find('>', i);
                if (j == std::string::npos || open.size() <= 1) { err = "unbalanced closing tag"; return false; }
                open.pop_back();
                i = j + 1;
                continue;
            }
            size_t j = i + 1;
            while (j < n && !std::isspace((unsigned char)s[j]) && s[j] != '>' && s[j] != '/') ++j;
            Elem e;
            e.name.assign(s, i + 1, j - i - 1);
            size_t k = j;
            while (k < n && s[k] != '>') {
                if (s[k] == '"') {
                    k = s.find('"', k + 1);
                    if (k == std::string::npos) { err = "unterminated attribute"; return false; }
                }
                ++k;
            }
            if (k >= n) { err = "unterminated tag"; return false; }
            bool self_close = s[k - 1] == '/';
            e.attr_off = j;
            e.attr_len = k - j;
            int id = (int)el.size();
            el.push_back(std::move(e));
            el[open.back()].kids.push_back(id);
            if (!self_close) open.push_back(id);
            i = k + 1;
        }
        return true;
    }

    int child(int parent, const char* name) const {
        if (parent < 0) return -1;
        for (int k : el[parent].kids)
            if (el[k].name == name) return k;
        return -1;
    }
    std::vector<int> children(int parent, const char* name) const {
        std::vector<int> out;
        if (parent < 0) return out;
        for (int k : el[parent].kids)
            if (el[k].name == name) out.push_back(k);
        return out;
    }
    const char* text(int k) const { return src->data() + (el[k].has_text ? el[k].text_off : src->size()); }
    size_t text_len(int k) const { return el[k].has_text ? el[k].text_len : 0; }
    bool attr_has(int k, const char* needle) const {
        return std::string_view(src->data() + el[k].attr_off, el[k].attr_len).find(needle) != std::string_view::npos;
    }
};

// Token reader over one element's text (a pointer into the NUL-terminated
// file buffer; the text is followed by '<' or the end of the buffer).
class Tok {
  public:
    explicit Tok(const char* p) : p_(p) {}
    bool f(float& v) {
        char* e;
        float x = std::strtof(p_, &e);
        if (e == p_) return false;
        v = x; p_ = e; return true;
    }
    bool i(int& v) {
        char* e;
        long x = std::strtol(p_, &e, 10);
        if (e == p_) return false;
        v = (int)x; p_ = e; return true;
    }
    bool v3(V3& v) { return f(v.x) && f(v.y) && f(v.z); }
    bool word(std::string& w) {
        while (*p_ && *p_ != '<' && std::isspace((unsigned char)*p_)) ++p_;
        const char* b = p_;
        while (*p_ && *p_ != '<' && !std::isspace((unsigned char)*p_)) ++p_;
        w.assign(b, p_ - b);
        return !w.empty();
    }

  private:
    const char* p_;
};

// All tokens of a number list [p, p+len) (floats or ints), stopping at the
// first token that does not parse, exactly like repeated Tok::f / Tok::i.
// Texts above kParMin bytes are split at whitespace into `threads` chunks
// parsed concurrently; a chunk that stops early ends the list there.
constexpr size_t kParMin = 64 * 1024;

template <class T>
std::vector<T> number_list(const char* p, size_t len, int threads) {
    auto scan = [](const char* b, const char* e, std::vector<T>& out) -> bool {   // false: stopped early
        const char* q = b;
        while (true) {
            while (q < e && std::isspace((unsigned char)*q)) ++q;
            if (q >= e) return true;
            char* end;
            T v;
            if constexpr (std::is_same<T, float>::value) v = std::strtof(q, &end);
            else v = (T)std::strtol(q, &end, 10);
            if (end == q) return false;
            out.push_back(v);
            q = end;
        }
    };
    std::vector<T> out;
    const int nch = len < kParMin ? 1 : std::max(1, std::min(threads, 16));
    if (nch == 1) {
        out.reserve(len / 6);
        scan(p, p + len, out);
        return out;
    }
    std::vector<const char*> cut{p};
    for (int c = 1; c < nch; ++c) {
        const char* q = std::max(cut.back(), p + len * c / nch);
        while (q < p + len && !std::isspace((unsigned char)*q)) ++q;     // a cut never splits a token
        cut.push_back(q);
    }
    cut.push_back(p + len);
    std::vector<std::vector<T>> part(nch);
    std::vector<char> full(nch, 1);
    std::vector<std::future<void>> fs;
    for (int c = 1; c < nch; ++c)
        fs.push_back(std::async(std::launch::async, [&, c] {
            part[c].reserve((cut[c + 1] - cut[c]) / 6);
            full[c] = scan(cut[c], cut[c + 1], part[c]);
        }));
    part[0].reserve((cut[1] - cut[0]) / 6);
    full[0] = scan(cut[0], cut[1], part[0]);
    for (auto& f : fs) f.get();
    size_t total = 0;
    for (int c = 0; c < nch; ++c) {
        total += part[c].size();
        if (!full[c]) break;
    }
    out.reserve(total);
    for (int c = 0; c < nch; ++c) {
        out.insert(out.end(), part[c].begin(), part[c].end());
        if (!full[c]) break;
    }
    return out;
}

struct Need {
    const Dom& d;
    std::string& err;
    int get(int parent, const char* name) {
        int k = d.child(parent, name);
        if (k < 0 && err.empty()) err = std::string("Error: missing element <") + name + ">";
        return k;
    }
    const char* text(int parent, const char* name) {
        int k = get(parent, name);
        return k < 0 ? "" : d.text(k);
    }
};

bool read_file(const char* path, std::string& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) { std::fclose(f); return false; }
    out.resize((size_t)n);
    const size_t got = n > 0 ? std::fread(&out[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    out.resize(got);
    return true;
}

}  // namespace

std::string load_xml(const char* path, HostScene& sc, int threads) {
    std::string buf;
    if (!read_file(path, buf)) return "Error: The xml file cannot be loaded.";   // parser.cpp:14
    threads = build_threads(threads);
    Dom d;
    std::string err;
    if (!d.parse(buf, err)) return "Error: The xml file cannot be loaded. (" + err + ")";
    if (d.el[0].kids.empty()) return "Error: Root is not found.";   // parser.cpp:20
    int root = d.el[0].kids.front();
    Need need{d, err};
    sc = HostScene();

    if (int e = d.child(root, "BackgroundColor"); e >= 0) {          // parser.cpp:24-33
        Tok t(d.text(e));
        t.i(sc.bg[0]); t.i(sc.bg[1]); t.i(sc.bg[2]);
    }
    if (int e = d.child(root, "ShadowRayEpsilon"); e >= 0) {         // :36-45 (default 0.001)
        Tok t(d.text(e));
        t.f(sc.eps);
    }
    if (int e = d.child(root, "MaxRecursionDepth"); e >= 0) {        // :48-57 (default 0)
        Tok t(d.text(e));
        t.i(sc.max_depth);
    }
    int cams = need.get(root, "Cameras");                            // :60-90
    for (int c : d.children(cams, "Camera")) {
        CameraRec cam{};
        Tok(need.text(c, "Position")).v3(cam.position);
        Tok(need.text(c, "Gaze")).v3(cam.gaze);
        Tok(need.text(c, "Up")).v3(cam.up);
        Tok np(need.text(c, "NearPlane"));
        for (float& v : cam.near_plane) np.f(v);
        Tok(need.text(c, "NearDistance")).f(cam.near_distance);
        Tok res(need.text(c, "ImageResolution"));
        res.i(cam.width); res.i(cam.height);
        Tok(need.text(c, "ImageName")).word(cam.name);
        sc.cameras.push_back(cam);
    }
    int lights = need.get(root, "Lights");                           // :93-111
    Tok(need.text(lights, "AmbientLight")).v3(sc.ambient);
    for (int l : d.children(lights, "PointLight")) {
        LightRec L{};
        Tok(need.text(l, "Position")).v3(L.position);
        Tok(need.text(l, "Intensity")).v3(L.intensity);
        sc.lights.push_back(L);
    }
    int mats = need.get(root, "Materials");                          // :114-140
    for (int m : d.children(mats, "Material")) {
        MaterialRec M{};
        M.is_mirror = d.attr_has(m, "type=\"mirror\"");              // :119
        Tok(need.text(m, "AmbientReflectance")).v3(M.ambient);
        Tok(need.text(m, "DiffuseReflectance")).v3(M.diffuse);
        Tok(need.text(m, "SpecularReflectance")).v3(M.specular);
        Tok(need.text(m, "MirrorReflectance")).v3(M.mirror);
        Tok(need.text(m, "PhongExponent")).f(M.phong);
        sc.materials.push_back(M);
    }
    if (int e = need.get(root, "VertexData"); e >= 0) {              // :143-151, complete triples
        const std::vector<float> v = number_list<float>(d.text(e), d.text_len(e), threads);
        sc.verts.resize(v.size() / 3);
        for (size_t i = 0; i < sc.verts.size(); ++i) sc.verts[i] = V3{v[3 * i], v[3 * i + 1], v[3 * i + 2]};
    }
    int objs = need.get(root, "Objects");
    // raytracer.cpp:336-341: standalone triangles first, then mesh faces.
    for (int tr : d.children(objs, "Triangle")) {                    // :180-195
        TriRec T{};
        Tok(need.text(tr, "Material")).i(T.material_id);
        Tok ix(need.text(tr, "Indices"));
        ix.i(T.v0); ix.i(T.v1); ix.i(T.v2);
        sc.tris.push_back(T);
    }
    for (int me : d.children(objs, "Mesh")) {                        // :154-177
        int mat = 0;
        Tok(need.text(me, "Material")).i(mat);
        const int fe = need.get(me, "Faces");
        if (fe < 0) continue;
        const std::vector<int> f = number_list<int>(d.text(fe), d.text_len(fe), threads);
        const size_t nf = f.size() / 3;
        sc.tris.reserve(sc.tris.size() + nf);
        for (size_t i = 0; i < nf; ++i) sc.tris.push_back(TriRec{mat, f[3 * i], f[3 * i + 1], f[3 * i + 2], {0, 0, 0}, {0, 0, 0}});
    }
    for (int sp : d.children(objs, "Sphere")) {                      // :198-217
        SphereRec S{};
        Tok(need.text(sp, "Material")).i(S.material_id);
        Tok(need.text(sp, "Center")).i(S.center_id);
        Tok(need.text(sp, "Radius")).f(S.radius);
        sc.spheres.push_back(S);
    }
    if (!err.empty()) return err;
    // Validate ids (the reference would read out of bounds instead).
    const int nv = (int)sc.verts.size(), nm = (int)sc.materials.size();
    for (const TriRec& t : sc.tris)
        if (t.v0 < 1 || t.v1 < 1 || t.v2 < 1 || t.v0 > nv || t.v1 > nv || t.v2 > nv || t.material_id < 1 || t.material_id > nm)
            return "Error: triangle references a missing vertex or material";
    for (const SphereRec& s : sc.spheres)
        if (s.center_id < 1 || s.center_id > nv || s.material_id < 1 || s.material_id > nm)
            return "Error: sphere references a missing vertex or material";
    return "";
}

// ---------------------------------------------------------------------------
// raytracer.cpp:342-348
// ---------------------------------------------------------------------------
void prepare_triangles(HostScene& s) {
    for (TriRec& t : s.tris) {
        const V3 a = s.verts[t.v0 - 1], b = s.verts[t.v1 - 1], c = s.verts[t.v2 - 1];
        const V3 ba{b.x - a.x, b.y - a.y, b.z - a.z}, ca{c.x - a.x, c.y - a.y, c.z - a.z};
        V3 n{ba.y * ca.z - ba.z * ca.y, ba.z * ca.x - ba.x * ca.z, ba.x * ca.y - ba.y * ca.x};
        const float len = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
        t.normal = V3{n.x / len, n.y / len, n.z / len};
        const V3 sum{(a.x + b.x) + c.x, (a.y + b.y) + c.y, (a.z + b.z) + c.z};
        t.center = V3{sum.x / 3, sum.y / 3, sum.z / 3};
    }
}

// ---------------------------------------------------------------------------
// BVH (bvh.h:48-163).  Build recursion is the reference's; the output is the
// pre-order device layout.
// ---------------------------------------------------------------------------
namespace {

constexpr int kMaxDepth = 19;    // bvh.h:18
constexpr int kMaxTries = 19;    // bvh.h:117

struct BNode {
    V3 lo, hi;
    int axis = 0, depth = 0;
    int left = -1, right = -1;
    int t0 = 0, t1 = 0, s0 = 0, s1 = 0;   // leaf: its triangles pt[t0, t1), spheres ps[s0, s1)
    int used = 0;                         // 1: a node of the tree (unused slots stay default)
};


// Dynamic fork-join: a split starts its right half on a new thread while `spare` (the threads the build
// may still start) allows, so the biggest subtrees get the threads whatever the split balance; the task
// gives its thread back when done.  The trees do not depend on it (every subtree owns fixed node slots).
constexpr int kForkMinSah = 1024;
inline bool take_thread(std::atomic<int>* spare) {
    if (spare->fetch_sub(1) > 0) return true;
    spare->fetch_add(1);
    return false;
}

// fn(i) for i in [0, n) on `threads` threads (contiguous chunks; fn must only write item i's outputs).
template <class F>
void parallel_for(int n, int threads, F&& fn) {
    const int t = std::max(1, std::min(threads, n / 64));
    if (t <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(t - 1);
    auto run = [&](int k) {
        const int b = (int)((long long)n * k / t), e = (int)((long long)n * (k + 1) / t);
        for (int i = b; i < e; ++i) fn(i);
    };
    for (int k = 1; k < t; ++k) pool.emplace_back(run, k);
    run(0);
    for (auto& th : pool) th.join();
}


// Per-triangle box (the three vertices folded with the reference's `<` / `>`
// updates, parser.h:272-317) and split key, computed once: a node's box is the
// same fold over its triangles' boxes (min/max of the same values; NaN never
// wins a comparison in either form), so every node box is bit-identical.
struct TriBox { float lo[3], hi[3], c[3]; };

// The reference recursion (bvh.h:48-79) over index ranges: a node's
// triangles are pt[t0, t1) and spheres ps[s0, s1); a split is a stable
// in-place partition (left keys first, order kept, as bvh.h:138-150 fills its
// two vectors), so a leaf's range lists its primitives in the reference's
// order.  Subtrees below a split touch disjoint ranges, so the top levels run
// as concurrent tasks, each into its own node pool (spliced afterwards).
constexpr int kForkMin = 1024;   // a split forks only when both sides have this many primitives

class Builder {
  public:
    // nodes: the shared node array, 2 (triangles + spheres) - 1 slots: a subtree over n primitives
    // (n >= 1) has at most 2n - 1 nodes, so rooted at slot `at` it owns [at, at + 2n - 1) -- the left
    // subtree from at + 1, the right one from at + 2 nl -- and concurrent subtrees write disjoint slots
    // (unused slots stay default nodes, never reached from the root)
    Builder(const HostScene& s, const std::vector<TriBox>& tb, std::vector<int>& pt, std::vector<int>& ps,
            std::atomic<int>* spare, std::vector<BNode>& nodes)
        : nodes(nodes), s_(s), tb_(tb), pt_(pt), ps_(ps), spare_(spare) {}
    std::vector<BNode>& nodes;

    int build(int t0, int t1, int s0, int s1, int depth, int at) {
        if (t0 == t1 && s0 == s1) return -1;
        const int id = at;
        BNode nd;
        nd.depth = depth;
        nd.used = 1;
        bounds(t0, t1, s0, s1, nd.lo, nd.hi);
        int tm = 0, sm = 0;
        bool leaf = (t1 - t0) + (s1 - s0) <= 1 || depth >= kMaxDepth;
        if (!leaf) {
            nd.axis = widest(nd.lo, nd.hi);
            leaf = !split(nd.axis, nd.lo, nd.hi, t0, t1, s0, s1, &tm, &sm);
        }
        if (leaf) {
            nd.t0 = t0; nd.t1 = t1; nd.s0 = s0; nd.s1 = s1;
            nodes[id] = nd;
            return id;
        }
        nodes[id] = nd;
        int r, l;
        const int nl = (tm - t0) + (sm - s0), nr = (t1 - tm) + (s1 - sm);
        const int lat = at + 1, rat = at + 2 * nl;
        if (std::min(nl, nr) >= kForkMin && take_thread(spare_)) {
            Builder rb(s_, tb_, pt_, ps_, spare_, nodes);
            auto fr = std::async(std::launch::async, [&] {
                const int v = rb.build(tm, t1, sm, s1, depth + 1, rat);
                spare_->fetch_add(1);
                return v;
            });
            l = build(t0, tm, s0, sm, depth + 1, lat);
            r = fr.get();
        } else {
            r = build(tm, t1, sm, s1, depth + 1, rat);     // right first (bvh.h:69-70)
            l = build(t0, tm, s0, sm, depth + 1, lat);
        }
        nodes[id].right = r;
        nodes[id].left = l;
        return id;
    }

  private:
    const HostScene& s_;
    const std::vector<TriBox>& tb_;
    std::vector<int>& pt_;
    std::vector<int>& ps_;
    std::atomic<int>* spare_;
    std::vector<int> scratch_;

    // Scene::getBoundingBox + extendBoundingBox (parser.h:272-317)
    void bounds(int t0, int t1, int s0, int s1, V3& lo, V3& hi) const {
        float l[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int i = t0; i < t1; ++i) {
            const TriBox& b = tb_[pt_[i]];
            for (int ax = 0; ax < 3; ++ax) {
                if (b.lo[ax] < l[ax]) l[ax] = b.lo[ax];
                if (b.hi[ax] > h[ax]) h[ax] = b.hi[ax];
            }
        }
        for (int i = s0; i < s1; ++i) {
            const SphereRec& sp = s_.spheres[ps_[i]];
            const V3& c = s_.verts[sp.center_id - 1];
            const float cc[3] = {c.x, c.y, c.z};
            for (int ax = 0; ax < 3; ++ax) {
                if (cc[ax] - sp.radius < l[ax]) l[ax] = cc[ax] - sp.radius;
                if (cc[ax] + sp.radius > h[ax]) h[ax] = cc[ax] + sp.radius;
            }
        }
        lo = V3{l[0], l[1], l[2]};
        hi = V3{h[0], h[1], h[2]};
    }

    static int widest(const V3& lo, const V3& hi) {                           // parser.h:227-235
        int w = 0;
        for (int ax = 1; ax < 3; ++ax)
            if (vget(hi, ax) - vget(lo, ax) > vget(hi, w) - vget(lo, w)) w = ax;
        return w;
    }

    float key_tri(int t, int axis) const { return tb_[t].c[axis]; }
    float key_sph(int k, int axis) const { return vget(s_.verts[s_.spheres[k].center_id - 1], axis); }

    // Stable partition of v[b, e) by pred (true first); returns the split point.
    template <class P>
    int stable_split(std::vector<int>& v, int b, int e, P pred) {
        scratch_.clear();
        int w = b;
        for (int i = b; i < e; ++i) {
            if (pred(v[i])) v[w++] = v[i];
            else scratch_.push_back(v[i]);
        }
        std::copy(scratch_.begin(), scratch_.end(), v.begin() + w);
        return w;
    }

    // BVHNode::partition (bvh.h:111-163): spatial midpoint of the widest axis,
    // moved toward the populated side up to 19 times.  One pass finds the
    // smallest and largest non-NaN key and whether a NaN key exists: "no key
    // < mid" is !(kmin < mid), "every key < mid" is !nan && kmax < mid, so a
    // retry costs O(1) instead of a pass.
    bool split(int axis, const V3& lo, const V3& hi, int t0, int t1, int s0, int s1, int* tm, int* sm) {
        float kmin = INFINITY, kmax = -INFINITY;
        bool nan = false;
        auto see = [&](float k) {
            if (k != k) { nan = true; return; }
            if (k < kmin) kmin = k;
            if (k > kmax) kmax = k;
        };
        for (int i = t0; i < t1; ++i) see(key_tri(pt_[i], axis));
        for (int i = s0; i < s1; ++i) see(key_sph(ps_[i], axis));
        float start = vget(lo, axis), end = vget(hi, axis);
        float mid = (start + end) / 2;
        for (int attempt = 0; attempt < kMaxTries; ++attempt) {
            const bool left_empty = !(kmin < mid);
            const bool right_empty = !nan && kmax < mid;
            if (left_empty) {
                start = mid;
                mid = (start + end) / 2;
            } else if (right_empty) {
                end = mid;
                mid = (start + end) / 2;
            } else {
                *tm = stable_split(pt_, t0, t1, [&](int t) { return key_tri(t, axis) < mid; });
                *sm = stable_split(ps_, s0, s1, [&](int k) { return key_sph(k, axis) < mid; });
                return true;
            }
        }
        return false;
    }
};

constexpr int kMaxWideSlotsHost = dl::kWideSlots;
inline int32_t fbits(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }
inline float ibits(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

// fp16 plane offsets of the wide nodes (dl::Wide): a plane decodes as
// fma(h, 2^e, origin) in f32.  h16_down / h16_up: the largest / smallest
// fp16 value <= / >= x (x >= 0, finite, < 65504 for up), normal or zero
// (offsets below the smallest normal go to 0 / 2^-14, so no decode depends on
// the device's fp16 denormal mode).  Values are returned as floats (exact).
// (Bit arithmetic; the same values as the ldexp / frexp / floor / ceil definitions: for a normal double
// x in [2^E, 2^(E+1)) the fp16 mantissa of floor(x) on the 2^(E-10) grid is its top 10 mantissa bits.)
float h16_value(uint16_t b) {
    const uint32_t ex = (b >> 10) & 31u, man = b & 1023u;
    return ex == 0 ? (float)man * 0x1p-24f : ibits((int32_t)(((ex - 15u + 127u) << 23) | (man << 13)));
}
inline uint64_t dbits(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }
uint16_t h16_down(double x) {
    if (!(x >= 0x1p-14)) return 0;
    if (x >= 65504.0) return 0x7bff;
    const uint64_t u = dbits(x);
    const int E = (int)((u >> 52) & 0x7ff) - 1023;        // x in [2^E, 2^(E+1)), E in [-14, 15]
    return (uint16_t)(((E + 15) << 10) | (int)((u >> 42) & 1023u));
}
uint16_t h16_up(double x) {
    if (!(x > 0.0)) return 0;
    if (x <= 0x1p-14) return (uint16_t)(1 << 10);       // smallest normal
    const uint64_t u = dbits(x);
    int ex = (int)((u >> 52) & 0x7ff) - 1023 + 15;
    int m = 1024 + (int)((u >> 42) & 1023u) + ((u & ((uint64_t(1) << 42) - 1)) != 0 ? 1 : 0);   // [1024, 2048]
    if (m == 2048) { m = 1024; ++ex; }
    if (ex >= 31) return 0x7bff;                         // caller keeps offsets far below 65504
    return (uint16_t)((ex << 10) | (m - 1024));
}

// One wide node's boxes: the slots in `mask` (n slots) quantized as fp16
// offsets from the union box's low corner on a power-of-two scale per axis
// (offsets up to ~2^15, i.e. 11 significant bits of the node's extent).
// Every decoded box is checked, with the device's arithmetic (the fp16 value
// is exact in f32, then one fma), to CONTAIN the child's exact box; false if
// one does not.  Fills origin, exps (with the slot mask) and the plane words.
bool quantize_wide(const float (*lo)[3], const float (*hi)[3], int n, unsigned mask, dl::Wide& w) {
    auto pow2 = [](int x) { return ibits(x << 23); };                       // 2^(x-127), x in [1, 254]
    auto dec = [](float org, uint16_t h, float sc) { return std::fma(h16_value(h), sc, org); };
    float o[3], top[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int a = 0; a < 3; ++a) o[a] = FLT_MAX;
    for (int i = 0; i < n; ++i)
        if (mask >> i & 1u)
            for (int a = 0; a < 3; ++a) { o[a] = std::min(o[a], lo[i][a]); top[a] = std::max(top[a], hi[i][a]); }
    if (mask == 0)
        for (int a = 0; a < 3; ++a) o[a] = top[a] = 0.0f;
    bool ok = true;
    int e[3];
    float sc[3];
    for (int a = 0; a < 3; ++a) {
        const double ext = (double)top[a] - o[a];
        e[a] = 127;
        if (ext > 0) e[a] = std::max(1, std::min(254, (int)std::ceil(std::log2(ext)) - 15 + 127));
        sc[a] = pow2(e[a]);
    }
    // the device's fused slab arithmetic (traverse2.hpp wide_slabs) needs |origin| <= 2^60 and
    // scale <= 2^40 to stay free of overflow; a scene beyond that keeps the binary trees
    for (int a = 0; a < 3; ++a)
        if (!(std::fabs(o[a]) <= 0x1p60f) || !(sc[a] <= 0x1p40f)) ok = false;
    // empty slots: lo = +inf, hi = -inf on every axis, so the device's slab test rejects them by
    // itself (entry +inf, exit -inf, or NaN when a plane product underflows to 0: every comparison
    // false) and needs no slot-mask test
    uint16_t hl[kMaxWideSlotsHost][3], hh[kMaxWideSlotsHost][3];
    for (int i = 0; i < kMaxWideSlotsHost; ++i)
        for (int a = 0; a < 3; ++a) { hl[i][a] = 0x7c00; hh[i][a] = 0xfc00; }
    for (int i = 0; i < n; ++i) {
        if (!(mask >> i & 1u)) continue;
        for (int a = 0; a < 3; ++a) {
            uint16_t ql = h16_down(((double)lo[i][a] - o[a]) / sc[a]);
            while (ql > 0 && dec(o[a], ql, sc[a]) > lo[i][a]) ql = ql == (1 << 10) ? 0 : ql - 1;   // monotone codes
            uint16_t qh = h16_up(((double)hi[i][a] - o[a]) / sc[a]);
            while (qh < 0x7bff && dec(o[a], qh, sc[a]) < hi[i][a]) qh = qh == 0 ? (1 << 10) : qh + 1;
            if (dec(o[a], ql, sc[a]) > lo[i][a] || dec(o[a], qh, sc[a]) < hi[i][a]) ok = false;
            if (ql != 0 && ql < (1 << 10)) ok = false;                          // never a denormal code
            if (qh != 0 && qh < (1 << 10)) ok = false;
            hl[i][a] = ql;
            hh[i][a] = qh;
        }
    }
    w.ox = o[0]; w.oy = o[1]; w.oz = o[2];
    w.exps = (uint32_t)e[0] | (uint32_t)e[1] << 8 | (uint32_t)e[2] << 16 | (mask & 63u) << 24;
    for (int side = 0; side < 2; ++side)
        for (int a = 0; a < 3; ++a)
            for (int pr = 0; pr < 3; ++pr) {
                const uint16_t (*q)[3] = side ? hh : hl;
                w.h[side * 9 + a * 3 + pr] = (uint32_t)q[2 * pr][a] | (uint32_t)q[2 * pr + 1][a] << 16;
            }
    return ok;
}

}  // namespace

// One reference leaf under the occlusion tree: its exact box, the box centre, and the leaf's flat
// (pre-order) node index, resolved to its info word and leaf record once the flatten is done.
struct ShadowLeaf { float lo[3], hi[3], c[3]; int32_t f; };
// The flatten's per-node results the occlusion tree's finish reads, valid once ready() returns true
// (false: the flatten failed and there is nothing to finish).
struct FlatHandoff {
    std::function<bool()> ready;
    const std::vector<int32_t>* leaf_info;
    const std::vector<int32_t>* lrec_of;
};
void build_shadow_tree(FlatBVH& out, int threads, std::vector<ShadowLeaf>& leaves, const FlatHandoff& flat);
bool build_ref_wide(FlatBVH& out);

int build_threads(int requested) {
    if (requested > 0) return std::min(requested, 64);
    if (const char* e = std::getenv("RT_BUILD_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) return std::min(v, 64);
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc, 16u));
}

std::string build_bvh(const HostScene& s, FlatBVH& out, int threads, const std::function<void()>* on_flat) {
    auto t0 = std::chrono::steady_clock::now();
    out = FlatBVH();
    out.threads = build_threads(threads);
    std::vector<TriBox> tb(s.tris.size());
    for (size_t i = 0; i < tb.size(); ++i) {
        const TriRec& tr = s.tris[i];
        TriBox& b = tb[i];
        for (int ax = 0; ax < 3; ++ax) { b.lo[ax] = FLT_MAX; b.hi[ax] = -FLT_MAX; b.c[ax] = vget(tr.center, ax); }
        for (int vid : {tr.v0, tr.v1, tr.v2}) {
            const V3& v = s.verts[vid - 1];
            for (int ax = 0; ax < 3; ++ax) {
                if (vget(v, ax) < b.lo[ax]) b.lo[ax] = vget(v, ax);
                if (vget(v, ax) > b.hi[ax]) b.hi[ax] = vget(v, ax);
            }
        }
    }
    std::vector<int> pt(s.tris.size()), ps(s.spheres.size());
    for (size_t i = 0; i < pt.size(); ++i) pt[i] = (int)i;
    for (size_t i = 0; i < ps.size(); ++i) ps[i] = (int)i;
    std::vector<BNode> bnodes(std::max<size_t>(1, 2 * (pt.size() + ps.size())));
    std::atomic<int> spare(std::max(0, out.threads - 1));
    Builder b(s, tb, pt, ps, &spare, bnodes);
    const int root = b.build(0, (int)pt.size(), 0, (int)ps.size(), 0, 0);
    out.ref_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    out.tri_shade.resize(s.tris.size());
    for (size_t i = 0; i < s.tris.size(); ++i) {
        const TriRec& t = s.tris[i];
        out.tri_shade[i] = dl::TriShade{t.normal.x, t.normal.y, t.normal.z, t.material_id};
    }
    if (root < 0) return "";
    auto tms = [t0] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    double tr_num = 0, tr_sah = 0, tr_off = 0, tr_fill = 0;   // RT_BUILD_TRACE: the flatten's steps, ms from t0

    // Pre-order flatten (bvh.h:81-105): node, left subtree, right subtree.  That is the order of the
    // node slots (Builder: a subtree rooted at slot `at` has its left subtree from at + 1 and its right
    // one after the left's whole slot range), so a node's flat index is the count of used slots before it.
    std::vector<int> flat_of(b.nodes.size(), -1);
    std::vector<int> order;
    order.reserve(b.nodes.size());
    for (size_t i = 0; i < b.nodes.size(); ++i)
        if (b.nodes[i].used) {
            flat_of[i] = (int)order.size();
            order.push_back((int)i);
        }
    // Child-pair layout: one pair per interior node.  The top levels (every
    // walk passes through them) are numbered first, breadth-first, so a
    // kernel can cache pairs [0, top_pairs) in LDS; the rest follow in
    // pre-order, which keeps a node's left-child pair next to its own.  The
    // numbering needs only the tree's shape (interior f: left child f + 1,
    // right child rchild[f]; a leaf: -1), so it comes before the flatten, and
    // so can the occlusion tree's SAH, which reads the leaves in pair order.
    const size_t nn = order.size();
    std::vector<int32_t> rchild(nn, -1);
    for (size_t f = 0; f < nn; ++f) {
        const BNode& n = b.nodes[order[f]];
        if (!(n.left < 0 && n.right < 0)) rchild[f] = flat_of[n.right];   // bvh.h:107-109
    }
    std::vector<int32_t> pair_of(nn, -1), pair_node;
    int32_t npairs = 0;
    {
        std::vector<int> per_level(64, 0);
        for (size_t f = 0; f < nn; ++f)
            if (rchild[f] >= 0) per_level[std::min(b.nodes[order[f]].depth, 63)]++;
        int top_levels = 0, top_count = 0;
        while (top_levels < 63 && top_count + per_level[top_levels] <= dl::kTopPairs && per_level[top_levels] > 0)
            top_count += per_level[top_levels++];
        // level by level, each level left to right (= pre-order within a level): breadth-first
        std::vector<int> cur, nxt;
        if (rchild[0] >= 0) cur.push_back(0);
        for (int lvl = 0; lvl < top_levels && !cur.empty(); ++lvl) {
            nxt.clear();
            for (int f : cur) {
                pair_of[f] = npairs++;
                if (rchild[f + 1] >= 0) nxt.push_back(f + 1);
                if (rchild[rchild[f]] >= 0) nxt.push_back(rchild[f]);
            }
            cur.swap(nxt);
        }
        out.top_pairs = npairs;
        for (size_t f = 0; f < nn; ++f)
            if (rchild[f] >= 0 && pair_of[f] < 0) pair_of[f] = npairs++;
        pair_node.resize(npairs);
        for (size_t f = 0; f < nn; ++f)
            if (pair_of[f] >= 0) pair_node[pair_of[f]] = (int32_t)f;
    }
    tr_num = tms();
    // The occlusion tree's leaves: every leaf child of a pair, in pair order (left, then right).
    std::vector<ShadowLeaf> sleaves;
    sleaves.reserve((size_t)npairs + 1);
    auto add_leaf = [&](int32_t f) {
        const BNode& n = b.nodes[order[f]];
        const float lo[3] = {(float)n.lo.x, (float)n.lo.y, (float)n.lo.z};
        const float hi[3] = {(float)n.hi.x, (float)n.hi.y, (float)n.hi.z};
        ShadowLeaf l;
        for (int a = 0; a < 3; ++a) { l.lo[a] = lo[a]; l.hi[a] = hi[a]; l.c[a] = 0.5f * (lo[a] + hi[a]); }
        l.f = f;
        sleaves.push_back(l);
    };
    for (int32_t i = 0; i < npairs; ++i) {
        const int32_t f = pair_node[i];
        if (rchild[f + 1] < 0) add_leaf(f + 1);
        if (rchild[rchild[f]] < 0) add_leaf(rchild[f]);
    }
    // Large scenes build the occlusion tree's SAH in its own task while this thread flattens; the task
    // then waits for the flatten's leaf info words and records (flat_done; false when the flatten fails,
    // set on every return by `release`) to finish its pairs and wide nodes.
    std::vector<int32_t> leaf_info(nn, 0), lrec_of(nn, -1);
    std::promise<bool> flat_done;
    std::shared_future<bool> flat_ready = flat_done.get_future().share();
    const FlatHandoff hand{[flat_ready] { return flat_ready.get(); }, &leaf_info, &lrec_of};
    double stree_ms = 0.0;
    const int sthreads = std::max(1, out.threads - out.threads / 4);   // the wide tree's quantization takes the rest
    auto shadow = [&out, &stree_ms, &sleaves, &hand, sthreads] {
        const auto ts = std::chrono::steady_clock::now();
        build_shadow_tree(out, sthreads, sleaves, hand);
        stree_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
    };
    std::future<void> fs;
    struct Release {
        std::promise<bool>& p;
        bool done = false;
        void operator()(bool ok) { if (!done) { done = true; p.set_value(ok); } }
        ~Release() { (*this)(false); }   // before fs joins the task (declared after it)
    } release{flat_done};
    if (out.threads > 1 && npairs >= 4096) fs = std::async(std::launch::async, shadow);   // large scenes
    tr_sah = tms();

    // Flatten.  A serial pass in pre-order gives every leaf its first prim slot and its leaf-record
    // offset (the order a serial fill pushes them in) and checks the encodings; the nodes, prims, leaf
    // records and pairs are then filled in parallel (beside the occlusion tree's SAH when it runs).
    out.nodes.resize(nn);
    bool lrec_ok = true;
    {
        size_t np = 0, nrec = 0;
        for (size_t f = 0; f < nn; ++f) {
            const BNode& n = b.nodes[order[f]];
            out.max_depth = std::max(out.max_depth, n.depth);
            if (rchild[f] >= 0) continue;
            const int ntri = n.t1 - n.t0, nsph = n.s1 - n.s0;
            if (ntri > dl::kNtriMask || nsph > dl::kMaxLeafSpheres)
                return "Error: BVH leaf exceeds the device encoding limits";
            out.leaves++;
            out.max_leaf = std::max(out.max_leaf, ntri + nsph);
            dl::Node& o = out.nodes[f];
            o.a = (int32_t)np;
            o.b = dl::kLeafBit | ((int32_t)nsph << dl::kNtriBits) | (int32_t)ntri;
            const size_t count = (size_t)(ntri + nsph);
            // Leaf records (dl::LeafHead + copies of the leaf's prims), one per reference leaf in
            // pre-order (the closest-hit walk's visit order), shared by both 4-wide trees
            if (nrec > (size_t)INT32_MAX - 1 - (2 + 3 * count)) lrec_ok = false;
            lrec_of[f] = (int32_t)nrec;
            np += count;
            nrec += 2 + 3 * count;
        }
        out.prims.resize(np);
        // (+ 3: a leaf's first-prim loads may run past a 0-prim last leaf; zeros)
        out.lrec.resize(lrec_ok ? nrec + 3 : 0);
        if (lrec_ok) std::memset(out.lrec.data() + nrec, 0, 3 * sizeof(dl::Vec4));
    }
    (void)ibits; (void)fbits;
    tr_off = tms();
    // beside the occlusion tree's SAH task (its threads take the cores) the fill runs on this thread alone:
    // more threads only contend with it (C3 on the box: 3.1 ms with 4 threads beside it, 1.9 ms serial)
    const int fth = fs.valid() ? 1 : out.threads;
    parallel_for((int)nn, fth, [&](int f) {
        const BNode& n = b.nodes[order[f]];
        dl::Node& o = out.nodes[f];
        o.minx = n.lo.x; o.miny = n.lo.y; o.minz = n.lo.z;
        o.maxx = n.hi.x; o.maxy = n.hi.y; o.maxz = n.hi.z;
        if (rchild[f] >= 0) {                                        // bvh.h:107-109
            o.a = rchild[f];
            o.b = n.axis;
            return;
        }
        dl::Prim* pp = out.prims.data() + o.a;
        for (int j = n.t0; j < n.t1; ++j) {
            const int t = pt[j];
            const TriRec& tr = s.tris[t];
            const V3 a = s.verts[tr.v0 - 1], bb = s.verts[tr.v1 - 1], c = s.verts[tr.v2 - 1];
            dl::Prim p{};
            p.p0x = a.x; p.p0y = a.y; p.p0z = a.z; p.id = t;
            p.p1x = a.x - bb.x; p.p1y = a.y - bb.y; p.p1z = a.z - bb.z; p.p1w = 0;
            p.p2x = a.x - c.x; p.p2y = a.y - c.y; p.p2z = a.z - c.z; p.p2w = 0;
            *pp++ = p;
        }
        for (int j = n.s0; j < n.s1; ++j) {
            const int k = ps[j];
            const SphereRec& sp = s.spheres[k];
            const V3 c = s.verts[sp.center_id - 1];
            dl::Prim p{};
            p.p0x = c.x; p.p0y = c.y; p.p0z = c.z; p.id = ~k;   // negative id marks a sphere
            p.p1x = sp.radius; p.p1y = sp.radius * sp.radius; p.p1z = 0; p.p1w = 0;
            p.p2x = 0; p.p2y = 0; p.p2z = 0; p.p2w = sp.material_id;
            *pp++ = p;
        }
        if (!lrec_ok) return;
        const int32_t count = (o.b & dl::kNtriMask) + ((o.b >> dl::kNtriBits) & dl::kMaxLeafSpheres);
        dl::LeafHead h{};
        h.minx = o.minx; h.miny = o.miny; h.minz = o.minz; h.count = count;
        h.maxx = o.maxx; h.maxy = o.maxy; h.maxz = o.maxz; h.slot0 = o.a;
        const size_t off = (size_t)lrec_of[f];
        std::memcpy(&out.lrec[off], &h, sizeof(h));
        if (count > 0) std::memcpy(&out.lrec[off + 2], &out.prims[o.a], sizeof(dl::Prim) * (size_t)count);
    });

    tr_fill = tms();
    // a leaf's info word: inline (count and first prim slot) or an index into leaf_big, assigned in the
    // order a serial pairs fill meets the leaves (each leaf is one pair's child; the root last)
    auto leaf_word = [&](size_t f) -> int32_t {
        const dl::Node& n = out.nodes[f];
        const int32_t count = (n.b & dl::kNtriMask) + ((n.b >> dl::kNtriBits) & dl::kMaxLeafSpheres);
        if (count >= 1 && count <= dl::kLeafMaxCount && n.a <= dl::kLeafStartMask)
            return dl::kLeafBit | (count << dl::kLeafCountShift) | n.a;
        out.leaf_big.push_back(dl::LeafBig{n.a, count});
        return dl::kLeafBit | (int32_t)(out.leaf_big.size() - 1);
    };
    for (size_t f = 0; f < nn; ++f) {
        if (rchild[f] < 0) continue;
        if (rchild[f + 1] < 0) leaf_info[f + 1] = leaf_word(f + 1);
        if (rchild[rchild[f]] < 0) leaf_info[rchild[f]] = leaf_word(rchild[f]);
    }
    auto info_of = [&](size_t f) -> int32_t { return rchild[f] >= 0 ? pair_of[f] : leaf_info[f]; };
    out.pairs.resize(npairs);
    out.pair_lrec.assign(2 * (size_t)npairs, -1);
    parallel_for((int)nn, fth, [&](int f) {
        const dl::Node& n = out.nodes[f];
        if (n.b < 0) return;
        const dl::Node& L = out.nodes[f + 1];
        const dl::Node& R = out.nodes[n.a];
        dl::Pair& p = out.pairs[pair_of[f]];
        p.l_minx = L.minx; p.l_miny = L.miny; p.l_minz = L.minz; p.l_info = info_of(f + 1);
        p.l_maxx = L.maxx; p.l_maxy = L.maxy; p.l_maxz = L.maxz; p.axis = n.b;
        p.r_minx = R.minx; p.r_miny = R.miny; p.r_minz = R.minz; p.r_info = info_of(n.a);
        p.r_maxx = R.maxx; p.r_maxy = R.maxy; p.r_maxz = R.maxz; p.pad = 0;
        out.pair_lrec[2 * pair_of[f]] = lrec_of[f + 1];
        out.pair_lrec[2 * pair_of[f] + 1] = lrec_of[n.a];
    });
    if ((int)out.leaf_big.size() > dl::kLeafStartMask) return "Error: too many large BVH leaves";
    out.root_lo[0] = out.nodes[0].minx; out.root_lo[1] = out.nodes[0].miny; out.root_lo[2] = out.nodes[0].minz;
    out.root_hi[0] = out.nodes[0].maxx; out.root_hi[1] = out.nodes[0].maxy; out.root_hi[2] = out.nodes[0].maxz;
    out.root_info = rchild[0] >= 0 ? pair_of[0] : (leaf_info[0] = leaf_word(0));
    out.root_lrec = lrec_of[0];
    if (!lrec_ok) out.lrec.clear();                  // no 4-wide trees: the binary trees only
    release(true);
    if (on_flat) (*on_flat)();
    // The occlusion tree (its own task when threads allow) and the reference-order wide tree are
    // independent: both read the pairs and leaf records, each writes only its own fields.
    const auto t1 = std::chrono::steady_clock::now();
    out.flat_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() - out.ref_ms;
    if (!build_ref_wide(out) || out.lrec.empty()) out.wnodes.clear();
    out.refwide_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    const double tr_wide = tms();
    if (fs.valid()) fs.get(); else shadow();
    out.stree_ms = stree_ms;
    if (std::getenv("RT_BUILD_TRACE"))
        std::fprintf(stderr, "build: ref %.2f numbering %.2f leaves+sah start %.2f offsets %.2f fill %.2f pairs %.2f "
                             "refwide %.2f stree joined %.2f (ms from start)\n",
                     out.ref_ms, tr_num, tr_sah, tr_off, tr_fill, out.ref_ms + out.flat_ms, tr_wide, tms());
    // Ordered DFS pushes two children per interior pop: stack <= depth + 2.
    out.max_stack = out.max_depth + 2;
    if (out.max_stack > dl::kMaxStack) return "Error: BVH deeper than the device stack";
    if (out.smax_depth + 2 > dl::kMaxStack) return "Error: occlusion tree deeper than the device stack";
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return "";
}

// Occlusion (any-hit) tree.  The reference's any-hit answer is "some
// primitive of a leaf whose box the ray hits has t < dist" (raytracer.cpp:
// 227-280: no t pruning, the first such primitive in any order ends the
// walk).  For a NaN-free ray the slab test is monotone under box nesting
// (subtract and multiply are monotone in the plane coordinate), so a leaf
// box hit implies every enclosing box is hit: the reference's reachable
// leaves are exactly the leaves whose own box is hit, whatever hierarchy sits
// above them.  This tree keeps the reference's leaves (same prim ranges, same
// exact leaf boxes, tested exactly) and puts a binned-SAH hierarchy of union
// boxes above them, so shadow rays visit far fewer nodes with the same
// answers.  Kernels use it only for NaN-free rays outside counting passes.
void build_shadow_tree(FlatBVH& out, int threads, std::vector<ShadowLeaf>& leaves, const FlatHandoff& flat) {
    const auto T0 = std::chrono::steady_clock::now();
    auto since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    double t_sah = 0, t_wait = 0, t_shape = 0;
    using Leaf = ShadowLeaf;
    out.spairs.clear();
    out.smax_depth = 0;
    if (leaves.size() < 2) {           // empty tree or a single root leaf: same as the reference
        if (!flat.ready()) return;
        for (int a = 0; a < 3; ++a) { out.sroot_lo[a] = out.root_lo[a]; out.sroot_hi[a] = out.root_hi[a]; }
        out.sroot_info = out.root_info;
        return;
    }
    struct Box {
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        void grow(const float* l, const float* h) {
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], l[a]); hi[a] = std::max(hi[a], h[a]); }
        }
        double area() const {
            const double dx = std::max(0.0, (double)hi[0] - lo[0]), dy = std::max(0.0, (double)hi[1] - lo[1]),
                         dz = std::max(0.0, (double)hi[2] - lo[2]);
            return dx * dy + dy * dz + dz * dx;
        }
    };
    // binned SAH over leaf centroids; each tree leaf is one reference leaf.  The leaves themselves are
    // partitioned in place (std::partition's swaps depend only on the predicate, so the order -- and
    // with it the count split of equal centroids -- is what partitioning an index array gave, and the
    // tree is bit-identical to it), so every pass reads them sequentially; a node's box and centroid
    // box are one pass, the three axes' bins another.
    struct TNode { Box box; int left = -1, right = -1, axis = 0; int32_t info = 0, rec = -1; };
    // Subtrees are independent (disjoint ranges of the leaf array), and a subtree over leaves [b, e) has
    // exactly 2(e - b) - 1 nodes: rooted at node slot `at`, it takes slots [at, at + 2(e - b) - 1) of
    // one array (the left subtree from at + 1, the right one from at + 2(mid - b)), so the top levels run
    // as concurrent tasks that write disjoint slots, with no per-task pools to splice.
    struct Sah {
        std::vector<Leaf>& lv;
        std::atomic<int>* spare;   // threads that may still be started (a task returns its own when done)
        std::vector<TNode>& tn;
        int smax_depth = 0;
        int (*fn)(Sah&, int, int, int, int);
        int build(int b, int e, int depth, int at) { return fn(*this, b, e, depth, at); }
    };
    auto sah_build = [](Sah& me_, int b, int e, int depth, int at) -> int {
        std::vector<Leaf>& lv = me_.lv;
        std::vector<TNode>& tn = me_.tn;
        TNode node;
        Box cb;
        for (int i = b; i < e; ++i) {
            node.box.grow(lv[i].lo, lv[i].hi);
            cb.grow(lv[i].c, lv[i].c);
        }
        me_.smax_depth = std::max(me_.smax_depth, depth);
        const int me = at;
        tn[me] = node;
        if (e - b == 1) {
            tn[me].rec = lv[b].f;          // the flat index until the flatten's words resolve it
            return me;
        }
        if (e - b == 2) {
            // two leaves: what the binned code below gives, without its bins.  Each live axis puts the
            // leaves in bins 0 and 1 at the same cost (the two leaf areas), so the first live axis wins
            // the strict comparison; the leaf of bin 0 goes left; no finite cost (or no live axis): a
            // count split on axis 0 with the leaves as they are.
            int axis = -1;
            for (int a = 0; a < 3 && axis < 0; ++a)
                if ((double)cb.hi[a] - cb.lo[a] > 0) axis = a;
            Box A, B;
            A.grow(lv[b].lo, lv[b].hi);
            B.grow(lv[b + 1].lo, lv[b + 1].hi);
            if (axis >= 0 && A.area() * 1 + B.area() * 1 < 1e300) {
                const double ex = (double)cb.hi[axis] - cb.lo[axis];
                int k = (int)((lv[b].c[axis] - cb.lo[axis]) / ex * 2);
                k = std::min(1, std::max(0, k));
                if (k != 0) std::swap(lv[b], lv[b + 1]);
            } else {
                axis = 0;
            }
            tn[me].left = me_.build(b, b + 1, depth + 1, at + 1);
            tn[me].right = me_.build(b + 1, e, depth + 1, at + 2);
            tn[me].axis = axis;
            return me;
        }
        constexpr int kMaxBins = 32;
        const int kBins = std::min(kMaxBins, e - b);   // O(n) per node: small nodes use fewer bins
        double best = 1e300;
        int best_axis = -1, best_split = 0;
        // only the kBins bins in use are initialised (most nodes are small).  Large nodes bin into two
        // interleaved copies (even / odd items) merged afterwards: neighbouring leaves fall in the same bin,
        // and one copy makes every grow wait on the previous one's stores.  (min / max of the same values in
        // any order: the same box.)
        const int ncopy = e - b >= 256 ? 2 : 1;
        alignas(Box) unsigned char bb_raw[2 * 3 * kMaxBins * sizeof(Box)];
        Box* const bb = reinterpret_cast<Box*>(bb_raw);
        int cnt[2][3][kMaxBins];
        double ext[3];
        bool live[3];
        for (int a = 0; a < 3; ++a) {
            ext[a] = (double)cb.hi[a] - cb.lo[a];
            live[a] = ext[a] > 0;
            for (int cp = 0; cp < ncopy; ++cp)
                for (int k = 0; k < kBins; ++k) { new (&bb[(cp * 3 + a) * kMaxBins + k]) Box(); cnt[cp][a][k] = 0; }
        }
        for (int i = b; i < e; ++i) {
            const Leaf& l = lv[i];
            const int cp = ncopy > 1 ? (i & 1) : 0;
            for (int a = 0; a < 3; ++a) {
                if (!live[a]) continue;
                int k = (int)((l.c[a] - cb.lo[a]) / ext[a] * kBins);
                k = std::min(kBins - 1, std::max(0, k));
                bb[(cp * 3 + a) * kMaxBins + k].grow(l.lo, l.hi);
                cnt[cp][a][k]++;
            }
        }
        if (ncopy > 1)
            for (int a = 0; a < 3; ++a)
                for (int k = 0; k < kBins; ++k) {
                    bb[a * kMaxBins + k].grow(bb[(3 + a) * kMaxBins + k].lo, bb[(3 + a) * kMaxBins + k].hi);
                    cnt[0][a][k] += cnt[1][a][k];
                }
        for (int a = 0; a < 3; ++a) {
            if (!live[a]) continue;
            const Box* const ba = bb + a * kMaxBins;
            // (an area is recomputed only where its box grew: an empty bin leaves it, and the empty box's
            // area is 0)
            double right_area[kMaxBins];
            int right_cnt[kMaxBins];
            Box acc;
            double ra = 0.0;
            int n = 0;
            for (int k = kBins - 1; k > 0; --k) {
                if (cnt[0][a][k]) { acc.grow(ba[k].lo, ba[k].hi); ra = acc.area(); }
                n += cnt[0][a][k];
                right_area[k] = ra;
                right_cnt[k] = n;
            }
            Box lacc;
            double la = 0.0;
            int ln = 0;
            for (int k = 1; k < kBins; ++k) {
                if (cnt[0][a][k - 1]) { lacc.grow(ba[k - 1].lo, ba[k - 1].hi); la = lacc.area(); }
                ln += cnt[0][a][k - 1];
                if (ln == 0 || right_cnt[k] == 0) continue;
                const double cost = la * ln + right_area[k] * right_cnt[k];
                if (cost < best) { best = cost; best_axis = a; best_split = k; }
            }
        }
        int mid;
        int axis = best_axis;
        if (best_axis < 0) {                       // all centroids equal: split by count
            axis = 0;
            mid = (b + e) / 2;
        } else {
            const double ex = ext[axis];
            const float lo_a = cb.lo[axis];
            auto it = std::partition(lv.begin() + b, lv.begin() + e, [&](const Leaf& l) {
                int k = (int)((l.c[axis] - lo_a) / ex * kBins);
                k = std::min(kBins - 1, std::max(0, k));
                return k < best_split;
            });
            mid = (int)(it - lv.begin());
            if (mid == b || mid == e) mid = (b + e) / 2;
        }
        int l, r;
        if (std::min(mid - b, e - mid) >= kForkMinSah && take_thread(me_.spare)) {
            Sah rb{lv, me_.spare, tn, 0, me_.fn};
            const int rat = at + 2 * (mid - b);
            auto fr = std::async(std::launch::async, [&rb, mid, e, depth, rat] {
                const int v = rb.build(mid, e, depth + 1, rat);
                rb.spare->fetch_add(1);
                return v;
            });
            l = me_.build(b, mid, depth + 1, at + 1);
            r = fr.get();
            me_.smax_depth = std::max(me_.smax_depth, rb.smax_depth);
        } else {
            l = me_.build(b, mid, depth + 1, at + 1);
            r = me_.build(mid, e, depth + 1, at + 2 * (mid - b));
        }
        tn[me].left = l;
        tn[me].right = r;
        tn[me].axis = axis;
        return me;
    };
    std::vector<TNode> tn(2 * leaves.size());
    std::atomic<int> spare(std::max(0, threads - 1));
    Sah top{leaves, &spare, tn, 0, +sah_build};
    const int root = top.build(0, (int)leaves.size(), 0, 0);
    out.smax_depth = top.smax_depth;
    t_sah = since(T0);
    if (!flat.ready()) return;
    t_wait = since(T0);
    for (size_t n = 0; n + 1 < tn.size(); ++n)     // the 2L - 1 nodes: leaf info words and records
        if (tn[n].left < 0) {
            const int32_t f = tn[n].rec;
            tn[n].info = (*flat.leaf_info)[f];
            tn[n].rec = (*flat.lrec_of)[f];
        }
    // pairs in pre-order of interior nodes: the order of their slots (a subtree at slot `at` has its
    // left subtree from at + 1 and its right one after the left's whole range), so a count, no walk
    std::vector<int32_t> pair_of(tn.size(), -1);
    int32_t np = 0;
    for (size_t n = 0; n + 1 < tn.size(); ++n)
        if (tn[n].left >= 0) pair_of[n] = np++;
    auto info = [&](int n) { return tn[n].left < 0 ? tn[n].info : pair_of[n]; };
    out.spairs.resize(np);
    parallel_for((int)tn.size(), threads, [&](int n) {
        if (tn[n].left < 0) return;
        const TNode& L = tn[tn[n].left];
        const TNode& R = tn[tn[n].right];
        dl::Pair& p = out.spairs[pair_of[n]];
        p.l_minx = L.box.lo[0]; p.l_miny = L.box.lo[1]; p.l_minz = L.box.lo[2]; p.l_info = info(tn[n].left);
        p.l_maxx = L.box.hi[0]; p.l_maxy = L.box.hi[1]; p.l_maxz = L.box.hi[2]; p.axis = tn[n].axis;
        p.r_minx = R.box.lo[0]; p.r_miny = R.box.lo[1]; p.r_minz = R.box.lo[2]; p.r_info = info(tn[n].right);
        p.r_maxx = R.box.hi[0]; p.r_maxy = R.box.hi[1]; p.r_maxz = R.box.hi[2]; p.pad = 0;
    });
    for (int a = 0; a < 3; ++a) { out.sroot_lo[a] = tn[root].box.lo[a]; out.sroot_hi[a] = tn[root].box.hi[a]; }
    out.sroot_info = info(root);

    // Wide collapse (dl::Wide, quantize_wide: every decoded box contains the
    // child's box, all the any-hit argument needs): a node's slots are a
    // frontier below an SAH node, grown by replacing the interior slot of
    // largest box area by its two children.  Leaves are the shared leaf records.
    // The shape (slots, child codes, pre-order node numbers) is one cheap serial
    // recursion; the quantization of every node runs in parallel.
    out.swnodes.clear();
    out.swmax_stack = 0;
    bool contain_ok = !out.lrec.empty();
    struct Shape { int n = 0; int ch[dl::kWideSlots]; int32_t code[dl::kWideSlots]; };
    std::vector<Shape> shapes;
    shapes.reserve(leaves.size());
    // returns the node code; *stack = worst-case stack entries of a walk from here down
    std::function<int32_t(int, int*)> shape = [&](int n, int* stack) -> int32_t {
        const TNode& t = tn[n];
        *stack = 0;
        if (t.left < 0) {
            if (t.rec < 0) contain_ok = false;
            return dl::kLeafBit | t.rec;
        }
        int ch[dl::kWideSlots] = {t.left, t.right};
        int nch = 2;
        while (nch < dl::kWideSlots) {
            int best = -1;
            double ba = -1.0;
            for (int i = 0; i < nch; ++i)
                if (tn[ch[i]].left >= 0 && tn[ch[i]].box.area() > ba) { ba = tn[ch[i]].box.area(); best = i; }
            if (best < 0) break;
            const int c = ch[best];
            for (int i = nch; i > best + 1; --i) ch[i] = ch[i - 1];
            ch[best] = tn[c].left;
            ch[best + 1] = tn[c].right;
            ++nch;
        }
        const int me = (int)shapes.size();
        shapes.emplace_back();
        int deepest = 0;
        Shape sh;
        sh.n = nch;
        for (int i = 0; i < nch; ++i) {
            int st = 0;
            sh.ch[i] = ch[i];
            sh.code[i] = shape(ch[i], &st);
            deepest = std::max(deepest, st);
        }
        shapes[me] = sh;
        *stack = nch - 1 + deepest;        // a step pushes at most n - 1, then goes below one
        return me;
    };
    const double t_pairs = since(T0);
    int stack = 0;
    out.swroot = shape(root, &stack);
    out.swmax_stack = stack + 1;
    t_shape = since(T0);
    out.swnodes.resize(shapes.size());
    std::vector<char> qok(shapes.size(), 1);
    parallel_for((int)shapes.size(), threads, [&](int i) {
        const Shape& sh = shapes[i];
        dl::Wide w{};
        float lo[dl::kWideSlots][3] = {}, hi[dl::kWideSlots][3] = {};
        for (int j = 0; j < dl::kWideSlots; ++j) w.child[j] = INT32_MAX;
        for (int j = 0; j < sh.n; ++j) {
            w.child[j] = sh.code[j];
            for (int a = 0; a < 3; ++a) { lo[j][a] = tn[sh.ch[j]].box.lo[a]; hi[j][a] = tn[sh.ch[j]].box.hi[a]; }
        }
        if (!quantize_wide(lo, hi, sh.n, (1u << sh.n) - 1u, w)) qok[i] = 0;
        out.swnodes[i] = w;
    });
    for (char q : qok) contain_ok = contain_ok && q;
    if (std::getenv("RT_BUILD_TRACE"))          // diagnostics: the occlusion tree's phases, ms from its start
        std::fprintf(stderr, "stree: sah %.2f flatten-wait %.2f pairs %.2f shape %.2f quantize %.2f (%zu leaves, %zu nodes)\n",
                     t_sah, t_wait, t_pairs, t_shape, since(T0), leaves.size(), shapes.size());
    if (!contain_ok || out.swmax_stack > dl::kMaxStack) out.swnodes.clear();   // binary occlusion tree only
}

// Reference-order wide tree for closest-hit walks: the reference BVH collapsed
// to dl::Wide nodes of up to dl::kWideSlots children.  The node of interior
// node N holds a frontier of nodes below N, grown from N's two children by
// repeatedly replacing the interior slot of largest box area by its two
// children (as the occlusion tree's collapse does), slots kept in pre-order.
// The reference visits the nodes below N in DFS order, the left child first
// iff d[axis] > 0 at every expanded node (raytracer.cpp:200-206), so the
// visiting order of the slots is a function of the octant of d alone: the
// node stores, per octant, each slot's rank in that order.  The walk over it
// (traverse2.hpp wide_closest_step) is exact for NaN-free rays: it visits the
// reference's leaves in the reference's order with the same tMax (see there).
// Returns false when a decoded box does not contain its child's box or a walk
// could overflow the device stack (the walk then keeps the binary tree).
bool build_ref_wide(FlatBVH& out) {
    constexpr int W = dl::kWideSlots;
    out.wnodes.clear();
    out.wmax_stack = 0;
    if (out.nodes.empty()) return true;
    if (out.root_info < 0) {                 // a single leaf
        out.wroot = dl::kLeafBit | out.root_lrec;
        return out.root_lrec >= 0;
    }
    bool ok = true;
    struct Slot { int32_t info, rec; float lo[3], hi[3]; };   // info: pair index or < 0 (leaf)
    auto kids = [&](int32_t pi, Slot* a, Slot* b) {
        const dl::Pair& P = out.pairs[pi];
        *a = Slot{P.l_info, out.pair_lrec[2 * pi], {P.l_minx, P.l_miny, P.l_minz}, {P.l_maxx, P.l_maxy, P.l_maxz}};
        *b = Slot{P.r_info, out.pair_lrec[2 * pi + 1], {P.r_minx, P.r_miny, P.r_minz}, {P.r_maxx, P.r_maxy, P.r_maxz}};
        return P.axis;
    };
    auto area = [](const Slot& c) {
        const double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1], dz = (double)c.hi[2] - c.lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    // expansion tree over slot ranges: split (axis, lo, mid, hi) cuts [lo, hi) at mid
    struct Split { int axis, lo, mid, hi; };
    // A node's shape: its slots, the splits that produced them and the child codes.  The shapes come
    // from one serial recursion (pre-order node numbers); the rank words and quantization of every
    // node run in parallel.
    struct Shape { int n = 0; Slot fr[W]; Split sp[W]; int nsp = 0; int32_t code[W]; };
    std::vector<Shape> shapes;
    shapes.reserve(out.pairs.size() / 2 + 1);
    // returns the node index; *stack = worst-case stack entries of a walk from this node down
    std::function<int32_t(int32_t, int*)> shape = [&](int32_t pi, int* stack) -> int32_t {
        Shape sh;
        sh.n = 2;
        sh.sp[0] = {kids(pi, &sh.fr[0], &sh.fr[1]), 0, 1, 2};
        sh.nsp = 1;
        while (sh.n < W) {
            int best = -1;
            double ba = -1.0;
            for (int i = 0; i < sh.n; ++i)
                if (sh.fr[i].info >= 0 && area(sh.fr[i]) > ba) { ba = area(sh.fr[i]); best = i; }
            if (best < 0) break;
            Slot a, b;
            const int ax = kids(sh.fr[best].info, &a, &b);
            for (int i = sh.n; i > best + 1; --i) sh.fr[i] = sh.fr[i - 1];
            sh.fr[best] = a;
            sh.fr[best + 1] = b;
            ++sh.n;
            for (int k = 0; k < sh.nsp; ++k) {
                Split& e = sh.sp[k];
                if (e.lo > best) e.lo++;
                if (e.mid > best) e.mid++;
                if (e.hi > best) e.hi++;
            }
            sh.sp[sh.nsp++] = {ax, best, best + 1, best + 2};
        }
        const int me = (int)shapes.size();
        shapes.emplace_back();
        int deepest = 0;
        for (int i = 0; i < sh.n; ++i) {
            if (sh.fr[i].info < 0) {
                if (sh.fr[i].rec < 0) ok = false;
                sh.code[i] = dl::kLeafBit | sh.fr[i].rec;
            } else {
                int st = 0;
                sh.code[i] = shape(sh.fr[i].info, &st);
                deepest = std::max(deepest, st);
            }
        }
        shapes[me] = sh;
        // a step pushes at most n - 1 entries, then continues below one of them
        *stack = sh.n - 1 + deepest;
        return me;
    };
    int stack = 0;
    out.wroot = shape(out.root_info, &stack);
    out.wmax_stack = stack + 1;
    out.wnodes.resize(shapes.size());
    std::vector<char> nok(shapes.size(), 1);
    parallel_for((int)shapes.size(), std::max(1, out.threads / 4), [&](int idx) {   // beside the occlusion tree's build
        const Shape& sh = shapes[idx];
        const int n = sh.n;
        bool good = true;
        dl::Wide w{};
        // ranks for the octants o = 0..3 (d[2] <= 0); an octant o >= 4 visits in the reverse order of o ^ 7
        for (int oct = 0; oct < 8; ++oct) {
            int order[dl::kWideSlots], no = 0;
            // the DFS over the splits (left first iff d[axis] > 0), iteratively: a stack of slot ranges
            int rs[2 * W][2], nr = 0;
            rs[nr][0] = 0; rs[nr][1] = n; ++nr;
            while (nr > 0) {
                --nr;
                const int lo = rs[nr][0], hi = rs[nr][1];
                if (hi - lo == 1) { if (no < dl::kWideSlots) order[no++] = lo; continue; }
                int k = 0;
                while (k < sh.nsp && !(sh.sp[k].lo == lo && sh.sp[k].hi == hi)) ++k;
                if (k == sh.nsp || nr + 2 > 2 * W) { good = false; break; }
                const Split& e = sh.sp[k];
                const bool left_first = (oct >> e.axis) & 1;
                // pushed in reverse: the first visited range on top
                if (left_first) { rs[nr][0] = e.mid; rs[nr][1] = e.hi; ++nr; rs[nr][0] = e.lo; rs[nr][1] = e.mid; ++nr; }
                else { rs[nr][0] = e.lo; rs[nr][1] = e.mid; ++nr; rs[nr][0] = e.mid; rs[nr][1] = e.hi; ++nr; }
            }
            if (no != n) good = false;
            uint32_t rw = 0;
            for (int r = 0; r < no; ++r) rw |= (uint32_t)r << (3 * order[r]);
            for (int j = n; j < dl::kWideSlots; ++j) rw |= (uint32_t)(n - 1) << (3 * j);   // empty: never valid
            if (oct < 4) {
                w.rank[oct] = rw;
            } else {                        // check the reversal the device relies on (real slots)
                const uint32_t all = 01111111u & ((1u << (3 * dl::kWideSlots)) - 1u);   // one per 3-bit field
                const uint32_t real = (1u << (3 * n)) - 1u;
                if ((rw & real) != (((uint32_t)(n - 1) * all - w.rank[oct ^ 7]) & real)) good = false;
            }
        }
        float lo[dl::kWideSlots][3] = {}, hi[dl::kWideSlots][3] = {};
        for (int i = 0; i < dl::kWideSlots; ++i) w.child[i] = INT32_MAX;
        for (int i = 0; i < n; ++i) {
            std::memcpy(lo[i], sh.fr[i].lo, sizeof(lo[i]));
            std::memcpy(hi[i], sh.fr[i].hi, sizeof(hi[i]));
            w.child[i] = sh.code[i];
        }
        if (!quantize_wide(lo, hi, n, (1u << n) - 1u, w)) good = false;
        out.wnodes[idx] = w;
        nok[idx] = good ? 1 : 0;
    });
    for (char g : nok) ok = ok && g;
    return ok && out.wmax_stack <= dl::kMaxStack;
}

}  // namespace rtx
