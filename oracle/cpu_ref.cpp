/*
 * oracle/cpu_ref.cpp -- CPU restatement of nemjit001/surf-path-tracer's CPU path
 * tracer (the parity oracle and the timed CPU baseline).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing under surf-path-tracer_amd/ links it.
 *
 * Parity UNPINNED against a run of the reference (see cpu_ref.h for why and for
 * what pins it instead).  Every function cites the reference file:line whose
 * behaviour it restates (paths relative to the reference repository root).
 *
 * Floating point: compile with -O2 -ffp-contract=off -fno-fast-math (x86-64 SSE,
 * no FMA), the arithmetic g++ gives the reference's own sources.  Operation
 * order follows the reference expression by expression; libm sinf/cosf/expf/tanf
 * are called exactly where the reference calls them.
 */
#include "cpu_ref.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <chrono>
#include <omp.h>
#include <zlib.h>

namespace {

/* ---------------------------------------------------------------- math -- */
/* surf_math.h:13-23 */
const float kFarAway = 1e30f;
const float kEps = 1e-5f;
const float kPi = 3.14159265358979323846264f;
const float kInvPi = 0.31830988618379067153777f;
const float k2Pi = 6.28318530717958647692528f;
const uint32_t kUnset = ~0u;

struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };

inline V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
inline V3 splat(float s) { return mk(s, s, s); }
inline V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator/(V3 a, V3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
inline V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
/* F32 * Float3 goes through Float3(F32) and the component product. */
inline V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
inline V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      /* surf_math.h:160 */
inline V3 cross(V3 a, V3 b) {                                                   /* surf_math.h:163-170 */
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float rsq(float x) { return 1.0f / sqrtf(x); }                           /* surf_math.h:96 */
inline V3 normalize(V3 a) { float inv = rsq(dot(a, a)); return a * inv; }       /* surf_math.h:161 */
inline float magnitude(V3 a) { return sqrtf(dot(a, a)); }
/* ternary min/max: NaN behaviour of the reference (surf_math.h:104-117) */
inline float tmin(float a, float b) { return a < b ? a : b; }
inline float tmax(float a, float b) { return a > b ? a : b; }
inline V3 vmin(V3 a, V3 b) { return mk(tmin(a.x, b.x), tmin(a.y, b.y), tmin(a.z, b.z)); }
inline V3 vmax(V3 a, V3 b) { return mk(tmax(a.x, b.x), tmax(a.y, b.y), tmax(a.z, b.z)); }
inline float clampf(float a, float lo, float hi) { return a < lo ? lo : (a > hi ? hi : a); }
inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
/* reflect, surf_math.h:225 */
inline V3 reflect(V3 d, V3 n) { return d - (2.0f * dot(n, d)) * n; }
/* depthInBounds, surf_math.h:227 */
inline bool depthOk(float t, float maxT) { return kEps <= t && t < maxT; }
/* radians, surf_math.h:231 */
inline float radiansf(float deg) { return (deg * kPi) * 0.005555555555555f; }

/* ------------------------------------------------------- RNG  (surf_math.cpp) */
uint32_t wang(uint32_t s) {                                                     /* :31-42 */
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
inline uint32_t seedOf(uint32_t s) { return wang((s + 1u) * 0x11u); }          /* :44-47 */
inline uint32_t rndU(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; } /* :57-63 */
inline float rndF(uint32_t& s) { return (float)rndU(s) * 2.3283064365387e-10f; } /* :70-73 */
inline float rndRange(uint32_t& s, float lo, float hi) { float r = hi - lo; return (rndF(s) * r) + lo; } /* :81-85 */
inline uint32_t rndRangeU(uint32_t& s, uint32_t lo, uint32_t hi) { return (rndU(s) + lo) % hi; }       /* :92-95 */

/* ------------------------------------------------------------ glm subset --
 * Matrix arithmetic of glm 0.9.9 (column major, non-SIMD code path).  The
 * reference's glm submodule commit is unrecoverable: this arithmetic is
 * "parity unpinned" (SURVEY.md 8c). */
struct M4 { float c[4][4]; };
M4 identity() { M4 m; memset(&m, 0, sizeof m); for (int i = 0; i < 4; ++i) m.c[i][i] = 1.0f; return m; }
inline V4 mul(const M4& m, V4 v) {
    /* type_mat4x4.inl operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
    V4 r; float* o = &r.x;
    for (int i = 0; i < 4; ++i)
        o[i] = (m.c[0][i] * v.x + m.c[1][i] * v.y) + (m.c[2][i] * v.z + m.c[3][i] * v.w);
    return r;
}
M4 translate(const M4& m, V3 v) {                /* matrix_transform.inl translate */
    M4 r = m;
    for (int i = 0; i < 4; ++i)
        r.c[3][i] = ((m.c[0][i] * v.x + m.c[1][i] * v.y) + m.c[2][i] * v.z) + m.c[3][i];
    return r;
}
M4 scale(const M4& m, V3 v) {                    /* matrix_transform.inl scale */
    M4 r = m;
    for (int i = 0; i < 4; ++i) { r.c[0][i] = m.c[0][i] * v.x; r.c[1][i] = m.c[1][i] * v.y; r.c[2][i] = m.c[2][i] * v.z; }
    return r;
}
M4 rotate(const M4& m, float angle, V3 v) {      /* matrix_transform.inl rotate */
    const float c = cosf(angle), s = sinf(angle);
    float inv = 1.0f / sqrtf((v.x * v.x + v.y * v.y) + v.z * v.z);
    V3 ax = mk(v.x * inv, v.y * inv, v.z * inv);
    V3 tp = mk((1.0f - c) * ax.x, (1.0f - c) * ax.y, (1.0f - c) * ax.z);
    float R[3][3];
    R[0][0] = c + tp.x * ax.x;  R[0][1] = tp.x * ax.y + s * ax.z;  R[0][2] = tp.x * ax.z - s * ax.y;
    R[1][0] = tp.y * ax.x - s * ax.z;  R[1][1] = c + tp.y * ax.y;  R[1][2] = tp.y * ax.z + s * ax.x;
    R[2][0] = tp.z * ax.x + s * ax.y;  R[2][1] = tp.z * ax.y - s * ax.x;  R[2][2] = c + tp.z * ax.z;
    M4 r;
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 4; ++i)
            r.c[k][i] = (m.c[0][i] * R[k][0] + m.c[1][i] * R[k][1]) + m.c[2][i] * R[k][2];
    for (int i = 0; i < 4; ++i) r.c[3][i] = m.c[3][i];
    return r;
}
M4 inverse(const M4& m) {                        /* func_matrix.inl compute_inverse<4,4> */
    auto M = [&](int a, int b) { return m.c[a][b]; };
    float c00 = M(2,2) * M(3,3) - M(3,2) * M(2,3), c02 = M(1,2) * M(3,3) - M(3,2) * M(1,3), c03 = M(1,2) * M(2,3) - M(2,2) * M(1,3);
    float c04 = M(2,1) * M(3,3) - M(3,1) * M(2,3), c06 = M(1,1) * M(3,3) - M(3,1) * M(1,3), c07 = M(1,1) * M(2,3) - M(2,1) * M(1,3);
    float c08 = M(2,1) * M(3,2) - M(3,1) * M(2,2), c10 = M(1,1) * M(3,2) - M(3,1) * M(1,2), c11 = M(1,1) * M(2,2) - M(2,1) * M(1,2);
    float c12 = M(2,0) * M(3,3) - M(3,0) * M(2,3), c14 = M(1,0) * M(3,3) - M(3,0) * M(1,3), c15 = M(1,0) * M(2,3) - M(2,0) * M(1,3);
    float c16 = M(2,0) * M(3,2) - M(3,0) * M(2,2), c18 = M(1,0) * M(3,2) - M(3,0) * M(1,2), c19 = M(1,0) * M(2,2) - M(2,0) * M(1,2);
    float c20 = M(2,0) * M(3,1) - M(3,0) * M(2,1), c22 = M(1,0) * M(3,1) - M(3,0) * M(1,1), c23 = M(1,0) * M(2,1) - M(2,0) * M(1,1);
    float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    float V0[4] = {M(1,0), M(0,0), M(0,0), M(0,0)}, V1[4] = {M(1,1), M(0,1), M(0,1), M(0,1)};
    float V2[4] = {M(1,2), M(0,2), M(0,2), M(0,2)}, V3_[4] = {M(1,3), M(0,3), M(0,3), M(0,3)};
    float I0[4], I1[4], I2[4], I3[4];
    for (int i = 0; i < 4; ++i) {
        I0[i] = (V1[i] * F0[i] - V2[i] * F1[i]) + V3_[i] * F2[i];
        I1[i] = (V0[i] * F0[i] - V2[i] * F3[i]) + V3_[i] * F4[i];
        I2[i] = (V0[i] * F1[i] - V1[i] * F3[i]) + V3_[i] * F5[i];
        I3[i] = (V0[i] * F2[i] - V1[i] * F4[i]) + V2[i] * F5[i];
    }
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    M4 inv;
    for (int i = 0; i < 4; ++i) { inv.c[0][i] = I0[i] * SA[i]; inv.c[1][i] = I1[i] * SB[i]; inv.c[2][i] = I2[i] * SA[i]; inv.c[3][i] = I3[i] * SB[i]; }
    float d0 = m.c[0][0] * inv.c[0][0], d1 = m.c[0][1] * inv.c[1][0], d2 = m.c[0][2] * inv.c[2][0], d3 = m.c[0][3] * inv.c[3][0];
    float det = (d0 + d1) + (d2 + d3);
    float oneOver = 1.0f / det;
    for (int k = 0; k < 4; ++k) for (int i = 0; i < 4; ++i) inv.c[k][i] = inv.c[k][i] * oneOver;
    return inv;
}
inline V3 xyz(V4 v) { return mk(v.x, v.y, v.z); }
inline V4 v4(V3 a, float w) { V4 r; r.x = a.x; r.y = a.y; r.z = a.z; r.w = w; return r; }

/* --------------------------------------------------------------- OBJ load --
 * tinyobjloader semantics the reference relies on (mesh.cpp:69-154): v / vt /
 * vn records, 1-based or negative indices, triangulate = true.  Quads are split
 * on the shorter diagonal, ties -> [0,1,3],[1,2,3] (tinyobjloader 2.x); larger
 * polygons fan from vertex 0.  Only plane.obj has a quad.  (Parity unpinned:
 * the tinyobjloader commit is unrecoverable.) */
struct ObjIdx { int v, t, n; };
bool readAll(const std::string& path, std::string& out) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) return false;
    char buf[1 << 16];
    int k;
    while ((k = gzread(f, buf, sizeof buf)) > 0) out.append(buf, (size_t)k);
    gzclose(f);
    return true;
}
int fixIdx(long i, size_t n) { if (i > 0) return (int)(i - 1); if (i < 0) return (int)((long)n + i); return -1; }

struct Tri { V3 v0, v1, v2, c; };            /* mesh.h:14-25 */
struct TriExt { V3 n0, n1, n2; float uv[6]; }; /* mesh.h:26-30 */
struct Mesh { std::vector<Tri> tris; std::vector<TriExt> ext; };

/* Triangle::Triangle(v1, v0, v2): OBJ vertex 0 lands in v1 (mesh.cpp:13-21). */
Tri makeTri(V3 a, V3 b, V3 c) {
    Tri t; t.v0 = b; t.v1 = a; t.v2 = c;
    t.c = (t.v0 + t.v1 + t.v2) * 0.333f;
    return t;
}

bool loadObj(const std::string& path, Mesh& mesh) {
    std::string text;
    if (!readAll(path, text)) return false;
    std::vector<float> V, N, T;
    std::vector<ObjIdx> tri;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        std::string line = text.substr(pos, eol - pos);
        pos = eol + 1;
        const char* s = line.c_str();
        while (*s == ' ' || *s == '\t') ++s;
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
            char* e; const char* p = s + 2;
            for (int i = 0; i < 3; ++i) { double d = strtod(p, &e); V.push_back((float)d); p = e; }
        } else if (s[0] == 'v' && s[1] == 'n') {
            char* e; const char* p = s + 2;
            for (int i = 0; i < 3; ++i) { double d = strtod(p, &e); N.push_back((float)d); p = e; }
        } else if (s[0] == 'v' && s[1] == 't') {
            char* e; const char* p = s + 2;
            for (int i = 0; i < 2; ++i) { double d = strtod(p, &e); T.push_back((float)d); p = e; }
        } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            std::vector<ObjIdx> poly;
            const char* p = s + 1;
            for (;;) {
                while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
                if (!*p) break;
                ObjIdx ix = {-1, -1, -1};
                char* e;
                long a = strtol(p, &e, 10); ix.v = fixIdx(a, V.size() / 3); p = e;
                if (*p == '/') {
                    ++p;
                    if (*p != '/') { long b = strtol(p, &e, 10); ix.t = fixIdx(b, T.size() / 2); p = e; }
                    if (*p == '/') { ++p; long c = strtol(p, &e, 10); ix.n = fixIdx(c, N.size() / 3); p = e; }
                }
                poly.push_back(ix);
                while (*p && *p != ' ' && *p != '\t') ++p;
            }
            if (poly.size() < 3) continue;
            if (poly.size() == 4) {
                auto P = [&](int k) { int v = poly[k].v; return mk(V[3 * v], V[3 * v + 1], V[3 * v + 2]); };
                V3 e02 = P(2) - P(0), e13 = P(3) - P(1);
                float s02 = e02.x * e02.x + e02.y * e02.y + e02.z * e02.z;
                float s13 = e13.x * e13.x + e13.y * e13.y + e13.z * e13.z;
                if (s02 < s13) { tri.push_back(poly[0]); tri.push_back(poly[1]); tri.push_back(poly[2]);
                                 tri.push_back(poly[0]); tri.push_back(poly[2]); tri.push_back(poly[3]); }
                else           { tri.push_back(poly[0]); tri.push_back(poly[1]); tri.push_back(poly[3]);
                                 tri.push_back(poly[1]); tri.push_back(poly[2]); tri.push_back(poly[3]); }
            } else {
                for (size_t k = 1; k + 1 < poly.size(); ++k) { tri.push_back(poly[0]); tri.push_back(poly[k]); tri.push_back(poly[k + 1]); }
            }
        }
    }
    auto vert = [&](const ObjIdx& i) { return mk(V[3 * i.v], V[3 * i.v + 1], V[3 * i.v + 2]); };
    auto nrm = [&](const ObjIdx& i) { return i.n >= 0 ? mk(N[3 * i.n], N[3 * i.n + 1], N[3 * i.n + 2]) : splat(0.0f); };
    for (size_t k = 0; k + 2 < tri.size(); k += 3) {
        mesh.tris.push_back(makeTri(vert(tri[k]), vert(tri[k + 1]), vert(tri[k + 2])));
        TriExt x;
        x.n0 = nrm(tri[k]); x.n1 = nrm(tri[k + 1]); x.n2 = nrm(tri[k + 2]);
        for (int j = 0; j < 3; ++j) {
            const ObjIdx& i = tri[k + j];
            x.uv[2 * j] = i.t >= 0 ? T[2 * i.t] : 0.0f;
            x.uv[2 * j + 1] = i.t >= 0 ? T[2 * i.t + 1] : 0.0f;
        }
        mesh.ext.push_back(x);
    }
    return true;
}

/* -------------------------------------------------------------- AABB / BVH */
struct Box { V3 mn, mx; };                    /* bvh.h:12-26, default inf / -inf */
inline Box emptyBox() { Box b; b.mn = splat(INFINITY); b.mx = splat(-INFINITY); return b; }
inline void grow(Box& b, V3 p) { b.mn = vmin(b.mn, p); b.mx = vmax(b.mx, p); }           /* bvh.cpp:17-21 */
inline void grow(Box& b, const Box& o) { b.mn = vmin(b.mn, o.mn); b.mx = vmax(b.mx, o.mx); } /* :23-27 */
inline float area(const Box& b) { V3 e = b.mx - b.mn; return e.x * e.y + e.y * e.z + e.z * e.x; } /* :29-33 */
inline V3 halfExtent(const Box& b) { return 0.5f * (b.mx - b.mn); }  /* AABB::center quirk, :35-38 */

struct Node { uint32_t lf, cnt; Box box; };    /* bvh.h:36-46 */

/* AABB::intersect, bvh.cpp:40-66 */
inline float slab(const Box& b, V3 o, V3 d, float depth) {
    V3 rd = splat(1.0f) / d;
    float tx0 = (b.mn.x - o.x) * rd.x, tx1 = (b.mx.x - o.x) * rd.x;
    float t0 = tmin(tx0, tx1), t1 = tmax(tx0, tx1);
    float ty0 = (b.mn.y - o.y) * rd.y, ty1 = (b.mx.y - o.y) * rd.y;
    t0 = tmax(t0, tmin(ty0, ty1)); t1 = tmin(t1, tmax(ty0, ty1));
    float tz0 = (b.mn.z - o.z) * rd.z, tz1 = (b.mx.z - o.z) * rd.z;
    t0 = tmax(t0, tmin(tz0, tz1)); t1 = tmin(t1, tmax(tz0, tz1));
    if (t1 >= t0 && t0 < depth && t1 > 0.0f) return t0;
    return kFarAway;
}

/* Triangle::intersect, mesh.cpp:23-62 (Moller-Trumbore). */
inline bool hitTri(const Tri& tr, V3 o, V3 d, float& depth, float& hu, float& hv) {
    V3 e1 = tr.v1 - tr.v0, e2 = tr.v2 - tr.v0;
    V3 h = cross(d, e2);
    float a = dot(e1, h);
    if (fabsf(a) < kEps) return false;
    float f = 1.0f / a;
    V3 s = o - tr.v0;
    float u = f * dot(s, h);
    if (0.0f > u || u > 1.0f) return false;
    V3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (0.0f > v || (u + v) > 1.0f) return false;
    float t = f * dot(e2, q);
    if (!depthOk(t, depth)) return false;
    depth = t; hu = u; hv = v;
    return true;
}

/* Binned-SAH build shared by BLAS (keys = triangle centroids, boxes = triangle
 * vertices) and TLAS (keys = AABB::center() half extents, boxes = instance
 * bounds): BvhBLAS::build/findSplitPlane/partitionNode/updateNodeBounds/
 * subdivide (bvh.cpp:255-265, 294-465) and their TLAS twins (:780-993). */
struct Prims {
    virtual float key(uint32_t prim, int axis) const = 0;
    virtual void growBox(Box& b, uint32_t prim) const = 0;
    virtual ~Prims() {}
};
struct Bvh {
    std::vector<uint32_t> idx;
    std::vector<Node> nodes;
    uint32_t used = 2;
};

void updateBounds(Bvh& b, const Prims& P, uint32_t ni) {
    Node& n = b.nodes[ni];
    for (uint32_t i = 0; i < n.cnt; ++i) P.growBox(n.box, b.idx[n.lf + i]);
}

float splitPlane(const Bvh& b, const Prims& P, const Node& n, float& cost, uint32_t& axisOut) {
    float bestCost = INFINITY, bestSplit = 0.0f; uint32_t bestAxis = 0;
    for (uint32_t axis = 0; axis < 3; ++axis) {
        float lo = 3.40282347e+38f, hi = 1.17549435e-38f;   /* FLT_MAX / FLT_MIN quirk, :303-304 */
        for (uint32_t i = 0; i < n.cnt; ++i) {
            float c = P.key(b.idx[n.lf + i], axis);
            lo = tmin(lo, c); hi = tmax(hi, c);
        }
        if (lo == hi) continue;
        const float binScale = 8.0f / (hi - lo);
        uint32_t bc[8] = {0}; Box bb[8];
        for (int k = 0; k < 8; ++k) bb[k] = emptyBox();
        for (uint32_t i = 0; i < n.cnt; ++i) {
            uint32_t p = b.idx[n.lf + i];
            size_t sec = (size_t)((P.key(p, axis) - lo) * binScale);
            size_t bin = sec < 7 ? sec : 7;
            bc[bin]++;
            P.growBox(bb[bin], p);
        }
        float la[7], ra[7]; uint32_t lc[7], rc[7];
        Box lb = emptyBox(), rb = emptyBox(); uint32_t ls = 0, rs = 0;
        for (int k = 0; k < 7; ++k) {
            ls += bc[k]; lc[k] = ls; grow(lb, bb[k]); la[k] = area(lb);
            int rbin = 7 - k, rplane = rbin - 1;
            rs += bc[rbin]; rc[rplane] = rs; grow(rb, bb[rbin]); ra[rplane] = area(rb);
        }
        float ext = (hi - lo) / 8.0f;
        for (int k = 0; k < 7; ++k) {
            float c = (float)lc[k] * la[k] + (float)rc[k] * ra[k];
            if (c < bestCost) { bestCost = c; bestSplit = lo + ext * (float)(k + 1); bestAxis = axis; }
        }
    }
    cost = bestCost; axisOut = bestAxis;
    return bestSplit;
}

uint32_t partition(Bvh& b, const Prims& P, const Node& n, float split, uint32_t axis) {
    int32_t pivot = (int32_t)n.lf;
    int32_t last = (int32_t)(n.lf + (n.cnt - 1));
    while (pivot <= last) {
        if (P.key(b.idx[pivot], (int)axis) < split) pivot++;
        else { uint32_t t = b.idx[pivot]; b.idx[pivot] = b.idx[last]; b.idx[last] = t; last--; }
    }
    return (uint32_t)pivot;
}

void subdivide(Bvh& b, const Prims& P, uint32_t ni) {
    float cost = INFINITY; uint32_t axis = 0;
    float split = splitPlane(b, P, b.nodes[ni], cost, axis);
    float parentCost = (float)b.nodes[ni].cnt * area(b.nodes[ni].box);
    if (cost >= parentCost) return;
    uint32_t pivot = partition(b, P, b.nodes[ni], split, axis);
    uint32_t leftCount = pivot - b.nodes[ni].lf;
    if (leftCount == 0 || leftCount == b.nodes[ni].cnt) return;
    uint32_t li = b.used, ri = b.used + 1;
    b.used += 2;
    Node& L = b.nodes[li]; L.lf = b.nodes[ni].lf; L.cnt = leftCount; L.box = emptyBox();
    Node& R = b.nodes[ri]; R.lf = pivot; R.cnt = b.nodes[ni].cnt - leftCount; R.box = emptyBox();
    b.nodes[ni].lf = li; b.nodes[ni].cnt = 0;
    updateBounds(b, P, li); updateBounds(b, P, ri);
    subdivide(b, P, li); subdivide(b, P, ri);
}

void buildBvh(Bvh& b, const Prims& P, uint32_t count) {
    b.idx.resize(count);
    for (uint32_t i = 0; i < count; ++i) b.idx[i] = i;
    /* node pool is memset to zero (bvh.cpp:77): the root box starts at (0,0,0)-(0,0,0) */
    Node z; memset(&z, 0, sizeof z);
    b.nodes.assign(2 * (size_t)count, z);
    b.used = 2;
    b.nodes[0].lf = 0; b.nodes[0].cnt = count;
    updateBounds(b, P, 0);
    subdivide(b, P, 0);
}

uint32_t bvhDepth(const Bvh& b, uint32_t ni) {
    const Node& n = b.nodes[ni];
    if (n.cnt != 0) return 0;
    uint32_t l = bvhDepth(b, n.lf), r = bvhDepth(b, n.lf + 1);
    return 1 + (l > r ? l : r);
}

struct TriPrims : Prims {
    const Mesh* m;
    float key(uint32_t p, int axis) const override { return comp(m->tris[p].c, axis); }
    void growBox(Box& b, uint32_t p) const override { const Tri& t = m->tris[p]; grow(b, t.v0); grow(b, t.v1); grow(b, t.v2); }
};

struct Blas { const Mesh* mesh; Bvh bvh; };

/* ------------------------------------------------------------ Material --- */
struct Material {                               /* material.h:6-19 */
    float emit = 0.0f, refl = 0.0f, refr = 0.0f, ior = 1.0f;
    V3 emitColor = {0, 0, 0}, albedo = {0, 0, 0}, absorption = {0, 0, 0};
    bool isLight() const { return emit > 0.0f && (emitColor.x > 0.0f || emitColor.y > 0.0f || emitColor.z > 0.0f); }
    V3 emittance() const { return emit * emitColor; }
};

/* ------------------------------------------------------------ Instance --- */
struct Instance {                               /* bvh.h:104-147, bvh.cpp:467-594 */
    const Blas* blas;
    const Material* mat;
    M4 M, Minv;
    Box bounds;
    float area;
};

Instance makeInstance(const Blas* blas, const Material* mat, const M4& M) {
    Instance in; in.blas = blas; in.mat = mat; in.M = M;
    in.Minv = inverse(M);                                                     /* :524-531 */
    /* updateBounds, :554-575 -- the BLAS root box (including the memset origin) */
    const Box& lb = blas->bvh.nodes[0].box;
    in.bounds = emptyBox();
    V3 corners[8] = {
        mk(lb.mx.x, lb.mx.y, lb.mx.z), mk(lb.mn.x, lb.mx.y, lb.mx.z), mk(lb.mx.x, lb.mn.y, lb.mx.z), mk(lb.mn.x, lb.mn.y, lb.mx.z),
        mk(lb.mx.x, lb.mx.y, lb.mn.z), mk(lb.mn.x, lb.mx.y, lb.mn.z), mk(lb.mx.x, lb.mn.y, lb.mn.z), mk(lb.mn.x, lb.mn.y, lb.mn.z)};
    for (int k = 0; k < 8; ++k) { V4 t = mul(M, v4(corners[k], 1.0f)); grow(in.bounds, xyz(t) / t.w); }
    /* calculateMeshArea, :577-594 */
    in.area = 0.0f;
    for (const Tri& t : blas->mesh->tris) {
        V4 a4 = mul(M, v4(t.v0, 1.0f)), b4 = mul(M, v4(t.v1, 1.0f)), c4 = mul(M, v4(t.v2, 1.0f));
        V3 a = xyz(a4) / a4.w, b = xyz(b4) / b4.w, c = xyz(c4) / c4.w;
        V3 e1 = b - a, e2 = c - a;
        in.area += 0.5f * magnitude(cross(e1, e2));
    }
    return in;
}

struct InstPrims : Prims {
    const std::vector<Instance>* inst;
    float key(uint32_t p, int axis) const override { return comp(halfExtent((*inst)[p].bounds), axis); }
    void growBox(Box& b, uint32_t p) const override { grow(b, (*inst)[p].bounds); }
};

/* ------------------------------------------------------------ traversal -- */
struct Hit { float t, u, v; uint32_t inst, prim; };

/* BvhBLAS::intersect (bvh.cpp:129-191) and intersectAny (:193-253), with the
 * instance world->object transform of Instance::intersect(Any) (:481-513).
 * Returns true when a triangle test succeeded; updates depth / hit. */
/* Optional traversal statistics (orc_trace_visits): node visits and triangle
 * tests of the current instance; never set during renders. */
thread_local uint32_t* tVisitNodes = nullptr;
thread_local uint32_t* tVisitTris = nullptr;
thread_local uint32_t* tVisitBaseN = nullptr;   /* per-instance arrays of the current ray */
thread_local uint32_t* tVisitBaseT = nullptr;

template <bool ANY>
bool blasTrace(const Blas& B, V3 o, V3 d, float& depth, Hit& hit, uint32_t& stackMax) {
    const Bvh& b = B.bvh;
    uint32_t stack[64]; uint32_t sp = 0;
    uint32_t ni = 0;
    bool any = false;
    for (;;) {
        const Node& n = b.nodes[ni];
        if (tVisitNodes) ++*tVisitNodes;
        if (n.cnt != 0) {
            if (tVisitTris) *tVisitTris += n.cnt;
            for (uint32_t i = 0; i < n.cnt; ++i) {
                uint32_t p = b.idx[n.lf + i];
                float u, v;
                if (hitTri(B.mesh->tris[p], o, d, depth, u, v)) {
                    if (ANY) return true;
                    any = true; hit.prim = p; hit.u = u; hit.v = v; hit.t = depth;
                }
            }
            if (sp == 0) break;
            ni = stack[--sp];
            continue;
        }
        uint32_t cn = n.lf, cf = n.lf + 1;
        float dn = slab(b.nodes[cn].box, o, d, depth), df = slab(b.nodes[cf].box, o, d, depth);
        if (dn > df) { float t = dn; dn = df; df = t; uint32_t c = cn; cn = cf; cf = c; }
        if (dn == kFarAway) { if (sp == 0) break; ni = stack[--sp]; }
        else {
            ni = cn;
            if (df != kFarAway) { if (sp >= 64) { fprintf(stderr, "oracle: BLAS stack overflow\n"); abort(); } stack[sp++] = cf; if (sp > stackMax) stackMax = sp; }
        }
    }
    return any;
}

struct Scene {
    std::vector<Mesh*> meshes;
    std::vector<Blas*> blases;
    std::vector<Material*> materials;
    std::vector<Instance> inst;
    Bvh tlas;
    std::vector<uint32_t> lights;
    /* SceneBackground (scene.h:18-26), main.cpp:343-346 */
    int bgType = 1; V3 bgColor = {0, 0, 0}, bgA = {0.8f, 0.8f, 0.8f}, bgB = {0.1f, 0.4f, 0.6f};
    /* camera, camera.h:27-57 */
    V3 camPos, camFwd, camUp; float scrW = 0, scrH = 0, fovY = 70.0f, focal = 7.0f, defocus = 0.5f;
    V3 firstPixel, uVec, vVec;
    uint32_t stackMax = 0;
    ~Scene() { for (auto* m : meshes) delete m; for (auto* b : blases) delete b; for (auto* m : materials) delete m; }
};

/* BvhTLAS::intersect (bvh.cpp:654-716) / intersectAny (:718-778). */
template <bool ANY>
bool tlasTrace(const Scene& S, V3 o, V3 d, float& depth, Hit& hit, uint32_t& stackMax) {
    const Bvh& b = S.tlas;
    uint32_t stack[64]; uint32_t sp = 0;
    uint32_t ni = 0;
    bool any = false;
    for (;;) {
        const Node& n = b.nodes[ni];
        if (n.cnt != 0) {
            for (uint32_t i = 0; i < n.cnt; ++i) {
                uint32_t ii = b.idx[n.lf + i];
                const Instance& in = S.inst[ii];
                V4 tp = mul(in.Minv, v4(o, 1.0f)), td = mul(in.Minv, v4(d, 0.0f));
                V3 oo = xyz(tp) / tp.w, dd = xyz(td);
                uint32_t sm = 0;
                if (tVisitBaseN) { tVisitNodes = tVisitBaseN + ii; tVisitTris = tVisitBaseT + ii; }
                bool h = blasTrace<ANY>(*in.blas, oo, dd, depth, hit, sm);
                if (sp + sm > stackMax) stackMax = sp + sm;
                if (h) { if (ANY) return true; any = true; hit.inst = ii; }
            }
            if (sp == 0) break;
            ni = stack[--sp];
            continue;
        }
        uint32_t cn = n.lf, cf = n.lf + 1;
        float dn = slab(b.nodes[cn].box, o, d, depth), df = slab(b.nodes[cf].box, o, d, depth);
        if (dn > df) { float t = dn; dn = df; df = t; uint32_t c = cn; cn = cf; cf = c; }
        if (dn == kFarAway) { if (sp == 0) break; ni = stack[--sp]; }
        else { ni = cn; if (df != kFarAway) { stack[sp++] = cf; if (sp > stackMax) stackMax = sp; } }
    }
    return any;
}

/* ------------------------------------------------------------ scene setup */
Scene* buildIndoor(const std::string& dir, int variant) {
    Scene* S = new Scene();
    const char* names[4] = {"susanne", "cube", "lens", "plane"};       /* main.cpp:163-166 */
    for (int i = 0; i < 4; ++i) {
        Mesh* m = new Mesh();
        std::string p = dir + "/" + names[i] + ".obj";
        if (!loadObj(p, *m) && !loadObj(p + ".gz", *m)) { fprintf(stderr, "oracle: cannot read %s\n", p.c_str()); delete m; delete S; return nullptr; }
        S->meshes.push_back(m);
    }
    Mesh *susM = S->meshes[0], *cubeM = S->meshes[1], *lensM = S->meshes[2], *planeM = S->meshes[3];
    Mesh* lattice = nullptr;
    if (variant == 1) {
        /* C5: 648 Suzanne copies at translate(-8+2i, -0.4+1.2j, -4+1.5k) * scale(0.5) baked in one mesh. */
        lattice = new Mesh();
        for (int i = 0; i < 9; ++i) for (int j = 0; j < 8; ++j) for (int k = 0; k < 9; ++k) {
            M4 X = scale(translate(identity(), mk(-8.0f + 2.0f * (float)i, -0.4f + 1.2f * (float)j, -4.0f + 1.5f * (float)k)), splat(0.5f));
            for (size_t t = 0; t < susM->tris.size(); ++t) {
                const Tri& s = susM->tris[t];
                /* the stored triangle keeps the OBJ order: OBJ vertex 0 is s.v1 */
                V4 a = mul(X, v4(s.v1, 1.0f)), b = mul(X, v4(s.v0, 1.0f)), c = mul(X, v4(s.v2, 1.0f));
                lattice->tris.push_back(makeTri(xyz(a) / a.w, xyz(b) / b.w, xyz(c) / c.w));
                lattice->ext.push_back(susM->ext[t]);
            }
        }
        S->meshes.push_back(lattice);
    }
    auto mkBlas = [&](Mesh* m) { Blas* b = new Blas(); b->mesh = m; TriPrims P; P.m = m; buildBvh(b->bvh, P, (uint32_t)m->tris.size()); S->blases.push_back(b); return b; };
    Blas *susB = mkBlas(susM), *cubeB = mkBlas(cubeM), *lensB = mkBlas(lensM), *planeB = mkBlas(planeM);   /* main.cpp:168-171 */
    Blas* latB = lattice ? mkBlas(lattice) : nullptr;

    auto mat = [&]() { Material* m = new Material(); S->materials.push_back(m); return m; };   /* main.cpp:173-202 */
    Material* floorM = mat(); floorM->albedo = splat(0.8f); floorM->refl = 0.01f;
    Material* redM = mat(); redM->albedo = mk(1.0f, 0.0f, 0.0f);
    Material* greenM = mat(); greenM->albedo = mk(0.0f, 1.0f, 0.0f);
    Material* diffM = mat(); diffM->albedo = mk(1.0f, 0.0f, 0.0f);
    Material* dielM = mat(); dielM->albedo = mk(0.7f, 0.7f, 0.2f); dielM->absorption = mk(0.03f, 0.04f, 0.03f); dielM->refr = 1.0f; dielM->ior = 1.42f;
    Material* specM = mat(); specM->albedo = mk(0.2f, 0.9f, 1.0f); specM->refl = 0.8f;
    Material* softL = mat(); softL->emitColor = mk(1.0f, 0.8f, 0.6f); softL->emit = 5.0f;
    Material* redL = mat(); redL->emitColor = mk(1.0f, 0.5f, 0.2f); redL->emit = 5.0f;

    const M4 I = identity();
    const V3 fwd = mk(0.0f, 0.0f, -1.0f), right = mk(1.0f, 0.0f, 0.0f);   /* camera.h:7-9 */
    Instance cubeL = makeInstance(cubeB, softL, scale(translate(I, mk(-8.0f, 7.0f, 5.0f)), mk(0.5f, 0.5f, 0.5f)));        /* :204-214 */
    Instance cubeR = makeInstance(cubeB, redL, scale(translate(I, mk(9.0f, 5.0f, -5.0f)), mk(1.0f, 1.0f, 1.0f)));         /* :216-226 */
    Instance floorI = makeInstance(planeB, floorM, scale(translate(I, mk(0.0f, -1.0f, 0.0f)), mk(10.0f, 10.0f, 10.0f)));   /* :228-238 */
    Instance sus0 = makeInstance(susB, diffM, translate(I, mk(0.0f, 0.0f, -1.0f)));                                        /* :240-247 */
    Instance sus1 = makeInstance(susB, specM, translate(I, mk(3.0f, 0.0f, -1.0f)));                                        /* :249-256 */
    Instance lens0 = makeInstance(lensB, dielM, translate(I, mk(-3.0f, 0.0f, -1.0f)));                                     /* :258-265 */
    Instance wallL = makeInstance(planeB, redM, scale(rotate(translate(I, mk(-10.0f, 4.0f, 0.0f)), radiansf(90.0f), fwd), mk(5.0f, 10.0f, 10.0f)));   /* :267-281 */
    Instance wallR = makeInstance(planeB, greenM, scale(rotate(translate(I, mk(10.0f, 4.0f, 0.0f)), radiansf(90.0f), fwd), mk(5.0f, 10.0f, 10.0f))); /* :283-297 */
    Instance wallTop = makeInstance(planeB, floorM, scale(translate(I, mk(0.0f, 9.0f, 0.0f)), mk(10.0f, 10.0f, 10.0f)));   /* :299-309 */
    Instance wallFront = makeInstance(planeB, floorM, scale(rotate(translate(I, mk(0.0f, 4.0f, -10.0f)), radiansf(90.0f), right), mk(10.0f, 10.0f, 5.0f))); /* :311-325 */
    Instance wallBack = makeInstance(planeB, floorM, scale(rotate(translate(I, mk(0.0f, 4.0f, 10.0f)), radiansf(90.0f), right), mk(10.0f, 10.0f, 5.0f)));   /* :327-341 */
    S->inst = {floorI, cubeL, cubeR, sus0, sus1, lens0, wallL, wallR, wallTop, wallFront, wallBack};          /* :360 */
    if (latB) S->inst.push_back(makeInstance(latB, diffM, I));
    if (variant == 2 || variant == 3) {
        /* general-TLAS test scenes (not in the reference's main.cpp): extra
         * instances of the cube / Suzanne / lens meshes, sizes 0.3-0.9 and
         * rotations varied so that BvhTLAS::build splits (bvh.cpp:780-993):
         * 40 extras (51 instances, LDS tables) or 80 (91, global tables) */
        const Blas* meshes[3] = {cubeB, susB, lensB};
        Material* mats[5] = {floorM, diffM, specM, dielM, greenM};
        const int extra = variant == 2 ? 40 : 80;
        for (int k = 0; k < extra; ++k) {
            const float x = -8.5f + 1.0f * (float)((k * 7) % 18);
            const float y = -0.4f + 0.9f * (float)((k * 5) % 10);
            float z = -8.5f + 1.0f * (float)((k * 11) % 18);
            if (x > -2.5f && x < 2.5f && y < 2.5f && z < -4.5f) z = z + 6.0f;   /* keep clear of the camera (0, 0, -7) */
            const float sc = 0.3f + 0.15f * (float)(k % 5);
            M4 X = translate(I, mk(x, y, z));
            if (k % 3 == 1) X = rotate(X, radiansf(17.0f * (float)(k % 7)), mk(0.0f, 1.0f, 0.0f));
            X = scale(X, mk(sc, sc, sc));
            S->inst.push_back(makeInstance(meshes[k % 3], mats[k % 5], X));
        }
    }

    /* Scene::Scene, scene.cpp:17-33 */
    InstPrims P; P.inst = &S->inst;
    buildBvh(S->tlas, P, (uint32_t)S->inst.size());
    for (uint32_t i = 0; i < S->inst.size(); ++i) if (S->inst[i].mat->isLight()) S->lights.push_back(i);
    return S;
}

/* Camera::Camera + generateViewPlane, camera.cpp:9-46; main.cpp:141-149 */
void setCamera(Scene& S, uint32_t W, uint32_t H) {
    S.camPos = mk(0.0f, 0.0f, -7.0f);
    V3 target = mk(0.0f, 0.0f, 0.0f);
    S.scrW = (float)W; S.scrH = (float)H;
    S.camFwd = normalize(target - S.camPos);
    V3 r = normalize(cross(mk(0.0f, 1.0f, 0.0f), S.camFwd));
    S.camUp = normalize(cross(S.camFwd, r));
    const float heightScale = tanf(radiansf(S.fovY) / 2.0f);
    const float aspect = S.scrW / S.scrH;
    const float vh = 2.0f * heightScale * S.focal;
    const float vw = aspect * vh;
    V3 right = normalize(cross(S.camUp, S.camFwd));                    /* Camera::right, camera.h:54-57 */
    const V3 u = right * vw;
    const V3 v = (-1.0f * S.camUp) * vh;
    const V3 du = u / S.scrW, dv = v / S.scrH;
    const V3 topLeft = ((S.camPos + (S.camFwd * S.focal)) - (0.5f * u)) - (0.5f * v);
    S.firstPixel = topLeft + 0.5f * (du + dv);
    S.uVec = u; S.vVec = v;
}

/* Camera::getPrimaryRay + sampleDefocusDisk, camera.h:59-87.  GCC evaluates
 * the Float2(...) arguments right to left: the y draw comes first. */
void primaryRay(const Scene& S, uint32_t& seed, float x, float y, V3& o, V3& d) {
    const float u = x * (1.0f / S.scrW), v = y * (1.0f / S.scrH);
    V3 origin = S.camPos;
    if (!(S.defocus == 0.0f)) {
        const float radius = S.focal * tanf(radiansf(S.defocus / 2.0f));
        const V3 right = normalize(cross(S.camUp, S.camFwd));
        const V3 du = right * radius, dv = (-1.0f * S.camUp) * radius;
        float sx, sy;
        do {
            sy = rndRange(seed, -1.0f, 1.0f);
            sx = rndRange(seed, -1.0f, 1.0f);
        } while (sx * sx + sy * sy > 1.0f);
        origin = S.camPos + ((sx * du) + (sy * dv));
    }
    const V3 plane = (S.firstPixel + u * S.uVec) + v * S.vVec;
    o = origin;
    d = normalize(plane - origin);
}

/* randomOnHemisphereCosineWeighted, surf_math.cpp:116-134 */
V3 cosineSample(uint32_t& seed, V3 n) {
    for (;;) {
        float r0 = rndF(seed), r1 = rndF(seed);
        float r = sqrtf(r0);
        float theta = k2Pi * r1;
        V3 dir = mk(r * cosf(theta), r * sinf(theta), sqrtf(1.0f - r0));
        const float xMax = 1.0f - kEps;
        V3 tmp = (fabsf(n.x) > xMax) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
        V3 B = normalize(cross(n, tmp));
        V3 T = cross(B, n);
        V3 out = ((dir.x * T) + (dir.y * B)) + (dir.z * n);
        if (!(dot(out, n) == 0.0f)) return out;
    }
}

struct Recorder {
    uint32_t maxExt, maxSh, nExt = 0, nSh = 0;
    float *eo, *ed, *so, *sd, *st;
};

struct Counters { uint64_t ext = 0, hit = 0, cont = 0, sh = 0, acc = 0, unocc = 0, maxSeg = 0; };

/* Optional early end of a path whose throughput T has every channel below
 * FLT_MIN (zero or denormal).  Such a path is Russian-roulette-terminated with
 * certainty at its next diffuse bounce (p = max(T) < the smallest positive
 * randomF32, 2^-32), so at most two more contributions remain, each below
 * 1.2e-38 * (emission or light term): radiance-neutral in f32 except for a
 * pixel whose energy is itself ~1e-38.  It ends the total-internal-reflection
 * orbits in the glass lens that the reference traces forever (throughput stuck
 * at the smallest denormal: 1.4e-45 * 0.69 rounds back up).  Off by default:
 * the reference has no such exit (renderer.cpp:336-460) and the CPU baseline
 * times the reference algorithm. */
bool gZeroCutoff = false;

/* Renderer::trace, iterative branch (renderer.cpp:332-463). */
V3 trace(const Scene& S, uint32_t& seed, V3 o, V3 d, uint32_t maxSeg, Counters& C, Recorder* rec, uint32_t& stackMax) {
    V3 energy = splat(0.0f), T = splat(1.0f);
    bool lastSpecular = true, inMedium = false;
    uint32_t seg = 0;
    for (;;) {
        seg++;
        float depth = kFarAway;
        Hit h; h.inst = kUnset; h.prim = kUnset; h.u = 0.0f; h.v = 0.0f; h.t = kFarAway;
        C.ext++;
        if (rec && rec->nExt < rec->maxExt) {
            float* a = rec->eo + 3 * rec->nExt; float* b = rec->ed + 3 * rec->nExt;
            a[0] = o.x; a[1] = o.y; a[2] = o.z; b[0] = d.x; b[1] = d.y; b[2] = d.z; rec->nExt++;
        }
        bool hit = tlasTrace<false>(S, o, d, depth, h, stackMax);
        if (!hit) {                                                        /* :338-342 */
            V3 bg = splat(0.0f);
            if (S.bgType == 0) bg = S.bgColor;
            else if (S.bgType == 1) { float a = 0.5f * (1.0f + d.y); bg = (a * S.bgB) + ((1.0f - a) * S.bgA); }  /* scene.cpp:35-51 */
            energy = energy + T * bg; C.acc++;
            break;
        }
        C.hit++;
        const Instance& in = S.inst[h.inst];
        const Mesh* mesh = in.blas->mesh;
        const Material* m = in.mat;
        if (m->isLight()) {                                               /* :348-352 */
            energy = energy + (lastSpecular ? T * m->emittance() : splat(0.0f));
            if (lastSpecular) C.acc++;
            break;
        }
        V3 medium = splat(1.0f);
        if (inMedium) { float nd = -depth; V3 a = m->absorption * nd; medium = mk(expf(a.x), expf(a.y), expf(a.z)); }   /* :354-356 */
        V3 I = o + depth * d;                                              /* Ray::hitPosition, ray.h:63-66 */
        /* Instance::normal (bvh.cpp:515-522) over Mesh::normal (mesh.h:63-68) */
        const TriExt& x = mesh->ext[h.prim];
        float w = (1.0f - h.u) - h.v;
        V3 nObj = ((h.u * x.n0) + (h.v * x.n2)) + (w * x.n1);
        V4 nw = mul(in.M, v4(nObj, 0.0f));
        float nn = (nw.x * nw.x + nw.y * nw.y) + (nw.z * nw.z + nw.w * nw.w);   /* glm dot(vec4) */
        float ninv = 1.0f / sqrtf(nn);                                          /* glm inversesqrt */
        V3 N = mk(nw.x * ninv, nw.y * ninv, nw.z * ninv);
        float rng = rndF(seed);                                            /* :361 */
        V3 R = splat(0.0f);
        bool nextMedium = inMedium;
        if (dot(d, N) > 0.0f) N = N * -1.0f;                               /* :367-368 */
        if (rng < m->refl) {                                               /* :370-375 */
            R = reflect(d, N);
            lastSpecular = true;
            T = T * (m->albedo * medium);
        } else if (rng < (m->refl + m->refr)) {                            /* :376-404 */
            bool mustRefract = false;
            R = reflect(d, N);
            float n1 = inMedium ? m->ior : 1.0f, n2 = inMedium ? 1.0f : m->ior;
            float ratio = n1 / n2;
            float cosI = -dot(d, N);
            float cos2 = 1.0f - (ratio * ratio) * (1.0f - cosI * cosI);
            if (cos2 > 0.0f) {
                float a = n1 - n2, b = n1 + n2;
                float r0 = (a * a) / (b * b);
                float c = 1.0f - cosI;
                float fres = r0 + (1.0f - r0) * ((((c * c) * c) * c) * c);
                mustRefract = rndF(seed) > fres;
                if (mustRefract) R = (ratio * d) + ((ratio * cosI - sqrtf(fabsf(cos2))) * N);
            }
            lastSpecular = true;
            T = T * (m->albedo * medium);
            nextMedium = mustRefract ? !inMedium : inMedium;
        } else {                                                           /* :405-455 */
            R = cosineSample(seed, N);
            uint32_t nL = (uint32_t)S.lights.size();
            float cosT = dot(N, R);
            float pdf = cosT * kInvPi;
            V3 brdf = m->albedo * kInvPi;
            if (nL > 0) {
                const Instance& L = S.inst[S.lights[rndRangeU(seed, 0, nL)]];   /* Scene::sampleLights, scene.h:53 */
                /* Instance::samplePoint, bvh.cpp:533-552 */
                const Mesh* lm = L.blas->mesh;
                float u = rndRange(seed, 0.0f, 1.0f);
                float v = rndRange(seed, 0.0f, 1.0f - u);
                uint32_t ti = rndRangeU(seed, 0, (uint32_t)lm->tris.size());
                const Tri& lt = lm->tris[ti];
                float lw = (1.0f - u) - v;
                V3 lp = ((u * lt.v0) + (v * lt.v2)) + (lw * lt.v1);        /* Mesh::position, mesh.h:56-61 */
                const TriExt& lx = lm->ext[ti];
                V3 ln = ((u * lx.n0) + (v * lx.n2)) + (lw * lx.n1);
                V4 tp = mul(L.M, v4(lp, 1.0f)), tn = mul(L.M, v4(ln, 0.0f));
                V3 P = xyz(tp) / tp.w;
                V3 LN = normalize(xyz(tn));
                V3 IL = P - I;
                V3 Ldir = normalize(IL);
                V3 SO = I + kEps * Ldir;
                float srDepth = magnitude(IL) - 2.0f * kEps;
                float falloff = 1.0f / dot(IL, IL);
                float cosO = dot(N, Ldir);
                float cosI = dot(LN, -1.0f * Ldir);
                if (cosO > 0.0f && cosI > 0.0f) {
                    float SA = (cosI * L.area) * falloff;
                    float lightPdf = 1.0f / SA;
                    C.sh++;
                    if (rec && rec->nSh < rec->maxSh) {
                        float* a = rec->so + 3 * rec->nSh; float* b = rec->sd + 3 * rec->nSh;
                        a[0] = SO.x; a[1] = SO.y; a[2] = SO.z; b[0] = Ldir.x; b[1] = Ldir.y; b[2] = Ldir.z; rec->st[rec->nSh] = srDepth; rec->nSh++;
                    }
                    float sd = srDepth; Hit sh;
                    if (!tlasTrace<true>(S, SO, Ldir, sd, sh, stackMax)) {
                        float invPdf = 1.0f / lightPdf;
                        V3 Ld = (((L.mat->emittance() * invPdf) * brdf) * cosO) * (float)nL;
                        energy = energy + T * Ld;
                        C.acc++; C.unocc++;
                    }
                }
            }
            const float p = clampf(tmax(T.x, tmax(T.y, T.z)), 0.0f, 1.0f);   /* :446-448 */
            if (p < rndF(seed)) break;
            float rr = 1.0f / p;
            float invPdf = 1.0f / pdf;
            lastSpecular = false;
            T = T * ((((cosT * invPdf) * brdf) * medium) * rr);
        }
        if (maxSeg != 0 && seg >= maxSeg) break;     /* C2 path-length cap */
        if (gZeroCutoff && T.x < 1.17549435e-38f && T.y < 1.17549435e-38f && T.z < 1.17549435e-38f) break;
        C.cont++;
        o = I + kEps * R;                                                  /* :458-460 */
        d = R;
        inMedium = nextMedium;
    }
    if (seg > C.maxSeg) C.maxSeg = seg;
    return energy;
}

}  // namespace

/* =========================================================== C API ====== */
struct orc_scene { Scene* s; };

extern "C" {

orc_scene* orc_scene_create(const char* dir, int variant) {
    Scene* s = buildIndoor(dir ? dir : ".", variant);
    if (!s) return nullptr;
    orc_scene* h = new orc_scene; h->s = s;
    setCamera(*s, 1280, 720);
    return h;
}
void orc_scene_destroy(orc_scene* h) { if (h) { delete h->s; delete h; } }

int orc_scene_mesh_tris(const orc_scene* h, uint32_t* out, int max) {
    int n = 0;
    for (auto* m : h->s->meshes) { if (n < max) out[n] = (uint32_t)m->tris.size(); n++; }
    return n;
}
uint32_t orc_scene_instance_count(const orc_scene* h) { return (uint32_t)h->s->inst.size(); }
uint32_t orc_scene_light_count(const orc_scene* h) { return (uint32_t)h->s->lights.size(); }

void orc_scene_set_camera(orc_scene* h, uint32_t w, uint32_t ht) { setCamera(*h->s, w, ht); }

void orc_camera_ubo(const orc_scene* h, void* out) {
    const Scene& S = *h->s;
    float u[32]; memset(u, 0, sizeof u);
    auto put = [&](int at, V3 v) { u[at] = v.x; u[at + 1] = v.y; u[at + 2] = v.z; };
    V3 right = normalize(cross(S.camUp, S.camFwd));
    put(0, S.camPos); put(4, S.camUp); put(8, S.camFwd); put(12, right);       /* renderer.cpp:972-979 */
    put(16, S.firstPixel); put(20, S.uVec); put(24, S.vVec);
    u[28] = S.scrW; u[29] = S.scrH; u[30] = S.focal; u[31] = S.defocus;
    memcpy(out, u, 128);
}

/* GPUBatcher::createBatchInfo (scene.cpp:61-157) -- first-use order instead of
 * pointer order for meshes/BLASes/materials (the reference's order is address
 * dependent; any consistent order is equivalent). */
uint64_t orc_scene_export(const orc_scene* h, int which, void* dst) {
    const Scene& S = *h->s;
    std::vector<const Mesh*> meshes; std::vector<const Blas*> blases; std::vector<const Material*> mats;
    for (const Instance& in : S.inst) {
        bool f = false; for (auto* m : meshes) f |= (m == in.blas->mesh); if (!f) meshes.push_back(in.blas->mesh);
        f = false; for (auto* b : blases) f |= (b == in.blas); if (!f) blases.push_back(in.blas);
        f = false; for (auto* m : mats) f |= (m == in.mat); if (!f) mats.push_back(in.mat);
    }
    std::vector<uint8_t> out;
    auto putf = [&](float v) { uint8_t b[4]; memcpy(b, &v, 4); out.insert(out.end(), b, b + 4); };
    auto putu = [&](uint32_t v) { uint8_t b[4]; memcpy(b, &v, 4); out.insert(out.end(), b, b + 4); };
    auto put3 = [&](V3 v) { putf(v.x); putf(v.y); putf(v.z); putf(0.0f); };
    auto putNode = [&](const Node& n) { putu(n.lf); putu(n.cnt); putu(0); putu(0); put3(n.box.mn); put3(n.box.mx); };
    switch (which) {
    case 0: for (auto* m : meshes) for (const Tri& t : m->tris) { put3(t.v0); put3(t.v1); put3(t.v2); put3(t.c); } break;
    case 1: for (auto* m : meshes) for (const TriExt& x : m->ext) { put3(x.n0); put3(x.n1); put3(x.n2); for (int k = 0; k < 6; ++k) putf(x.uv[k]); putf(0); putf(0); } break;
    case 2: for (auto* b : blases) for (uint32_t i : b->bvh.idx) putu(i); break;
    case 3: for (auto* b : blases) for (uint32_t i = 0; i < b->bvh.used; ++i) putNode(b->bvh.nodes[i]); break;
    case 4: for (auto* m : mats) { putf(m->emit); putf(m->refl); putf(m->refr); putf(m->ior); put3(m->emitColor); put3(m->albedo); put3(m->absorption); } break;
    case 5: for (const Instance& in : S.inst) {
                uint32_t to = 0, io = 0, no = 0, mo = 0;
                for (auto* m : meshes) { if (m == in.blas->mesh) break; to += (uint32_t)m->tris.size(); }
                for (auto* b : blases) { if (b == in.blas) break; io += (uint32_t)b->mesh->tris.size(); }
                for (auto* b : blases) { if (b == in.blas) break; no += b->bvh.used; }
                for (auto* m : mats) { if (m == in.mat) break; mo++; }
                putu(to); putu(io); putu(no); putu(mo); putf(in.area); putu(0); putu(0); putu(0);
                for (int k = 0; k < 4; ++k) for (int i = 0; i < 4; ++i) putf(in.M.c[k][i]);
                for (int k = 0; k < 4; ++k) for (int i = 0; i < 4; ++i) putf(in.Minv.c[k][i]);
            } break;
    case 6: for (uint32_t i : S.tlas.idx) putu(i); break;
    case 7: for (uint32_t i = 0; i < S.tlas.used; ++i) putNode(S.tlas.nodes[i]); break;
    case 8: for (uint32_t i : S.lights) { putu(i); putu((uint32_t)S.inst[i].blas->mesh->tris.size()); } break;
    case 9: putu((uint32_t)S.bgType); putu(0); putu(0); putu(0); put3(S.bgColor); put3(S.bgA); put3(S.bgB); break;
    default: return 0;
    }
    if (dst && !out.empty()) memcpy(dst, out.data(), out.size());
    return out.size();
}

/* Renderer::render (renderer.cpp:148-201) over an arbitrary list of image
 * rows: rows dynamic over OpenMP threads (renderer.cpp:163), then per pixel
 * and per frame: one seed initSeed(p + totalSamples*1799) with totalSamples =
 * first + f*spp the sample count before the frame (renderer.cpp:169), then
 * `spp` samples in sequence, each drawing its jitter, disk sample and path
 * from the RNG state the previous sample's path left (renderer.cpp:171-181),
 * acc += (rgb, 1) per sample in sample order (renderer.cpp:180).  acc holds
 * nrows x W RGBA floats in list order. */
double orc_render_rows_spp(orc_scene* h, uint32_t W, uint32_t H, const uint32_t* rows, uint32_t nrows,
                           uint32_t first, uint32_t frames, uint32_t spp, uint32_t maxSeg, int threads,
                           float* acc, orc_counters* cnt) {
    Scene& S = *h->s;
    if (S.scrW != (float)W || S.scrH != (float)H) setCamera(S, W, H);
    if (threads > 0) omp_set_num_threads(threads);
    if (spp == 0) spp = 1;
    Counters tot; uint32_t smax = 0;
    auto t0 = std::chrono::steady_clock::now();
    #pragma omp parallel
    {
        Counters C; uint32_t sm = 0;
        #pragma omp for schedule(dynamic)
        for (int64_t k = 0; k < (int64_t)nrows; ++k) {
            const uint32_t y = rows[k];
            for (uint32_t x = 0; x < W; ++x) {
                uint64_t p = (uint64_t)x + (uint64_t)y * W;
                float* a = acc + 4 * ((uint64_t)k * W + x);
                for (uint32_t f = 0; f < frames; ++f) {
                    /* SizeType arithmetic truncated to U32 (renderer.cpp:169) */
                    uint32_t seed = seedOf((uint32_t)(p + ((uint64_t)first + (uint64_t)f * spp) * 1799u));
                    for (uint32_t s = 0; s < spp; ++s) {
                        float jy = rndRange(seed, -0.5f, 0.5f);   /* GCC: last argument first */
                        float jx = rndRange(seed, -0.5f, 0.5f);
                        V3 o, d;
                        primaryRay(S, seed, (float)x + jx, (float)y + jy, o, d);
                        V3 c = trace(S, seed, o, d, maxSeg, C, nullptr, sm);
                        a[0] += c.x; a[1] += c.y; a[2] += c.z; a[3] += 1.0f;
                    }
                }
            }
        }
        #pragma omp critical
        {
            tot.ext += C.ext; tot.hit += C.hit; tot.cont += C.cont; tot.sh += C.sh; tot.acc += C.acc; tot.unocc += C.unocc;
            if (C.maxSeg > tot.maxSeg) tot.maxSeg = C.maxSeg;
            if (sm > smax) smax = sm;
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    if (smax > S.stackMax) S.stackMax = smax;
    if (cnt) {
        cnt->samples = (uint64_t)nrows * W * frames * spp;
        cnt->n_ext = tot.ext; cnt->n_hit = tot.hit; cnt->n_cont = tot.cont; cnt->n_shadow = tot.sh;
        cnt->n_acc = tot.acc; cnt->n_unocc = tot.unocc; cnt->max_segments = tot.maxSeg;
    }
    return std::chrono::duration<double>(t1 - t0).count();
}

double orc_render_rows(orc_scene* h, uint32_t W, uint32_t H, const uint32_t* rows, uint32_t nrows,
                       uint32_t first, uint32_t frames, uint32_t maxSeg, int threads,
                       float* acc, orc_counters* cnt) {
    return orc_render_rows_spp(h, W, H, rows, nrows, first, frames, 1, maxSeg, threads, acc, cnt);
}

double orc_render_spp(orc_scene* h, uint32_t W, uint32_t H, uint32_t r0, uint32_t r1,
                      uint32_t first, uint32_t frames, uint32_t spp, uint32_t maxSeg, int threads,
                      float* acc, orc_counters* cnt) {
    std::vector<uint32_t> rows;
    for (uint32_t y = r0; y < r1; ++y) rows.push_back(y);
    return orc_render_rows_spp(h, W, H, rows.data(), (uint32_t)rows.size(), first, frames, spp, maxSeg, threads, acc, cnt);
}

double orc_render(orc_scene* h, uint32_t W, uint32_t H, uint32_t r0, uint32_t r1,
                  uint32_t first, uint32_t frames, uint32_t maxSeg, int threads,
                  float* acc, orc_counters* cnt) {
    return orc_render_spp(h, W, H, r0, r1, first, frames, 1, maxSeg, threads, acc, cnt);
}

void orc_scene_update(orc_scene* h, float dt) {
    /* Scene::update / GPUScene::update (scene.cpp:53-59, 267-282): rotate
     * instance 3 by 1.0*dt about WORLD_UP (camera.h:9), setTransform (inverse,
     * bounds, area, bvh.cpp:524-531), then BvhTLAS::refit (bvh.cpp:793-819):
     * leaves re-derive their instances' bounds and GROW their box (no reset,
     * updateNodeBounds :933-944), interior nodes take min/max of children. */
    Scene& S = *h->s;
    Instance& in = S.inst[3];
    in = makeInstance(in.blas, in.mat, rotate(in.M, 1.0f * dt, mk(0.0f, 1.0f, 0.0f)));
    Bvh& b = S.tlas;
    for (int64_t i = (int64_t)b.used - 1; i >= 0; --i) {
        if (i == 1) continue;
        Node& n = b.nodes[(size_t)i];
        if (n.cnt != 0) {
            for (uint32_t k = 0; k < n.cnt; ++k) {
                Instance& x = S.inst[b.idx[n.lf + k]];
                x = makeInstance(x.blas, x.mat, x.M);   /* updateInstanceData: same bounds/area recomputation */
            }
            for (uint32_t k = 0; k < n.cnt; ++k) grow(n.box, S.inst[b.idx[n.lf + k]].bounds);
            continue;
        }
        const Node& l = b.nodes[n.lf];
        const Node& r = b.nodes[n.lf + 1];
        n.box.mn = mk(tmin(l.box.mn.x, r.box.mn.x), tmin(l.box.mn.y, r.box.mn.y), tmin(l.box.mn.z, r.box.mn.z));
        n.box.mx = mk(tmax(l.box.mx.x, r.box.mx.x), tmax(l.box.mx.y, r.box.mx.y), tmax(l.box.mx.z, r.box.mx.z));
    }
}

void orc_path_lengths(orc_scene* h, uint32_t W, uint32_t H, uint32_t frame, uint32_t* out) {
    Scene& S = *h->s;
    if (S.scrW != (float)W || S.scrH != (float)H) setCamera(S, W, H);
    #pragma omp parallel for schedule(dynamic)
    for (int64_t y = 0; y < (int64_t)H; ++y) {
        Counters C; uint32_t sm = 0;
        for (uint32_t x = 0; x < W; ++x) {
            const uint64_t p = (uint64_t)x + (uint64_t)y * W;
            uint32_t seed = seedOf((uint32_t)(p + (uint64_t)frame * 1799u));
            float jy = rndRange(seed, -0.5f, 0.5f);
            float jx = rndRange(seed, -0.5f, 0.5f);
            V3 o, d;
            primaryRay(S, seed, (float)x + jx, (float)y + jy, o, d);
            const uint64_t e0 = C.ext;
            trace(S, seed, o, d, 0, C, nullptr, sm);
            out[p] = (uint32_t)(C.ext - e0);
        }
    }
}

void orc_trace_closest(const orc_scene* h, uint32_t n, const float* o, const float* d,
                       float* ot, float* ou, float* ov, uint32_t* oi, uint32_t* op) {
    const Scene& S = *h->s;
    #pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        float depth = kFarAway;
        Hit hh; hh.inst = kUnset; hh.prim = kUnset; hh.u = 0.0f; hh.v = 0.0f; hh.t = kFarAway;
        uint32_t sm = 0;
        bool hit = tlasTrace<false>(S, mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]), depth, hh, sm);
        ot[i] = depth; ou[i] = hit ? hh.u : 0.0f; ov[i] = hit ? hh.v : 0.0f;
        oi[i] = hit ? hh.inst : kUnset; op[i] = hit ? hh.prim : kUnset;
    }
}

void orc_trace_visits(const orc_scene* h, uint32_t n, const float* o, const float* d, uint32_t* nodes, uint32_t* tris) {
    const Scene& S = *h->s;
    const size_t ni = S.inst.size();
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        float depth = kFarAway;
        Hit hh; hh.inst = kUnset; hh.prim = kUnset; hh.u = 0.0f; hh.v = 0.0f; hh.t = kFarAway;
        uint32_t sm = 0;
        tVisitBaseN = nodes + i * ni; tVisitBaseT = tris + i * ni;
        tlasTrace<false>(S, mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]), depth, hh, sm);
        tVisitBaseN = tVisitBaseT = tVisitNodes = tVisitTris = nullptr;
    }
}

void orc_trace_any(const orc_scene* h, uint32_t n, const float* o, const float* d, const float* tm, uint8_t* out) {
    const Scene& S = *h->s;
    #pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        float depth = tm[i]; Hit hh; uint32_t sm = 0;
        out[i] = tlasTrace<true>(S, mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]), depth, hh, sm) ? 1 : 0;
    }
}

void orc_trace_brute(const orc_scene* h, uint32_t n, const float* o, const float* d, float* ot, uint32_t* oi, uint32_t* op) {
    const Scene& S = *h->s;
    #pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        float depth = kFarAway; uint32_t bi = kUnset, bp = kUnset;
        V3 wo = mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), wd = mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
        for (uint32_t k = 0; k < S.inst.size(); ++k) {
            const Instance& in = S.inst[k];
            V4 tp = mul(in.Minv, v4(wo, 1.0f)), td = mul(in.Minv, v4(wd, 0.0f));
            V3 oo = xyz(tp) / tp.w, dd = xyz(td);
            const Mesh* m = in.blas->mesh;
            for (uint32_t p = 0; p < m->tris.size(); ++p) {
                float u, v;
                if (hitTri(m->tris[p], oo, dd, depth, u, v)) { bi = k; bp = p; }
            }
        }
        ot[i] = depth; oi[i] = bi; op[i] = bp;
    }
}

void orc_record_rays(orc_scene* h, uint32_t W, uint32_t H, uint32_t frame, uint32_t pb, uint32_t pe,
                     uint32_t maxExt, float* eo, float* ed, uint32_t* nExt,
                     uint32_t maxSh, float* so, float* sd, float* st, uint32_t* nSh) {
    Scene& S = *h->s;
    if (S.scrW != (float)W || S.scrH != (float)H) setCamera(S, W, H);
    Recorder rec; rec.maxExt = maxExt; rec.maxSh = maxSh; rec.eo = eo; rec.ed = ed; rec.so = so; rec.sd = sd; rec.st = st;
    Counters C; uint32_t sm = 0;
    for (uint32_t p = pb; p < pe; ++p) {
        uint32_t x = p % W, y = p / W;
        uint32_t seed = seedOf((uint32_t)(p + (uint64_t)frame * 1799u));
        float jy = rndRange(seed, -0.5f, 0.5f);
        float jx = rndRange(seed, -0.5f, 0.5f);
        V3 o, d;
        primaryRay(S, seed, (float)x + jx, (float)y + jy, o, d);
        trace(S, seed, o, d, 0, C, &rec, sm);
    }
    *nExt = rec.nExt; *nSh = rec.nSh;
}

void orc_bvh_depths(const orc_scene* h, uint32_t* td, uint32_t* bd) {
    const Scene& S = *h->s;
    *td = bvhDepth(S.tlas, 0);
    uint32_t m = 0;
    for (auto* b : S.blases) { uint32_t d = bvhDepth(b->bvh, 0); if (d > m) m = d; }
    *bd = m;
}

/* Mesh(path): returns the triangle count (-1 if unreadable); with non-NULL
 * outputs writes 64-B Triangle and 80-B TriExtension records (up to cap). */
long orc_obj_load(const char* path, float* trisOut, float* extOut, uint64_t cap) {
    Mesh m;
    if (!loadObj(path, m)) return -1;
    if (trisOut && extOut) {
        const size_t n = std::min<size_t>(m.tris.size(), cap);
        for (size_t i = 0; i < n; ++i) {
            float* t = trisOut + 16 * i;
            memset(t, 0, 64);
            const Tri& r = m.tris[i];
            t[0] = r.v0.x; t[1] = r.v0.y; t[2] = r.v0.z; t[4] = r.v1.x; t[5] = r.v1.y; t[6] = r.v1.z;
            t[8] = r.v2.x; t[9] = r.v2.y; t[10] = r.v2.z; t[12] = r.c.x; t[13] = r.c.y; t[14] = r.c.z;
            float* x = extOut + 20 * i;
            memset(x, 0, 80);
            const TriExt& e = m.ext[i];
            x[0] = e.n0.x; x[1] = e.n0.y; x[2] = e.n0.z; x[4] = e.n1.x; x[5] = e.n1.y; x[6] = e.n1.z;
            x[8] = e.n2.x; x[9] = e.n2.y; x[10] = e.n2.z;
            for (int j = 0; j < 6; ++j) x[12 + j] = e.uv[j];
        }
    }
    return (long)m.tris.size();
}

/* BvhBLAS::build over raw reference Triangles (64 B: v0, v1, v2, centroid at
 * 16-B strides); writes the index permutation and the node pool as 48-B
 * BvhNode records (leftFirst, count, pad, bbMin, pad, bbMax, pad).  Sequential,
 * the reference's recursion order. */
uint32_t orc_bvh_build(const float* tris, uint32_t n, uint32_t* idxOut, float* nodesOut) {
    Mesh m;
    m.tris.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        const float* t = tris + 16 * (size_t)i;
        Tri& d = m.tris[i];
        d.v0 = V3{t[0], t[1], t[2]}; d.v1 = V3{t[4], t[5], t[6]}; d.v2 = V3{t[8], t[9], t[10]}; d.c = V3{t[12], t[13], t[14]};
    }
    TriPrims P; P.m = &m;
    Bvh b;
    buildBvh(b, P, n);
    memcpy(idxOut, b.idx.data(), (size_t)n * 4);
    for (uint32_t k = 0; k < b.used; ++k) {
        float* o = nodesOut + 12 * (size_t)k;
        memset(o, 0, 48);
        memcpy(o, &b.nodes[k].lf, 4); memcpy(o + 1, &b.nodes[k].cnt, 4);
        o[4] = b.nodes[k].box.mn.x; o[5] = b.nodes[k].box.mn.y; o[6] = b.nodes[k].box.mn.z;
        o[8] = b.nodes[k].box.mx.x; o[9] = b.nodes[k].box.mx.y; o[10] = b.nodes[k].box.mx.z;
    }
    return b.used;
}

void orc_set_zero_cutoff(int on) { gZeroCutoff = on != 0; }

uint32_t orc_init_seed(uint32_t s) { return seedOf(s); }
uint32_t orc_random_u32(uint32_t* s) { return rndU(*s); }
float orc_random_f32(uint32_t* s) { return rndF(*s); }

/* RgbaToU32 with SSE semantics (surf_math.cpp:13-29): x*255 -> cvtps (round to
 * nearest even, NaN/overflow -> INT_MIN) -> unsigned-saturating packs. */
void orc_finalize_rgba8(const float* acc, uint32_t n, float inv, uint32_t* out) {
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t r = 0;
        for (int c = 0; c < 4; ++c) {
            float v = (acc[4 * i + c] * inv) * 255.0f;
            int32_t q;
            if (!(v >= -2147483648.0f && v < 2147483648.0f)) q = INT32_MIN;
            else q = (int32_t)nearbyintf(v);
            uint32_t b = q < 0 ? 0u : (q > 255 ? 255u : (uint32_t)q);
            r |= b << (8 * c);
        }
        out[i] = r;
    }
}

}  // extern "C"
