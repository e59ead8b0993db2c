/*
 * scene_host.cpp -- host half of the product: the reference's Renderer/Scene/BVH
 * host API (surf/surf_host.hpp) and the C-ABI scene helpers of surf_hip.h.
 *
 * Everything here runs once per scene (OBJ parse, BLAS/TLAS binned-SAH build,
 * instance setup, GPUBatcher flattening).  It must produce the exact node
 * arrays the reference would, because BVH topology fixes traversal order and
 * therefore which of two equal-depth hits wins.  Floating point is built with
 * -ffp-contract=off (plain SSE arithmetic, like g++ on the reference).
 */
#include "surf/surf_host.hpp"

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <array>
#include <chrono>
#include <atomic>
#include <cmath>
#include <memory>
#include <thread>
#include <stdexcept>

namespace surf {

/* =================================================================== Mat4 */
Mat4::Mat4(F32 diag) {
    std::memset(c, 0, sizeof c);
    for (int i = 0; i < 4; ++i) c[i][i] = diag;
}

/* glm operator*(mat4, vec4): pairwise column sums (m0 v0 + m1 v1) + (m2 v2 + m3 v3) */
Float4 Mat4::operator*(const Float4& v) const {
    F32 r[4];
    for (int i = 0; i < 4; ++i) {
        const F32 a = c[0][i] * v.x + c[1][i] * v.y;
        const F32 b = c[2][i] * v.z + c[3][i] * v.w;
        r[i] = a + b;
    }
    return Float4(r[0], r[1], r[2], r[3]);
}

Mat4 translate(const Mat4& m, const Float3& v) {
    Mat4 r = m;
    for (int i = 0; i < 4; ++i) {
        F32 s = m.c[0][i] * v.x + m.c[1][i] * v.y;
        s = s + m.c[2][i] * v.z;
        r.c[3][i] = s + m.c[3][i];
    }
    return r;
}

Mat4 scale(const Mat4& m, const Float3& v) {
    Mat4 r = m;
    const F32 k[3] = {v.x, v.y, v.z};
    for (int col = 0; col < 3; ++col)
        for (int i = 0; i < 4; ++i) r.c[col][i] = m.c[col][i] * k[col];
    return r;
}

Mat4 rotate(const Mat4& m, F32 angle, const Float3& axisIn) {
    const F32 cs = cosf(angle), sn = sinf(angle);
    const F32 len2 = (axisIn.x * axisIn.x + axisIn.y * axisIn.y) + axisIn.z * axisIn.z;
    const F32 inv = 1.0f / sqrtf(len2);
    const F32 a[3] = {axisIn.x * inv, axisIn.y * inv, axisIn.z * inv};
    const F32 omc = 1.0f - cs;
    const F32 t[3] = {omc * a[0], omc * a[1], omc * a[2]};
    F32 rot[3][3];
    rot[0][0] = cs + t[0] * a[0];
    rot[0][1] = t[0] * a[1] + sn * a[2];
    rot[0][2] = t[0] * a[2] - sn * a[1];
    rot[1][0] = t[1] * a[0] - sn * a[2];
    rot[1][1] = cs + t[1] * a[1];
    rot[1][2] = t[1] * a[2] + sn * a[0];
    rot[2][0] = t[2] * a[0] + sn * a[1];
    rot[2][1] = t[2] * a[1] - sn * a[0];
    rot[2][2] = cs + t[2] * a[2];
    Mat4 r(0.0f);
    for (int col = 0; col < 3; ++col)
        for (int i = 0; i < 4; ++i) {
            F32 s = m.c[0][i] * rot[col][0] + m.c[1][i] * rot[col][1];
            r.c[col][i] = s + m.c[2][i] * rot[col][2];
        }
    for (int i = 0; i < 4; ++i) r.c[3][i] = m.c[3][i];
    return r;
}

/* glm compute_inverse<4,4>: cofactors, sign pattern, det from row 0. */
Mat4 inverse(const Mat4& m) {
    const auto& a = m.c;
    const F32 k00 = a[2][2] * a[3][3] - a[3][2] * a[2][3];
    const F32 k02 = a[1][2] * a[3][3] - a[3][2] * a[1][3];
    const F32 k03 = a[1][2] * a[2][3] - a[2][2] * a[1][3];
    const F32 k04 = a[2][1] * a[3][3] - a[3][1] * a[2][3];
    const F32 k06 = a[1][1] * a[3][3] - a[3][1] * a[1][3];
    const F32 k07 = a[1][1] * a[2][3] - a[2][1] * a[1][3];
    const F32 k08 = a[2][1] * a[3][2] - a[3][1] * a[2][2];
    const F32 k10 = a[1][1] * a[3][2] - a[3][1] * a[1][2];
    const F32 k11 = a[1][1] * a[2][2] - a[2][1] * a[1][2];
    const F32 k12 = a[2][0] * a[3][3] - a[3][0] * a[2][3];
    const F32 k14 = a[1][0] * a[3][3] - a[3][0] * a[1][3];
    const F32 k15 = a[1][0] * a[2][3] - a[2][0] * a[1][3];
    const F32 k16 = a[2][0] * a[3][2] - a[3][0] * a[2][2];
    const F32 k18 = a[1][0] * a[3][2] - a[3][0] * a[1][2];
    const F32 k19 = a[1][0] * a[2][2] - a[2][0] * a[1][2];
    const F32 k20 = a[2][0] * a[3][1] - a[3][0] * a[2][1];
    const F32 k22 = a[1][0] * a[3][1] - a[3][0] * a[1][1];
    const F32 k23 = a[1][0] * a[2][1] - a[2][0] * a[1][1];
    const F32 f0[4] = {k00, k00, k02, k03}, f1[4] = {k04, k04, k06, k07}, f2[4] = {k08, k08, k10, k11};
    const F32 f3[4] = {k12, k12, k14, k15}, f4[4] = {k16, k16, k18, k19}, f5[4] = {k20, k20, k22, k23};
    const F32 w0[4] = {a[1][0], a[0][0], a[0][0], a[0][0]};
    const F32 w1[4] = {a[1][1], a[0][1], a[0][1], a[0][1]};
    const F32 w2[4] = {a[1][2], a[0][2], a[0][2], a[0][2]};
    const F32 w3[4] = {a[1][3], a[0][3], a[0][3], a[0][3]};
    Mat4 inv(0.0f);
    for (int i = 0; i < 4; ++i) {
        const F32 sa = (i & 1) ? -1.0f : 1.0f, sb = -sa;
        inv.c[0][i] = ((w1[i] * f0[i] - w2[i] * f1[i]) + w3[i] * f2[i]) * sa;
        inv.c[1][i] = ((w0[i] * f0[i] - w2[i] * f3[i]) + w3[i] * f4[i]) * sb;
        inv.c[2][i] = ((w0[i] * f1[i] - w1[i] * f3[i]) + w3[i] * f5[i]) * sa;
        inv.c[3][i] = ((w0[i] * f2[i] - w1[i] * f4[i]) + w2[i] * f5[i]) * sb;
    }
    const F32 d01 = a[0][0] * inv.c[0][0] + a[0][1] * inv.c[1][0];
    const F32 d23 = a[0][2] * inv.c[2][0] + a[0][3] * inv.c[3][0];
    const F32 rdet = 1.0f / (d01 + d23);
    for (int col = 0; col < 4; ++col)
        for (int i = 0; i < 4; ++i) inv.c[col][i] = inv.c[col][i] * rdet;
    return inv;
}

static inline Float3 dehomog(const Float4& v) { return Float3(v.x, v.y, v.z) / v.w; }

/* =================================================================== Mesh */
Triangle::Triangle(Float3 a, Float3 b, Float3 c) : v0(b), v1(a), v2(c), centroid(0.0f) {
    centroid = (v0 + v1 + v2) * 0.333f;               /* mesh.cpp:20 */
}

unsigned defaultBuildThreads() {
    if (const char* e = getenv("SURF_BUILD_THREADS")) { const int v = atoi(e); if (v > 0) return (unsigned)v; }
    if (const char* e = getenv("OMP_NUM_THREADS")) { const int v = atoi(e); if (v > 0) return (unsigned)v; }
    const unsigned hc = std::thread::hardware_concurrency();
    return hc ? std::min(hc, 64u) : 1u;
}

namespace {

/* Runs f(chunk) for chunk in [0, n) on up to `threads` threads. */
template <class F>
void forChunks(U32 n, unsigned threads, F&& f) {
    const unsigned t = std::min<unsigned>(threads, n);
    if (t <= 1) { for (U32 c = 0; c < n; ++c) f(c); return; }
    std::atomic<U32> next{0};
    auto work = [&]() { for (U32 c; (c = next.fetch_add(1)) < n;) f(c); };
    std::vector<std::thread> pool;
    for (unsigned i = 1; i < t; ++i) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

std::string slurp(const std::string& path) {
    /* plain files in one read; gzip (magic 1f 8b) through zlib */
    if (FILE* f = fopen(path.c_str(), "rb")) {
        unsigned char magic[2] = {0, 0};
        const size_t m = fread(magic, 1, 2, f);
        if (!(m == 2 && magic[0] == 0x1f && magic[1] == 0x8b) && fseek(f, 0, SEEK_END) == 0) {
            const long size = ftell(f);
            std::string out;
            if (size >= 0) {
                out.resize((size_t)size);
                rewind(f);
                const size_t got = size ? fread(&out[0], 1, (size_t)size, f) : 0;
                fclose(f);
                if (got != (size_t)size) throw std::runtime_error("short read " + path);
                return out;
            }
        }
        fclose(f);
    }
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open " + path);
    std::string out;
    std::vector<char> buf(1 << 20);
    for (;;) {
        const int k = gzread(f, buf.data(), (unsigned)buf.size());
        if (k <= 0) break;
        out.append(buf.data(), (size_t)k);
    }
    gzclose(f);
    return out;
}

/* Resolves a 1-based / negative OBJ index against `count` records. */
inline long objIndex(long raw, size_t count) {
    if (raw > 0) return raw - 1;
    if (raw < 0) return (long)count + raw;
    return -1;
}

struct Corner { long v = -1, t = -1, n = -1; };

/* OBJ ingestion: tinyobjloader-compatible semantics
 * (mesh.cpp:69-154, triangulate = true) parsed in parallel chunks.
 *
 * The text is cut into chunks at line starts.  Pass 1 (parallel) parses every
 * chunk on its own: v / vn / vt records into chunk-local arrays and faces as
 * raw OBJ indices together with the chunk-local record counts at that line --
 * all a relative (negative) index needs.  A prefix sum over the chunks' counts
 * then fixes every record's global position, so pass 2 (parallel) resolves the
 * indices exactly as a front-to-back reader would (1-based, or relative to the
 * records read so far) and writes the triangles at their global offsets.
 * Lines are cut at '\n' in place, so every number is parsed from a
 * NUL-terminated line, exactly like the line-by-line reader.  Floats go through
 * strtod then narrow to float (tinyobj's real_t = float path). */
struct ObjFace {
    uint32_t first, n;               /* corners [first, first + n) of the chunk */
    uint32_t lv, lt, ln;             /* chunk-local record counts before this face */
};
struct RawCorner { long v, t, n; bool hasT, hasN; };
struct ObjChunk {
    char* b = nullptr;
    char* e = nullptr;
    std::vector<F32> pos, nrm, tex;
    std::vector<RawCorner> corners;
    std::vector<ObjFace> faces;
    size_t tris = 0;
};

void parseChunk(ObjChunk& C) {
    char* p = C.b;
    while (p < C.e) {
        char* eol = static_cast<char*>(memchr(p, '\n', (size_t)(C.e - p)));
        if (!eol) eol = C.e;
        *eol = '\0';                                    /* one NUL-terminated line */
        const char* s = p;
        p = eol + 1;
        while (*s == ' ' || *s == '\t') ++s;
        auto floats = [&](const char* q, int k, std::vector<F32>& dst) {
            char* e = nullptr;
            for (int i = 0; i < k; ++i) { dst.push_back((F32)strtod(q, &e)); q = e; }
        };
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) floats(s + 2, 3, C.pos);
        else if (s[0] == 'v' && s[1] == 'n') floats(s + 2, 3, C.nrm);
        else if (s[0] == 'v' && s[1] == 't') floats(s + 2, 2, C.tex);
        else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            ObjFace f;
            f.first = (uint32_t)C.corners.size();
            f.lv = (uint32_t)(C.pos.size() / 3); f.lt = (uint32_t)(C.tex.size() / 2); f.ln = (uint32_t)(C.nrm.size() / 3);
            const char* q = s + 1;
            while (true) {
                while (*q == ' ' || *q == '\t' || *q == '\r') ++q;
                if (*q == '\0') break;
                RawCorner c{0, 0, 0, false, false};
                char* e = nullptr;
                c.v = strtol(q, &e, 10);
                q = e;
                if (*q == '/') {
                    ++q;
                    if (*q != '/') { c.t = strtol(q, &e, 10); c.hasT = true; q = e; }
                    if (*q == '/') { ++q; c.n = strtol(q, &e, 10); c.hasN = true; q = e; }
                }
                C.corners.push_back(c);
                while (*q && *q != ' ' && *q != '\t') ++q;
            }
            f.n = (uint32_t)(C.corners.size() - f.first);
            if (f.n < 3) { C.corners.resize(f.first); continue; }
            C.faces.push_back(f);
            C.tris += f.n - 2;                          /* quad: 2, n-gon fan: n - 2 */
        }
    }
}

void parseObj(std::string& text, Mesh& mesh, unsigned threads) {
    const size_t len = text.size();
    if (len == 0) return;
    char* base = &text[0];
    /* chunks of >= 1 MiB starting at line starts */
    const size_t want = std::max<size_t>(1, std::min<size_t>((size_t)threads * 4, len / (1u << 20) + 1));
    std::vector<ObjChunk> chunks;
    size_t at = 0;
    for (size_t k = 0; k < want && at < len; ++k) {
        size_t end = (k + 1 == want) ? len : std::max(at, len * (k + 1) / want);
        if (end < len) {
            const char* nl = static_cast<const char*>(memchr(base + end, '\n', len - end));
            end = nl ? (size_t)(nl - base) + 1 : len;
        }
        ObjChunk c;
        c.b = base + at;
        c.e = base + end;
        chunks.push_back(std::move(c));
        at = end;
    }
    const U32 nc = (U32)chunks.size();
    forChunks(nc, threads, [&](U32 k) { parseChunk(chunks[k]); });
    /* global record offsets of every chunk */
    std::vector<size_t> vBase(nc + 1, 0), tBase(nc + 1, 0), nBase(nc + 1, 0), triBase(nc + 1, 0);
    for (U32 k = 0; k < nc; ++k) {
        vBase[k + 1] = vBase[k] + chunks[k].pos.size() / 3;
        tBase[k + 1] = tBase[k] + chunks[k].tex.size() / 2;
        nBase[k + 1] = nBase[k] + chunks[k].nrm.size() / 3;
        triBase[k + 1] = triBase[k] + chunks[k].tris;
    }
    std::vector<F32> pos(3 * vBase[nc]), nrm(3 * nBase[nc]), tex(2 * tBase[nc]);
    forChunks(nc, threads, [&](U32 k) {
        std::copy(chunks[k].pos.begin(), chunks[k].pos.end(), pos.begin() + 3 * vBase[k]);
        std::copy(chunks[k].nrm.begin(), chunks[k].nrm.end(), nrm.begin() + 3 * nBase[k]);
        std::copy(chunks[k].tex.begin(), chunks[k].tex.end(), tex.begin() + 2 * tBase[k]);
        std::vector<F32>().swap(chunks[k].pos);
        std::vector<F32>().swap(chunks[k].nrm);
        std::vector<F32>().swap(chunks[k].tex);
    });
    const size_t nt = triBase[nc];
    mesh.triangles.assign(nt, Triangle(Float3(0.0f), Float3(0.0f), Float3(0.0f)));
    mesh.triExtensions.assign(nt, TriExtension{});
    std::atomic<bool> bad{false};
    forChunks(nc, threads, [&](U32 k) {
        const ObjChunk& C = chunks[k];
        size_t out = triBase[k];
        auto resolve = [&](const RawCorner& r, const ObjFace& f) {
            Corner c;
            c.v = objIndex(r.v, vBase[k] + f.lv);
            if (r.hasT) c.t = objIndex(r.t, tBase[k] + f.lt);
            if (r.hasN) c.n = objIndex(r.n, nBase[k] + f.ln);
            return c;
        };
        auto vtx = [&](const Corner& c, bool& ok) {
            if (c.v < 0 || (size_t)(3 * c.v + 2) >= pos.size()) { ok = false; return Float3(0.0f); }
            return Float3(pos[3 * c.v], pos[3 * c.v + 1], pos[3 * c.v + 2]);
        };
        auto nor = [&](const Corner& c) {
            if (c.n < 0 || (size_t)(3 * c.n + 2) >= nrm.size()) return Float3(0.0f);
            return Float3(nrm[3 * c.n], nrm[3 * c.n + 1], nrm[3 * c.n + 2]);
        };
        auto uv = [&](const Corner& c) {
            if (c.t < 0 || (size_t)(2 * c.t + 1) >= tex.size()) return Float2(0.0f, 0.0f);
            return Float2(tex[2 * c.t], tex[2 * c.t + 1]);
        };
        bool ok = true;
        Corner face[64];
        std::vector<Corner> big;
        for (const ObjFace& f : C.faces) {
            Corner* fc = face;
            if (f.n > 64) { big.resize(f.n); fc = big.data(); }
            for (uint32_t j = 0; j < f.n; ++j) fc[j] = resolve(C.corners[f.first + j], f);
            auto emit = [&](const Corner& a, const Corner& b, const Corner& c) {
                mesh.triangles[out] = Triangle(vtx(a, ok), vtx(b, ok), vtx(c, ok));
                TriExtension& x = mesh.triExtensions[out];
                x.n0 = nor(a); x.n1 = nor(b); x.n2 = nor(c);
                x.uv0 = uv(a); x.uv1 = uv(b); x.uv2 = uv(c);
                ++out;
            };
            if (f.n == 4) {
                /* quad: split on the shorter diagonal; ties -> (0,1,3),(1,2,3) */
                const Float3 d02 = vtx(fc[2], ok) - vtx(fc[0], ok), d13 = vtx(fc[3], ok) - vtx(fc[1], ok);
                const F32 l02 = d02.x * d02.x + d02.y * d02.y + d02.z * d02.z;
                const F32 l13 = d13.x * d13.x + d13.y * d13.y + d13.z * d13.z;
                if (l02 < l13) { emit(fc[0], fc[1], fc[2]); emit(fc[0], fc[2], fc[3]); }
                else { emit(fc[0], fc[1], fc[3]); emit(fc[1], fc[2], fc[3]); }
            } else {
                for (uint32_t j = 1; j + 1 < f.n; ++j) emit(fc[0], fc[j], fc[j + 1]);
            }
        }
        if (!ok) bad = true;
    });
    if (bad) throw std::runtime_error("OBJ vertex index out of range");
}

}  // namespace

Mesh::Mesh(const std::string& path) : Mesh(path, defaultBuildThreads()) {}

Mesh::Mesh(const std::string& path, unsigned threads) {
    const bool log = getenv("SURF_BUILD_LOG") != nullptr;
    auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = now();
    std::string text;
    try { text = slurp(path); }
    catch (const std::exception&) { text = slurp(path + ".gz"); }
    const double t1 = now();
    parseObj(text, *this, std::max(1u, threads));
    if (log) fprintf(stderr, "[surf obj] %s: read %.3f s, parse %.3f s, %zu triangles\n", path.c_str(), t1 - t0, now() - t1, triangles.size());
}

/* =================================================================== AABB */
F32 AABB::area() const { const Float3 e = bbMax - bbMin; return e.x * e.y + e.y * e.z + e.z * e.x; }
Float3 AABB::center() const { return 0.5f * (bbMax - bbMin); }

/* ========================================================= binned SAH build
 * One builder for both levels.  Prim access is a policy: key(p, axis) is the
 * binning coordinate, addTo(box, p) grows a box by the primitive.  Build order
 * reproduces the reference's recursive subdivide exactly (pre-order, children
 * allocated in pairs at split time).
 *
 * Parallel build.  Two facts make a multi-threaded build
 * produce the reference's arrays byte for byte:
 *   - every reduction in findSplitPlane/updateNodeBounds is a min, a max or an
 *     integer count, which are order-independent for finite inputs (checked
 *     once; a non-finite key or vertex selects the sequential builder), and the
 *     sweep over the 8 bins is done exactly as the reference does it;
 *   - subdivide(X) allocates all nodes of X's subtree in one contiguous block
 *     of the pool that starts at the `used` value on entry, so a subtree built
 *     elsewhere with local numbering only needs its interior child indices
 *     shifted by the block's final base.
 * Large nodes bin in parallel chunks and run their two children concurrently;
 * the index partition stays the reference's sequential swap loop (it defines
 * the index order).  Subtrees below kSeqPrims are built by the sequential
 * builder into a local block, then placed with one offset. */
namespace {

constexpr int kBins = 8;
constexpr int kPlanes = kBins - 1;
constexpr U32 kSeqPrims = 1u << 15;          /* subtree size built sequentially */
constexpr U32 kChunk = 1u << 16;             /* prims per binning chunk */

}  // namespace

namespace {

/* Per-axis bins of one node (bvh.cpp:302-340). */
struct Bins {
    F32 lo[3], hi[3];
    U32 cnt[3][kBins];
    AABB box[3][kBins];
};

/* A primitive as the build sees it: its binning key, its id and its box (the
 * box of its vertices, or the instance bounds).  The build permutes these
 * records in place of the reference's index array (same swaps), so every pass
 * streams through memory; the index array is read off the ids at the end. */
struct alignas(16) PrimRef {
    F32 key[3];
    U32 id;
    AABB box;
};

template <class Prims>
struct SahBuilder {
    const Prims& prims;
    std::vector<U32>& idx;
    std::vector<PrimRef>& refs;
    std::vector<BvhNode>& nodes;
    U32& used;
    unsigned threads = 1;
    std::atomic<int>* active = nullptr;           /* concurrent subtree builders */

    unsigned chunkThreads() const {
        const int a = active ? active->load() : 0;      /* extra builder threads */
        return std::max(1u, threads / (unsigned)(1 + a));
    }

    void bounds(BvhNode& n) const {
        for (U32 i = 0; i < n.count; ++i) n.boundingBox.grow(refs[n.leftFirst + i].box);
    }

    /* updateNodeBounds over parallel chunks (min/max: exact in any order) */
    void boundsPar(BvhNode& n) const {
        const U32 nc = (n.count + kChunk - 1) / kChunk;
        std::vector<AABB> part(nc);
        forChunks(nc, chunkThreads(), [&](U32 c) {
            const U32 b = n.leftFirst + c * kChunk, e = std::min(n.leftFirst + n.count, b + kChunk);
            for (U32 i = b; i < e; ++i) part[c].grow(refs[i].box);
        });
        for (const AABB& p : part) n.boundingBox.grow(p);
    }

    /* The sweep over the bins and the cost comparison (bvh.cpp:341-377). */
    static void sweep(const U32* cnt, const AABB* box, F32 lo, F32 hi, U32 axis, F32& bestCost, F32& bestSplit,
                      U32& bestAxis) {
        F32 lArea[kPlanes], rArea[kPlanes];
        U32 lCnt[kPlanes], rCnt[kPlanes];
        AABB lBox, rBox;
        U32 lSum = 0, rSum = 0;
        for (int k = 0; k < kPlanes; ++k) {
            lSum += cnt[k];
            lCnt[k] = lSum;
            lBox.grow(box[k]);
            lArea[k] = lBox.area();
            const int rb = kBins - 1 - k;
            rSum += cnt[rb];
            rCnt[rb - 1] = rSum;
            rBox.grow(box[rb]);
            rArea[rb - 1] = rBox.area();
        }
        const F32 extent = (hi - lo) / (F32)kBins;
        for (int k = 0; k < kPlanes; ++k) {
            const F32 c = (F32)lCnt[k] * lArea[k] + (F32)rCnt[k] * rArea[k];
            if (c < bestCost) {
                bestCost = c;
                bestSplit = lo + extent * (F32)(k + 1);
                bestAxis = axis;
            }
        }
    }

    static U32 binOf(F32 key, F32 lo, F32 scaleK) {
        const size_t s = (size_t)((key - lo) * scaleK);
        return (U32)(s < (size_t)(kBins - 1) ? s : (size_t)(kBins - 1));
    }

    /* findSplitPlane (bvh.cpp:294-377); returns split position, cost/axis out.
     * The reference makes two passes per axis (key range, then bins); here one
     * pass finds all three key ranges and one pass fills all three axes' bins
     * from the triangle's box.  Same values: min, max and counts only. */
    F32 plane(const BvhNode& n, F32& bestCost, U32& bestAxis) const {
        bestCost = INFINITY;
        bestAxis = 0;
        F32 bestSplit = 0.0f;
        const U32 first = n.leftFirst, cnt = n.count;
        F32 lo[3] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f};   /* F32_MAX / F32_MIN (sic) */
        F32 hi[3] = {1.17549435e-38f, 1.17549435e-38f, 1.17549435e-38f};
        for (U32 i = 0; i < cnt; ++i)
            for (U32 a = 0; a < 3; ++a) {
                const F32 k = refs[first + i].key[a];
                lo[a] = lo[a] < k ? lo[a] : k;
                hi[a] = hi[a] > k ? hi[a] : k;
            }
        F32 scaleK[3];
        U32 binCount[3][kBins] = {};
        AABB binBox[3][kBins];
        for (U32 a = 0; a < 3; ++a) scaleK[a] = lo[a] == hi[a] ? 0.0f : (F32)kBins / (hi[a] - lo[a]);
        for (U32 i = 0; i < cnt; ++i) {
            const PrimRef& pr = refs[first + i];
            const AABB& tb = pr.box;
            for (U32 a = 0; a < 3; ++a) {
                if (lo[a] == hi[a]) continue;
                const U32 k = binOf(pr.key[a], lo[a], scaleK[a]);
                binCount[a][k]++;
                binBox[a][k].grow(tb);
            }
        }
        for (U32 a = 0; a < 3; ++a)
            if (lo[a] != hi[a]) sweep(binCount[a], binBox[a], lo[a], hi[a], a, bestCost, bestSplit, bestAxis);
        return bestSplit;
    }

    /* Same result as plane(): the three axes' key ranges and bins are min/max
     * and count reductions over parallel chunks, merged in chunk order. */
    F32 planePar(const BvhNode& n, F32& bestCost, U32& bestAxis) const {
        bestCost = INFINITY;
        bestAxis = 0;
        F32 bestSplit = 0.0f;
        const U32 first = n.leftFirst, cnt = n.count;
        const U32 nc = (cnt + kChunk - 1) / kChunk;
        std::vector<std::array<F32, 6>> rng(nc);
        forChunks(nc, chunkThreads(), [&](U32 c) {
            F32 lo[3] = {3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f};
            F32 hi[3] = {1.17549435e-38f, 1.17549435e-38f, 1.17549435e-38f};
            const U32 b = first + c * kChunk, e = std::min(first + cnt, b + kChunk);
            for (U32 i = b; i < e; ++i)
                for (U32 a = 0; a < 3; ++a) {
                    const F32 k = refs[i].key[a];
                    lo[a] = lo[a] < k ? lo[a] : k;
                    hi[a] = hi[a] > k ? hi[a] : k;
                }
            rng[c] = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
        });
        Bins B;
        for (U32 a = 0; a < 3; ++a) {
            F32 lo = 3.40282347e+38f, hi = 1.17549435e-38f;
            for (U32 c = 0; c < nc; ++c) { lo = lo < rng[c][a] ? lo : rng[c][a]; hi = hi > rng[c][3 + a] ? hi : rng[c][3 + a]; }
            B.lo[a] = lo; B.hi[a] = hi;
        }
        std::vector<Bins> part(nc);
        forChunks(nc, chunkThreads(), [&](U32 c) {
            Bins& P = part[c];
            F32 scaleK[3];
            for (U32 a = 0; a < 3; ++a) {
                scaleK[a] = B.lo[a] == B.hi[a] ? 0.0f : (F32)kBins / (B.hi[a] - B.lo[a]);
                for (int k = 0; k < kBins; ++k) { P.cnt[a][k] = 0; P.box[a][k] = AABB(); }
            }
            const U32 b = first + c * kChunk, e = std::min(first + cnt, b + kChunk);
            for (U32 i = b; i < e; ++i) {
                const PrimRef& pr = refs[i];
                const AABB& tb = pr.box;
                for (U32 a = 0; a < 3; ++a) {
                    if (B.lo[a] == B.hi[a]) continue;
                    const U32 k = binOf(pr.key[a], B.lo[a], scaleK[a]);
                    P.cnt[a][k]++;
                    P.box[a][k].grow(tb);
                }
            }
        });
        for (U32 a = 0; a < 3; ++a) {
            if (B.lo[a] == B.hi[a]) continue;
            for (int k = 0; k < kBins; ++k) {
                B.cnt[a][k] = 0; B.box[a][k] = AABB();
                for (U32 c = 0; c < nc; ++c) { B.cnt[a][k] += part[c].cnt[a][k]; B.box[a][k].grow(part[c].box[a][k]); }
            }
            sweep(B.cnt[a], B.box[a], B.lo[a], B.hi[a], a, bestCost, bestSplit, bestAxis);
        }
        return bestSplit;
    }

    /* partitionNode (bvh.cpp:379-399): the reference's swap loop */
    U32 split(const BvhNode& n, F32 pos, U32 axis) {
        I32 i = (I32)n.leftFirst;
        I32 j = (I32)(n.leftFirst + (n.count - 1));
        while (i <= j) {
            if (refs[i].key[axis] < pos) ++i;
            else { std::swap(refs[i], refs[j]); --j; }
        }
        return (U32)i;
    }

    /* subdivide (bvh.cpp:401-465) from `start` with an explicit stack; nodes
     * are appended at `used` (pairs), left subtree first like the recursion. */
    void grow(U32 start) {
        std::vector<U32> todo{start};
        while (!todo.empty()) {
            const U32 ni = todo.back();
            todo.pop_back();
            F32 cost; U32 axis;
            const F32 pos = plane(nodes[ni], cost, axis);
            if (cost >= (F32)nodes[ni].count * nodes[ni].boundingBox.area()) continue;
            const U32 pivot = split(nodes[ni], pos, axis);
            const U32 nl = pivot - nodes[ni].leftFirst;
            if (nl == 0 || nl == nodes[ni].count) continue;
            const U32 l = used, r = used + 1;
            used += 2;
            if (nodes.size() < used) nodes.resize(std::max<size_t>(used, 2 * nodes.size()));
            nodes[l].leftFirst = nodes[ni].leftFirst; nodes[l].count = nl; nodes[l].boundingBox = AABB();
            nodes[r].leftFirst = pivot; nodes[r].count = nodes[ni].count - nl; nodes[r].boundingBox = AABB();
            nodes[ni].leftFirst = l;
            nodes[ni].count = 0;
            bounds(nodes[l]);
            bounds(nodes[r]);
            todo.push_back(r);
            todo.push_back(l);
        }
    }

    /* A subtree built away from the pool: its root record, and either a local
     * block (sequential build; local slot 0 is the root, children from 1) or
     * two child subtrees.  size = nodes the subtree allocates in the pool. */
    struct Sub {
        BvhNode root;
        std::vector<BvhNode> block;
        std::unique_ptr<Sub> l, r;
        size_t size = 0;
    };

    std::unique_ptr<Sub> buildSub(BvhNode root) {
        auto s = std::make_unique<Sub>();
        if (root.count < kSeqPrims) {
            std::vector<BvhNode> loc(1, root);
            U32 u = 1;
            SahBuilder<Prims> seq{prims, idx, refs, loc, u, 1, nullptr};
            seq.grow(0);
            loc.resize(u);
            s->root = loc[0];
            s->size = u - 1;
            s->block = std::move(loc);
            return s;
        }
        F32 cost; U32 axis;
        const F32 pos = planePar(root, cost, axis);
        s->root = root;
        if (cost >= (F32)root.count * root.boundingBox.area()) return s;
        const U32 pivot = split(root, pos, axis);
        const U32 nl = pivot - root.leftFirst;
        if (nl == 0 || nl == root.count) return s;
        BvhNode L, R;
        L.leftFirst = root.leftFirst; L.count = nl; L.boundingBox = AABB();
        R.leftFirst = pivot; R.count = root.count - nl; R.boundingBox = AABB();
        if (L.count >= kSeqPrims) boundsPar(L); else bounds(L);
        if (R.count >= kSeqPrims) boundsPar(R); else bounds(R);
        /* the children own disjoint index ranges: the left one runs on a new
         * thread while fewer than threads-1 extra builder threads exist */
        int cur = active->load();
        bool spawn = false;
        while (cur < (int)threads - 1 && !(spawn = active->compare_exchange_weak(cur, cur + 1))) {}
        if (spawn) {
            std::thread lt([&]() { s->l = buildSub(L); });
            s->r = buildSub(R);
            lt.join();
            active->fetch_sub(1);
        } else {
            s->l = buildSub(L);
            s->r = buildSub(R);
        }
        s->root.count = 0;
        s->size = 2 + s->l->size + s->r->size;
        return s;
    }

    /* Writes subtree s with its root at pool slot `at` and its block at
     * `base`; sequential blocks are queued for a parallel copy. */
    void place(Sub& s, U32 at, U32 base, std::vector<std::pair<Sub*, U32>>& jobs) {
        nodes[at] = s.root;
        if (!s.block.empty()) {
            if (s.size == 0) return;
            nodes[at].leftFirst = base + (s.root.leftFirst - 1);
            jobs.emplace_back(&s, base);
            return;
        }
        if (!s.l) return;                                /* leaf */
        nodes[at].leftFirst = base;
        place(*s.l, base, base + 2, jobs);
        place(*s.r, base + 1, base + 2 + (U32)s.l->size, jobs);
    }

    void run(U32 count, bool finite) {
        const bool log = getenv("SURF_BUILD_LOG") != nullptr && count >= kSeqPrims;
        auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        double t0 = now();
        auto phase = [&](const char* what) {
            if (log) fprintf(stderr, "[surf build]   %-12s %8.3f s\n", what, now() - t0);
            t0 = now();
        };
        refs.resize(count);
        forChunks((count + kChunk - 1) / kChunk, threads, [&](U32 c) {
            const U32 b = c * kChunk, e = std::min(count, b + kChunk);
            for (U32 i = b; i < e; ++i) {
                PrimRef& r = refs[i];
                for (U32 a = 0; a < 3; ++a) r.key[a] = prims.key(i, a);
                r.id = i;
                r.box = AABB();
                prims.addTo(r.box, i);
            }
        });
        auto ids = [&]() {
            idx.resize(count);
            forChunks((count + kChunk - 1) / kChunk, threads, [&](U32 c) {
                const U32 b = c * kChunk, e = std::min(count, b + kChunk);
                for (U32 i = b; i < e; ++i) idx[i] = refs[i].id;
            });
            std::vector<PrimRef>().swap(refs);
        };
        BvhNode zero;                                /* MALLOC64 + memset(0): root box starts at the origin */
        zero.leftFirst = 0;
        zero.count = 0;
        zero.boundingBox.bbMin = Float3(0.0f);
        zero.boundingBox.bbMax = Float3(0.0f);
        if (threads <= 1 || !finite || count < kSeqPrims) {
            nodes.assign(2 * (size_t)count, zero);
            used = 2;
            nodes[0].leftFirst = 0;
            nodes[0].count = count;
            bounds(nodes[0]);
            grow(0);
            ids();
            return;
        }
        /* only [0, used) of the reference's 2*count pool is ever read; node 1 stays zero */
        BvhNode root = zero;
        root.count = count;
        std::atomic<int> act{0};
        active = &act;
        boundsPar(root);
        phase("root bounds");
        std::unique_ptr<Sub> tree = buildSub(root);
        phase("subtrees");
        used = 2 + (U32)tree->size;
        nodes.clear();
        nodes.resize(used, zero);
        phase("pool alloc");
        std::vector<std::pair<Sub*, U32>> jobs;
        place(*tree, 0, 2, jobs);
        forChunks((U32)jobs.size(), threads, [&](U32 j) {
            const Sub& b = *jobs[j].first;
            const U32 base = jobs[j].second;
            for (size_t k = 1; k < b.block.size(); ++k) {
                BvhNode n = b.block[k];
                if (n.count == 0) n.leftFirst = base + (n.leftFirst - 1);
                nodes[base + (k - 1)] = n;
            }
        });
        phase("place");
        tree.reset();
        ids();
        phase("ids, free");
    }
};

struct MeshPrims {
    const Mesh* mesh;
    F32 key(U32 p, U32 axis) const { return (&mesh->triangles[p].centroid.x)[axis]; }
    void addTo(AABB& b, U32 p) const {
        const Triangle& t = mesh->triangles[p];
        b.grow(t.v0); b.grow(t.v1); b.grow(t.v2);
    }
};

struct InstancePrims {
    const std::vector<Instance>* inst;
    F32 key(U32 p, U32 axis) const { return (*inst)[p].bounds.center()[axis]; }
    void addTo(AABB& b, U32 p) const { b.grow((*inst)[p].bounds); }
};

U32 depthOf(const std::vector<BvhNode>& nodes, U32 root) {
    U32 best = 0;
    std::vector<std::pair<U32, U32>> st{{root, 0}};
    while (!st.empty()) {
        auto [n, d] = st.back();
        st.pop_back();
        if (nodes[n].count != 0) { best = std::max(best, d); continue; }
        st.push_back({nodes[n].leftFirst, d + 1});
        st.push_back({nodes[n].leftFirst + 1, d + 1});
    }
    return best;
}

}  // namespace

/* ================================================================= BvhBLAS */
BvhBLAS::BvhBLAS(Mesh* mesh) : m_mesh(mesh) { build(); }
BvhBLAS::BvhBLAS(Mesh* mesh, unsigned threads) : m_mesh(mesh) { build(threads); }

void BvhBLAS::build() { build(defaultBuildThreads()); }

void BvhBLAS::build(unsigned threads) {
    MeshPrims prims{m_mesh};
    std::vector<PrimRef> refs;
    SahBuilder<MeshPrims> b{prims, m_indices, refs, m_nodes, m_nodesUsed, threads};
    bool finite = true;
    for (const Triangle& t : m_mesh->triangles)
        for (const Float3* v : {&t.v0, &t.v1, &t.v2, &t.centroid})
            finite = finite && std::isfinite(v->x) && std::isfinite(v->y) && std::isfinite(v->z);
    b.run((U32)m_mesh->triangles.size(), finite);
}

/* bvh.cpp:268-287 */
void BvhBLAS::refit() {
    MeshPrims prims{m_mesh};
    for (int64_t i = (int64_t)m_nodesUsed - 1; i >= 0; --i) {
        if (i == 1) continue;
        BvhNode& n = m_nodes[(size_t)i];
        if (n.isLeaf()) {
            for (U32 k = 0; k < n.count; ++k) prims.addTo(n.boundingBox, m_indices[n.leftFirst + k]);
            continue;
        }
        const BvhNode& l = m_nodes[n.leftFirst];
        const BvhNode& r = m_nodes[n.leftFirst + 1];
        n.boundingBox.bbMin = min(l.boundingBox.bbMin, r.boundingBox.bbMin);
        n.boundingBox.bbMax = max(l.boundingBox.bbMax, r.boundingBox.bbMax);
    }
}

U32 BvhBLAS::depth() const { return depthOf(m_nodes, 0); }

/* ================================================================ Instance */
Instance::Instance(BvhBLAS* blas, Material* mat, Mat4 transform)
    : bvh(blas), material(mat), m_transform(transform), m_invTransform(1.0f) {
    setTransform(transform);
}

void Instance::setTransform(const Mat4& transform) {            /* bvh.cpp:524-531 */
    m_invTransform = inverse(transform);
    m_transform = transform;
    updateBounds();
    calculateMeshArea();
}

void Instance::updateBounds() {                                  /* bvh.cpp:554-575 */
    const AABB& lb = bvh->bounds();
    bounds = AABB();
    for (int k = 0; k < 8; ++k) {
        /* corner order of the reference: x alternates fastest, max before min */
        const Float3 corner((k & 1) ? lb.bbMin.x : lb.bbMax.x,
                            (k & 2) ? lb.bbMin.y : lb.bbMax.y,
                            (k & 4) ? lb.bbMin.z : lb.bbMax.z);
        bounds.grow(dehomog(m_transform * Float4(corner, 1.0f)));
    }
}

void Instance::calculateMeshArea() {                             /* bvh.cpp:577-594 */
    area = 0.0f;
    for (const Triangle& t : bvh->mesh()->triangles) {
        const Float3 a = dehomog(m_transform * Float4(t.v0, 1.0f));
        const Float3 b = dehomog(m_transform * Float4(t.v1, 1.0f));
        const Float3 c = dehomog(m_transform * Float4(t.v2, 1.0f));
        area = area + 0.5f * (b - a).cross(c - a).magnitude();
    }
}

GPUInstance Instance::toGPUInstance() const {
    GPUInstance g;
    std::memset(&g, 0, sizeof g);
    g.area = area;
    std::memcpy(g.transform, m_transform.c, sizeof g.transform);
    std::memcpy(g.inv_transform, m_invTransform.c, sizeof g.inv_transform);
    return g;
}

/* ================================================================= BvhTLAS */
BvhTLAS::BvhTLAS(std::vector<Instance> instances) : m_instances(std::move(instances)) { build(); }

void BvhTLAS::build() {
    InstancePrims prims{&m_instances};
    std::vector<PrimRef> refs;
    SahBuilder<InstancePrims> b{prims, m_indices, refs, m_nodes, m_nodesUsed, 1};
    b.run((U32)m_instances.size(), false);
}

/* bvh.cpp:793-819 */
void BvhTLAS::refit() {
    InstancePrims prims{&m_instances};
    for (int64_t i = (int64_t)m_nodesUsed - 1; i >= 0; --i) {
        if (i == 1) continue;
        BvhNode& n = m_nodes[(size_t)i];
        if (n.isLeaf()) {
            for (U32 k = 0; k < n.count; ++k) m_instances[m_indices[n.leftFirst + k]].updateInstanceData();
            for (U32 k = 0; k < n.count; ++k) prims.addTo(n.boundingBox, m_indices[n.leftFirst + k]);
            continue;
        }
        const BvhNode& l = m_nodes[n.leftFirst];
        const BvhNode& r = m_nodes[n.leftFirst + 1];
        n.boundingBox.bbMin = min(l.boundingBox.bbMin, r.boundingBox.bbMin);
        n.boundingBox.bbMax = max(l.boundingBox.bbMax, r.boundingBox.bbMax);
    }
}

U32 BvhTLAS::depth() const { return depthOf(m_nodes, 0); }

/* ============================================================== GPUBatcher */
GPUBatchInfo GPUBatcher::createBatchInfo(const std::vector<Instance>& instances) {
    GPUBatchInfo out;
    std::vector<const Mesh*> meshes;
    std::vector<const BvhBLAS*> blases;
    std::vector<const Material*> mats;
    auto slot = [](auto& list, auto* key) {
        for (size_t i = 0; i < list.size(); ++i) if (list[i] == key) return i;
        list.push_back(key);
        return list.size() - 1;
    };
    for (const Instance& in : instances) {
        slot(meshes, in.bvh->mesh());
        slot(blases, in.bvh);
        slot(mats, in.material);
    }
    std::vector<U32> triBase, idxBase, nodeBase;
    for (const Mesh* m : meshes) {
        triBase.push_back((U32)out.triBuffer.size());
        out.triBuffer.insert(out.triBuffer.end(), m->triangles.begin(), m->triangles.end());
        out.triExtBuffer.insert(out.triExtBuffer.end(), m->triExtensions.begin(), m->triExtensions.end());
    }
    for (const BvhBLAS* b : blases) {
        idxBase.push_back((U32)out.BLASIndices.size());
        out.BLASIndices.insert(out.BLASIndices.end(), b->indices(), b->indices() + b->triCount());
    }
    for (const BvhBLAS* b : blases) {
        nodeBase.push_back((U32)out.BLASNodes.size());
        out.BLASNodes.insert(out.BLASNodes.end(), b->nodePool(), b->nodePool() + b->nodesUsed());
    }
    for (const Material* m : mats) out.materials.push_back(*m);
    for (const Instance& in : instances) {
        GPUInstance g = in.toGPUInstance();
        const size_t mi = std::find(meshes.begin(), meshes.end(), in.bvh->mesh()) - meshes.begin();
        const size_t bi = std::find(blases.begin(), blases.end(), in.bvh) - blases.begin();
        g.tri_offset = triBase[mi];
        g.bvh_idx_offset = idxBase[bi];
        g.bvh_node_offset = nodeBase[bi];
        g.material_offset = (U32)(std::find(mats.begin(), mats.end(), in.material) - mats.begin());
        if (in.material->isLight())
            out.lights.push_back(GPULightData{(U32)out.gpuInstances.size(), (U32)in.bvh->triCount()});
        out.gpuInstances.push_back(g);
    }
    return out;
}

/* ================================================================ GPUScene */
GPUScene::GPUScene(RenderContext* context, SceneBackground background, std::vector<Instance> instances)
    : m_context(context), m_background(background), m_sceneTlas(instances),
      m_batchInfo(GPUBatcher::createBatchInfo(instances)) {}

void GPUScene::update(F32 deltaTime) {
    Instance& in = m_sceneTlas.instance(3);
    in.setTransform(rotate(in.transform(), 1.0f * deltaTime, WORLD_UP));
    m_sceneTlas.refit();
    m_batchInfo = GPUBatcher::createBatchInfo(m_sceneTlas.instances());
    ++m_generation;
}

surf_scene_desc GPUScene::descriptor() const {
    surf_scene_desc d;
    std::memset(&d, 0, sizeof d);
    d.triangles = reinterpret_cast<const surf_triangle*>(m_batchInfo.triBuffer.data());
    d.triangle_count = (U32)m_batchInfo.triBuffer.size();
    d.tri_ext = reinterpret_cast<const surf_tri_extension*>(m_batchInfo.triExtBuffer.data());
    d.blas_indices = m_batchInfo.BLASIndices.data();
    d.blas_index_count = (U32)m_batchInfo.BLASIndices.size();
    d.blas_nodes = reinterpret_cast<const surf_bvh_node*>(m_batchInfo.BLASNodes.data());
    d.blas_node_count = (U32)m_batchInfo.BLASNodes.size();
    d.materials = reinterpret_cast<const surf_material*>(m_batchInfo.materials.data());
    d.material_count = (U32)m_batchInfo.materials.size();
    d.instances = m_batchInfo.gpuInstances.data();
    d.instance_count = (U32)m_batchInfo.gpuInstances.size();
    d.tlas_indices = m_sceneTlas.indices();
    d.tlas_nodes = reinterpret_cast<const surf_bvh_node*>(m_sceneTlas.nodePool());
    d.tlas_node_count = m_sceneTlas.nodesUsed();
    d.lights = reinterpret_cast<const surf_light*>(m_batchInfo.lights.data());
    d.light_count = (U32)m_batchInfo.lights.size();
    d.background = reinterpret_cast<const surf_background*>(&m_background);
    return d;
}

/* ================================================================== Camera */
Camera::Camera(Float3 pos, Float3 target, U32 w, U32 h, F32 fov, F32 focal, F32 defocus)
    : position(pos), forward(0.0f), up(0.0f), screenWidth((F32)w), screenHeight((F32)h),
      fovY(fov), focalLength(focal), defocusAngle(defocus), viewPlane{} {
    forward = (target - position).normalize();                   /* camera.cpp:21-23 */
    const Float3 r = WORLD_UP.cross(forward).normalize();
    up = forward.cross(r).normalize();
    generateViewPlane();
}

void Camera::generateViewPlane() {                               /* camera.cpp:28-46 */
    const F32 heightScale = tanf(radians(fovY) / 2.0f);
    const F32 aspect = screenWidth / screenHeight;
    const F32 vh = 2.0f * heightScale * focalLength;
    const F32 vw = aspect * vh;
    const Float3 u = right() * vw;
    const Float3 v = (-1.0f * up) * vh;
    const Float3 du = u / screenWidth, dv = v / screenHeight;
    const Float3 topLeft = ((position + (forward * focalLength)) - (0.5f * u)) - (0.5f * v);
    viewPlane.firstPixel = topLeft + 0.5f * (du + dv);
    viewPlane.uVector = u;
    viewPlane.vVector = v;
}

CameraUBO Camera::toUBO() const {
    CameraUBO u;
    std::memset(&u, 0, sizeof u);
    auto put = [](surf_float3_16& d, const Float3& s) { d.x = s.x; d.y = s.y; d.z = s.z; d._pad = 0.0f; };
    put(u.position, position); put(u.up, up); put(u.fwd, forward); put(u.right, right());
    put(u.first_pixel, viewPlane.firstPixel); put(u.u_vector, viewPlane.uVector); put(u.v_vector, viewPlane.vVector);
    u.resolution[0] = screenWidth; u.resolution[1] = screenHeight;
    u.focal_length = focalLength; u.defocus_angle = defocusAngle;
    return u;
}

}  // namespace surf

/* ====================================================== C-ABI scene helpers */
struct surf_scene {
    std::vector<std::unique_ptr<surf::Mesh>> meshes;
    std::vector<std::unique_ptr<surf::BvhBLAS>> blases;
    std::vector<std::unique_ptr<surf::Material>> materials;
    std::unique_ptr<surf::GPUScene> scene;
    surf::RenderContext context;
};

namespace {

/* The scene of the reference's main.cpp:161-346 (and the C5 deep variant). */
void buildIndoor(surf_scene& S, const std::string& dir, int variant) {
    using namespace surf;
    /* SURF_BUILD_LOG=1: phase times on stderr */
    const bool log = getenv("SURF_BUILD_LOG") != nullptr;
    auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t0 = now();
    auto phase = [&](const char* what) {
        if (log) fprintf(stderr, "[surf build] %-14s %8.3f s\n", what, now() - t0);
        t0 = now();
    };
    for (const char* name : {"susanne", "cube", "lens", "plane"})
        S.meshes.push_back(std::make_unique<Mesh>(dir + "/" + name + ".obj"));
    Mesh* sus = S.meshes[0].get();
    Mesh* cube = S.meshes[1].get();
    Mesh* lens = S.meshes[2].get();
    Mesh* plane = S.meshes[3].get();
    Mesh* lattice = nullptr;
    phase("obj load");
    if (variant == 1) {
        /* C5: 648 Suzannes, translate(-8+2i, -0.4+1.2j, -4+1.5k) * scale(0.5), one mesh */
        auto m = std::make_unique<Mesh>();
        m->triangles.reserve(648 * sus->triangles.size());
        m->triExtensions.reserve(648 * sus->triangles.size());
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 8; ++j)
                for (int k = 0; k < 9; ++k) {
                    const Mat4 X = scale(translate(Mat4(1.0f), Float3(-8.0f + 2.0f * (F32)i, -0.4f + 1.2f * (F32)j, -4.0f + 1.5f * (F32)k)), Float3(0.5f));
                    for (size_t t = 0; t < sus->triangles.size(); ++t) {
                        const Triangle& s = sus->triangles[t];
                        /* OBJ order is (v1, v0, v2) of the stored triangle */
                        m->triangles.emplace_back(dehomog(X * Float4(s.v1, 1.0f)), dehomog(X * Float4(s.v0, 1.0f)), dehomog(X * Float4(s.v2, 1.0f)));
                        m->triExtensions.push_back(sus->triExtensions[t]);
                    }
                }
        lattice = m.get();
        S.meshes.push_back(std::move(m));
    }
    phase("lattice mesh");
    for (Mesh* m : {sus, cube, lens, plane}) S.blases.push_back(std::make_unique<BvhBLAS>(m));
    phase("blas build");
    if (lattice) S.blases.push_back(std::make_unique<BvhBLAS>(lattice));
    phase("lattice blas");
    BvhBLAS* susB = S.blases[0].get();
    BvhBLAS* cubeB = S.blases[1].get();
    BvhBLAS* lensB = S.blases[2].get();
    BvhBLAS* planeB = S.blases[3].get();

    auto mat = [&]() { S.materials.push_back(std::make_unique<Material>()); return S.materials.back().get(); };
    Material* floorM = mat(); floorM->albedo = Float3(0.8f); floorM->reflectivity = 0.01f;
    Material* wallRed = mat(); wallRed->albedo = Float3(1.0f, 0.0f, 0.0f);
    Material* wallGreen = mat(); wallGreen->albedo = Float3(0.0f, 1.0f, 0.0f);
    Material* diffuse = mat(); diffuse->albedo = Float3(1.0f, 0.0f, 0.0f);
    Material* dielectric = mat(); dielectric->albedo = Float3(0.7f, 0.7f, 0.2f); dielectric->absorption = Float3(0.03f, 0.04f, 0.03f);
    dielectric->refractivity = 1.0f; dielectric->indexOfRefraction = 1.42f;
    Material* specular = mat(); specular->albedo = Float3(0.2f, 0.9f, 1.0f); specular->reflectivity = 0.8f;
    Material* softLight = mat(); softLight->emissionColor = Float3(1.0f, 0.8f, 0.6f); softLight->emissionStrength = 5.0f;
    Material* redLight = mat(); redLight->emissionColor = Float3(1.0f, 0.5f, 0.2f); redLight->emissionStrength = 5.0f;

    const Mat4 I(1.0f);
    std::vector<Instance> inst;
    inst.emplace_back(planeB, floorM, scale(translate(I, Float3(0.0f, -1.0f, 0.0f)), Float3(10.0f, 10.0f, 10.0f)));
    inst.emplace_back(cubeB, softLight, scale(translate(I, Float3(-8.0f, 7.0f, 5.0f)), Float3(0.5f, 0.5f, 0.5f)));
    inst.emplace_back(cubeB, redLight, scale(translate(I, Float3(9.0f, 5.0f, -5.0f)), Float3(1.0f, 1.0f, 1.0f)));
    inst.emplace_back(susB, diffuse, translate(I, Float3(0.0f, 0.0f, -1.0f)));
    inst.emplace_back(susB, specular, translate(I, Float3(3.0f, 0.0f, -1.0f)));
    inst.emplace_back(lensB, dielectric, translate(I, Float3(-3.0f, 0.0f, -1.0f)));
    inst.emplace_back(planeB, wallRed, scale(rotate(translate(I, Float3(-10.0f, 4.0f, 0.0f)), radians(90.0f), WORLD_FORWARD), Float3(5.0f, 10.0f, 10.0f)));
    inst.emplace_back(planeB, wallGreen, scale(rotate(translate(I, Float3(10.0f, 4.0f, 0.0f)), radians(90.0f), WORLD_FORWARD), Float3(5.0f, 10.0f, 10.0f)));
    inst.emplace_back(planeB, floorM, scale(translate(I, Float3(0.0f, 9.0f, 0.0f)), Float3(10.0f, 10.0f, 10.0f)));
    inst.emplace_back(planeB, floorM, scale(rotate(translate(I, Float3(0.0f, 4.0f, -10.0f)), radians(90.0f), WORLD_RIGHT), Float3(10.0f, 10.0f, 5.0f)));
    inst.emplace_back(planeB, floorM, scale(rotate(translate(I, Float3(0.0f, 4.0f, 10.0f)), radians(90.0f), WORLD_RIGHT), Float3(10.0f, 10.0f, 5.0f)));
    if (lattice) inst.emplace_back(S.blases[4].get(), diffuse, I);
    if (variant == 2 || variant == 3) {
        /* general-TLAS test scenes (not in the reference's main.cpp): extra
         * instances of the cube / Suzanne / lens meshes, sizes 0.3-0.9 and
         * rotations varied so that BvhTLAS::build splits (bvh.cpp:780-993):
         * 40 extras (51 instances, LDS tables) or 80 (91, global tables) */
        BvhBLAS* meshes[3] = {cubeB, susB, lensB};
        Material* mats[5] = {floorM, diffuse, specular, dielectric, wallGreen};
        const int extra = variant == 2 ? 40 : 80;
        for (int k = 0; k < extra; ++k) {
            const F32 x = -8.5f + 1.0f * (F32)((k * 7) % 18);
            const F32 y = -0.4f + 0.9f * (F32)((k * 5) % 10);
            F32 z = -8.5f + 1.0f * (F32)((k * 11) % 18);
            if (x > -2.5f && x < 2.5f && y < 2.5f && z < -4.5f) z = z + 6.0f;   /* keep clear of the camera (0, 0, -7) */
            const F32 sc = 0.3f + 0.15f * (F32)(k % 5);
            Mat4 X = translate(I, Float3(x, y, z));
            if (k % 3 == 1) X = rotate(X, radians(17.0f * (F32)(k % 7)), WORLD_UP);
            X = scale(X, Float3(sc, sc, sc));
            inst.emplace_back(meshes[k % 3], mats[k % 5], X);
        }
    }

    SceneBackground bg;
    bg.type = BackgroundType::ColorGradient;
    bg.gradient.colorA = Float3(0.8f, 0.8f, 0.8f);
    bg.gradient.colorB = Float3(0.1f, 0.4f, 0.6f);
    phase("instances");
    S.scene = std::make_unique<GPUScene>(&S.context, bg, std::move(inst));
    phase("tlas + batch");
}

}  // namespace

extern "C" {

int surf_scene_build_indoor(const char* assets_dir, int variant, surf_scene** out) {
    if (!out || variant < 0 || variant > 3) return SURF_ERR_INVALID;
    *out = nullptr;
    auto s = std::make_unique<surf_scene>();
    try {
        buildIndoor(*s, assets_dir ? assets_dir : ".", variant);
    } catch (const std::exception& e) {
        fprintf(stderr, "surf_scene_build_indoor: %s\n", e.what());
        return SURF_ERR_IO;
    }
    *out = s.release();
    return SURF_OK;
}

int surf_scene_update(surf_scene* scene, float delta_time) {
    if (!scene) return SURF_ERR_INVALID;
    scene->scene->update(delta_time);   /* scene.cpp:267-282: rotate instance 3 about WORLD_UP, TLAS refit, re-batch */
    return SURF_OK;
}

int surf_scene_desc_get(const surf_scene* scene, surf_scene_desc* out) {
    if (!scene || !out) return SURF_ERR_INVALID;
    *out = scene->scene->descriptor();
    return SURF_OK;
}

int surf_scene_camera(const surf_scene* scene, uint32_t width, uint32_t height, surf_camera_ubo* out) {
    if (!scene || !out || width == 0 || height == 0) return SURF_ERR_INVALID;
    /* main.cpp:141-149 */
    surf::Camera cam(surf::Float3(0.0f, 0.0f, -7.0f), surf::Float3(0.0f, 0.0f, 0.0f), width, height, 70.0f, 7.0f, 0.5f);
    *out = cam.toUBO();
    return SURF_OK;
}

int surf_scene_bvh_depths(const surf_scene* scene, uint32_t* tlas_depth, uint32_t* max_blas_depth) {
    if (!scene || !tlas_depth || !max_blas_depth) return SURF_ERR_INVALID;
    *tlas_depth = scene->scene->tlas().depth();
    uint32_t m = 0;
    for (const auto& b : scene->blases) m = std::max(m, b->depth());
    *max_blas_depth = m;
    return SURF_OK;
}

void surf_scene_destroy(surf_scene* scene) { delete scene; }

int surf_write_ppm(const char* path, uint32_t width, uint32_t height, const uint32_t* rgba8) {
    if (!path || !rgba8 || width == 0 || height == 0) return SURF_ERR_INVALID;
    FILE* f = fopen(path, "wb");
    if (!f) return SURF_ERR_IO;
    fprintf(f, "P6\n%u %u\n255\n", width, height);
    std::vector<unsigned char> row((size_t)width * 3);
    bool ok = true;
    for (uint32_t y = 0; y < height && ok; ++y) {
        for (uint32_t x = 0; x < width; ++x) {
            const uint32_t p = rgba8[(size_t)y * width + x];
            row[3 * x] = (unsigned char)(p & 0xffu);
            row[3 * x + 1] = (unsigned char)((p >> 8) & 0xffu);
            row[3 * x + 2] = (unsigned char)((p >> 16) & 0xffu);
        }
        ok = fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    return (fclose(f) == 0 && ok) ? SURF_OK : SURF_ERR_IO;
}

int surf_write_png(const char* path, uint32_t width, uint32_t height, const uint32_t* rgba8) {
    if (!path || !rgba8 || width == 0 || height == 0) return SURF_ERR_INVALID;
    /* scanlines: filter byte 0 + RGBA bytes (R from the low byte) */
    const size_t stride = (size_t)width * 4 + 1;
    std::vector<unsigned char> raw(stride * height);
    for (uint32_t y = 0; y < height; ++y) {
        unsigned char* r = &raw[stride * y];
        r[0] = 0;
        for (uint32_t x = 0; x < width; ++x) {
            const uint32_t p = rgba8[(size_t)y * width + x];
            r[1 + 4 * x] = (unsigned char)(p & 0xffu);
            r[2 + 4 * x] = (unsigned char)((p >> 8) & 0xffu);
            r[3 + 4 * x] = (unsigned char)((p >> 16) & 0xffu);
            r[4 + 4 * x] = (unsigned char)(p >> 24);
        }
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<unsigned char> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return SURF_ERR_IO;
    FILE* f = fopen(path, "wb");
    if (!f) return SURF_ERR_IO;
    bool ok = true;
    auto put = [&](const void* p, size_t n) { ok = ok && fwrite(p, 1, n, f) == n; };
    auto be32 = [](uint32_t v, unsigned char* b) { b[0] = (unsigned char)(v >> 24); b[1] = (unsigned char)(v >> 16); b[2] = (unsigned char)(v >> 8); b[3] = (unsigned char)v; };
    auto chunk = [&](const char* type, const unsigned char* data, size_t n) {
        unsigned char b[4];
        be32((uint32_t)n, b); put(b, 4);
        put(type, 4);
        if (n) put(data, n);
        uLong crc = crc32(0L, Z_NULL, 0);
        crc = crc32(crc, reinterpret_cast<const Bytef*>(type), 4);
        if (n) crc = crc32(crc, data, (uInt)n);
        be32((uint32_t)crc, b); put(b, 4);
    };
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    put(sig, 8);
    unsigned char ihdr[13];
    be32(width, ihdr); be32(height, ihdr + 4);
    ihdr[8] = 8; ihdr[9] = 6; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;    /* 8-bit RGBA, deflate, no interlace */
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), zlen);
    chunk("IEND", nullptr, 0);
    return (fclose(f) == 0 && ok) ? SURF_OK : SURF_ERR_IO;
}

struct surf_mesh { surf::Mesh mesh; };

int surf_obj_load(const char* path, uint32_t threads, surf_mesh** out) {
    if (!path || !out) return SURF_ERR_INVALID;
    *out = nullptr;
    try {
        auto m = std::make_unique<surf_mesh>();
        m->mesh = surf::Mesh(path, threads ? threads : surf::defaultBuildThreads());
        *out = m.release();
    } catch (const std::exception& e) {
        fprintf(stderr, "surf_obj_load: %s\n", e.what());
        return SURF_ERR_IO;
    }
    return SURF_OK;
}

int surf_mesh_data(const surf_mesh* m, const surf_triangle** triangles, const surf_tri_extension** tri_ext, uint32_t* count) {
    if (!m || !triangles || !tri_ext || !count) return SURF_ERR_INVALID;
    *triangles = reinterpret_cast<const surf_triangle*>(m->mesh.triangles.data());
    *tri_ext = reinterpret_cast<const surf_tri_extension*>(m->mesh.triExtensions.data());
    *count = (uint32_t)m->mesh.triangles.size();
    return SURF_OK;
}

void surf_mesh_destroy(surf_mesh* m) { delete m; }

int surf_bvh_build(const surf_triangle* triangles, uint32_t count, uint32_t threads, uint32_t* indices_out,
                   surf_bvh_node* nodes_out, uint32_t* nodes_used) {
    if (!triangles || count == 0 || !indices_out || !nodes_out || !nodes_used) return SURF_ERR_INVALID;
    try {
        surf::Mesh mesh;
        mesh.triangles.resize(count, surf::Triangle(surf::Float3(0.0f), surf::Float3(0.0f), surf::Float3(0.0f)));
        std::memcpy(static_cast<void*>(mesh.triangles.data()), triangles, (size_t)count * sizeof(surf_triangle));
        surf::BvhBLAS b(&mesh, threads ? threads : surf::defaultBuildThreads());
        std::memcpy(indices_out, b.indices(), (size_t)count * sizeof(uint32_t));
        std::memcpy(nodes_out, b.nodePool(), (size_t)b.nodesUsed() * sizeof(surf_bvh_node));
        *nodes_used = b.nodesUsed();
    } catch (const std::exception& e) {
        fprintf(stderr, "surf_bvh_build: %s\n", e.what());
        return SURF_ERR_OOM;
    }
    return SURF_OK;
}

}  // extern "C"
