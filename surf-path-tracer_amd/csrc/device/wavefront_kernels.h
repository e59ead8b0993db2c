/*
 * wavefront_kernels.h -- the hot path: HIP kernels for gfx950 (CDNA4, wave64).
 *
 * Pipeline per wavefront iteration ("phase", parity par = phase & 1; pool[par]
 * is read, pool[par^1] is written):
 *
 *   k_extend   closest hit of every path in pool[par]        ray_extend.comp:26-185
 *   k_shade    material eval, NEE shadow-ray emission, RR,   ray_shade.comp:44-191
 *              compacted append of continuing paths           (CPU oracle: renderer.cpp:336-460)
 *   k_connect  any-hit of the shadow queue + contribution    ray_connect.comp:34-212
 *   k_regen    refill pool[par^1] with new camera samples    ray_generation.comp:32-80
 *
 * plus k_accumulate (frame-ordered per-pixel sum, renderer.cpp:180) and
 * k_finalize (wavefront_finalize.comp:15-26 with RgbaToU32 rounding).
 *
 * Semantics follow the reference CPU renderer (the parity target), not the
 * GLSL: one RNG stream per (pixel, frame) carried in the path record, GCC
 * argument order for the jitter/disk draws, CPU cosine-frame constants, queues
 * drained completely (no WF_RAY_DIFF_THRESHOLD early exit), no racy
 * accumulator updates (per-sample radiance slots, each written by one lane).
 *
 * Memory layout (HBM, SoA, 16-B aligned float4 records, coalesced per lane):
 *   path pool   o  : float4(origin.xyz, sample id bits)
 *               d  : float4(dir.xyz,    flags bits: b0 inMedium, b1 lastSpecular, b2.. segments)
 *               T  : float4(transmission.xyz, rng state bits)
 *   hit         tuv: float4(t, u, v, prim bits), inst: u32
 *   shadow q.   od : float4(origin.xyz, tmax), float4(dir.xyz, sample id bits) interleaved, c: float4(T*Ld, 0)
 *   radiance    float4 per sample of the frame batch (energy of the path)
 */
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include "surf_math.h"

namespace surfdev {

constexpr uint32_t kUnset = 0xffffffffu;
constexpr uint32_t kFlagMedium = 1u, kFlagSpecular = 2u;
constexpr int kBlock = 256;
/* Minimum waves per SIMD the register allocator must allow (occupancy). */
#ifndef SURF_SHADE_WAVES
#define SURF_SHADE_WAVES 4
#endif
#ifndef SURF_SEG_TIMING
#define SURF_SEG_TIMING 0
#endif
#ifndef SURF_TAIL_WAVES
#define SURF_TAIL_WAVES 3          /* k_tail waves per SIMD (2, 3: same speed; 4, 6: slower) */
#endif
#ifndef SURF_TRACE_WAVES
#define SURF_TRACE_WAVES 2
#endif
/* k_extend over one-level records (the L2/MALL-resident BVHs): 6 waves per
 * SIMD -- 80 VGPRs, a few spills -- beside the 16-bit stack that lets 6 fit
 * the LDS (C3 k_extend 117 -> 114 ms per render, MEASUREMENTS round 6); the
 * two-level lane walk (HBM-resident BVHs) keeps SURF_TRACE_WAVES (6 would
 * spill 96 of its registers) */
#ifndef SURF_TRACE_WAVES_EXT
#define SURF_TRACE_WAVES_EXT 6
#endif
#ifndef SURF_COOP_WAVES
#define SURF_COOP_WAVES 4          /* k_tail_coop waves per SIMD (launch bounds; 3: 136 VGPRs, 5: spills) */
#endif

struct DevInstance {          /* 160 B */
    float Minv[16];
    float M[16];
    uint32_t triOffset, idxOffset, nodeOffset, material;
    float area;
    uint32_t affineInv;       /* Minv row 3 == (0,0,0,1): w == 1 exactly for finite points */
    uint32_t affine;          /* M row 3 == (0,0,0,1) */
    uint32_t _pad;
};

struct DevMaterial {          /* = Material (64 B) */
    float emit, refl, refr, ior;
    float ec[4], albedo[4], absorb[4];
};

/* Per-instance traversal record (144 B), host-built at upload: rows of M^-1
 * (row i = m[i], m[4+i], m[8+i], m[12+i]), offsets, and the BLAS root record.
 * Kernels stage the table in LDS, so the per-instance loop of every ray reads
 * LDS instead of paying two dependent memory trips per instance. */
struct TraceInst {
    float4 m0, m1, m2, m3;
    uint4 meta;               /* nodeOffset, idxOffset, affineInv, instance id */
    float4 r0, r1, r2, r3;    /* root node record */
    float4 wlo, whi;          /* conservative world box of the BLAS's triangles (wlo.w != 0: usable) */
};
constexpr uint32_t kLdsTraceInst = 64;   /* instances staged in LDS (9 KB) */

struct DevScene {
    const TraceInst* tinst;   /* [nInst], instance-id order */
    const float4* nodes;      /* BLAS: 4 float4 per node (see upload) */
    const float4* tris;       /* 3 float4 per BLAS index slot: (v0, prim), e1, e2 */
    const float4* normals;    /* 3 float4 per global triangle: n0, n1, n2 */
    const float4* verts;      /* reference Triangle records (v0, v1, v2, centroid) */
    const float4* tlasNodes;  /* 4 float4 per TLAS node */
    const uint32_t* tlasIdx;
    const DevInstance* inst;
    const DevMaterial* mats;
    const uint2* lights;      /* (instance, primitive count) */
    uint32_t nLights;
    /* the emitters' BLAS k_connect stages in LDS (sbRecN = 0: none): the
     * instances whose BLAS root is node sbNode0 walk its sbRecN interior records
     * in compact form (sbRec: the children's boxes, each child an interior
     * record index or a leaf's triangle range -- no leaf records) and its sbTriN
     * triangle slots (S.tris + 3 * sbTri0) from LDS */
    uint32_t sbNode0, sbRecN, sbTri0, sbTriN;
    const float4* sbRec;
    uint32_t nInst, nMats;
    uint32_t tlasLeafCount;   /* TLAS root is a leaf with this many instances (0: general TLAS) */
    uint32_t finiteBoxes;     /* every BLAS node box is finite: slabFinite is exact */
    uint32_t nodes4G;         /* every BLAS-local record offset (64 B each) fits 32 bits: the asm wave walk's buffer offsets */
    const float* wnodes;      /* two-level records (48 floats per BLAS node, see surf_upload_scene), or null */
    uint32_t nWnodes;         /* nodes in wnodes (every 192-B offset fits 32 bits) */
    uint32_t laneW;           /* the one-ray-per-lane traversal walks the two-level records too (HBM-resident BVHs) */
    uint32_t bgType;
    float bgColor[3], bgA[3], bgB[3];
    float cellLo[3], cellScale[3];   /* ray-order cells: the TLAS root box split in 2 per axis (scale 0: one cell) */
    /* ray-order membership key (single-leaf TLAS): the world boxes of the (at
     * most 3) instances with the largest BLASes; keyMode 1: pool key by them */
    uint32_t nHeavy, keyMode;
    float4 hvLo[3], hvHi[3];
};

struct DevCamera {
    float pos[3], firstPixel[3], uVec[3], vVec[3], diskU[3], diskV[3];
    float invW, invH;
    uint32_t defocus;
};

/* Path pool: od[2i] = (origin, sample id), od[2i + 1] = (direction, flags) --
 * the ray a traversal reads is one 32-B piece of one cache line, also when it
 * is gathered through the ray order -- T[i] = (throughput, rng state),
 * key[i] = ray-order bin (start instance). */
struct Pool { float4* od; float4* T; uint8_t* key; };
/* Where a path that used up its segment budget goes. */
struct Sink { Pool q; uint32_t* n; uint32_t cap; };
/* Shadow queue: od[2i] = (origin, tmax), od[2i + 1] = (direction, sample id)
 * -- the ray k_connect traverses is one 32-B piece of one cache line --
 * c[i] = (T * Ld, 0), read only for an unoccluded ray.  k_shade appends each
 * shadow ray straight into the region of its order bin (shadowKey: kShBins
 * regions of `region` slots, then an overflow region of the pool's capacity
 * for a bin that outgrows its region), so k_connect reads the rays in bin
 * order sequentially: no sort pass and no gather through an order array. */
constexpr uint32_t kShBins = 16;     /* shadow-ray order bins: light slot (mod 2) x octant cell */
/* Each bin's cursor and region are split by XCD (SURF_SH_XCDS parts, the
 * appending workgroup's HW_REG_XCC_ID) and the cursors lie SURF_SH_STRIDE words
 * apart: every workgroup iteration of k_shade reserves once per non-empty bin,
 * and same-address device atomics serialize. */
#ifndef SURF_SH_XCDS
#define SURF_SH_XCDS 1
#endif
#ifndef SURF_SH_STRIDE
#define SURF_SH_STRIDE 32
#endif
constexpr uint32_t kShXcds = SURF_SH_XCDS, kShStride = SURF_SH_STRIDE;
constexpr uint32_t kShSegs = kShBins * kShXcds + 1u;      /* queue segments: (bin, XCD) regions, then the overflow */
struct ShadowQ {
    float4* od; float4* c;
    uint32_t* cur;        /* [2 parities][kShSegs] cursors, kShStride words apart (may count past a region's end) */
    uint32_t region;      /* slots per (bin, XCD) region */
    uint32_t bins;        /* kShBins, or 1: no shadow order (SURF_SORT=0/2) */
};
__device__ __forceinline__ uint32_t* shCursor(const ShadowQ& Q, int par, uint32_t seg) {
    return Q.cur + ((size_t)par * kShSegs + seg) * kShStride;
}
__device__ __forceinline__ uint32_t xccId() {
    if constexpr (kShXcds == 1u) return 0u;
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x % kShXcds;
}

/* Device counters of the sample stream.  Double-buffered by phase parity so no
 * kernel writes a word another block of the same launch still reads. */
struct Counters {
    uint32_t nIn[2];                 /* paths in pool[p] when a phase reads it */
    uint32_t app[2];                 /* phase parity p: paths appended to pool[p^1] (the shadow
                                        queue's cursors are ShadowQ::cur) */
    uint32_t maxSeg;                 /* 0 = unbounded */
    uint32_t zeroCutoff;             /* end paths whose throughput is exactly 0 (radiance-neutral) */
    uint32_t segMax;                 /* longest finished path (extension rays), diagnostics */
    uint32_t survN;                  /* k_tail survivors appended (may exceed survCap) */
    uint32_t survCap;
    uint32_t rowNext;                /* k_tail_pair path queue: next path to hand out */
    /* issue order of the stream's first permFrames frames: every frame's
     * samples of the permA pixels listed first in StreamGeom::perm, then each
     * frame's other pixels frame by frame (0: frame-major throughout) */
    uint32_t permFrames, permA;
    /* samples per frame (config().samplesPerFrame, renderer.cpp:171): a frame's
     * samples of one pixel form a chain -- sample k + 1 starts from the RNG state
     * sample k's path left -- so k_regen issues only the first sample of each
     * (frame, pixel) and the kernel that ends a sample's path starts the next */
    uint32_t spp;
    unsigned long long issued[2];    /* stream chains issued (first samples of (frame, pixel)), per parity */
    unsigned long long limit;        /* host-written issue limit (frame window) */
    unsigned long long baseFrame;    /* absolute frame index of stream frame 0 */
    unsigned long long ev[16];       /* ext, hit, cont, shadow, acc, unocc, tail paths, capped paths, wavefront ext, resumed rays */
    uint32_t capped[64];             /* sample ids of paths ended by the segment cap, slot blockIdx % 64 (diagnostics, ~0 = none) */
    /* event counts striped over kStripes cache lines (block b adds to stripe
     * b % kStripes): a counter shared by every block of a launch serializes its
     * atomics (~12 ns each, measured); totals = ev + sum over stripes */
    unsigned long long evS[32][16];
    unsigned long long dbg[8];       /* SURF_SEG_TIMING builds: k_tail_coop cycles (extend, shade, connect, segments) */
    uint32_t resumeN[2];             /* capped lane walks: resume records written by k_extend of parity p (k_regen zeroes) */
};
constexpr uint32_t kStripes = 32;    /* frameDone and event-count stripes */
constexpr int kEvents = 10;          /* event kinds counted (ev / evS index; 9: rays k_extend_cont finished) */

/* A path ended by the segment cap: counted in the event stripes; its sample
 * id is also stored in slot blockIdx % 64 (diagnostics: a racy overwrite, so
 * every workgroup that caps a path leaves some id behind).  No single shared
 * address is touched per path: a same-address atomic or load per capped path
 * serialized k_shade under C2's 8-segment cap (33 -> 88 ms). */
__device__ __forceinline__ void noteCappedSid(bool capped, Counters* C, uint32_t sid) {
    if (capped) C->capped[blockIdx.x % 64u] = sid;
}
__device__ __forceinline__ void noteCapped(Counters* C, uint32_t sid) {
    atomicAdd(&C->evS[blockIdx.x % kStripes][7], 1ull);
    noteCappedSid(true, C, sid);
}

/* Where a stream sample lives: radiance slot sid = (pass % window) * npx + pixel,
 * pass = the sample's index in the stream (frame * spp + its place in the
 * frame; window is a multiple of spp, so a frame's samples occupy consecutive
 * slots and slot % spp is the place in the frame). */
struct StreamGeom {
    const uint32_t* rows;            /* shard rows */
    uint32_t width, npx, window;
    const uint32_t* perm;            /* local pixels, class A (Counters::permA of them) first */
};

SURF_HD V3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

/* Streaming (non-temporal) access to the path pools, hit records and shadow
 * queue: each record is touched once per phase, so it should not evict the
 * BVH nodes and triangles the traversal re-reads from L2. */
#ifndef SURF_STREAM_NT
#define SURF_STREAM_NT 1
#endif
typedef float ntf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldS(const float4* p) {
#if SURF_STREAM_NT
    const ntf4 v = __builtin_nontemporal_load(reinterpret_cast<const ntf4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ void stS(float4* p, float4 v) {
#if SURF_STREAM_NT
    const ntf4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<ntf4*>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ uint32_t ldSu(const uint32_t* p) {
#if SURF_STREAM_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ void stSu(uint32_t* p, uint32_t v) {
#if SURF_STREAM_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
SURF_HD V3 xyz(float4 v) { return mk3(v.x, v.y, v.z); }

/* ------------------------------------------------------------------ traversal
 * Stack in LDS: entry k of thread t at stk[k * stride] (stk = lds + t,
 * stride = blockDim.x) -> consecutive lanes hit consecutive banks.
 * BvhBLAS::intersect / intersectAny (bvh.cpp:129-253): near child first
 * (left unless dist(left) > dist(right)), far child pushed when it hits,
 * leaves in index order, LIFO pops.  Node record (64 B) of node n holds its
 * own leftFirst/count and, if interior, both children's boxes:
 *   q0 = (left.min.xyz,  leftFirst)   q1 = (left.max.xyz,  count)
 *   q2 = (right.min.xyz, 0)           q3 = (right.max.xyz, 0)
 * The root record is read once per instance before the per-lane loop: when
 * the instance index is wave-uniform (single-leaf TLAS) those are scalar
 * loads, as are the triangles of a root leaf (the room's planes). */
/* Pins a loaded record in registers: the compiler may not sink any part of the
 * load below this point, so all 16-B loads of a node or triangle are issued
 * together and paid as one memory round trip (without it, the leaf/count words
 * are fetched first and the boxes only after the leaf branch: two trips). */
__device__ __forceinline__ void pin(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ uint32_t laneIdx() { return __lane_id(); }

template <bool ANY>
__device__ __forceinline__ bool leafTest(const float4* tri, uint32_t lf, uint32_t cnt, V3 o, V3 d, float& depth,
                                         float& hu, float& hv, uint32_t& hprim) {
    bool any = false;
    for (uint32_t k = 0; k < cnt; ++k) {
        const float4* tp = tri + 3u * (lf + k);
        float4 a = tp[0], b = tp[1], c = tp[2];
        pin(a); pin(b); pin(c);
        float u, v;
        if (triHit(xyz(a), xyz(b), xyz(c), o, d, depth, u, v)) {
            if (ANY) return true;
            any = true;
            hu = u; hv = v; hprim = f2u(a.w);
        }
    }
    return any;
}

/* Scalar (wave-uniform) variant for a root leaf: no pinning, s_load path. */
template <bool ANY>
__device__ __forceinline__ bool leafTestUniform(const float4* tri, uint32_t lf, uint32_t cnt, V3 o, V3 d, float& depth,
                                                float& hu, float& hv, uint32_t& hprim) {
    bool any = false;
    for (uint32_t k = 0; k < cnt; ++k) {
        const float4 a = tri[3u * (lf + k)], b = tri[3u * (lf + k) + 1u], c = tri[3u * (lf + k) + 2u];
        float u, v;
        if (triHit(xyz(a), xyz(b), xyz(c), o, d, depth, u, v)) {
            if (ANY) return true;
            any = true;
            hu = u; hv = v; hprim = f2u(a.w);
        }
    }
    return any;
}

template <bool FIN>
__device__ __forceinline__ float boxDist(float4 lo, float4 hi, V3 o, V3 rd, float depth) {
    return FIN ? slabFinite(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, o, rd, depth)
               : slab(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, o, rd, depth);
}

/* Any-hit walk of the emitters' BLAS staged in LDS (k_connect, S.sbRecN):
 * record r = (L.min, refL), (L.max, refR), (R.min, -), (R.max, -) of interior
 * node r (root 0); a child reference is an interior record index or, for a
 * leaf, kLeafTag | count << 16 | leftFirst into the staged triangles (v0, e1,
 * e2 per BVH slot, after the records).  The reference's box tests at the
 * fixed shadow-ray depth decide which leaves are tested (a leaf is box-tested
 * at its parent and never again, bvh.cpp:193-253); the answer is an OR over
 * them, so testing a hit leaf's triangles as soon as its parent is visited --
 * no leaf record, no stack entry -- returns what blasTrace<true> does. */
constexpr uint32_t kLeafTagC = 0x80000000u;
__device__ __forceinline__ bool leafAnyStaged(const float4* sT, uint32_t ref, V3 o, V3 d, float depth) {
    const uint32_t cnt = (ref >> 16) & 0x7fffu, lf = ref & 0xffffu;
    for (uint32_t k = 0; k < cnt; ++k) {
        const float4* tp = sT + 3u * (lf + k);
        const float4 a = tp[0], b = tp[1], c = tp[2];
        float dd = depth, u, v;
        if (triHit(xyz(a), xyz(b), xyz(c), o, d, dd, u, v)) return true;
    }
    return false;
}
template <bool FIN, typename SK>
__device__ __forceinline__ bool blasAnyStaged(uint32_t recN, const float4* sR, V3 o, V3 d, V3 rd, float depth, SK* stk,
                                              uint32_t stride, uint32_t base) {
    const float4* sT = sR + 4u * recN;
    SK* const bottom = stk + base * stride;
    SK* sp = bottom;
    uint32_t node = 0u;
    for (;;) {
        const float4* nd = sR + 4u * node;
        const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        const uint32_t rl = f2u(q0.w), rr = f2u(q1.w);
        bool hl = boxDist<FIN>(q0, q1, o, rd, depth) != kFarAway;
        bool hr = boxDist<FIN>(q2, q3, o, rd, depth) != kFarAway;
        if (hl && (rl & kLeafTagC)) {
            if (leafAnyStaged(sT, rl, o, d, depth)) return true;
            hl = false;
        }
        if (hr && (rr & kLeafTagC)) {
            if (leafAnyStaged(sT, rr, o, d, depth)) return true;
            hr = false;
        }
        if (hl) {
            node = rl;
            if (hr) { *sp = (SK)rr; sp += stride; }
        } else if (hr) {
            node = rr;
        } else {
            if (sp == bottom) return false;
            sp -= stride;
            node = *sp;
        }
    }
}

/* The capped lane walk (k_extend with a cap): a lane whose BLAS walk has
 * taken its `left` iterations (node visits; W-record visits in the two-level
 * walk) reserves a resume record and stops, its state here -- the node (ref)
 * it was about to visit -- and the entries below it still on its LDS stack;
 * k_extend writes the record and k_extend_cont continues the walk from that
 * state, 64 such rays to a wave.  Exact: the continuation takes the
 * reference's decisions from the same state (same boxes, order, pruning and
 * leaf order), so the ray ends as the uncapped walk would end it. */
struct LaneCap {
    uint32_t left;        /* iterations the lane may still take */
    uint32_t ref, depthN, turn;
    bool capped;
};

/* FIN: o, rd and every box finite (slabFinite is exact); else the reference's
 * ternary slab with its NaN behaviour. */
/* STG: the BLAS is the emitters' one staged in LDS (S.sbNode0, sN; any-hit
 * only: blasAnyStaged).  SK: the stack entry type (16-bit when every node
 * index fits). */
template <bool ANY, bool FIN, bool STG = false, typename SK = uint32_t, bool CAP = false, bool RES = false>
__device__ __forceinline__ bool blasTrace(const DevScene& S, const TraceInst& I, V3 o, V3 d, V3 rd, float& depth,
                                          float& hu, float& hv, uint32_t& hprim,
                                          SK* stk, uint32_t stride, uint32_t base, const float4* sN = nullptr,
                                          LaneCap* lc = nullptr, uint32_t ref0 = 0u, uint32_t n0 = 0u) {
    const uint32_t nodeOff = I.meta.x;
    const float4* tri = S.tris + 3u * I.meta.y;
    /* root: never box-tested (bvh.cpp:131), only its children are */
    const float4 r0 = I.r0, r1 = I.r1;
    const uint32_t rlf = f2u(r0.w), rcnt = f2u(r1.w);
    if (rcnt != 0u) return leafTestUniform<ANY>(tri, rlf, rcnt, o, d, depth, hu, hv, hprim);
    if constexpr (STG && ANY) return blasAnyStaged<FIN, SK>(S.sbRecN, sN, o, d, rd, depth, stk, stride, base);
    /* stack pointer walks in steps of `stride` words (lane-interleaved LDS) */
    SK* const bottom = stk + base * stride;
    SK* sp = bottom;
    uint32_t node;
    bool any = false;
    if (RES) {
        node = ref0;
        sp = bottom + n0 * stride;
    } else {
        const float4 r2 = I.r2, r3 = I.r3;
        float dn = boxDist<FIN>(r0, r1, o, rd, depth);
        float df = boxDist<FIN>(r2, r3, o, rd, depth);
        uint32_t cn = nodeOff + rlf, cf = cn + 1u;
        if (ANY) {
            /* any-hit: the answer is an OR over every leaf the fixed-depth box
             * tests admit, whatever the order -- left child first, no ordering */
            if (dn == kFarAway && df == kFarAway) return false;
            node = dn != kFarAway ? cn : cf;
            if (dn != kFarAway && df != kFarAway) { *sp = cf; sp += stride; }
        } else {
            if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
            if (dn == kFarAway) return false;
            node = cn;
            if (df != kFarAway) { *sp = cf; sp += stride; }
        }
    }
    for (;;) {
        if (CAP) {
            if (lc->left == 0u) {
                lc->ref = node; lc->depthN = (uint32_t)((sp - bottom) / stride); lc->capped = true;
                return any;
            }
            --lc->left;
        }
        const float4* nd = S.nodes + 4u * node;
        float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        pin(q0); pin(q1); pin(q2); pin(q3);
        const uint32_t lf = f2u(q0.w), cnt = f2u(q1.w);
        if (cnt != 0u) {
            if (leafTest<ANY>(tri, lf, cnt, o, d, depth, hu, hv, hprim)) {
                if (ANY) return true;
                any = true;
            }
            if (sp == bottom) break;
            sp -= stride;
            node = *sp;
            continue;
        }
        float dn = boxDist<FIN>(q0, q1, o, rd, depth);
        float df = boxDist<FIN>(q2, q3, o, rd, depth);
        uint32_t cn = nodeOff + lf, cf = cn + 1u;
        if (ANY) {
            if (dn == kFarAway && df == kFarAway) {
                if (sp == bottom) break;
                sp -= stride;
                node = *sp;
            } else {
                node = dn != kFarAway ? cn : cf;
                if (dn != kFarAway && df != kFarAway) { *sp = cf; sp += stride; }
            }
            continue;
        }
        if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
        if (dn == kFarAway) {
            if (sp == bottom) break;
            sp -= stride;
            node = *sp;
        } else {
            node = cn;
            if (df != kFarAway) { *sp = cf; sp += stride; }
        }
    }
    return any;
}

/* blasTrace over the two-level records (S.wnodes, S.laneW): one memory round
 * trip per two BVH levels -- for BVHs that live in HBM, where every level of
 * the one-level walk waits for a DRAM access.  A W record holds three node
 * records (X, X.left, X.right) in the lanes-as-planes order (surf_upload_scene):
 * per row the two child boxes (min.x, max.x, min.y, max.y, min.z, max.z),
 * leftFirst, count, and, for an interior row node, its two children as packed
 * leaf references (kLeafTag | count << 24 | leftFirst when they are leaves
 * that fit, else 0).  The decisions are blasTrace's (near child first, far
 * pushed when hit, pop when both miss), taken for two levels from one record:
 * exact, as no leaf lies between the levels (the depth is the same).  Stack
 * entries are node indices, or packed leaf references (a popped leaf needs no
 * record). */
constexpr uint32_t kLeafTag = 0x80000000u;
struct WRow { float4 a, b, c, d; };
template <bool FIN>
__device__ __forceinline__ void wBoxes(const WRow& r, V3 o, V3 rd, float depth, float& d0, float& d1) {
    d0 = FIN ? slabFinite(r.a.x, r.a.z, r.b.x, r.a.y, r.a.w, r.b.y, o, rd, depth) : slab(r.a.x, r.a.z, r.b.x, r.a.y, r.a.w, r.b.y, o, rd, depth);
    d1 = FIN ? slabFinite(r.b.z, r.c.x, r.c.z, r.b.w, r.c.y, r.c.w, o, rd, depth) : slab(r.b.z, r.c.x, r.c.z, r.b.w, r.c.y, r.c.w, o, rd, depth);
}
__device__ __forceinline__ WRow wSel(bool c, const WRow& x, const WRow& y) {
    WRow r;
    r.a = c ? y.a : x.a; r.b = c ? y.b : x.b; r.c = c ? y.c : x.c; r.d = c ? y.d : x.d;
    return r;
}
/* RES (k_extend_cont): the walk continues from a capped lane's state -- ref0
 * next, n0 refs already on the stack -- instead of from the root. */
template <bool ANY, bool FIN, bool CAP = false, bool RES = false>
__device__ __forceinline__ bool blasTraceW(const DevScene& S, const TraceInst& I, V3 o, V3 d, V3 rd, float& depth,
                                           float& hu, float& hv, uint32_t& hprim, uint32_t* stk, uint32_t stride, uint32_t base,
                                           LaneCap* lc = nullptr, uint32_t ref0 = 0u, uint32_t n0 = 0u) {
    const uint32_t nodeOff = I.meta.x;
    const float4* tri = S.tris + 3u * I.meta.y;
    const uint32_t rlf = f2u(I.r0.w), rcnt = f2u(I.r1.w);
    if (rcnt != 0u) return leafTestUniform<ANY>(tri, rlf, rcnt, o, d, depth, hu, hv, hprim);
    const float4* W = reinterpret_cast<const float4*>(S.wnodes);
    uint32_t* const bottom = stk + base * stride;
    uint32_t* sp = RES ? bottom + n0 * stride : bottom;
    uint32_t ref = RES ? ref0 : nodeOff;    /* the root: its children are tested in its first visit */
    bool any = false;
    for (;;) {
        if (CAP) {
            if (lc->left == 0u) {
                lc->ref = ref; lc->depthN = (uint32_t)((sp - bottom) / stride); lc->capped = true;
                return any;
            }
            --lc->left;
        }
        uint32_t lf = 0u, cnt = 0u;
        if (ref & kLeafTag) {
            lf = ref & 0xFFFFFFu; cnt = (ref >> 24) & 0x7Fu;
        } else {
            const float4* w = W + 12u * ref;
            WRow r0{w[0], w[1], w[2], w[3]}, r1{w[4], w[5], w[6], w[7]}, r2{w[8], w[9], w[10], w[11]};
            pin(r0.a); pin(r0.b); pin(r0.c); pin(r0.d); pin(r1.a); pin(r1.b); pin(r1.c); pin(r1.d);
            pin(r2.a); pin(r2.b); pin(r2.c); pin(r2.d);
            cnt = f2u(r0.d.y);
            lf = f2u(r0.d.x);
            if (cnt == 0u) {
                /* level 1: X's children */
                float dL, dR;
                wBoxes<FIN>(r0, o, rd, depth, dL, dR);
                bool c;                       /* near child is the right one */
                if (ANY) c = dL == kFarAway;
                else c = dL > dR;
                const float dn = c ? dR : dL, df = c ? dL : dR;
                if (dn == kFarAway) goto pop;
                {
                    const WRow rc = wSel(c, r1, r2), rf = wSel(c, r2, r1);
                    const uint32_t cC = f2u(rc.d.y), lC = f2u(rc.d.x), cF = f2u(rf.d.y), lF = f2u(rf.d.x);
                    /* the far child as a stack entry: a packed leaf, or its node index */
                    const uint32_t refF = (cF != 0u && lF < (1u << 24) && cF < 128u) ? (kLeafTag | (cF << 24) | lF)
                                                                                       : nodeOff + lf + (c ? 0u : 1u);
                    if (cC != 0u) {
                        /* near child is a leaf: the far child pushed, then the leaf */
                        if (df != kFarAway) { *sp = refF; sp += stride; }
                        lf = lC; cnt = cC;
                    } else {
                        /* level 2: the near child's children, at the same depth */
                        float eL, eR;
                        wBoxes<FIN>(rc, o, rd, depth, eL, eR);
                        bool g;
                        if (ANY) g = eL == kFarAway;
                        else g = eL > eR;
                        const float en = g ? eR : eL, ef = g ? eL : eR;
                        if (en == kFarAway) {
                            /* the reference pushes the far child and pops it at once */
                            if (df == kFarAway) goto pop;
                            ref = refF;
                            continue;
                        }
                        if (df != kFarAway) { *sp = refF; sp += stride; }
                        const uint32_t pN = f2u(g ? rc.d.w : rc.d.z), pF = f2u(g ? rc.d.z : rc.d.w);
                        if (ef != kFarAway) { *sp = pF ? pF : nodeOff + lC + (g ? 0u : 1u); sp += stride; }
                        ref = pN ? pN : nodeOff + lC + (g ? 1u : 0u);
                        continue;
                    }
                }
            }
        }
        /* a leaf */
        if (leafTest<ANY>(tri, lf, cnt, o, d, depth, hu, hv, hprim)) {
            if (ANY) return true;
            any = true;
        }
    pop:
        if (sp == bottom) break;
        sp -= stride;
        ref = *sp;
    }
    return any;
}

/* Instance::intersect(Any) (bvh.cpp:481-513): origin (M^-1 (o,1)).xyz / w,
 * direction (M^-1 (d,0)).xyz (not renormalized: t is shared with world space).
 * For an affine M^-1 (row 3 = 0,0,0,1) w is exactly 1 for finite o and x/1 = x,
 * so the division is skipped without changing a bit.  Row products keep glm's
 * pairwise sum (m0 x + m1 y) + (m2 z + m3 w) (mrow). */
__device__ __forceinline__ float rowDot(float4 r, float x, float y, float z, float w) {
    const float a = r.x * x + r.y * y;
    const float b = r.z * z + r.w * w;
    return a + b;
}

template <bool ANY, bool LW = false, bool STG = false, typename SK = uint32_t, bool CAP = false>
__device__ __forceinline__ bool instanceTrace(const DevScene& S, const TraceInst& I, V3 o, V3 d, float& depth, float& hu,
                                              float& hv, uint32_t& hprim, SK* stk, uint32_t stride, uint32_t base,
                                              const float4* sN = nullptr, LaneCap* lc = nullptr);
/* The rest of a capped lane walk's BLAS walk (k_extend_cont): the instance's
 * object-space ray formed as instanceTrace forms it, then blasTraceW from the
 * saved ref with the saved refs on the stack (a capped walk was a finite one) */
template <bool LW, typename SK>
__device__ __forceinline__ bool instanceResume(const DevScene& S, const TraceInst& I, V3 o, V3 d, float& depth, float& hu, float& hv,
                                               uint32_t& hprim, SK* stk, uint32_t stride, uint32_t ref0, uint32_t n0) {
    V3 oo = mk3(rowDot(I.m0, o.x, o.y, o.z, 1.0f), rowDot(I.m1, o.x, o.y, o.z, 1.0f), rowDot(I.m2, o.x, o.y, o.z, 1.0f));
    if (!I.meta.z) oo = divs(oo, rowDot(I.m3, o.x, o.y, o.z, 1.0f));
    const V3 dd = mk3(rowDot(I.m0, d.x, d.y, d.z, 0.0f), rowDot(I.m1, d.x, d.y, d.z, 0.0f), rowDot(I.m2, d.x, d.y, d.z, 0.0f));
    const V3 rd = mk3(1.0f / dd.x, 1.0f / dd.y, 1.0f / dd.z);
    if constexpr (LW)
        return blasTraceW<false, true, false, true>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, 0u, nullptr, ref0, n0);
    return blasTrace<false, true, false, SK, false, true>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, 0u, nullptr, nullptr,
                                                         ref0, n0);
}
template <bool ANY, bool LW, bool STG, typename SK, bool CAP>
__device__ __forceinline__ bool instanceTrace(const DevScene& S, const TraceInst& I, V3 o, V3 d, float& depth, float& hu,
                                              float& hv, uint32_t& hprim, SK* stk, uint32_t stride, uint32_t base,
                                              const float4* sN, LaneCap* lc) {
    V3 oo = mk3(rowDot(I.m0, o.x, o.y, o.z, 1.0f), rowDot(I.m1, o.x, o.y, o.z, 1.0f), rowDot(I.m2, o.x, o.y, o.z, 1.0f));
    if (!I.meta.z) oo = divs(oo, rowDot(I.m3, o.x, o.y, o.z, 1.0f));
    const V3 dd = mk3(rowDot(I.m0, d.x, d.y, d.z, 0.0f), rowDot(I.m1, d.x, d.y, d.z, 0.0f), rowDot(I.m2, d.x, d.y, d.z, 0.0f));
    /* a root leaf (the room's walls) needs no 1/d: its triangles are tested directly */
    if (f2u(I.r1.w) != 0u)
        return leafTestUniform<ANY>(S.tris + 3u * I.meta.y, f2u(I.r0.w), f2u(I.r1.w), oo, dd, depth, hu, hv, hprim);
    const V3 rd = mk3(1.0f / dd.x, 1.0f / dd.y, 1.0f / dd.z);
    /* S.finiteBoxes: every BLAS box is finite (checked at upload) */
    const bool fin = S.finiteBoxes && finite3(oo) && finite3(rd);
    if constexpr (LW)
        return fin ? blasTraceW<ANY, true, CAP>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, base, lc)
                   : blasTraceW<ANY, false>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, base);
    if (fin) return blasTrace<ANY, true, STG, SK, CAP>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, base, sN, lc);
    return blasTrace<ANY, false, STG, SK>(S, I, oo, dd, rd, depth, hu, hv, hprim, stk, stride, base, sN);
}

/* Instance tables a traversal reads: LDS copies (stageTrace) or global. */
struct TraceTables {
    const TraceInst* inst;    /* by instance id */
    const uint32_t* order;    /* TLAS leaf index array (tlasIndices) */
};

/* Dynamic LDS layout of the traversal kernels: [stack: depth x blockDim u32]
 * [TraceInst x nInst][tlasIdx x nInst].  Every thread of the block calls this. */
__device__ __forceinline__ TraceTables stageTrace(const DevScene& S, uint32_t* lds, uint32_t stackWords) {
    TraceInst* tab = reinterpret_cast<TraceInst*>(lds + stackWords);
    uint32_t* order = reinterpret_cast<uint32_t*>(tab + S.nInst);
    const uint32_t n16 = S.nInst * (uint32_t)(sizeof(TraceInst) / 16);
    for (uint32_t k = threadIdx.x; k < n16; k += blockDim.x) reinterpret_cast<float4*>(tab)[k] = reinterpret_cast<const float4*>(S.tinst)[k];
    for (uint32_t k = threadIdx.x; k < S.nInst; k += blockDim.x) order[k] = S.tlasIdx[k];
    __syncthreads();
    return TraceTables{tab, order};
}

template <bool LDS_INST>
__device__ __forceinline__ TraceTables traceTables(const DevScene& S, uint32_t* lds, uint32_t stackWords) {
    if (LDS_INST) return stageTrace(S, lds, stackWords);
    return TraceTables{S.tinst, S.tlasIdx};
}

/* BvhTLAS::intersect / intersectAny (bvh.cpp:654-778). */
/* CAP (single-leaf TLAS, LW): the walk stops where the lane's cap ran out
 * (LaneCap); lc->turn is then the instance's place in TLAS order */
/* RES (closest hit, LW): continue a capped lane's walk -- the instance at
 * TLAS place lc->turn from lc->ref / lc->depthN (instanceResume), then the
 * instances after it; any / hinst come in as the lane left them */
template <bool ANY, bool LW = false, bool STG = false, typename SK = uint32_t, bool CAP = false, bool RES = false>
__device__ __forceinline__ bool traceScene(const DevScene& S, const TraceTables& Tt, V3 o, V3 d, float& depth, float& hu, float& hv,
                                           uint32_t& hinst, uint32_t& hprim, SK* stk, uint32_t stride, const float4* sN = nullptr,
                                           LaneCap* lc = nullptr, bool any0 = false) {
    bool any = any0;
    if (RES) {
        const uint32_t ii = Tt.order[lc->turn];
        if (instanceResume<LW, SK>(S, Tt.inst[ii], o, d, depth, hu, hv, hprim, stk, stride, lc->ref, lc->depthN)) {
            any = true;
            hinst = ii;
        }
    }
    if (S.tlasLeafCount) {
        /* single-leaf TLAS (the bundled scene): every lane visits the same
         * instances in the same order -> wave-uniform loop over LDS records.
         * A lane skips an instance whose conservative world box (the BLAS's
         * triangles under M, padded far beyond float rounding) its ray misses
         * within [0, depth): no triangle of it can produce an accepted hit, so
         * the skip changes no result; a wave skips the instance's transform,
         * divisions and traversal when all its lanes do (coherent rays: the
         * shadow queue is ordered by light and origin cell). */
        const V3 rdw = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        const bool cullOk = finite3(o) && finite3(rdw);
        for (uint32_t k = RES ? lc->turn + 1u : 0u; k < S.tlasLeafCount; ++k) {
            const uint32_t ii = Tt.order[k];
            const TraceInst& I = Tt.inst[ii];
            if (cullOk && I.wlo.w != 0.0f) {
                const float tx0 = (I.wlo.x - o.x) * rdw.x, tx1 = (I.whi.x - o.x) * rdw.x;
                const float ty0 = (I.wlo.y - o.y) * rdw.y, ty1 = (I.whi.y - o.y) * rdw.y;
                const float tz0 = (I.wlo.z - o.z) * rdw.z, tz1 = (I.whi.z - o.z) * rdw.z;
                const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
                const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
                if (t1 < t0 || t1 < 0.0f || t0 >= depth) continue;
            }
            /* (wave-uniform: the staged BLAS's instances walk it in LDS; the
             * staged triangles are those at S.sbTri0, so both offsets must match) */
            const bool hitI = (STG && !LW && I.meta.x == S.sbNode0 && I.meta.y == S.sbTri0)
                                  ? instanceTrace<ANY, false, true, SK>(S, I, o, d, depth, hu, hv, hprim, stk, stride, 0u, sN)
                                  : instanceTrace<ANY, LW, false, SK, CAP>(S, I, o, d, depth, hu, hv, hprim, stk, stride, 0u, nullptr, lc);
            if (hitI) {
                if (ANY) return true;
                any = true;
                hinst = ii;
            }
            if (CAP && lc->capped) { lc->turn = k; return any; }
        }
        return any;
    }
    const V3 rd = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    uint32_t sp = 0, node = 0;
    for (;;) {
        const float4* nd = S.tlasNodes + 4u * node;
        float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        pin(q0); pin(q1); pin(q2); pin(q3);
        const uint32_t lf = f2u(q0.w), cnt = f2u(q1.w);
        if (cnt != 0u) {
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t ii = Tt.order[lf + k];
                if (instanceTrace<ANY, LW, false, SK>(S, Tt.inst[ii], o, d, depth, hu, hv, hprim, stk, stride, sp)) {
                    if (ANY) return true;
                    any = true;
                    hinst = ii;
                }
            }
            if (sp == 0) break;
            node = stk[(--sp) * stride];
            continue;
        }
        float dn = slab(q0.x, q0.y, q0.z, q1.x, q1.y, q1.z, o, rd, depth);
        float df = slab(q2.x, q2.y, q2.z, q3.x, q3.y, q3.z, o, rd, depth);
        uint32_t cn = lf, cf = lf + 1u;
        if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
        if (dn == kFarAway) {
            if (sp == 0) break;
            node = stk[(--sp) * stride];
        } else {
            node = cn;
            if (df != kFarAway) stk[(sp++) * stride] = cf;
        }
    }
    return any;
}

/* Object-space ray of instance I (Instance::intersect, bvh.cpp:481-513). */
__device__ __forceinline__ void instanceRay(const TraceInst& I, V3 o, V3 d, V3& oo, V3& dd) {
    oo = mk3(rowDot(I.m0, o.x, o.y, o.z, 1.0f), rowDot(I.m1, o.x, o.y, o.z, 1.0f), rowDot(I.m2, o.x, o.y, o.z, 1.0f));
    if (!I.meta.z) oo = divs(oo, rowDot(I.m3, o.x, o.y, o.z, 1.0f));
    dd = mk3(rowDot(I.m0, d.x, d.y, d.z, 0.0f), rowDot(I.m1, d.x, d.y, d.z, 0.0f), rowDot(I.m2, d.x, d.y, d.z, 0.0f));
}

/* ------------------------------------------------- one ray per wave, lanes as planes
 * For the last long paths of a drain (whose single-path segment latency is
 * what the drain waits for): every lane holds the same ray and the wave walks
 * the reference's DFS itself -- same boxes, same near/far order, same pruning,
 * same leaf order -- with the work of one node visit spread over lanes:
 *   lanes 0..11 each load one bound of the node record (box b = l / 6,
 *   axis a = (l % 6) / 2, side s = l & 1), lanes 12 / 13 its leftFirst / count;
 *   (bound - o_a) * rd_a for all 12 planes is one multiply;
 *   the reference's ternary min/max (same operand order, so NaN/inf cases
 *   stay bit-identical) run on lane pairs and lane triples via DPP moves;
 *   near/far, the stack (one VGPR, entry k in lane k) and the loop are scalar;
 *   a leaf's triangles are tested in parallel lanes and accepted in index order.
 * The DFS is the same sequence of decisions as blasTrace, so results equal
 * traceScene's bit for bit (also for any-hit).  Needs all 64 lanes active, a
 * single-leaf TLAS and a stack depth <= 64. */
template <int CTRL>
__device__ __forceinline__ float dppMov(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppSwap1 = 0xB1;             /* quad_perm [1,0,3,2]: lane l <- l ^ 1 */
constexpr int kDppShr2 = 0x112, kDppShr4 = 0x114;   /* row_shr: lane l <- l - n (within 16) */

__device__ __forceinline__ uint32_t planeDword(uint32_t l) {
    if (l < 12u) return (l / 6u) * 8u + (l & 1u) * 4u + ((l % 6u) >> 1);
    return l == 12u ? 3u : (l == 13u ? 7u : 0u);
}
__device__ __forceinline__ float pick3(V3 v, uint32_t a) { return a == 0u ? v.x : (a == 1u ? v.y : v.z); }

/* Both children's slab distances from this lane's bound v (lanes 0..11):
 * dn = box 0 (left child), df = box 1 (right), kFarAway on a miss (slab()). */
__device__ __forceinline__ void slabPair(float v, float oA, float rdA, float depth, float& d0, float& d1) {
    const float t = (v - oA) * rdA;
    const float tp = dppMov<kDppSwap1>(t);
    const float t0a = tmin(t, tp), t1a = tmax(t, tp);          /* even lanes: (lo, hi) of one axis */
    const float t0x = dppMov<kDppShr4>(t0a), t0y = dppMov<kDppShr2>(t0a);
    const float t1x = dppMov<kDppShr4>(t1a), t1y = dppMov<kDppShr2>(t1a);
    const float m0 = tmax(tmax(t0x, t0y), t0a);                /* lane 6b+4: t0a is the z axis */
    const float m1 = tmin(tmin(t1x, t1y), t1a);
    const float dist = (m1 >= m0 && m0 < depth && m1 > 0.0f) ? m0 : kFarAway;
    d0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dist), 4));
    d1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dist), 10));
}

/* Triangles [lf, lf + cnt) of a BLAS leaf, one per lane, accepted in index order. */
template <bool ANY>
__device__ __forceinline__ bool leafWave(const float4* tri, uint32_t lf, uint32_t cnt, V3 o, V3 d, float& depth,
                                         float& hu, float& hv, uint32_t& hprim) {
    bool any = false;
    const uint32_t lane = __lane_id();
    for (uint32_t b = 0; b < cnt; b += 64u) {
        const uint32_t k = b + lane;
        float t = depth, u = 0.0f, v = 0.0f;
        uint32_t prim = 0;
        bool h = false;
        if (k < cnt) {
            const float4* tp = tri + 3u * (lf + k);
            const float4 a = tp[0], e1 = tp[1], e2 = tp[2];
            prim = f2u(a.w);
            h = triHitFlat(xyz(a), xyz(e1), xyz(e2), o, d, depth, t, u, v);
        }
        unsigned long long m = __ballot(h);
        if (ANY) { if (m) return true; continue; }
        while (m) {
            const int j = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const float tj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), j));
            if (tj < depth) {
                depth = tj;
                hu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j));
                hv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
                hprim = (uint32_t)__builtin_amdgcn_readlane((int)prim, j);
                any = true;
            }
        }
    }
    return any;
}

/* SURF_SEG_TIMING builds: per-segment breakdown of traceWave (diagnostics).
 * segClock waits for every outstanding memory operation, then reads the
 * shader clock, so a section's time includes its loads. */
#if SURF_SEG_TIMING
__device__ __forceinline__ unsigned long long segClock() {
    unsigned long long t;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    return t;
}
__device__ unsigned long long g_segStats[8];
#endif
struct SegStats { unsigned long long cycInst, cycLoop, visits, leaves, tris, entered, cycWait, cycLeaf; };

/* SURF_DRAIN_TRACE builds: (end time, segments, start time, state at the
 * start: age | inMedium << 16 | lastSpecular << 17 | 255 max(T) << 24) of every
 * path the cooperative drain kernels finish, real-time clock (diagnostics). */
#ifndef SURF_DRAIN_TRACE
#define SURF_DRAIN_TRACE 0
#endif
#if SURF_DRAIN_TRACE
constexpr uint32_t kDrainTraceCap = 1u << 18;
__device__ uint4 g_drainEnd[kDrainTraceCap];
__device__ uint32_t g_drainEndN;
__device__ __forceinline__ uint32_t drainState(float4 d4, float4 T4) {
    const uint32_t fl = f2u(d4.w);
    const float m = fminf(fmaxf(fmaxf(T4.x, T4.y), T4.z), 1.0f);
    return min(fl >> 2, 0xffffu) | ((fl & 3u) << 16) | ((uint32_t)(m * 255.0f) << 24);
}
__device__ __forceinline__ void drainTraceEnd(unsigned long long t0, uint32_t seg, uint32_t state) {
    const unsigned long long t = wall_clock64();
    const uint32_t k = atomicAdd(&g_drainEndN, 1u);
    if (k < kDrainTraceCap) g_drainEnd[k] = make_uint4((uint32_t)t, state, seg, (uint32_t)t0);
}
#endif

/* Lanes-as-planes slab distances of the record held in row `row` (lanes
 * 16 row .. 16 row + 13) of v: the DPP moves of slabPair stay inside a row of
 * 16 lanes, so every row evaluates its own record. */
template <bool FIN>
__device__ __forceinline__ void slabPairRow(float v, float oA, float rdA, float depth, uint32_t row, float& d0, float& d1) {
    const float t = (v - oA) * rdA;
    float m0, m1;
    if (FIN) {
        /* o, 1/d and every box finite: no NaN can arise, the ternary min/max
         * equal IEEE min/max (slabFinite), and the lane moves fold into the
         * min/max as DPP operands (6 VALU ops instead of 17).  m0 / m1 are
         * valid in lanes 4 and 10 of each row (their l-4, l-2 sources). */
        float t0a, t1a;
        asm volatile(
            "s_nop 1\n\t"
            "v_min_f32_dpp %0, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %1, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_max_f32_dpp %2, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_min_f32_dpp %3, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_max_f32_dpp %2, %0, %2 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
            "v_min_f32_dpp %3, %1, %3 row_shr:2 row_mask:0xf bank_mask:0xf"
            : "=&v"(t0a), "=&v"(t1a), "=&v"(m0), "=&v"(m1)
            : "v"(t));
    } else {
        const float tp = dppMov<kDppSwap1>(t);
        const float t0a = tmin(t, tp), t1a = tmax(t, tp);
        const float t0x = dppMov<kDppShr4>(t0a), t0y = dppMov<kDppShr2>(t0a);
        const float t1x = dppMov<kDppShr4>(t1a), t1y = dppMov<kDppShr2>(t1a);
        m0 = tmax(tmax(t0x, t0y), t0a);
        m1 = tmin(tmin(t1x, t1y), t1a);
    }
    const float dist = (m1 >= m0 && m0 < depth && m1 > 0.0f) ? m0 : kFarAway;
    d0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dist), (int)(4u + 16u * row)));
    d1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dist), (int)(10u + 16u * row)));
}

/* slabPairRow's decision without leaving the vector unit: lane 10 of the row
 * takes box 0's distance from lane 4 (DPP row_shr:6) and forms blasTrace's
 * choices -- bit 0: the right child is nearer (dn > df), bit 1: the nearer
 * child is hit, bit 2: the farther child is hit -- read out with one readlane
 * (instead of two readlanes and float compares on scalar operands). */
constexpr int kDppShr6 = 0x116;
template <bool FIN>
__device__ __forceinline__ uint32_t slabDecide(float v, float oA, float rdA, float depth, uint32_t row) {
    const float t = (v - oA) * rdA;
    float m0, m1;
    if (FIN) {
        float t0a, t1a;
        asm volatile(
            "s_nop 1\n\t"
            "v_min_f32_dpp %0, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "v_max_f32_dpp %1, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_max_f32_dpp %2, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
            "v_min_f32_dpp %3, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_max_f32_dpp %2, %0, %2 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
            "v_min_f32_dpp %3, %1, %3 row_shr:2 row_mask:0xf bank_mask:0xf"
            : "=&v"(t0a), "=&v"(t1a), "=&v"(m0), "=&v"(m1)
            : "v"(t));
    } else {
        const float tp = dppMov<kDppSwap1>(t);
        const float t0a = tmin(t, tp), t1a = tmax(t, tp);
        const float t0x = dppMov<kDppShr4>(t0a), t0y = dppMov<kDppShr2>(t0a);
        const float t1x = dppMov<kDppShr4>(t1a), t1y = dppMov<kDppShr2>(t1a);
        m0 = tmax(tmax(t0x, t0y), t0a);
        m1 = tmin(tmin(t1x, t1y), t1a);
    }
    /* blasTrace: dist_b = hit_b ? m0_b : kFarAway, swap when dn > df.  With
     * hit_b = (m1 >= m0 && m0 < depth && m1 > 0) (false on NaN) and m0 < depth
     * <= kFarAway for a hit: swap = hit1 && (!hit0 || m0_0 > m0_1).  The three
     * facts come out of the compares as lane masks (SGPRs) and the choice is
     * scalar: no select / readlane chain in the vector unit. */
    const unsigned long long H = __ballot(m1 >= m0 && m0 < depth && m1 > 0.0f);   /* lanes 4 / 10: box 0 / box 1 hit */
    const float mp = dppMov<kDppShr6>(m0);              /* lane 10 <- lane 4 */
    const unsigned long long G = __ballot(mp > m0);      /* lane 10: m0 of box 0 > m0 of box 1 */
    const uint32_t sh = 16u * row;
    const uint32_t hit0 = (uint32_t)(H >> (4u + sh)) & 1u, hit1 = (uint32_t)(H >> (10u + sh)) & 1u;
    const uint32_t gt = (uint32_t)(G >> (10u + sh)) & 1u;
    const uint32_t sw = hit1 & (gt | (hit0 ^ 1u));
    const uint32_t farHit = sw ? hit0 : hit1;
    return sw | ((sw | hit0) << 1) | (farHit << 2);
}
__device__ __forceinline__ void waitLoadsAfterBits(float& v, uint32_t bits) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v) : "s"(bits));
}

/* slab()'s t0 / t1 before its hit test: the same operations in the same order. */
__device__ __forceinline__ void slabRange(float4 lo, float4 hi, V3 o, V3 rd, float& t0, float& t1) {
    const float tx0 = (lo.x - o.x) * rd.x, tx1 = (hi.x - o.x) * rd.x;
    t0 = tmin(tx0, tx1); t1 = tmax(tx0, tx1);
    const float ty0 = (lo.y - o.y) * rd.y, ty1 = (hi.y - o.y) * rd.y;
    t0 = tmax(t0, tmin(ty0, ty1)); t1 = tmin(t1, tmax(ty0, ty1));
    const float tz0 = (lo.z - o.z) * rd.z, tz1 = (hi.z - o.z) * rd.z;
    t0 = tmax(t0, tmin(tz0, tz1)); t1 = tmin(t1, tmax(tz0, tz1));
}
__device__ __forceinline__ float slabHit(float t0, float t1, float depth) {
    return (t1 >= t0 && t0 < depth && t1 > 0.0f) ? t0 : kFarAway;
}
__device__ __forceinline__ float bcast(float v, uint32_t l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l)); }

/* A load the compiler may not sink past the code between it and its use (it
 * would sink a load used on one branch into that branch, after the slab test
 * it is meant to overlap).  Its VGPR is outside the compiler's wait-count
 * tracking, so the value is passed through waitLoads() before any use. */
__device__ __forceinline__ float loadEarly(const float* p) {
    float v;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
    return v;
}
__device__ __forceinline__ void waitLoads(float& v) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(v)); }
/* ... and not before a and b are computed (the scheduler would hoist it). */
__device__ __forceinline__ void waitLoadsAfter(float& v, float a, float b) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v) : "s"(a), "s"(b));
}

/* blasWalk's interior visits (FIN: o, 1/d and every box finite) as one
 * instruction sequence: the compiler's structurized control flow spent ~70
 * instructions per visit on flag registers and loop-carried copies, while the
 * drain's throughput is set by instructions issued per segment (+24 per visit
 * of either kind: +15 % drain time, profiles/r2_experiments).  Same operations
 * as slabDecide<true> and the C++ loop, in the same order: the record's plane
 * distances, the DPP min/max fold, the hit / order masks, the near child
 * (row of the prefetched pair) or a pop, the far child's record to the LDS
 * stack.  Leaves the walk at a leaf (cnt != 0; lf, cnt of it) or with the
 * stack empty (cnt == 0).  Stack pointer in bytes (64 per entry); the
 * records are read through a raw buffer resource at byte offset
 * 64 (nodeOff + lf) + laneOff. */
typedef int surfI4 __attribute__((ext_vector_type(4)));
template <bool ANY>
__device__ __forceinline__ void walkInteriorFin(float& cur, uint32_t& row16, uint32_t& spb, uint32_t& lf, uint32_t& cnt,
                                                float oA, float rdA, float depth, uint32_t nodeOff, surfI4 rsrc,
                                                uint32_t laneOff, uint32_t stkLane) {
    float nxt, t, t0a, t1a, m0, m1, mp;
    uint32_t addr, idx, off;
    unsigned long long h, tt, g, a, save;
    const unsigned long long mask0 = 0x000000000000FFFFull, mask1 = 0x00000000FFFF0000ull;
    if (ANY) {
        asm volatile(
        /* lf / cnt of the current node are read where cur is set (entry, descend, pop) */
        "s_or_b32 %[idx], %[row], 13\n\t"
        "v_readlane_b32 %[cnt], %[cur], %[idx]\n\t"
        "s_or_b32 %[idx], %[row], 12\n\t"
        "v_readlane_b32 %[lf], %[cur], %[idx]\n"
        "L_top_%=:\n\t"
        "s_cmp_lg_u32 %[cnt], 0\n\t"
        "s_cbranch_scc1 L_exit_%=\n\t"
        "s_lshl_b32 %[off], %[lf], 6\n\t"
        "buffer_load_dword %[nxt], %[loff], %[rsrc], %[off] offen\n\t"
#if SURF_EXPOSE_LOAD   /* diagnostics: the record load's whole latency on the visit's path */
        "s_waitcnt vmcnt(0)\n\t"
#endif
        "v_sub_f32 %[t], %[cur], %[oA]\n\t"
        "v_mul_f32 %[t], %[t], %[rdA]\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %[t0a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %[t1a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %[m0], %[t0a], %[t0a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %[m1], %[t1a], %[t1a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %[m0], %[t0a], %[m0] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %[m1], %[t1a], %[m1] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        /* lanes 4 / 10 of the row: box 0 / box 1 hit (m1 >= m0, m0 < depth, m1 > 0) */
        "v_cmp_ge_f32_e64 %[h], %[m1], %[m0]\n\t"
        "v_cmp_gt_f32_e64 %[tt], %[depth], %[m0]\n\t"
        "s_and_b64 %[h], %[h], %[tt]\n\t"
        "v_cmp_lt_f32_e64 %[tt], 0, %[m1]\n\t"
        "s_and_b64 %[h], %[h], %[tt]\n\t"
        /* any-hit: no near/far order (the answer is an OR over the admitted
         * leaves): box 0 first when hit, box 1 pushed when both hit */
        "s_lshr_b64 %[h], %[h], %[row]\n\t"
        "s_bitcmp1_b64 %[h], 4\n\t"
        "s_cbranch_scc1 L_h0_%=\n\t"
        "s_bitcmp1_b64 %[h], 10\n\t"
        "s_cbranch_scc0 L_pop_%=\n\t"
        "s_mov_b32 %[row], 16\n\t"
        "s_branch L_desc_%=\n"
        "L_h0_%=:\n\t"
        "s_mov_b32 %[row], 0\n\t"
        "s_bitcmp1_b64 %[h], 10\n\t"
        "s_cbranch_scc0 L_desc_%=\n\t"
        "v_add_u32 %[addr], %[sp], %[stk]\n\t"
        "s_mov_b64 %[save], exec\n\t"
        "s_mov_b64 exec, %[mask1]\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "ds_write_b32 %[addr], %[nxt]\n\t"
        "s_mov_b64 exec, %[save]\n\t"
        "s_add_u32 %[sp], %[sp], 64\n"
        "L_desc_%=:\n\t"
        "s_or_b32 %[idx], %[row], 13\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "v_readlane_b32 %[cnt], %[nxt], %[idx]\n\t"
        "s_or_b32 %[idx], %[row], 12\n\t"
        "v_readlane_b32 %[lf], %[nxt], %[idx]\n\t"
        "v_mov_b32 %[cur], %[nxt]\n\t"
        "s_branch L_top_%=\n"
        /* both children missed: pop (every row reads the entry) or done */
        "L_pop_%=:\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_cmp_eq_u32 %[sp], 0\n\t"
        "s_cbranch_scc1 L_done_%=\n\t"
        "s_sub_u32 %[sp], %[sp], 64\n\t"
        "v_add_u32 %[addr], %[sp], %[stk]\n\t"
        "ds_read_b32 %[cur], %[addr]\n\t"
        "s_mov_b32 %[row], 0\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readlane_b32 %[cnt], %[cur], 13\n\t"
        "v_readlane_b32 %[lf], %[cur], 12\n\t"
        "s_branch L_top_%=\n"
        "L_done_%=:\n\t"
        "s_mov_b32 %[cnt], 0\n"
        "L_exit_%=:"
        : [cur] "+v"(cur), [row] "+s"(row16), [sp] "+s"(spb), [lf] "=&s"(lf), [cnt] "=&s"(cnt), [nxt] "=&v"(nxt),
          [t] "=&v"(t), [t0a] "=&v"(t0a), [t1a] "=&v"(t1a), [m0] "=&v"(m0), [m1] "=&v"(m1), [mp] "=&v"(mp),
          [addr] "=&v"(addr), [idx] "=&s"(idx), [off] "=&s"(off), [h] "=&s"(h), [tt] "=&s"(tt), [g] "=&s"(g),
          [a] "=&s"(a), [save] "=&s"(save)
        : [oA] "v"(oA), [rdA] "v"(rdA), [depth] "s"(depth), [noff] "s"(nodeOff), [rsrc] "s"(rsrc), [loff] "v"(laneOff),
          [stk] "v"(stkLane), [mask0] "s"(mask0), [mask1] "s"(mask1)
        : "memory", "scc");
    } else {
        asm volatile(
        /* lf / cnt of the current node are read where cur is set (entry, descend, pop) */
        "s_or_b32 %[idx], %[row], 13\n\t"
        "v_readlane_b32 %[cnt], %[cur], %[idx]\n\t"
        "s_or_b32 %[idx], %[row], 12\n\t"
        "v_readlane_b32 %[lf], %[cur], %[idx]\n"
        "L_top_%=:\n\t"
        "s_cmp_lg_u32 %[cnt], 0\n\t"
        "s_cbranch_scc1 L_exit_%=\n\t"
        "s_lshl_b32 %[off], %[lf], 6\n\t"
        "buffer_load_dword %[nxt], %[loff], %[rsrc], %[off] offen\n\t"
#if SURF_EXPOSE_LOAD   /* diagnostics: the record load's whole latency on the visit's path */
        "s_waitcnt vmcnt(0)\n\t"
#endif
        "v_sub_f32 %[t], %[cur], %[oA]\n\t"
        "v_mul_f32 %[t], %[t], %[rdA]\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %[t0a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %[t1a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %[m0], %[t0a], %[t0a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %[m1], %[t1a], %[t1a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %[m0], %[t0a], %[m0] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %[m1], %[t1a], %[m1] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        /* lanes 4 / 10 of the row: box 0 / box 1 hit (m1 >= m0, m0 < depth, m1 > 0) */
        "v_cmp_ge_f32_e64 %[h], %[m1], %[m0]\n\t"
        "v_cmp_gt_f32_e64 %[tt], %[depth], %[m0]\n\t"
        "s_and_b64 %[h], %[h], %[tt]\n\t"
        "v_cmp_lt_f32_e64 %[tt], 0, %[m1]\n\t"
        "s_and_b64 %[h], %[h], %[tt]\n\t"
        /* lane 10: m0 of box 0 > m0 of box 1 */
        "v_mov_b32_dpp %[mp], %[m0] row_shr:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_cmp_gt_f32_e64 %[g], %[mp], %[m0]\n\t"
        "s_lshr_b64 %[h], %[h], %[row]\n\t"
        /* bits 4 / 10 of a: box 0 / box 1 hit.  One hit: that child, nothing
         * pushed.  Both: the nearer (swap when m0 of box 0 > m0 of box 1, as
         * blasTrace's dn > df), the other pushed.  None: pop. */
        "s_and_b64 %[a], %[h], 0x410\n\t"
        "s_cbranch_scc0 L_pop_%=\n\t"
        "s_cmp_eq_u64 %[a], 0x410\n\t"
        "s_cbranch_scc1 L_both_%=\n\t"
        "s_cmp_eq_u64 %[a], 0x400\n\t"
        "s_cselect_b32 %[row], 16, 0\n\t"
        "s_branch L_desc_%=\n"
        "L_both_%=:\n\t"
        "s_lshr_b64 %[g], %[g], %[row]\n\t"
        "v_add_u32 %[addr], %[sp], %[stk]\n\t"
        "s_bitcmp1_b64 %[g], 10\n\t"
        "s_cselect_b32 %[row], 16, 0\n\t"
        "s_cselect_b64 %[a], %[mask0], %[mask1]\n\t"
        "s_mov_b64 %[save], exec\n\t"
        "s_mov_b64 exec, %[a]\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "ds_write_b32 %[addr], %[nxt]\n\t"
        "s_mov_b64 exec, %[save]\n\t"
        "s_add_u32 %[sp], %[sp], 64\n"
        "L_desc_%=:\n\t"
        "s_or_b32 %[idx], %[row], 13\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "v_readlane_b32 %[cnt], %[nxt], %[idx]\n\t"
        "s_or_b32 %[idx], %[row], 12\n\t"
        "v_readlane_b32 %[lf], %[nxt], %[idx]\n\t"
        "v_mov_b32 %[cur], %[nxt]\n\t"
        "s_branch L_top_%=\n"
        /* both children missed: pop (every row reads the entry) or done */
        "L_pop_%=:\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_cmp_eq_u32 %[sp], 0\n\t"
        "s_cbranch_scc1 L_done_%=\n\t"
        "s_sub_u32 %[sp], %[sp], 64\n\t"
        "v_add_u32 %[addr], %[sp], %[stk]\n\t"
        "ds_read_b32 %[cur], %[addr]\n\t"
        "s_mov_b32 %[row], 0\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readlane_b32 %[cnt], %[cur], 13\n\t"
        "v_readlane_b32 %[lf], %[cur], 12\n\t"
        "s_branch L_top_%=\n"
        "L_done_%=:\n\t"
        "s_mov_b32 %[cnt], 0\n"
        "L_exit_%=:"
        : [cur] "+v"(cur), [row] "+s"(row16), [sp] "+s"(spb), [lf] "=&s"(lf), [cnt] "=&s"(cnt), [nxt] "=&v"(nxt),
          [t] "=&v"(t), [t0a] "=&v"(t0a), [t1a] "=&v"(t1a), [m0] "=&v"(m0), [m1] "=&v"(m1), [mp] "=&v"(mp),
          [addr] "=&v"(addr), [idx] "=&s"(idx), [off] "=&s"(off), [h] "=&s"(h), [tt] "=&s"(tt), [g] "=&s"(g),
          [a] "=&s"(a), [save] "=&s"(save)
        : [oA] "v"(oA), [rdA] "v"(rdA), [depth] "s"(depth), [noff] "s"(nodeOff), [rsrc] "s"(rsrc), [loff] "v"(laneOff),
          [stk] "v"(stkLane), [mask0] "s"(mask0), [mask1] "s"(mask1)
        : "memory", "scc");
    }
}

/* The DFS below one BLAS root (blasTrace's loop), from the root's children:
 * near child cn at distance dn (!= kFarAway), far child cf at df.  Latency:
 * a visit issues the load of BOTH children's records (row 0 of the VGPR:
 * left child, row 1: right; rows 2/3 repeat them) before its own slab test,
 * so the near child's record is in registers when the decision is made; a
 * pop loads the popped node's record into every row. */
#define SURF_STR(x) #x
#define SURF_XSTR(x) SURF_STR(x)
template <bool ANY, bool FIN>
__device__ __forceinline__ bool blasWalk(const DevScene& S, uint32_t nodeOff, const float4* tri, V3 o, V3 d, V3 rd,
                                         float dn, float df, uint32_t cn, uint32_t cf, float& depth, float& hu, float& hv,
                                         uint32_t& hprim, float* rs, SegStats* ss) {
    const uint32_t lane = __lane_id(), l16 = lane & 15u;
    const uint32_t dw = planeDword(l16), ax = l16 < 12u ? (l16 % 6u) >> 1 : 0u;
    const uint32_t half = (lane >> 4) & 1u;
    const float oA = pick3(o, ax), rdA = pick3(rd, ax);
    const float* nodesF = reinterpret_cast<const float*>(S.nodes);
    /* the root's children: both records (rows 0/1), the far one to the stack */
    const uint32_t cmin = cn < cf ? cn : cf;
    float cur = nodesF[16u * (cmin + half) + dw];
    uint32_t row = cn - cmin, sp = 0;
    if (df != kFarAway) {
        if (half != row && lane < 32u) rs[l16] = cur;
        sp = 1;
    }
    bool any = false;
#if SURF_SEG_TIMING
    if (ss) ++ss->entered;
#endif
    /* walkInteriorFin's operands: node records as a raw buffer (gfx9 dword 3),
     * this lane's byte offset in a record pair, its LDS stack column */
    const uintptr_t nb = reinterpret_cast<uintptr_t>(S.nodes + 4u * (size_t)nodeOff);   /* this BLAS's records */
    const surfI4 rsrc = {(int)(uint32_t)nb, (int)(uint32_t)(nb >> 32), -1, 0x00020000};
    const uint32_t laneOff = 64u * half + 4u * dw;
    const uint32_t stkLane = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)rs) + 4u * l16;
    (void)rsrc; (void)laneOff; (void)stkLane;
    for (;;) {
        /* interior nodes: an inner loop that leaves depth and the hit untouched
         * (no loop-carried copies of them per visit) */
        uint32_t lf, cnt;
#if !SURF_PAD_VALU && !SURF_PAD_SALU   /* (timing builds count no interior visits on this path) */
        if (FIN && S.nodes4G) {
            uint32_t row16 = 16u * row, spb = 64u * sp;
            walkInteriorFin<ANY>(cur, row16, spb, lf, cnt, oA, rdA, depth, nodeOff, rsrc, laneOff, stkLane);
            row = row16 >> 4;
            sp = spb >> 6;
            if (cnt == 0u) return any;
#if SURF_SEG_TIMING
            if (ss) { ++ss->leaves; ss->tris += cnt; }
#endif
        } else
#endif
        for (;;) {
            lf = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(cur), (int)(12u + 16u * row));
            cnt = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(cur), (int)(13u + 16u * row));
#if SURF_SEG_TIMING
            if (ss) { if (cnt) { ++ss->leaves; ss->tris += cnt; } else ++ss->visits; }
#endif
            if (cnt != 0u) break;
#if SURF_PAD_VALU   /* diagnostics: extra VALU / SALU issue per interior visit */
            asm volatile(".rept " SURF_XSTR(SURF_PAD_VALU) "\n\tv_nop\n\t.endr");
#endif
#if SURF_PAD_SALU
            { uint32_t z = lf; asm volatile(".rept " SURF_XSTR(SURF_PAD_SALU) "\n\ts_add_u32 %0, %0, 1\n\t.endr" : "+s"(z)); }
#endif
            const uint32_t c0 = nodeOff + lf;
            float nxt = loadEarly(nodesF + 16u * (c0 + half) + dw);
            const uint32_t bits = slabDecide<FIN>(cur, oA, rdA, depth, row);
            const uint32_t nearRow = bits & 1u;
#if SURF_SEG_TIMING
            const unsigned long long tw0 = segClock();
#endif
            waitLoadsAfterBits(nxt, bits);   /* on every path: the register must not be reused while the load is in flight */
#if SURF_SEG_TIMING
            if (ss) { asm volatile("" : "+v"(nxt)); ss->cycWait += segClock() - tw0; }
#endif
            if (!(bits & 2u)) {
                if (sp == 0u) return any;
                cur = rs[16u * --sp + l16];
                row = 0;
            } else {
                cur = nxt;
                row = nearRow;
                /* the far child's record (already fetched, the other row) to the LDS stack */
                if (bits & 4u) {
                    if (half != nearRow && lane < 32u) rs[16u * sp + l16] = nxt;
                    ++sp;
                }
            }
        }
#if SURF_SEG_TIMING
        const unsigned long long tl0 = segClock();
#endif
        const bool lh = leafWave<ANY>(tri, lf, cnt, o, d, depth, hu, hv, hprim);
#if SURF_SEG_TIMING
        if (ss) ss->cycLeaf += segClock() - tl0;
#endif
        if (lh) {
            if (ANY) return true;
            any = true;
        }
        if (sp == 0u) break;
        cur = rs[16u * --sp + l16];
        row = 0;
    }
    return any;
}

template <bool ANY>
__device__ __forceinline__ bool blasWave(const DevScene& S, const TraceInst& I, V3 o, V3 d, float& depth, float& hu, float& hv,
                                         uint32_t& hprim, float* rs, SegStats* ss = nullptr) {
    const uint32_t lane = __lane_id();
    const uint32_t nodeOff = I.meta.x;
    const float4* tri = S.tris + 3u * I.meta.y;
    const uint32_t rlf = f2u(I.r0.w), rcnt = f2u(I.r1.w);
    if (rcnt != 0u) return leafWave<ANY>(tri, rlf, rcnt, o, d, depth, hu, hv, hprim);
    const V3 rd = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const uint32_t dw = planeDword(lane), ax = lane < 12u ? (lane % 6u) >> 1 : 0u;
    const float oA = pick3(o, ax), rdA = pick3(rd, ax);
    /* root: never box-tested (bvh.cpp:131); its children's boxes are in its record */
    float dn, df;
    slabPair(reinterpret_cast<const float*>(&I.r0)[dw], oA, rdA, depth, dn, df);
    uint32_t cn = nodeOff + rlf, cf = cn + 1u;
    if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
    if (dn == kFarAway) return false;
    if (S.finiteBoxes && finite3(o) && finite3(rd))
        return blasWalk<ANY, true>(S, nodeOff, tri, o, d, rd, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss);
    return blasWalk<ANY, false>(S, nodeOff, tri, o, d, rd, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss);
}

/* ---------------------------------------------------------------------------
 * Two BVH levels per wave visit (the drain's closest-hit and any-hit walks).
 *
 * The two-level record W(X) of node X (host-built, 48 floats = 192 B) holds
 * three node records in the lanes-as-planes order (lane l of a row holds dword
 * planeDword(l) of the 64-B record): row 0 = rec(X), row 1 = rec(X.left),
 * row 2 = rec(X.right) -- the boxes of X's two children and of its four
 * grandchildren, every child's and grandchild's leftFirst / count.  (A leaf's
 * W holds its own record in row 0.)
 *
 * One visit of X with W(X) in a VGPR:
 *   - issues the loads of W of X's four grandchildren (the candidates for the
 *     next visit) and of X's two children (what a push of the far child
 *     needs), all addresses read from W(X);
 *   - one slab pass over the three rows: the hit / order masks of X's
 *     children and of both children's children;
 *   - the reference's decisions for both levels (bvh.cpp:129-191: near child
 *     first, far child pushed when hit, pop when both miss), exact because no
 *     leaf lies between the two levels, so the depth is the same: near child
 *     C of X (a leaf: push the far child, leave for the leaf), then near
 *     child G of C with the far grandchild pushed after the far child, or --
 *     both of C's children missed -- the far child (pushed then popped at
 *     once in the reference), or a pop;
 *   - the next state W(G) is one of the four candidate loads, selected by
 *     v_cndmask on scalar masks; pushes write whole W records to the LDS
 *     stack (256 B per entry; ds_write2st64 writes both slots, the stack
 *     pointer advances by how many were real).
 * One memory round trip per two levels instead of one per level, and one
 * slab pass + one decision sequence per two levels. */
#define SURF_W2_HEAD                                                                                   \
    /* the state may be a leaf (entry, pop, descent): leave for it */                                  \
    "L_chk_%=:\n\t"                                                                                    \
    "v_readlane_b32 %[cnt], %[st], 13\n\t"                                                             \
    "v_readlane_b32 %[lf], %[st], 12\n\t"                                                              \
    "s_cmp_lg_u32 %[cnt], 0\n\t"                                                                       \
    "s_cbranch_scc1 L_exit_%=\n\t"                                                                     \
    SURF_W2_VISIT                                                                                      \
    /* candidate loads: W of the grandchildren (n0..n3) and of the children (f0, f1) */                \
    "v_readlane_b32 %[lfL], %[st], 28\n\t"                                                             \
    "v_readlane_b32 %[lfR], %[st], 44\n\t"                                                             \
    "s_mul_i32 %[o0], %[lfL], 192\n\t"                                                                 \
    "s_mul_i32 %[o2], %[lfR], 192\n\t"                                                                 \
    "s_mul_i32 %[of], %[lf], 192\n\t"                                                                  \
    "buffer_load_dword %[n0], %[loff], %[rsrc], %[o0] offen\n\t"                                       \
    "buffer_load_dword %[n1], %[loff], %[rsrc], %[o0] offen offset:192\n\t"                            \
    "buffer_load_dword %[n2], %[loff], %[rsrc], %[o2] offen\n\t"                                       \
    "buffer_load_dword %[n3], %[loff], %[rsrc], %[o2] offen offset:192\n\t"                            \
    "buffer_load_dword %[f0], %[loff], %[rsrc], %[of] offen\n\t"                                       \
    "buffer_load_dword %[f1], %[loff], %[rsrc], %[of] offen offset:192\n\t"                            \
    /* the 36 planes of rows 0..2: distances, the DPP min/max fold */                                  \
    "v_sub_f32 %[t], %[st], %[oA]\n\t"                                                                 \
    "v_mul_f32 %[t], %[t], %[rdA]\n\t"                                                                 \
    /* (the children's counts, for level 2: the two wait states the DPP read needs) */                 \
    "v_readlane_b32 %[cL], %[st], 29\n\t"                                                              \
    "v_readlane_b32 %[cR], %[st], 45\n\t"                                                              \
    "v_min_f32_dpp %[t0a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"             \
    "v_max_f32_dpp %[t1a], %[t], %[t] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"             \
    "s_nop 1\n\t"                                                                                      \
    "v_max_f32_dpp %[m0], %[t0a], %[t0a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"                    \
    "v_min_f32_dpp %[m1], %[t1a], %[t1a] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"                    \
    "s_nop 1\n\t"                                                                                      \
    "v_max_f32_dpp %[m0], %[t0a], %[m0] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"                     \
    "v_min_f32_dpp %[m1], %[t1a], %[m1] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"                     \
    /* lanes 16r+4 / 16r+10: box 0 / box 1 of row r hit (m1 >= m0, m0 < depth, m1 > 0) */             \
    "v_cmp_ge_f32_e64 %[h], %[m1], %[m0]\n\t"                                                          \
    "v_cmp_gt_f32_e64 %[tt], %[depth], %[m0]\n\t"                                                      \
    "s_and_b64 %[h], %[h], %[tt]\n\t"                                                                  \
    "v_cmp_lt_f32_e64 %[tt], 0, %[m1]\n\t"                                                             \
    "s_and_b64 %[h], %[h], %[tt]\n\t"

/* closest hit: lanes 16r+10 of g: m0 of box 0 > m0 of box 1 (blasTrace's dn > df) */
#define SURF_W2_ORDER                                                                                  \
    "v_mov_b32_dpp %[mp], %[m0] row_shr:6 row_mask:0xf bank_mask:0xf\n\t"                              \
    "v_cmp_gt_f32_e64 %[g], %[mp], %[m0]\n\t"

/* level 1 (X's children, row 0): none hit -> pop; b0: both hit (far pushed; 256 =
 * one stack entry, or 0; sb0 its lane mask); c: near child (non-zero: the right) */
#define SURF_W2_L1A                                                                                    \
    "s_and_b64 %[a], %[h], %[m410]\n\t"                                                                \
    "s_cbranch_scc0 L_pop_%=\n\t"                                                                      \
    "s_cmp_eq_u64 %[a], %[m410]\n\t"                                                                   \
    "s_cselect_b32 %[b0], 0x100, 0\n\t"                                                                \
    "s_cselect_b64 %[sb0], -1, 0\n\t"                                                                  \
    "s_cmp_eq_u64 %[a], 0x400\n\t"                                                                     \
    "s_cselect_b32 %[c], 1, 0\n\t"
/* closest hit, both hit: the nearer (swap when m0 of box 0 > m0 of box 1) */
#define SURF_W2_L1ORDER                                                                                \
    "s_bitcmp1_b64 %[g], 10\n\t"                                                                       \
    "s_cselect_b32 %[idx], %[b0], 0\n\t"                                                               \
    "s_or_b32 %[c], %[c], %[idx]\n\t"
/* near child C in row 1 + c; a leaf: push the far child, leave for C; else level 2 (row 1 + c) */
#define SURF_W2_L2A                                                                                    \
    "s_cmp_lg_u32 %[c], 0\n\t"                                                                         \
    "s_cselect_b64 %[sc], -1, 0\n\t"                                                                   \
    "s_cselect_b32 %[cnt], %[cR], %[cL]\n\t"                                                           \
    "s_cselect_b32 %[k16], 32, 16\n\t"                                                                 \
    "s_cmp_lg_u32 %[cnt], 0\n\t"                                                                       \
    "s_cbranch_scc1 L_leafC_%=\n\t"                                                                    \
    "s_lshr_b64 %[tt], %[h], %[k16]\n\t"                                                               \
    "s_and_b64 %[a], %[tt], %[m410]\n\t"                                                               \
    "s_cbranch_scc0 L_miss2_%=\n\t"                                                                    \
    "s_cmp_eq_u64 %[a], %[m410]\n\t"                                                                   \
    "s_cselect_b32 %[b1], 0x100, 0\n\t"                                                                \
    "s_cmp_eq_u64 %[a], 0x400\n\t"                                                                     \
    "s_cselect_b32 %[cc], 1, 0\n\t"
#define SURF_W2_L2ORDER                                                                                \
    "s_lshr_b64 %[tt], %[g], %[k16]\n\t"                                                               \
    "s_bitcmp1_b64 %[tt], 10\n\t"                                                                      \
    "s_cselect_b32 %[idx], %[b1], 0\n\t"                                                               \
    "s_or_b32 %[cc], %[cc], %[idx]\n\t"
/* descend to grandchild n[2c + cc]; push the far child f[1 - c] (b0) and the far
 * grandchild n[2c + 1 - cc] (b1): slot 0 = b0 ? far child : far grandchild,
 * slot 1 = far grandchild, the stack pointer advances by b0 + b1 (bytes of
 * 256-B entries).  SCC on entry: cc != 0 (the last op of L2A / L2ORDER). */
#define SURF_W2_TAIL                                                                                   \
    "s_cselect_b64 %[scc], -1, 0\n\t"                                                                  \
    "s_add_u32 %[b1], %[b1], %[b0]\n\t"                                                                \
    "v_add_u32 %[addr], %[sp], %[stk]\n\t"                                                             \
    "s_waitcnt vmcnt(0)\n\t"                                                                           \
    "v_cndmask_b32_e64 %[ta], %[n0], %[n1], %[scc]\n\t"                                                \
    "v_cndmask_b32_e64 %[tb], %[n2], %[n3], %[scc]\n\t"                                                \
    "v_cndmask_b32_e64 %[m0], %[n1], %[n0], %[scc]\n\t"                                                \
    "v_cndmask_b32_e64 %[m1], %[n3], %[n2], %[scc]\n\t"                                                \
    "v_cndmask_b32_e64 %[st], %[ta], %[tb], %[sc]\n\t"                                                 \
    "v_cndmask_b32_e64 %[mp], %[m0], %[m1], %[sc]\n\t"                                                 \
    "v_cndmask_b32_e64 %[t], %[f1], %[f0], %[sc]\n\t"                                                  \
    "v_cndmask_b32_e64 %[sl0], %[mp], %[t], %[sb0]\n\t"                                                \
    "ds_write2st64_b32 %[addr], %[sl0], %[mp] offset1:1\n\t"                                           \
    "s_add_u32 %[sp], %[sp], %[b1]\n\t"                                                                \
    "s_branch L_chk_%=\n"                                                                              \
    /* C is a leaf: push the far child (when both were hit), leave for C */                            \
    "L_leafC_%=:\n\t"                                                                                  \
    "s_cmp_lg_u32 %[c], 0\n\t"                                                                         \
    "s_cselect_b32 %[lf], %[lfR], %[lfL]\n\t"                                                          \
    "v_add_u32 %[addr], %[sp], %[stk]\n\t"                                                             \
    "s_waitcnt vmcnt(0)\n\t"                                                                           \
    "v_cndmask_b32_e64 %[t], %[f1], %[f0], %[sc]\n\t"                                                  \
    "v_cndmask_b32_e64 %[st], %[f0], %[f1], %[sc]\n\t"   /* W(C): the leaf's triangles */              \
    "s_cmp_eq_u32 %[b0], 0\n\t"                                                                        \
    "s_cbranch_scc1 L_exit_%=\n\t"                                                                     \
    "ds_write_b32 %[addr], %[t]\n\t"                                                                   \
    "s_add_u32 %[sp], %[sp], 256\n\t"                                                                  \
    "s_branch L_exit_%=\n"                                                                             \
    /* both of C's children missed: the reference pushes the far child and pops   \
     * it at once -- visit it (when hit), else pop */                                                  \
    "L_miss2_%=:\n\t"                                                                                  \
    "s_waitcnt vmcnt(0)\n\t"                                                                           \
    "s_cmp_eq_u32 %[b0], 0\n\t"                                                                        \
    "s_cbranch_scc1 L_pop_%=\n\t"                                                                      \
    "v_cndmask_b32_e64 %[st], %[f1], %[f0], %[sc]\n\t"                                                 \
    "s_nop 1\n\t"                                                                                      \
    "s_branch L_chk_%=\n"                                                                              \
    /* pop (every load of the visit has landed) */                                                     \
    "L_pop_%=:\n\t"                                                                                    \
    "s_waitcnt vmcnt(0)\n\t"                                                                           \
    "s_cmp_eq_u32 %[sp], 0\n\t"                                                                        \
    "s_cbranch_scc1 L_done_%=\n\t"                                                                     \
    "s_sub_u32 %[sp], %[sp], 256\n\t"                                                                  \
    "v_add_u32 %[addr], %[sp], %[stk]\n\t"                                                             \
    "ds_read_b32 %[st], %[addr]\n\t"                                                                   \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                         \
    "s_branch L_chk_%=\n"                                                                              \
    "L_done_%=:\n\t"                                                                                   \
    "s_mov_b32 %[cnt], 0\n"                                                                            \
    "L_exit_%=:"

#define SURF_W2_OPERANDS                                                                               \
    : [st] "+v"(st), [sp] "+s"(spb), [nv] "+s"(nv), [lf] "=&s"(lf), [cnt] "=&s"(cnt), [n0] "=&v"(n0), [n1] "=&v"(n1),  \
      [n2] "=&v"(n2), [n3] "=&v"(n3), [f0] "=&v"(f0), [f1] "=&v"(f1), [t] "=&v"(t), [t0a] "=&v"(t0a),    \
      [t1a] "=&v"(t1a), [m0] "=&v"(m0), [m1] "=&v"(m1), [mp] "=&v"(mp), [ta] "=&v"(ta), [tb] "=&v"(tb),  \
      [sl0] "=&v"(sl0), [addr] "=&v"(addr), [lfL] "=&s"(lfL), [lfR] "=&s"(lfR), [o0] "=&s"(o0),          \
      [o2] "=&s"(o2), [of] "=&s"(of), [c] "=&s"(c), [cc] "=&s"(cc), [k16] "=&s"(k16), [idx] "=&s"(idx),   \
      [b0] "=&s"(b0), [b1] "=&s"(b1), [h] "=&s"(h), [tt] "=&s"(tt), [g] "=&s"(g), [a] "=&s"(a),           \
      [sc] "=&s"(sc), [scc] "=&s"(scc), [sb0] "=&s"(sb0), [cL] "=&s"(cL), [cR] "=&s"(cR)                \
    : [oA] "v"(oA), [rdA] "v"(rdA), [depth] "s"(depth), [rsrc] "s"(rsrc), [loff] "v"(laneOff),            \
      [stk] "v"(stkLane), [m410] "s"(m410)                                                               \
    : "memory", "scc"

/* SURF_WALK_PROFILE builds (diagnostics, surf_debug_segment_cycles): cycles and
 * counts of the wave walk's parts, accumulated by lane 0 of a lone wave */
#ifndef SURF_WALK_PROFILE
#define SURF_WALK_PROFILE 0
#endif
__device__ unsigned long long g_walkProf[8];   /* interior cycles, leaf cycles, walks, leaves, triangles, 2-level visits, prologue cycles, instance loop cycles */
__device__ __forceinline__ unsigned long long profClock() {
    __builtin_amdgcn_s_waitcnt(0);
    return __builtin_amdgcn_s_memtime();
}
__device__ __forceinline__ void profAdd(int k, unsigned long long v) {
    if (SURF_WALK_PROFILE && __lane_id() == 0) g_walkProf[k] += v;
}
#if SURF_WALK_PROFILE
#define SURF_W2_VISIT "s_add_u32 %[nv], %[nv], 1\n\t"
#else
#define SURF_W2_VISIT ""
#endif

template <bool ANY>
__device__ __forceinline__ void walk2Fin(float& st, uint32_t& spb, uint32_t& lf, uint32_t& cnt, float oA, float rdA, float depth,
                                         surfI4 rsrc, uint32_t laneOff, uint32_t stkLane, uint32_t& nv) {
    float n0, n1, n2, n3, f0, f1, t, t0a, t1a, m0, m1, mp, ta, tb, sl0;
    uint32_t addr, lfL, lfR, o0, o2, of, c, cc, k16, idx, b0, b1, cL, cR;
    unsigned long long h, tt, g = 0, a, sc, scc, sb0;
    const unsigned long long m410 = 0x410ull;
    if (ANY) {
        /* any-hit: no near/far order (the answer is an OR over the admitted
         * leaves): box 0 first when hit, box 1 pushed when both hit */
        asm volatile(SURF_W2_HEAD SURF_W2_L1A SURF_W2_L2A SURF_W2_TAIL SURF_W2_OPERANDS);
    } else {
        asm volatile(SURF_W2_HEAD SURF_W2_ORDER SURF_W2_L1A SURF_W2_L1ORDER SURF_W2_L2A SURF_W2_L2ORDER SURF_W2_TAIL
                     SURF_W2_OPERANDS);
    }
}

/* A leaf of <= 3 triangles whose two-level record W(leaf) holds them (row j:
 * lanes 0..2 v0, 3..5 e1, 6..8 e2, 9 prim -- surf_upload_scene), in st: every
 * lane of row j takes triangle j's components by DPP row_newbcast, tests it
 * (triHitFlat), and the hits are accepted in index order as leafWave does --
 * with no memory trip: the record came with the visit's candidate loads. */
template <int L>
__device__ __forceinline__ float rowBcast(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + L, 0xF, 0xF, false));
}
template <bool ANY>
__device__ __forceinline__ bool leafWaveW(float st, uint32_t cnt, V3 o, V3 d, float& depth, float& hu, float& hv, uint32_t& hprim) {
    const uint32_t row = __lane_id() >> 4;
    const V3 v0 = mk3(rowBcast<0>(st), rowBcast<1>(st), rowBcast<2>(st));
    const V3 e1 = mk3(rowBcast<3>(st), rowBcast<4>(st), rowBcast<5>(st));
    const V3 e2 = mk3(rowBcast<6>(st), rowBcast<7>(st), rowBcast<8>(st));
    const uint32_t prim = f2u(rowBcast<9>(st));
    float t = depth, u = 0.0f, v = 0.0f;
    const bool h = row < cnt && triHitFlat(v0, e1, e2, o, d, depth, t, u, v);
    unsigned long long m = __ballot(h) & 0x0000000100010001ull;   /* lane 16 j: triangle j hit */
    if (ANY) return m != 0ull;
    bool any = false;
    while (m) {
        const int j = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const float tj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), j));
        if (tj < depth) {
            depth = tj;
            hu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), j));
            hv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
            hprim = (uint32_t)__builtin_amdgcn_readlane((int)prim, j);
            any = true;
        }
    }
    return any;
}
constexpr uint32_t kLeafInW = 3;     /* triangles a two-level leaf record holds */

/* blasWalk with two-level visits (S.wnodes): the DFS below one BLAS root from
 * W(root) -- its first visit re-tests the root's children at the current
 * depth (the caller's entry test gave the same answer) and their children. */
template <bool ANY>
__device__ __forceinline__ bool blasWalk2(const DevScene& S, uint32_t nodeOff, const float4* tri, V3 o, V3 d, V3 rd, float& depth,
                                          float& hu, float& hv, uint32_t& hprim, float* rs) {
    const uint32_t lane = __lane_id(), l16 = lane & 15u;
    const uint32_t ax = l16 < 12u ? (l16 % 6u) >> 1 : 0u;
    const float oA = pick3(o, ax), rdA = pick3(rd, ax);
    const float* wb = S.wnodes + 48u * (size_t)nodeOff;                 /* this BLAS's W records */
    const uintptr_t nb = reinterpret_cast<uintptr_t>(wb);
    const surfI4 rsrc = {(int)(uint32_t)nb, (int)(uint32_t)(nb >> 32), (int)((S.nWnodes - nodeOff) * 192u), 0x00020000};
    const uint32_t laneOff = 4u * lane;
    const uint32_t stkLane = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)rs) + 4u * lane;
    float st = loadEarly(wb + lane);                                     /* W(root) */
    waitLoads(st);
    uint32_t sp = 0u;
    bool any = false;
    uint32_t nv = 0u;
    if (SURF_WALK_PROFILE) profAdd(2, 1);
    for (;;) {
        uint32_t lf, cnt;
        const float dS = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(depth)));   /* wave-uniform */
        unsigned long long tA = 0;
        if (SURF_WALK_PROFILE) tA = profClock();
        walk2Fin<ANY>(st, sp, lf, cnt, oA, rdA, dS, rsrc, laneOff, stkLane, nv);
        if (SURF_WALK_PROFILE) { const unsigned long long tB = profClock(); profAdd(0, tB - tA); tA = tB; }
        if (cnt == 0u) { if (SURF_WALK_PROFILE) profAdd(5, nv); return any; }
        const bool lh = cnt <= kLeafInW ? leafWaveW<ANY>(st, cnt, o, d, depth, hu, hv, hprim)
                                         : leafWave<ANY>(tri, lf, cnt, o, d, depth, hu, hv, hprim);
        if (SURF_WALK_PROFILE) { profAdd(1, profClock() - tA); profAdd(3, 1); profAdd(4, cnt); }
        if (lh) {
            if (ANY) { if (SURF_WALK_PROFILE) profAdd(5, nv); return true; }
            any = true;
        }
        if (sp == 0u) { if (SURF_WALK_PROFILE) profAdd(5, nv); return any; }
        sp -= 256u;
        st = rs[sp / 4u + lane];
    }
}

/* LDS prologue table of the wave traversal: 16 floats per instance */
__device__ __forceinline__ uint32_t proWords(const DevScene& S) { return 16u * S.nInst; }

/* Prologue entry of one instance (lane-parallel: one instance per lane): its
 * object-space ray, 1/d, the slab ranges of its BLAS root's two children and
 * the range of its conservative world box (the lane traversal's instance
 * cull, traceScene; the full line when unusable), as blasWave forms them.
 * None of it depends on depth: the depth tests are applied at the instance's
 * turn.  Returns whether the instance can still yield a hit at `depth`. */
__device__ __forceinline__ bool waveProEntry(const TraceInst& I, V3 o, V3 d, V3 rdw, bool cullOk, float depth, float4* p) {
    float w0 = -kFarAway, w1 = kFarAway;
    if (cullOk && I.wlo.w != 0.0f) {
        const float tx0 = (I.wlo.x - o.x) * rdw.x, tx1 = (I.whi.x - o.x) * rdw.x;
        const float ty0 = (I.wlo.y - o.y) * rdw.y, ty1 = (I.whi.y - o.y) * rdw.y;
        const float tz0 = (I.wlo.z - o.z) * rdw.z, tz1 = (I.whi.z - o.z) * rdw.z;
        w0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
        w1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    }
    V3 oo = mk3(rowDot(I.m0, o.x, o.y, o.z, 1.0f), rowDot(I.m1, o.x, o.y, o.z, 1.0f), rowDot(I.m2, o.x, o.y, o.z, 1.0f));
    if (!I.meta.z) oo = divs(oo, rowDot(I.m3, o.x, o.y, o.z, 1.0f));
    const V3 dd = mk3(rowDot(I.m0, d.x, d.y, d.z, 0.0f), rowDot(I.m1, d.x, d.y, d.z, 0.0f), rowDot(I.m2, d.x, d.y, d.z, 0.0f));
    const V3 rd = mk3(1.0f / dd.x, 1.0f / dd.y, 1.0f / dd.z);
    float a0, a1, b0, b1;
    slabRange(I.r0, I.r1, oo, rd, a0, a1);
    slabRange(I.r2, I.r3, oo, rd, b0, b1);
    p[0] = make_float4(oo.x, oo.y, oo.z, a0);
    p[1] = make_float4(dd.x, dd.y, dd.z, a1);
    p[2] = make_float4(rd.x, rd.y, rd.z, b0);
    p[3] = make_float4(b1, w0, w1, 0.0f);
    /* a root child that misses at this depth misses at every later (smaller)
     * depth too; root leaves are always taken */
    const bool wMiss = w1 < w0 || w1 < 0.0f || w0 >= depth;
    return !wMiss && (f2u(I.r1.w) != 0u || slabHit(a0, a1, depth) != kFarAway || slabHit(b0, b1, depth) != kFarAway);
}

/* The one-level walk (no two-level records, or a non-finite ray / box). */
template <bool ANY>
__device__ __forceinline__ bool blasWalkFallback(const DevScene& S, uint32_t nodeOff, const float4* tri, V3 o, V3 d, V3 rd, float dn, float df,
                                              uint32_t cn, uint32_t cf, float& depth, float& hu, float& hv, uint32_t& hprim, float* rs,
                                              SegStats* ss, bool fin) {
    return fin ? blasWalk<ANY, true>(S, nodeOff, tri, o, d, rd, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss)
               : blasWalk<ANY, false>(S, nodeOff, tri, o, d, rd, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss);
}

/* Instance::intersect(Any) (bvh.cpp:481-513) of one instance at its turn, from
 * its prologue entry pk (LDS, one address for the wave: a broadcast): the
 * world-box cull and the root children's depth tests at the current depth,
 * then the BLAS walk (or the root leaf's triangles). */
template <bool ANY, bool W2 = false>
__device__ __forceinline__ bool waveInstance(const DevScene& S, const TraceInst& I, const float4* pk, float& depth, float& hu,
                                             float& hv, uint32_t& hprim, float* rs, SegStats* ss) {
    /* wave-uniform (the tables may be read through a generic pointer: LDS or global) */
    const uint32_t nodeOff = (uint32_t)__builtin_amdgcn_readfirstlane((int)I.meta.x);
    const float4* tri = S.tris + 3u * (uint32_t)__builtin_amdgcn_readfirstlane((int)I.meta.y);
    const uint32_t rlf = (uint32_t)__builtin_amdgcn_readfirstlane((int)f2u(I.r0.w));
    const uint32_t rcnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)f2u(I.r1.w));
    const float4 q0 = pk[0], q1 = pk[1], q2 = pk[2], q3 = pk[3];
    if (q3.z < q3.y || q3.z < 0.0f || q3.y >= depth) return false;   /* world-box cull at the current depth */
    const V3 ok = xyz(q0);
    const V3 dk = xyz(q1);
    if (rcnt != 0u) return leafWave<ANY>(tri, rlf, rcnt, ok, dk, depth, hu, hv, hprim);
    /* root: never box-tested (bvh.cpp:131); its children's boxes are in its record */
    float dn = slabHit(q0.w, q1.w, depth);
    float df = slabHit(q2.w, q3.x, depth);
    uint32_t cn = nodeOff + rlf, cf = cn + 1u;
    if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
    if (dn == kFarAway) return false;
    const V3 rk = xyz(q2);
    const bool fin = S.finiteBoxes && finite3(ok) && finite3(rk);
    if (W2) {
        /* kernels built for two-level records carry no one-level asm walk (its
         * registers and code): a non-finite ray takes the C++ walk */
        if (fin) return blasWalk2<ANY>(S, nodeOff, tri, ok, dk, rk, depth, hu, hv, hprim, rs);
        return blasWalk<ANY, false>(S, nodeOff, tri, ok, dk, rk, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss);
    }
    return blasWalkFallback<ANY>(S, nodeOff, tri, ok, dk, rk, dn, df, cn, cf, depth, hu, hv, hprim, rs, ss, fin);
}

/* BvhTLAS::intersect / intersectAny (bvh.cpp:654-778) for any TLAS: the
 * prologue entries of every instance first (64 lanes at a time, by instance
 * id), then the reference's TLAS DFS on the wave -- the node record's 12
 * planes in lanes (slabPair: the ternary min/max in its operand order), near
 * child first, the far child pushed when hit (a stack of node indices, entry
 * k in lane k of one VGPR), a leaf's instances in index order, each at its
 * turn with the depth the earlier ones left (waveInstance). */
template <bool ANY, bool W2 = false>
__device__ __forceinline__ bool traceWaveTlas(const DevScene& S, const TraceTables& Tt, V3 o, V3 d, float& depth, float& hu,
                                              float& hv, uint32_t& hinst, uint32_t& hprim, float* rs, float4* pro, SegStats* ss) {
    const uint32_t lane = __lane_id();
    const V3 rdw = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const bool cullOk = finite3(o) && finite3(rdw);
    for (uint32_t b = 0; b < S.nInst; b += 64u)
        if (b + lane < S.nInst) (void)waveProEntry(Tt.inst[b + lane], o, d, rdw, cullOk, depth, pro + 4u * (b + lane));
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);              /* the entries are in LDS before any lane reads another's */
    const float* nodesF = reinterpret_cast<const float*>(S.tlasNodes);
    const uint32_t dw = planeDword(lane), ax = lane < 12u ? (lane % 6u) >> 1 : 0u;
    const float oA = pick3(o, ax), rdA = pick3(rdw, ax);
    bool any = false;
    uint32_t node = 0u, tsp = 0u;
    int tstk = 0;                                     /* TLAS stack: entry k in lane k */
    for (;;) {
        const float rec = nodesF[16u * node + dw];
        const uint32_t lf = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(rec), 12);
        const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(rec), 13);
        if (cnt != 0u) {
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t ii = Tt.order[lf + k];
                if (waveInstance<ANY, W2>(S, Tt.inst[ii], pro + 4u * ii, depth, hu, hv, hprim, rs, ss)) {
                    if (ANY) return true;
                    any = true;
                    hinst = ii;
                }
            }
            if (tsp == 0u) break;
            node = (uint32_t)__builtin_amdgcn_readlane(tstk, (int)--tsp);
            continue;
        }
        float dn, df;
        slabPair(rec, oA, rdA, depth, dn, df);
        uint32_t cn = lf, cf = lf + 1u;
        if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
        if (dn == kFarAway) {
            if (tsp == 0u) break;
            node = (uint32_t)__builtin_amdgcn_readlane(tstk, (int)--tsp);
        } else {
            node = cn;
            if (df != kFarAway) {
                if (lane == tsp) tstk = (int)cf;
                ++tsp;
            }
        }
    }
    return any;
}

/* BvhTLAS::intersect / intersectAny on the wave (bvh.cpp:654-778).  A
 * single-leaf TLAS of <= 64 instances (the bundled scene) takes the fast
 * path: lane k forms the prologue entry of the k-th instance in TLAS order,
 * the instances whose entry can still hit are taken in that order, each
 * applying the depth tests at its turn (a missed instance costs a few
 * readlanes instead of a serial transform, three divisions and a slab test).
 * Any other TLAS: traceWaveTlas. */
template <bool ANY, bool W2 = false>
__device__ __forceinline__ bool traceWave(const DevScene& S, const TraceTables& Tt, V3 o, V3 d, float& depth, float& hu,
                                          float& hv, uint32_t& hinst, uint32_t& hprim, float* rs, float4* pro, SegStats* ss = nullptr) {
    bool any = false;
    const uint32_t nI = S.tlasLeafCount;
    if (nI == 0u || nI > 64u) return traceWaveTlas<ANY, W2>(S, Tt, o, d, depth, hu, hv, hinst, hprim, rs, pro, ss);
#if SURF_SEG_TIMING
    unsigned long long t0 = segClock();
#endif
    const uint32_t lane = __lane_id();
    /* lane k: the k-th instance's entry, kept in the LDS prologue table (not
     * in registers through the walk); root-leaf instances (the room's walls)
     * are culled by their world box too, which otherwise cost a triangle test
     * and its loads every segment */
    const V3 rdw = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const bool cullOk = finite3(o) && finite3(rdw);
    unsigned long long tP = 0;
    if (SURF_WALK_PROFILE) tP = profClock();
    bool keep = false;
    if (lane < nI) keep = waveProEntry(Tt.inst[Tt.order[lane]], o, d, rdw, cullOk, depth, pro + 4u * lane);
    unsigned long long cand = __ballot(keep);
    if (SURF_WALK_PROFILE) { const unsigned long long t = profClock(); profAdd(6, t - tP); tP = t; }
    while (cand) {
        const uint32_t k = (uint32_t)(__ffsll((long long)cand) - 1);
        cand &= cand - 1ull;
        const uint32_t ii = Tt.order[k];
#if SURF_SEG_TIMING
        if (ss) { const unsigned long long t1 = segClock(); ss->cycInst += t1 - t0; t0 = t1; }
#endif
        const bool h = waveInstance<ANY, W2>(S, Tt.inst[ii], pro + 4u * k, depth, hu, hv, hprim, rs, ss);
#if SURF_SEG_TIMING
        if (ss) { const unsigned long long t1 = segClock(); ss->cycLoop += t1 - t0; t0 = t1; }
#endif
        if (h) {
            if (ANY) return true;
            any = true;
            hinst = ii;
        }
    }
#if SURF_SEG_TIMING
    if (ss) ss->cycInst += segClock() - t0;
#endif
    if (SURF_WALK_PROFILE) profAdd(7, profClock() - tP);
    return any;
}

/* --------------------------------------------------------------- wave helpers */
__device__ __forceinline__ uint32_t laneId() { return __lane_id(); }
__device__ __forceinline__ uint32_t rankBelow(unsigned long long mask) {
    return (uint32_t)__popcll(mask & ((1ull << laneId()) - 1ull));
}
/* One atomic per wave reserves `popc(mask)` slots; returns this lane's slot. */
__device__ __forceinline__ uint32_t waveAppend(uint32_t* counter, unsigned long long mask) {
    uint32_t base = 0;
    if (laneId() == 0 && mask) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = (uint32_t)__shfl((int)base, 0);
    return base + rankBelow(mask);
}
__device__ __forceinline__ void waveCount(unsigned long long* ctr, unsigned long long v) {
    if (laneId() == 0 && v) atomicAdd(ctr, v);
}

/* Block-level event counts: one atomic per counter per workgroup (the counters
 * are hot addresses shared by every wave of the launch).  vals are wave-uniform;
 * every thread of the block must call this. */
template <int N, int BLK = kBlock>   /* BLK: the largest workgroup the caller runs */
__device__ __forceinline__ void blockCount(Counters* C, const int (&idx)[N], const unsigned long long (&vals)[N]) {
    unsigned long long* ev = C->evS[blockIdx.x % kStripes];
    __shared__ unsigned long long sEv[N][BLK / 64];
    const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (laneId() == 0)
        for (int k = 0; k < N; ++k) sEv[k][w] = vals[k];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            unsigned long long t = 0;
            for (uint32_t j = 0; j < nw; ++j) t += sEv[k][j];
            if (t) atomicAdd(&ev[idx[k]], t);
        }
    }
}

/* ------------------------------------------------------------- ray order
 * Each phase's pool is traced in the order of a 4-bit key: the instance the
 * ray starts on (the one its path just hit; camera rays have their own bin).
 * Rays that start on the same surface enter the same BVHs, so a wave's
 * wave-uniform instance loop walks fewer instances: 1 M recorded extension
 * rays take 635 us shuffled, 355 us grouped by start instance (round 1;
 * DESIGN.md 4 "Ray order"; the probe script, tools/order_probe.py, was retired
 * in round 3 -- commit 5a920ae still holds it).  A counting sort of 4-byte indices per phase
 * (count, scan, scatter; ~2 us of kernels per 100 k paths) feeds k_extend and
 * k_shade through order[]; hit records stay in order i, so the paths, their
 * results and the append order of the next pool are unchanged in content --
 * only the interleaving of lanes changes. */
constexpr uint32_t kBins = 64;
constexpr uint32_t kSortBlocks = 256;
constexpr uint32_t kSortUnroll = 16;   /* keys per thread in flight in k_bincount / k_binscatter */
/* threads per k_bincount / k_binscatter / k_regen_count block: 256 -- four
 * waves, which find room beside the concurrent k_connect where a 1024-thread
 * workgroup (16 waves on one CU) waits for a CU to empty (MEASUREMENTS r6) */
#ifndef SURF_SORT_THREADS
#define SURF_SORT_THREADS 256
#endif
constexpr uint32_t kSortThreads = SURF_SORT_THREADS;
#ifndef SURF_SORT_FUSED_SCAN
#define SURF_SORT_FUSED_SCAN 1          /* k_binscatter scans the counts itself (no k_binscan launch) */
#endif
static_assert(kBins <= 256u, "pool/shadow keys are one byte");

/* Which of the heavy instances' world boxes the ray's line meets in [0, tmax)
 * (bit h for S.hvLo/hvHi[h]).  A sort key only -- approximate reciprocals and
 * any NaN outcome are fine: the order of traversal changes no ray's result. */
__device__ __forceinline__ uint32_t heavyMask(const DevScene& S, float4 o, float4 d, float tmax) {
    const float rx = __builtin_amdgcn_rcpf(d.x), ry = __builtin_amdgcn_rcpf(d.y), rz = __builtin_amdgcn_rcpf(d.z);
    uint32_t m = 0;
    for (uint32_t h = 0; h < S.nHeavy; ++h) {
        const float4 lo = S.hvLo[h], hi = S.hvHi[h];
        const float tx0 = (lo.x - o.x) * rx, tx1 = (hi.x - o.x) * rx;
        const float ty0 = (lo.y - o.y) * ry, ty1 = (hi.y - o.y) * ry;
        const float tz0 = (lo.z - o.z) * rz, tz1 = (hi.z - o.z) * rz;
        const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
        const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
        m |= (t1 >= t0 && t1 > 0.0f && t0 < tmax) ? (1u << h) : 0u;
    }
    return m;
}

/* Pool order key.  Default (single-leaf TLAS with heavy instances): which of
 * the heavy BLASes the ray's line reaches x the x/z quadrant of its origin, so
 * a wave's lanes enter the same expensive BVHs -- the wave-uniform instance
 * loop pays, per instance, its slowest lane in it (recorded C3 extension rays,
 * lock-step visit steps per 64 rays, tools/lockstep_sim.cpp: 53.8 by start
 * instance x quadrant, 37.7 by heavy-instance mask).  keyMode 2 (default)
 * orders the masks descending: the rays that reach the most heavy BLASes --
 * the costliest -- come first in the order, so k_extend's first-dispatched
 * workgroups take them and its last-dispatched ones the cheap ones (longest
 * jobs first).  In ascending order (keyMode 1) the costly bins sat at the end
 * of the grid's first pass, on the last-dispatched workgroups, unless enough
 * of them spilled into the grid-stride second pass (which the first workgroups
 * run): k_extend 119 -> 166 ms per C3 render between a 5- and a 4.5-frame pool
 * at the same grid, 117 -> 150 ms at 56 workgroups per CU; heavy-first: 119
 * and 117 (profiles/r4_experiments/cliff).  Otherwise the instance the path
 * starts on (<= 14; camera rays: kBins - 1) x the quadrant: 1 M recorded
 * extension rays (round 2, DESIGN 4 "Ray order"): 634 us shuffled, 345 by
 * start instance, 334 by start x quadrant. */
__device__ __forceinline__ uint8_t poolKey(const DevScene& S, uint32_t inst, float4 o, float4 d) {
    const uint32_t cx = (o.x - S.cellLo[0]) * S.cellScale[0] >= 1.0f ? 1u : 0u;
    const uint32_t cz = (o.z - S.cellLo[2]) * S.cellScale[2] >= 1.0f ? 1u : 0u;
    if (S.keyMode == 2u) return (uint8_t)((7u - heavyMask(S, o, d, kFarAway)) * 4u + cx + 2u * cz);
    if (S.keyMode) return (uint8_t)(heavyMask(S, o, d, kFarAway) * 4u + cx + 2u * cz);
    return (uint8_t)((inst < 14u ? inst : 14u) * 4u + cx + 2u * cz);
}

/* Shadow-ray order key: light slot (mod 2) x the octant cell of the scene box
 * holding the ray's origin.  1 M recorded shadow rays (round 2; the retired
 * tools/order_probe2.py, last in commit 5a920ae):
 * 340 us shuffled, 277 sorted by light, 238 by light x octant cell, 286 by
 * light x 4x4x4 cells (too fine: the bins stop sharing paths through the BVH).
 * The pool's heavy-instance mask (of the segment [0, tmax)) x light x x/z
 * quadrant was measured slower: k_connect 147 -> 174 ms per C3 render. */
__device__ __forceinline__ uint8_t shadowKey(const DevScene& S, uint32_t light, float4 o) {
    uint32_t cell = 0;
    const float p[3] = {o.x, o.y, o.z};
#pragma unroll
    for (int a = 0; a < 3; ++a)
        cell |= ((p[a] - S.cellLo[a]) * S.cellScale[a] >= 1.0f ? 1u : 0u) << a;
    return (uint8_t)((light & 1u) * 8u + cell);
}

/* Rays to order: which = 0 the pool read by phase par, 1 its shadow queue. */
__device__ __forceinline__ uint32_t sortCount(const Counters* C, int par, int which) {
    return which ? 0u : C->nIn[par];   /* (the shadow queue needs no sort: k_shade appends it in bin order) */
}
__device__ __forceinline__ void sortChunk(uint32_t n, uint32_t& a, uint32_t& b) {
    const uint32_t c = (n + gridDim.x - 1u) / gridDim.x;
    a = min(n, blockIdx.x * c);
    b = min(n, a + c);
}

__global__ __launch_bounds__(kSortThreads) void k_bincount(const uint8_t* __restrict__ key, const Counters* C, int par, int which,
                                                     uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kBins];
    if (threadIdx.x < kBins) h[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t a, b;
    sortChunk(sortCount(C, par, which), a, b);
    /* kSortUnroll key loads in flight per thread before their atomics (one
     * wave per SIMD: a rolled loop waited on each load in turn); same atomic
     * order as the rolled loop */
    uint32_t i = a + threadIdx.x;
    for (; i + (kSortUnroll - 1u) * blockDim.x < b; i += kSortUnroll * blockDim.x) {
        uint32_t k[kSortUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kSortUnroll; ++u) k[u] = key[i + u * blockDim.x];
#pragma unroll
        for (uint32_t u = 0; u < kSortUnroll; ++u) atomicAdd(&h[k[u]], 1u);
    }
    for (; i < b; i += blockDim.x) atomicAdd(&h[key[i]], 1u);
    __syncthreads();
    if (threadIdx.x < kBins) hist[threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

/* Exclusive scan of the bin-major [kBins][blocks] counts: one block of 1024. */
__global__ __launch_bounds__(1024) void k_binscan(uint32_t* __restrict__ hist, uint32_t total) {
    constexpr uint32_t kPer = kBins * kSortBlocks / 1024u;    /* counts per thread (the host passes total = kBins x blocks) */
    static_assert(kBins * kSortBlocks % 1024u == 0u, "scan layout");
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, a = t * kPer;
    (void)total;
    /* all kPer loads in flight at once (a rolled loop waited for each in turn: 20 us per launch) */
    uint32_t c[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) c[k] = hist[a + k];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) sum += c[k];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) { hist[a + k] = run; run += c[k]; }
}

__global__ __launch_bounds__(kSortThreads) void k_binscatter(const uint8_t* __restrict__ key, const Counters* C, int par, int which,
                                                       const uint32_t* __restrict__ hist, uint32_t* __restrict__ order) {
    __shared__ uint32_t base[kBins];
#if SURF_SORT_FUSED_SCAN
    /* this block's start in every bin, from the raw bin-major [kBins][blocks]
     * counts (no separate scan launch): kLanes consecutive lanes per bin sum
     * the bin's count over all blocks and over the blocks before this one,
     * then one wave scans the bin totals */
    {
        constexpr uint32_t kLanes = kSortThreads / kBins, kPer = kSortBlocks / kLanes;
        static_assert(kSortThreads % kBins == 0u && kSortBlocks % kLanes == 0u && kLanes <= 64u, "scan layout");
        __shared__ uint32_t tot[kBins];
        const uint32_t bin = threadIdx.x / kLanes, sub = threadIdx.x % kLanes;
        const uint32_t* row = hist + bin * kSortBlocks + sub * kPer;
        uint32_t c[kPer];
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) c[u] = row[u];
        uint32_t all = 0, below = 0;
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
            all += c[u];
            below += sub * kPer + u < blockIdx.x ? c[u] : 0u;
        }
#pragma unroll
        for (uint32_t off = 1; off < kLanes; off <<= 1) {
            all += __shfl_xor(all, off, kLanes);
            below += __shfl_xor(below, off, kLanes);
        }
        if (sub == 0u) { tot[bin] = all; base[bin] = below; }
        __syncthreads();
        if (threadIdx.x < kBins) {
            const uint32_t v = tot[threadIdx.x];
            uint32_t inc = v;
#pragma unroll
            for (uint32_t off = 1; off < kBins; off <<= 1) {
                const uint32_t t = __shfl_up(inc, off, kBins);
                if (threadIdx.x >= off) inc += t;
            }
            base[threadIdx.x] += inc - v;
        }
    }
#else
    if (threadIdx.x < kBins) base[threadIdx.x] = hist[threadIdx.x * gridDim.x + blockIdx.x];
#endif
    __syncthreads();
    uint32_t a, b;
    sortChunk(sortCount(C, par, which), a, b);
    uint32_t i = a + threadIdx.x;
    for (; i + (kSortUnroll - 1u) * blockDim.x < b; i += kSortUnroll * blockDim.x) {
        uint32_t k[kSortUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kSortUnroll; ++u) k[u] = key[i + u * blockDim.x];
#pragma unroll
        for (uint32_t u = 0; u < kSortUnroll; ++u) order[atomicAdd(&base[k[u]], 1u)] = i + u * blockDim.x;
    }
    for (; i < b; i += blockDim.x) order[atomicAdd(&base[key[i]], 1u)] = i;
}

/* ------------------------------------------------------------------ kernels */
/* SK: the traversal stack's entry type -- 16-bit when every BLAS and TLAS
 * node index fits (half the stack's LDS: more resident workgroups) */
constexpr uint32_t kResumeHead = 10;   /* words of a resume record before its stack refs (64 words in all) */
/* CAP (single-leaf TLAS): a lane leaves a ray after capIters node visits of
 * one BLAS walk (W-record visits in the two-level walk; LaneCap) and writes
 * its resume record (64 words: slot i, pool index j, TLAS turn, next node,
 * stack depth, depth, u, v, prim, instance, then the stack's entries bottom
 * first); k_extend_cont finishes those rays and writes their hit records. */
#ifndef SURF_TRACE_WAVES_CAP
#define SURF_TRACE_WAVES_CAP SURF_TRACE_WAVES_EXT
#endif
template <bool LDS, bool LW = false, typename SK = uint32_t, bool CAP = false>
__global__ __launch_bounds__(kBlock, LW ? SURF_TRACE_WAVES : (CAP ? SURF_TRACE_WAVES_CAP : SURF_TRACE_WAVES_EXT)) void k_extend(DevScene S, Pool cur, float4* __restrict__ hitTUV,
                                                   uint32_t* __restrict__ hitInst, const Counters* C, int par, uint32_t stackWords,
                                                   const uint32_t* __restrict__ order, uint32_t capIters, uint32_t* __restrict__ resumeRec,
                                                   uint32_t resumeCap) {
    extern __shared__ uint32_t lds[];
    const uint32_t n = C->nIn[par];
    /* blocks past the pool exit before staging: a small pool (the drain) costs
     * what it traces, not the fixed grid's LDS staging */
    if (blockIdx.x * blockDim.x >= n) return;
    /* (stackWords: 32-bit words of the stack; a 16-bit stack uses half of them) */
    const TraceTables Tt = traceTables<LDS>(S, lds, sizeof(SK) == 2 ? (stackWords + 1u) / 2u : stackWords);
    const uint32_t stride = blockDim.x;
    SK* stk = reinterpret_cast<SK*>(lds) + threadIdx.x;
    LaneCap lc;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t j = order ? order[i] : i;       /* ray order: hit records stay in order i */
        const float4 o = ldS(&cur.od[2u * (j)]), d = ldS(&cur.od[2u * (j) + 1u]);
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
        if (CAP) { lc.left = capIters; lc.capped = false; }
        const bool hit = traceScene<false, LW, false, SK, CAP>(S, Tt, xyz(o), xyz(d), depth, u, v, inst, prim, stk, stride, nullptr,
                                                               CAP ? &lc : nullptr);
        /* (the records hold a whole pool: every lane that stops has one) */
        uint32_t slot = 0u;
        if (CAP) {   /* one atomic per wave, by its first active lane (lanes past the pool have left the loop) */
            const unsigned long long m = __ballot(lc.capped);
            const int lead = __ffsll((long long)__ballot(true)) - 1;
            uint32_t base = 0u;
            if ((int)__lane_id() == lead && m) base = atomicAdd(&const_cast<Counters*>(C)->resumeN[par], (uint32_t)__popcll(m));
            slot = (uint32_t)__shfl((int)base, lead) + rankBelow(m);
        }
        if (CAP && lc.capped) {
            uint32_t* r = resumeRec + 64u * (size_t)slot;
            r[0] = i; r[1] = j; r[2] = lc.turn; r[3] = lc.ref; r[4] = lc.depthN;
            r[5] = f2u(depth); r[6] = f2u(u); r[7] = f2u(v); r[8] = prim; r[9] = inst;
            for (uint32_t e = 0; e < lc.depthN; ++e) r[kResumeHead + e] = (uint32_t)stk[e * stride];
            continue;
        }
        stS(&hitTUV[i], make_float4(depth, u, v, u2f(prim)));
        stSu(&hitInst[i], hit ? inst : kUnset);
    }
}

/* The second pass of the capped lane walk (LaneCap): each lane takes one
 * resume record of this phase, puts the capped lane's stack into its own LDS
 * column and continues that walk (traceScene RES) -- the rays that outlived
 * the cap, 64 to a wave again -- then writes the hit record k_extend would
 * have written.  Same traversal code and decisions: exact. */
template <bool LDS, bool LW, typename SK>
__global__ __launch_bounds__(kBlock, SURF_TRACE_WAVES) void k_extend_cont(DevScene S, Pool cur, float4* __restrict__ hitTUV,
                                                                         uint32_t* __restrict__ hitInst, const Counters* C, int par,
                                                                         uint32_t stackWords, const uint32_t* __restrict__ rec,
                                                                         uint32_t recCap) {
    extern __shared__ uint32_t lds[];
    const uint32_t n = min(C->resumeN[par], recCap);
    if (blockIdx.x * blockDim.x >= n) return;
    const TraceTables Tt = traceTables<LDS>(S, lds, sizeof(SK) == 2 ? (stackWords + 1u) / 2u : stackWords);
    const uint32_t stride = blockDim.x;
    SK* stk = reinterpret_cast<SK*>(lds) + threadIdx.x;
    uint32_t done = 0u;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x, ++done) {
        const uint32_t* r = rec + 64u * (size_t)q;
        const uint32_t i = r[0], j = r[1];
        LaneCap lc;
        lc.turn = r[2]; lc.ref = r[3]; lc.depthN = r[4];
        float depth = u2f(r[5]), u = u2f(r[6]), v = u2f(r[7]);
        uint32_t prim = r[8], inst = r[9];
        for (uint32_t e = 0; e < lc.depthN; ++e) stk[e * stride] = (SK)r[kResumeHead + e];
        const float4 o = ldS(&cur.od[2u * j]), d = ldS(&cur.od[2u * j + 1u]);
        const bool hit = traceScene<false, LW, false, SK, false, true>(S, Tt, xyz(o), xyz(d), depth, u, v, inst, prim, stk, stride,
                                                                    nullptr, &lc, inst != kUnset);
        stS(&hitTUV[i], make_float4(depth, u, v, u2f(prim)));
        stSu(&hitInst[i], hit ? inst : kUnset);
    }
    if (done) atomicAdd(&const_cast<Counters*>(C)->evS[blockIdx.x % kStripes][9], (unsigned long long)done);
}

/* randomOnHemisphereCosineWeighted, surf_math.cpp:116-134 (retry loop for R.N == 0) */
/* One try of the loop body (two draws); false when R.N == 0 (retry). */
__device__ __forceinline__ bool cosineTry(uint32_t& seed, V3 n, V3& out) {
    const float r0 = rndF(seed), r1 = rndF(seed);
    const float r = sqrtf(r0);
    const float theta = k2Pi * r1;
    float sn, cs;
    gSinCosf(theta, sn, cs);
    const V3 dir = mk3(r * cs, r * sn, sqrtf(1.0f - r0));
    const float xMax = 1.0f - kEps;
    const V3 tmp = (fabsf(n.x) > xMax) ? mk3(0.0f, 1.0f, 0.0f) : mk3(1.0f, 0.0f, 0.0f);
    const V3 B = normalize(cross(n, tmp));
    const V3 T = cross(B, n);
    out = add(add(lscl(dir.x, T), lscl(dir.y, B)), lscl(dir.z, n));
    return !(dot(out, n) == 0.0f);
}
__device__ __forceinline__ V3 cosineSample(uint32_t& seed, V3 n) {
    V3 out;
    while (!cosineTry(seed, n, out)) {}
    return out;
}

__device__ __forceinline__ void addRadiance(float4* rad, uint32_t sid, V3 c) {
    float4 r = rad[sid];
    r.x = r.x + c.x; r.y = r.y + c.y; r.z = r.z + c.z;
    rad[sid] = r;
}
/* The drain kernels keep the radiance of the sample they run in registers:
 * loaded once when the path is taken (what the wavefront phases added before
 * the hand-over), each contribution added in the reference's order
 * (renderer.cpp:415-444, the same float adds addRadiance makes), stored once
 * when the sample ends or leaves the kernel -- instead of a dependent global
 * read-modify-write on the path's chain every segment. */
__device__ __forceinline__ V3 loadRadiance(const float4* rad, uint32_t sid) { return xyz(rad[sid]); }
__device__ __forceinline__ void storeRadiance(float4* rad, uint32_t sid, V3 e) { rad[sid] = make_float4(e.x, e.y, e.z, 0.0f); }
/* One-path-per-wave kernels: the running sum is wave-uniform; kept in SGPRs
 * (readfirstlane after each add) so it costs no VGPRs across the walks. */
__device__ __forceinline__ float sgprF(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ V3 addU(V3 e, V3 c) {
    const V3 t = add(e, c);
    return mk3(sgprF(t.x), sgprF(t.y), sgprF(t.z));
}

/* Result of shading one hit: what the path does next. */
struct ShadeOut {
    bool cont, shadow, hitGeom, accd, capped;
    bool next;                       /* the path ended and its frame's next sample continues it (k_shade) */
    uint32_t seedOut;                /* RNG state after the bounce's draws (the next sample of a frame starts from it) */
    bool addRad;                     /* rad[sid] += radd (miss / light hit), done by the caller */
    uint32_t seg;                    /* extension rays of the path so far */
    V3 radd;
    float4 o, d, T;                  /* continuation path record */
    float4 so, sd, sc;               /* shadow ray: (origin, tmax), (dir, sid), (T*Ld, 0) */
    uint32_t light;                  /* slot of the sampled light in the light list (ray-order key) */
};

/* One bounce of Renderer::trace's loop body (renderer.cpp:338-460) for one path
 * whose extension ray has been traced (h4 = t,u,v,prim; inst = ~0 on a miss). */
/* Scene tables shading reads by per-lane (divergent) index: LDS copies when
 * they fit (k_shade / k_tail stage them per workgroup), else global. */
struct ShadeTables {
    const DevInstance* inst;
    const DevMaterial* mats;
    const uint2* lights;
};

constexpr uint32_t kLdsInst = 64, kLdsMats = 64, kLdsLights = 64;

__device__ __forceinline__ void stageTables(const DevScene& S, DevInstance* sInst, DevMaterial* sMat, uint2* sLights) {
    const uint32_t nI = S.nInst * (sizeof(DevInstance) / 16), nM = S.nMats * (sizeof(DevMaterial) / 16);
    for (uint32_t k = threadIdx.x; k < nI; k += blockDim.x) reinterpret_cast<float4*>(sInst)[k] = reinterpret_cast<const float4*>(S.inst)[k];
    for (uint32_t k = threadIdx.x; k < nM; k += blockDim.x) reinterpret_cast<float4*>(sMat)[k] = reinterpret_cast<const float4*>(S.mats)[k];
    for (uint32_t k = threadIdx.x; k < S.nLights; k += blockDim.x) sLights[k] = S.lights[k];
    __syncthreads();
}

/* The cooperative (one path per wave) kernels stage the trace and shading
 * tables in LDS when they fit; with more instances / materials / lights they
 * read them from global memory (wave-uniform reads).  The host sizes the
 * dynamic LDS the same way (surf_hip.hip coopLds / coopTailLds). */
/* (a compile-time choice: through a pointer that may be LDS or global, a
 * table load is a flat load the compiler cannot prove wave-uniform, and the
 * walk's scalar operands derive from those loads) */
template <bool LDS>
__device__ __forceinline__ TraceTables coopTrace(const DevScene& S, uint32_t* lds, uint32_t words) {
    if (LDS) return stageTrace(S, lds, words);
    return TraceTables{S.tinst, S.tlasIdx};
}
/* shading tables at LDS word `at` (16-B aligned) when they fit */
template <bool LDS>
__device__ __forceinline__ ShadeTables coopShade(const DevScene& S, uint32_t* lds, uint32_t at) {
    if (!LDS) return ShadeTables{S.inst, S.mats, S.lights};
    DevInstance* const sInst = reinterpret_cast<DevInstance*>(lds + at);
    DevMaterial* const sMat = reinterpret_cast<DevMaterial*>(sInst + S.nInst);
    uint2* const sLights = reinterpret_cast<uint2*>(sMat + S.nMats);
    stageTables(S, sInst, sMat, sLights);            /* ends with a barrier */
    return ShadeTables{sInst, sMat, sLights};
}

/* Next-event estimation of one diffuse bounce (Scene::sampleLights +
 * Instance::samplePoint, scene.h:53, bvh.cpp:533-552; renderer.cpp:384-415):
 * four draws from seed; sets r's shadow ray when the light faces P. */
__device__ __forceinline__ void sampleNEE(const DevScene& S, const ShadeTables& Tb, uint32_t& seed, V3 P, V3 N, V3 T, V3 brdf,
                                          uint32_t sid, ShadeOut& r) {
    /* Scene::sampleLights + Instance::samplePoint (scene.h:53, bvh.cpp:533-552) */
    const uint32_t li = rndRangeU(seed, 0u, S.nLights);
    const uint2 L = Tb.lights[li];
    const DevInstance& LI = Tb.inst[L.x];
    const float lu = rndRange(seed, 0.0f, 1.0f);
    const float lv = rndRange(seed, 0.0f, 1.0f - lu);
    const uint32_t ti = rndRangeU(seed, 0u, L.y);
    const float4* tv = S.verts + 4u * (LI.triOffset + ti);
    const float4* tn = S.normals + 3u * (LI.triOffset + ti);
    const float lw = (1.0f - lu) - lv;
    const V3 lp = add(add(lscl(lu, xyz(tv[0])), lscl(lv, xyz(tv[2]))), lscl(lw, xyz(tv[1])));
    const V3 ln = add(add(lscl(lu, xyz(tn[0])), lscl(lv, xyz(tn[2]))), lscl(lw, xyz(tn[1])));
    const float* LM = LI.M;
    V3 Pl = mk3(mrow(LM, 0, lp.x, lp.y, lp.z, 1.0f), mrow(LM, 1, lp.x, lp.y, lp.z, 1.0f), mrow(LM, 2, lp.x, lp.y, lp.z, 1.0f));
    if (!LI.affine) Pl = divs(Pl, mrow(LM, 3, lp.x, lp.y, lp.z, 1.0f));   /* w == 1 exactly when affine */
    const V3 LN = normalize(mk3(mrow(LM, 0, ln.x, ln.y, ln.z, 0.0f), mrow(LM, 1, ln.x, ln.y, ln.z, 0.0f),
                                mrow(LM, 2, ln.x, ln.y, ln.z, 0.0f)));
    const V3 IL = sub(Pl, P);
    const V3 Ld = normalize(IL);
    const V3 SO = add(P, lscl(kEps, Ld));
    const float srDepth = sqrtf(dot(IL, IL)) - 2.0f * kEps;
    const float falloff = 1.0f / dot(IL, IL);
    const float cosO = dot(N, Ld);
    const float cosL = dot(LN, lscl(-1.0f, Ld));
    if (cosO > 0.0f && cosL > 0.0f) {
        const float SA = (cosL * LI.area) * falloff;
        const float lightPdf = 1.0f / SA;
        const float invPdf = 1.0f / lightPdf;
        const DevMaterial& lm = Tb.mats[LI.material];
        const V3 le = lscl(lm.emit, ld3(lm.ec));
        const V3 Lc = scl(scl(mul(scl(le, invPdf), brdf), cosO), (float)S.nLights);
        const V3 contrib = mul(T, Lc);
        r.shadow = true;
        r.light = li;
        r.so = make_float4(SO.x, SO.y, SO.z, srDepth);
        r.sd = make_float4(Ld.x, Ld.y, Ld.z, u2f(sid));
        r.sc = make_float4(contrib.x, contrib.y, contrib.z, 0.0f);
    }
}

template <bool SPEC = false>
__device__ __forceinline__ void shadePath(const DevScene& S, const ShadeTables& Tb, float4 o4, float4 d4, float4 T4, float4 h4,
                                          uint32_t inst, uint32_t maxSeg, uint32_t zeroCutoff, ShadeOut& r) {
    r.cont = r.shadow = r.hitGeom = r.accd = r.capped = r.addRad = r.next = false;
    const uint32_t sid = f2u(o4.w);
    uint32_t flags = f2u(d4.w);
    uint32_t seed = f2u(T4.w);
    r.seedOut = seed;
    const V3 o = xyz(o4), d = xyz(d4);
    V3 T = xyz(T4);
    bool lastSpecular = (flags & kFlagSpecular) != 0u;
    const bool inMedium = (flags & kFlagMedium) != 0u;
    const uint32_t seg = flags >> 2;
    r.seg = seg;
    if (inst == kUnset) {
        /* miss: energy += T * background (scene.cpp:35-51) */
        V3 bg = mk3(0.0f, 0.0f, 0.0f);
        if (S.bgType == 0u) bg = ld3(S.bgColor);
        else if (S.bgType == 1u) {
            const float a = 0.5f * (1.0f + d.y);
            bg = add(lscl(a, ld3(S.bgB)), lscl(1.0f - a, ld3(S.bgA)));
        }
        r.addRad = true; r.radd = mul(T, bg);
        r.accd = true;
        return;
    }
    r.hitGeom = true;
    const DevInstance& I = Tb.inst[inst];
    const DevMaterial& m = Tb.mats[I.material];
    const bool isLight = m.emit > 0.0f && (m.ec[0] > 0.0f || m.ec[1] > 0.0f || m.ec[2] > 0.0f);
    if (isLight) {
        const V3 le = lscl(m.emit, ld3(m.ec));
        r.addRad = true; r.radd = lastSpecular ? mul(T, le) : mk3(0.0f, 0.0f, 0.0f);
        r.accd = lastSpecular;
        return;
    }
    const float t = h4.x, hu = h4.y, hv = h4.z;
    const uint32_t prim = f2u(h4.w);
    V3 medium = mk3(1.0f, 1.0f, 1.0f);
    if (inMedium) {
        const float nd = -t;
        medium = mk3(gExpf(m.absorb[0] * nd), gExpf(m.absorb[1] * nd), gExpf(m.absorb[2] * nd));
    }
    const V3 P = add(o, lscl(t, d));
    /* Instance::normal: M (u n0 + v n2 + w n1, 0), glm::normalize(vec4) */
    const float4* nr = S.normals + 3u * (I.triOffset + prim);
    const float4 n0 = nr[0], n1 = nr[1], n2 = nr[2];
    const float w = (1.0f - hu) - hv;
    const V3 no = add(add(lscl(hu, xyz(n0)), lscl(hv, xyz(n2))), lscl(w, xyz(n1)));
    const float* M = I.M;
    const float nx4 = mrow(M, 0, no.x, no.y, no.z, 0.0f), ny4 = mrow(M, 1, no.x, no.y, no.z, 0.0f);
    const float nz4 = mrow(M, 2, no.x, no.y, no.z, 0.0f), nw4 = mrow(M, 3, no.x, no.y, no.z, 0.0f);
    const float nn = (nx4 * nx4 + ny4 * ny4) + (nz4 * nz4 + nw4 * nw4);
    const float ninv = 1.0f / sqrtf(nn);
    V3 N = mk3(nx4 * ninv, ny4 * ninv, nz4 * ninv);
    const float rng = rndF(seed);
    V3 R = mk3(0.0f, 0.0f, 0.0f);
    bool nextMedium = inMedium;
    bool alive = true;
    if (dot(d, N) > 0.0f) N = scl(N, -1.0f);
    if (rng < m.refl) {
        R = sub(d, lscl(2.0f * dot(N, d), N));
        lastSpecular = true;
        T = mul(T, mul(ld3(m.albedo), medium));
    } else if (rng < (m.refl + m.refr)) {
        bool mustRefract = false;
        R = sub(d, lscl(2.0f * dot(N, d), N));
        const float n1f = inMedium ? m.ior : 1.0f, n2f = inMedium ? 1.0f : m.ior;
        const float ratio = n1f / n2f;
        const float cosI = -dot(d, N);
        const float cos2 = 1.0f - (ratio * ratio) * (1.0f - cosI * cosI);
        if (cos2 > 0.0f) {
            const float a = n1f - n2f, b = n1f + n2f;
            const float r0 = (a * a) / (b * b);
            const float c = 1.0f - cosI;
            const float fres = r0 + (1.0f - r0) * ((((c * c) * c) * c) * c);
            mustRefract = rndF(seed) > fres;
            if (mustRefract) R = add(lscl(ratio, d), lscl(ratio * cosI - sqrtf(fabsf(cos2)), N));
        }
        lastSpecular = true;
        T = mul(T, mul(ld3(m.albedo), medium));
        nextMedium = mustRefract ? !inMedium : inMedium;
    } else {
        const V3 brdf = scl(ld3(m.albedo), kInvPi);
        if (SPEC) {
            /* the light sample depends on the cosine sample only through the RNG
             * state after its draws: formed from the state after the first try
             * (almost always accepted) beside the cosine sample, so the two
             * dependency chains interleave; formed again after a retry */
            uint32_t sC = seed;
            V3 R1;
            const bool ok1 = cosineTry(sC, N, R1);
            uint32_t sL = sC;
            if (S.nLights > 0u) sampleNEE(S, Tb, sL, P, N, T, brdf, sid, r);
            if (ok1) {
                R = R1;
            } else {
                R = cosineSample(sC, N);
                sL = sC;
                r.shadow = false;
                if (S.nLights > 0u) sampleNEE(S, Tb, sL, P, N, T, brdf, sid, r);
            }
            seed = sL;
        } else {
            R = cosineSample(seed, N);
            if (S.nLights > 0u) sampleNEE(S, Tb, seed, P, N, T, brdf, sid, r);
        }
        const float cosT = dot(N, R);
        const float pdf = cosT * kInvPi;
        const float pm = tmax(T.x, tmax(T.y, T.z));
        const float pr = pm < 0.0f ? 0.0f : (pm > 1.0f ? 1.0f : pm);   /* clamp(max(T), 0, 1) */
        if (pr < rndF(seed)) alive = false;
        else {
            const float rr = 1.0f / pr;
            const float invPdf = 1.0f / pdf;
            lastSpecular = false;
            T = mul(T, scl(mul(lscl(cosT * invPdf, brdf), medium), rr));
        }
    }
    /* throughput cutoff: every channel of T below FLT_MIN.  Russian roulette ends
     * such a path with certainty at its next diffuse bounce (p < 2^-32 <= rand);
     * what is dropped is the emitter hits along the specular / dielectric chain
     * up to that bounce plus its NEE term, each < 1.2e-38 * L; it also ends the
     * TIR orbits in the glass lens that never terminate in the reference. */
    if (zeroCutoff && T.x < 1.17549435e-38f && T.y < 1.17549435e-38f && T.z < 1.17549435e-38f) alive = false;
    r.capped = alive && (maxSeg != 0u && seg >= maxSeg);
    r.seedOut = seed;
    if (alive && !(maxSeg != 0u && seg >= maxSeg)) {
        r.cont = true;
        const V3 O = add(P, lscl(kEps, R));
        flags = (nextMedium ? kFlagMedium : 0u) | (lastSpecular ? kFlagSpecular : 0u) | ((seg + 1u) << 2);
        r.o = make_float4(O.x, O.y, O.z, u2f(sid));
        r.d = make_float4(R.x, R.y, R.z, u2f(flags));
        r.T = make_float4(T.x, T.y, T.z, u2f(seed));
    }
}

/* Camera::getPrimaryRay + sampleDefocusDisk (camera.h:59-87) with the jitter
 * of renderer.cpp:173-177, drawn from `seed` in g++'s order (last argument
 * first): the path record of sample `sid` at shard pixel lp. */
__device__ __forceinline__ void cameraSample(const DevCamera& cam, const StreamGeom& G, uint32_t lp, uint32_t sid, uint32_t seed,
                                             float4& o4, float4& d4, float4& T4) {
    const uint32_t rowi = lp / G.width;
    const uint32_t x = lp - rowi * G.width;
    const uint32_t row = G.rows[rowi];
    const float jy = rndRange(seed, -0.5f, 0.5f);
    const float jx = rndRange(seed, -0.5f, 0.5f);
    const float u = ((float)x + jx) * cam.invW, v = ((float)row + jy) * cam.invH;
    V3 origin = ld3(cam.pos);
    if (cam.defocus) {
        float sx, sy;
        do {
            sy = rndRange(seed, -1.0f, 1.0f);
            sx = rndRange(seed, -1.0f, 1.0f);
        } while (sx * sx + sy * sy > 1.0f);
        origin = add(origin, add(lscl(sx, ld3(cam.diskU)), lscl(sy, ld3(cam.diskV))));
    }
    const V3 plane = add(add(ld3(cam.firstPixel), lscl(u, ld3(cam.uVec))), lscl(v, ld3(cam.vVec)));
    const V3 dir = normalize(sub(plane, origin));
    o4 = make_float4(origin.x, origin.y, origin.z, u2f(sid));
    d4 = make_float4(dir.x, dir.y, dir.z, u2f(kFlagSpecular | (1u << 2)));
    T4 = make_float4(1.0f, 1.0f, 1.0f, u2f(seed));
}

/* The next sample of a multi-sample frame (Renderer::render's sample loop,
 * renderer.cpp:171-181): when the path of sample `sid` ended and its frame has
 * samples left for the pixel, the pixel's next camera sample -- radiance slot
 * sid + npx (the frame's samples occupy consecutive slots) -- drawn from the
 * RNG state the ended path left.  False for a frame's last sample. */
__device__ __forceinline__ bool chainNext(const DevCamera& cam, const StreamGeom& G, uint32_t spp, uint32_t sid, uint32_t slot,
                                          uint32_t seed, float4& o4, float4& d4, float4& T4) {
    if (spp <= 1u || slot % spp == spp - 1u) return false;
    cameraSample(cam, G, sid - slot * G.npx, sid + G.npx, seed, o4, d4, T4);
    return true;
}

/* Frame completion: one atomic per distinct frame slot in the wave (lanes of a
 * wave almost always share one frame). */
__device__ __forceinline__ void frameDoneAdd(uint32_t* frameDone, bool done, uint32_t slot) {
    unsigned long long pending = __ballot(done);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t ls = (uint32_t)__shfl((int)slot, leader);
        const unsigned long long same = __ballot(done && slot == ls) & pending;
        if (laneId() == (uint32_t)leader) atomicAdd(&frameDone[ls], (uint32_t)__popcll(same));
        pending &= ~same;
    }
}

template <bool LDS_TABLES>
__global__ __launch_bounds__(kBlock, SURF_SHADE_WAVES) void k_shade(DevScene S, Pool cur, Pool nxt, const float4* __restrict__ hitTUV,
                                                  const uint32_t* __restrict__ hitInst, ShadowQ Q,
                                                  float4* __restrict__ rad, uint32_t* __restrict__ frameDone,
                                                  uint32_t npx, uint32_t window, Counters* C, int par,
                                                  const uint32_t* __restrict__ order, DevCamera cam, StreamGeom G) {
    if (blockIdx.x * blockDim.x >= C->nIn[par]) return;     /* nothing to shade in this block */
    __shared__ DevInstance sInst[LDS_TABLES ? kLdsInst : 1];
    __shared__ DevMaterial sMat[LDS_TABLES ? kLdsMats : 1];
    __shared__ uint2 sLights[LDS_TABLES ? kLdsLights : 1];
    ShadeTables Tb{S.inst, S.mats, S.lights};
    if (LDS_TABLES) {
        stageTables(S, sInst, sMat, sLights);
        Tb = ShadeTables{sInst, sMat, sLights};
    }
    /* block-level compaction: per iteration one packed 64-bit atomic reserves the
     * block's continuation and shadow slots (LDS double-buffered by iteration) */
    __shared__ uint32_t sWave[2][kBlock / 64];
    __shared__ uint32_t sBase[2];
    /* shadow rays per bin of the iteration (a lane's LDS atomic returns its rank
     * in its bin) and each bin's reservation: region base, the part that fits
     * the region, the overflow base of the rest */
    __shared__ uint32_t sShCnt[2][kShBins];
    __shared__ uint32_t sShBase[2][kShBins], sShOk[2][kShBins], sShOv[2][kShBins];
    if (threadIdx.x < 2u * kShBins) (&sShCnt[0][0])[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t n = C->nIn[par];
    const uint32_t maxSeg = C->maxSeg, zeroCutoff = C->zeroCutoff, spp = C->spp;
    const uint32_t wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t it = 0;
    unsigned long long cHit = 0, cCont = 0, cSh = 0, cAcc = 0, cCap = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x, it ^= 1u) {
        const uint32_t i = base + threadIdx.x;
        ShadeOut r;
        r.cont = r.shadow = r.hitGeom = r.accd = r.capped = r.addRad = r.next = false;
        r.seg = 0;
        uint32_t slot = 0, sid = 0, hinst = kUnset;
        const bool active = i < n;
        if (active) {
            const uint32_t j = order ? order[i] : i;   /* the path k_extend traced as ray i */
            const float4 o4 = ldS(&cur.od[2u * (j)]);
            sid = f2u(o4.w);
            slot = sid / npx;
            hinst = ldSu(&hitInst[i]);
            shadePath(S, Tb, o4, ldS(&cur.od[2u * (j) + 1u]), ldS(&cur.T[j]), ldS(&hitTUV[i]), hinst, maxSeg, zeroCutoff, r);
            if (r.addRad) addRadiance(rad, sid, r.radd);
            /* the sample ended: its frame's next sample of this pixel takes its
             * place in the next pool (a camera ray, not a continuation) */
            if (!r.cont && chainNext(cam, G, spp, sid, slot, r.seedOut, r.o, r.d, r.T)) {
                r.next = true;
                rad[sid + npx] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
        }
        const unsigned long long mCont = __ballot(r.cont || r.next);
        if (laneId() == 0) sWave[it][wv] = (uint32_t)__popcll(mCont);
        /* the shadow ray's bin -- toward the same light from the same octant of
         * the scene -- and its rank among the iteration's rays of that bin */
        const uint32_t kb = r.shadow ? (Q.bins > 1u ? shadowKey(S, r.light, r.so) : 0u) : kShBins;
        uint32_t rk = 0;
        if (r.shadow) rk = atomicAdd(&sShCnt[it][kb], 1u);
        __syncthreads();
        if (threadIdx.x <= kShBins) {
            /* the iteration's reservations in ONE atomic instruction of wave 0
             * (a round trip each would serialize): lanes 0..kShBins-1 the
             * non-empty shadow bins (this XCD's part of each), lane kShBins the
             * continuations; shadow rays that do not fit their bin's region go
             * to the overflow region */
            const uint32_t t = threadIdx.x;
            const uint32_t seg = t * kShXcds + xccId();
            uint32_t tot = 0;
            uint32_t* cur = reinterpret_cast<uint32_t*>(&C->app[par]);
            if (t < kShBins) {
                tot = sShCnt[it][t];
                sShCnt[it ^ 1u][t] = 0u;           /* the next iteration's counts (last read an iteration ago) */
                cur = shCursor(Q, par, seg);
            } else {
                for (uint32_t k = 0; k < nw; ++k) tot += sWave[it][k];
            }
            const uint32_t b0 = tot ? atomicAdd(cur, tot) : 0u;
            if (t == kShBins) {
                sBase[it] = b0;
            } else {
                const uint32_t ok = b0 >= Q.region ? 0u : min(tot, Q.region - b0);
                const uint32_t ov = ok < tot ? atomicAdd(shCursor(Q, par, kShSegs - 1u), tot - ok) : 0u;
                sShBase[it][t] = seg * Q.region + b0; sShOk[it][t] = ok; sShOv[it][t] = ov;
            }
        }
        __syncthreads();
        uint32_t jc = sBase[it];
        for (uint32_t k = 0; k < wv; ++k) jc += sWave[it][k];
        jc += rankBelow(mCont);
        if (r.cont || r.next) {
            stS(&nxt.od[2u * (jc)], r.o); stS(&nxt.od[2u * (jc) + 1u], r.d); stS(&nxt.T[jc], r.T);
            /* starts on the instance it hit, from this quadrant; camera rays in their own bin */
            nxt.key[jc] = r.next ? (uint8_t)(kBins - 1u) : poolKey(S, hinst, r.o, r.d);
        }
        if (r.shadow) {
            const uint32_t ok = sShOk[it][kb];
            const uint32_t js = rk < ok ? sShBase[it][kb] + rk : (kShSegs - 1u) * Q.region + sShOv[it][kb] + (rk - ok);
            stS(&Q.od[2u * js], r.so); stS(&Q.od[2u * js + 1u], r.sd); stS(&Q.c[js], r.sc);
        }
        /* a path that ends here may still have this phase's shadow ray pending:
         * connect runs before the host reads frameDone (end of the phase). */
        frameDoneAdd(frameDone + (blockIdx.x % kStripes) * window, active && !r.cont, slot);
        if (active && !r.cont && r.seg > 32u) atomicMax(&C->segMax, r.seg);   /* rare: RR ends most paths early */
        noteCappedSid(r.capped, C, sid);
        cCap += (unsigned long long)__popcll(__ballot(r.capped));
        cHit += (unsigned long long)__popcll(__ballot(r.hitGeom));
        cCont += (unsigned long long)__popcll(__ballot(r.cont));
        cSh += (unsigned long long)__popcll(__ballot(r.shadow));
        cAcc += (unsigned long long)__popcll(__ballot(r.accd));
    }
    blockCount<5>(C, {1, 2, 3, 4, 7}, {cHit, cCont, cSh, cAcc, cCap});
}

/* Where shadow ray i of the bin order lives: the (bin, XCD) regions in bin
 * order, then the overflow region (pre: the first ray index of each segment,
 * kShSegs + 1 entries, the last = the count). */
__device__ __forceinline__ uint32_t shadowSlot(const ShadowQ& Q, const uint32_t* pre, uint32_t i) {
    uint32_t lo = 0, hi = kShSegs;            /* pre[lo] <= i < pre[hi] */
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (i >= pre[mid]) lo = mid; else hi = mid;
    }
    return lo * Q.region + (i - pre[lo]);
}

template <bool LDS, bool LW = false, bool STG = false>
__global__ __launch_bounds__(kBlock, STG ? 5 : SURF_TRACE_WAVES) void k_connect(DevScene S, ShadowQ Q, float4* __restrict__ rad, Counters* C, int par,
                                                    uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t sPre[kShSegs + 1];
    if (threadIdx.x < 64u) {
        /* first ray index of every queue segment: a wave scan of the cursors */
        uint32_t carry = 0;
        if (threadIdx.x == 0) sPre[0] = 0u;
        for (uint32_t b0 = 0; b0 < kShSegs; b0 += 64u) {
            const uint32_t b = b0 + threadIdx.x;
            uint32_t v = b < kShSegs ? min(*shCursor(Q, par, b), b + 1u < kShSegs ? Q.region : 0xffffffffu) : 0u;
#pragma unroll
            for (uint32_t off = 1; off < 64u; off <<= 1) {
                const uint32_t t = __shfl_up(v, off);
                if (threadIdx.x >= off) v += t;
            }
            if (b < kShSegs) sPre[b + 1] = carry + v;
            carry += (uint32_t)__shfl((int)v, 63);
        }
    }
    __syncthreads();
    const uint32_t n = sPre[kShSegs];
    if (blockIdx.x * blockDim.x >= n) return;               /* no shadow rays for this block */
    /* STG: the emitters' BLAS node records (every unoccluded shadow ray walks
     * that BLAS down to its sampled triangle) staged after a stack of 16-bit
     * entries (every node index < 65536) and the trace tables; stageTrace's
     * barrier publishes them */
    const uint32_t stackWordsUsed = STG ? stackWords / 2u : stackWords;
    float4* sN = nullptr;
    if (STG) {
        sN = reinterpret_cast<float4*>(lds + ((stackWordsUsed + S.nInst * (uint32_t)((sizeof(TraceInst) + 4u) / 4u) + 3u) & ~3u));
        for (uint32_t k = threadIdx.x; k < 4u * S.sbRecN; k += blockDim.x) sN[k] = S.sbRec[k];
        float4* const sT = sN + 4u * S.sbRecN;
        for (uint32_t k = threadIdx.x; k < 3u * S.sbTriN; k += blockDim.x) sT[k] = S.tris[3u * S.sbTri0 + k];
    }
    const TraceTables Tt = traceTables<LDS>(S, lds, stackWordsUsed);
    const uint32_t stride = blockDim.x;
    using SK = typename std::conditional<STG, uint16_t, uint32_t>::type;
    SK* stk = reinterpret_cast<SK*>(lds) + threadIdx.x;
    unsigned long long cUn = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i0 = base + threadIdx.x;
        bool unocc = false;
        if (i0 < n) {
            const uint32_t i = shadowSlot(Q, sPre, i0);
            const float4 o = ldS(&Q.od[2u * i]), d = ldS(&Q.od[2u * i + 1u]);
            float depth = o.w, u = 0.0f, v = 0.0f;
            uint32_t inst = kUnset, prim = kUnset;
            const bool occ = traceScene<true, LW, STG, SK>(S, Tt, xyz(o), xyz(d), depth, u, v, inst, prim, stk, stride, sN);
            if (!occ) {
                const float4 c = ldS(&Q.c[i]);
                addRadiance(rad, f2u(d.w), xyz(c));
                unocc = true;
            }
        }
        cUn += (unsigned long long)__popcll(__ballot(unocc));
    }
    blockCount<2>(C, {5, 4}, {cUn, cUn});
}

/* What k_regen issues in phase par: chains [iss, iss + nnew) into pool slots
 * [cont, cont + nnew) of pool[par^1], and where the stream's permuted head ends. */
struct RegenPlan {
    uint32_t cont, nnew, lp0, nA, nB;
    unsigned long long iss, base, f0, endA, endP;
    uint32_t spp;
};
__device__ __forceinline__ RegenPlan regenPlan(const Counters* C, int par, uint32_t capacity, const StreamGeom& G) {
    RegenPlan R;
    R.cont = C->app[par];
    R.iss = C->issued[par];
    const unsigned long long lim = C->limit;
    R.base = C->baseFrame;
    R.spp = C->spp;
    const uint32_t room = capacity - R.cont;
    const unsigned long long left = lim > R.iss ? lim - R.iss : 0ull;
    R.nnew = (unsigned long long)room < left ? room : (uint32_t)left;
    /* frame / pixel of the first new chain, then step without 64-bit divisions */
    R.f0 = R.iss / G.npx;
    R.lp0 = (uint32_t)(R.iss - R.f0 * G.npx);
    /* the permuted head of the stream (surf_hip.hip classifyPixels) */
    R.nA = C->permA; R.nB = G.npx - C->permA;
    R.endA = (unsigned long long)R.nA * C->permFrames; R.endP = (unsigned long long)G.npx * C->permFrames;
    return R;
}
/* The k-th new chain's first sample into pool slot cont + k. */
__device__ __forceinline__ void regenSample(const DevCamera& cam, const Pool& nxt, float4* __restrict__ rad, const StreamGeom& G,
                                            const RegenPlan& R, uint32_t k) {
    uint32_t lp;
    unsigned long long f;
    if (R.iss + k < R.endP) {
        const unsigned long long s = R.iss + k;
        if (s < R.endA) { f = s / R.nA; lp = G.perm[(uint32_t)(s - f * R.nA)]; }
        else { const unsigned long long j = s - R.endA; f = j / R.nB; lp = G.perm[R.nA + (uint32_t)(j - f * R.nB)]; }
    } else {
        lp = R.lp0 + k;
        const uint32_t df = lp / G.npx;
        lp -= df * G.npx;
        f = R.f0 + df;
    }
    const unsigned long long pass = f * R.spp;
    const uint32_t slot = (uint32_t)(pass % G.window);
    const uint32_t rowi = lp / G.width;
    const uint32_t p = (lp - rowi * G.width) + G.rows[rowi] * G.width;
    const uint32_t sid = slot * G.npx + lp;
    float4 o4, d4, T4;
    cameraSample(cam, G, lp, sid, initSeed(p + (uint32_t)(R.base + pass) * 1799u), o4, d4, T4);
    const uint32_t slotIdx = R.cont + k;
    stS(&nxt.od[2u * (slotIdx)], o4);
    stS(&nxt.od[2u * (slotIdx) + 1u], d4);
    stS(&nxt.T[slotIdx], T4);
    nxt.key[slotIdx] = (uint8_t)(kBins - 1u);                      /* camera rays */
    rad[sid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}
/* The counters of the phase after par (one thread). */
__device__ __forceinline__ void regenCounters(Counters* C, int par, const RegenPlan& R) {
    const int nx = par ^ 1;
    C->resumeN[par] = 0u;          /* this phase's k_extend_cont has run */
    C->nIn[nx] = R.cont + R.nnew;
    C->issued[nx] = R.iss + R.nnew;
    C->app[nx] = 0u;               /* next phase's append cursor */
    C->ev[0] += R.cont + R.nnew;   /* extension rays of the next phase */
    C->ev[8] += R.cont + R.nnew;   /* ... traced by k_extend unless the drain takes the pool */
}

/* Fills pool[par^1] after the continuing paths, up to capacity and the issue
 * limit, with the first sample of the next (frame, pixel) chains in issue
 * order: frame f's first sample is stream pass f * spp, seeded
 * initSeed(p + 1799 * (baseFrame + f * spp)) (renderer.cpp:169; baseFrame =
 * the sample count before the stream). */
__global__ __launch_bounds__(kBlock) void k_regen(DevCamera cam, Pool nxt, float4* __restrict__ rad, Counters* C, int par,
                                                  uint32_t capacity, StreamGeom G, ShadowQ Q) {
    const RegenPlan R = regenPlan(C, par, capacity, G);
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < kShSegs) *shCursor(Q, par ^ 1, gid) = 0u;      /* the next phase's shadow-queue cursors */
    for (uint32_t k = gid; k < R.nnew; k += gridDim.x * blockDim.x) regenSample(cam, nxt, rad, G, R, k);
    if (gid == 0) regenCounters(C, par, R);
}

/* k_regen fused with the next phase's pool count (the default; SURF_REGEN_COUNT=0:
 * k_regen + k_bincount): one workgroup per sort chunk (k_binscatter's
 * sortChunk over the next pool's cont + nnew paths), which counts the
 * continuations' keys of its chunk and generates the chunk's new camera
 * samples (key kBins - 1), then writes the chunk's bin counts where k_bincount
 * would -- so the next phase's sort is k_binscatter alone, and one kernel
 * instead of two waits for CU slots beside k_connect. */
__global__ __launch_bounds__(kSortThreads) void k_regen_count(DevCamera cam, Pool nxt, float4* __restrict__ rad, Counters* C, int par,
                                                             uint32_t capacity, StreamGeom G, ShadowQ Q, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kBins];
    if (threadIdx.x < kBins) h[threadIdx.x] = 0u;
    const RegenPlan R = regenPlan(C, par, capacity, G);
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < kShSegs) *shCursor(Q, par ^ 1, gid) = 0u;      /* the next phase's shadow-queue cursors */
    __syncthreads();
    uint32_t a, b;
    sortChunk(R.cont + R.nnew, a, b);
    uint32_t cam0 = 0u;
    for (uint32_t i = a + threadIdx.x; i < b; i += blockDim.x) {
        if (i < R.cont) atomicAdd(&h[nxt.key[i]], 1u);
        else { regenSample(cam, nxt, rad, G, R, i - R.cont); ++cam0; }
    }
    if (cam0) atomicAdd(&h[kBins - 1u], cam0);
    __syncthreads();
    if (threadIdx.x < kBins) hist[threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
    if (gid == 0) regenCounters(C, par, R);
}

/* Finishes the last paths of the stream: one kernel, each active lane runs its
 * path (extend -> shade -> connect per segment), so the long Russian-roulette
 * tail pays no per-bounce launch.  Same device functions as the wavefront
 * kernels: identical results.  lanes < lpw of each wave work.
 * Two stages (runTail): pool 0 with a segment budget -- a path still alive
 * after `budget` segments is appended to `surv` instead of holding its wave --
 * then the survivors (lens TIR orbits run thousands of segments) one per wave,
 * so no long path shares a wave.  firstCounted: the first extension ray of
 * each input path is already in the event counts (regen counted it). */
/* One path run to its end (or for `budget` segments, after which the
 * continuation goes to `sink`): extend -> shade -> connect per segment with
 * the wavefront kernels' device functions.  Returns whether the path ended. */
__device__ __forceinline__ bool runPath(const DevScene& S, const TraceTables& Tt, const ShadeTables& Tb, float4 o4, float4 d4,
                                        float4 T4, uint32_t budget, const Sink& sink, float4* __restrict__ rad,
                                        uint32_t* __restrict__ frameDone, uint32_t npx, uint32_t window, Counters* C,
                                        uint32_t* stk, uint32_t stride, uint32_t firstCounted, const DevCamera& cam,
                                        const StreamGeom& G) {
    const uint32_t maxSeg = C->maxSeg, zeroCutoff = C->zeroCutoff, spp = C->spp;
    const uint32_t st = blockIdx.x % kStripes;
    uint32_t slot = f2u(o4.w) / npx;
    uint32_t nExt = 0, nHit = 0, nCont = 0, nSh = 0, nAcc = 0, nUn = 0, nDone = 0;   /* per path: 32 bits suffice */
    bool done = true;
    V3 E = loadRadiance(rad, f2u(o4.w));
    for (;;) {
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
        const bool hit = traceScene<false>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, stk, stride);
        ++nExt;
        ShadeOut r;
        shadePath(S, Tb, o4, d4, T4, make_float4(depth, u, v, u2f(prim)), hit ? inst : kUnset, maxSeg, zeroCutoff, r);
        if (r.addRad) E = add(E, r.radd);
        nHit += r.hitGeom; nAcc += r.accd;
        if (r.shadow) {
            ++nSh;
            float sdep = r.so.w, su = 0.0f, sv = 0.0f;
            uint32_t si = kUnset, sp = kUnset;
            if (!traceScene<true>(S, Tt, xyz(r.so), xyz(r.sd), sdep, su, sv, si, sp, stk, stride)) {
                E = add(E, xyz(r.sc));
                ++nUn; ++nAcc;
            }
        }
        if (r.capped) {
            noteCapped(C, f2u(o4.w));
        }
        if (!r.cont) {
            atomicMax(&C->segMax, r.seg);
            storeRadiance(rad, f2u(o4.w), E);
            __threadfence();      /* radiance before completion: other streams' kernels read it */
            atomicAdd(&frameDone[st * window + slot], 1u);
            ++nDone;
            /* the frame's next sample of this pixel continues on this lane */
            if (chainNext(cam, G, spp, f2u(o4.w), slot, r.seedOut, o4, d4, T4)) { ++slot; E = mk3(0.0f, 0.0f, 0.0f); continue; }
            break;
        }
        ++nCont;
        if (budget != 0u && nExt >= budget) {
            const uint32_t k = atomicAdd(sink.n, 1u);
            if (k < sink.cap) {
                storeRadiance(rad, f2u(o4.w), E);          /* the next stage reloads it */
                sink.q.od[2u * (k)] = r.o; sink.q.od[2u * (k) + 1u] = r.d; sink.q.T[k] = r.T;
                done = false;
                break;
            }
        }
        o4 = r.o; d4 = r.d; T4 = r.T;
    }
    unsigned long long* ev = C->evS[st];
    atomicAdd(&ev[0], (unsigned long long)(nExt - firstCounted)); atomicAdd(&ev[1], (unsigned long long)nHit);
    atomicAdd(&ev[2], (unsigned long long)nCont); atomicAdd(&ev[3], (unsigned long long)nSh);
    atomicAdd(&ev[4], (unsigned long long)nAcc); atomicAdd(&ev[5], (unsigned long long)nUn);
    if (nDone) atomicAdd(&ev[6], (unsigned long long)nDone);
    return done;
}

/* Finishes the last paths of the stream: one kernel, each active lane runs its
 * path (extend -> shade -> connect per segment), so the long Russian-roulette
 * tail pays no per-bounce launch.  lanes < lpw of each wave work.  With a
 * budget, paths still alive after `budget` segments go to `surv` for the next
 * drain stage.  firstCounted: the first extension ray of each input path is
 * already in the event counts (regen counted it). */
template <bool LDS_TABLES>
__global__ __launch_bounds__(64, SURF_TAIL_WAVES) void k_tail(DevScene S, Pool cur, uint32_t n, uint32_t lpw, float4* __restrict__ rad,
                                             uint32_t* __restrict__ frameDone, uint32_t npx, uint32_t window, Counters* C,
                                             uint32_t stackWords, uint32_t firstCounted, uint32_t budget, Pool surv,
                                             DevCamera cam, StreamGeom G) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = traceTables<LDS_TABLES>(S, lds, stackWords);
    __shared__ DevInstance sInst[LDS_TABLES ? kLdsInst : 1];
    __shared__ DevMaterial sMat[LDS_TABLES ? kLdsMats : 1];
    __shared__ uint2 sLights[LDS_TABLES ? kLdsLights : 1];
    ShadeTables Tb{S.inst, S.mats, S.lights};
    if (LDS_TABLES) {
        stageTables(S, sInst, sMat, sLights);
        Tb = ShadeTables{sInst, sMat, sLights};
    }
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x * lpw + lane;
    if (lane >= lpw || i >= n) return;
    runPath(S, Tt, Tb, cur.od[2u * (i)], cur.od[2u * (i) + 1u], cur.T[i], budget, Sink{surv, &C->survN, C->survCap}, rad, frameDone, npx, window, C,
            lds + threadIdx.x, blockDim.x, firstCounted, cam, G);
}

/* Cooperative tail: one path per 64-lane wave (block), for the long paths
 * left at the end of a drain, whose single-lane segment latency bounds the
 * drain.  Each segment: closest hit with the lanes-as-planes wave traversal
 * (traceWave), shading evaluated redundantly by every lane (same inputs, same
 * results, no broadcast), shadow ray any-hit with the same traversal; lane 0
 * does the writes.  Identical results to k_tail.  LDS: the record stack
 * (stackWords = 16 x depth words), then the trace tables; the shading tables
 * are read from global memory (wave-uniform reads): LDS copies would cap the
 * one-wave blocks at ~2 waves per SIMD. */
template <bool LDS, bool W2 = false>
__global__ __launch_bounds__(64, SURF_COOP_WAVES) void k_tail_coop(DevScene S, Pool cur, uint32_t n, float4* __restrict__ rad,
                                                  uint32_t* __restrict__ frameDone, uint32_t npx, uint32_t window, Counters* C,
                                                  uint32_t stackWords, uint32_t firstCounted, DevCamera cam, StreamGeom G) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = coopTrace<LDS>(S, lds, stackWords + proWords(S));
    /* shading's instance / material / light tables in LDS too: a path's
     * segments read them on its dependent chain (the drain's latency floor) */
    const ShadeTables Tb = coopShade<LDS>(S, lds, (stackWords + proWords(S) + S.nInst * (uint32_t)((sizeof(TraceInst) + 4u) / 4u) + 3u) & ~3u);
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const bool lead = threadIdx.x == 0;
    float* rstk = reinterpret_cast<float*>(lds);     /* the record stack (16 words per entry) */
    float4* pro = reinterpret_cast<float4*>(lds + stackWords);
    const uint32_t maxSeg = C->maxSeg, zeroCutoff = C->zeroCutoff, spp = C->spp;
    const uint32_t st = blockIdx.x % kStripes;
    float4 o4 = cur.od[2u * (i)], d4 = cur.od[2u * (i) + 1u], T4 = cur.T[i];
    uint32_t slot = f2u(o4.w) / npx;
    V3 E = loadRadiance(rad, __builtin_amdgcn_readfirstlane(f2u(o4.w)));            /* the running sample's radiance */
    unsigned long long nExt = 0, nHit = 0, nCont = 0, nSh = 0, nAcc = 0, nUn = 0, nDone = 0;
#if SURF_DRAIN_TRACE
    const unsigned long long tStart = wall_clock64();
    const uint32_t state0 = drainState(d4, T4);
#endif
#if SURF_SEG_TIMING
    unsigned long long cyc[3] = {0, 0, 0};
    SegStats ss{0, 0, 0, 0, 0, 0, 0, 0};
    SegStats* ssp = &ss;
#else
    SegStats* ssp = nullptr;
#endif
    for (;;) {
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
#if SURF_SEG_TIMING
        const unsigned long long c0 = segClock();
#endif
        const bool hit = traceWave<false, W2>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, rstk, pro, ssp);
        (void)ssp;
        ++nExt;
        ShadeOut r;
#if SURF_SEG_TIMING
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long c1 = segClock();
#endif
        shadePath<true>(S, Tb, o4, d4, T4, make_float4(depth, u, v, u2f(prim)), hit ? inst : kUnset, maxSeg, zeroCutoff, r);
        if (r.addRad) E = addU(E, r.radd);
#if SURF_SEG_TIMING
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long c2 = segClock();
#endif
        nHit += r.hitGeom; nAcc += r.accd;
        if (r.shadow) {
            ++nSh;
            float sdep = r.so.w, su = 0.0f, sv = 0.0f;
            uint32_t si = kUnset, sp = kUnset;
            const bool occ = traceWave<true, W2>(S, Tt, xyz(r.so), xyz(r.sd), sdep, su, sv, si, sp, rstk, pro);
            if (!occ) {
                E = addU(E, xyz(r.sc));
                ++nUn; ++nAcc;
            }
        }
#if SURF_SEG_TIMING
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long c3 = segClock();
        cyc[0] += c1 - c0; cyc[1] += c2 - c1; cyc[2] += c3 - c2;
#endif
        if (lead && r.capped) {
            noteCapped(C, f2u(o4.w));
        }
        if (!r.cont) {
            if (lead) {
                atomicMax(&C->segMax, r.seg);
                storeRadiance(rad, __builtin_amdgcn_readfirstlane(f2u(o4.w)), E);   /* (uniform: an SGPR address) */
                __threadfence();      /* radiance before completion */
                atomicAdd(&frameDone[st * window + slot], 1u);
            }
            ++nDone;
            /* the frame's next sample of this pixel continues on this wave */
            if (chainNext(cam, G, spp, f2u(o4.w), slot, r.seedOut, o4, d4, T4)) { ++slot; E = mk3(0.0f, 0.0f, 0.0f); continue; }
            break;
        }
        ++nCont;
        o4 = r.o; d4 = r.d; T4 = r.T;
    }
    if (lead) {
#if SURF_DRAIN_TRACE
        drainTraceEnd(tStart, (uint32_t)nExt, state0);
#endif
        unsigned long long* ev = C->evS[st];
        atomicAdd(&ev[0], nExt - (unsigned long long)firstCounted); atomicAdd(&ev[1], nHit); atomicAdd(&ev[2], nCont);
        atomicAdd(&ev[3], nSh); atomicAdd(&ev[4], nAcc); atomicAdd(&ev[5], nUn);
        atomicAdd(&ev[6], nDone);
#if SURF_SEG_TIMING
        atomicAdd(&C->dbg[0], cyc[0]); atomicAdd(&C->dbg[1], cyc[1]); atomicAdd(&C->dbg[2], cyc[2]);
        atomicAdd(&C->dbg[3], nExt); atomicAdd(&C->dbg[4], nSh);
        atomicAdd(&g_segStats[0], ss.cycInst); atomicAdd(&g_segStats[1], ss.cycLoop); atomicAdd(&g_segStats[2], ss.visits);
        atomicAdd(&g_segStats[3], ss.leaves); atomicAdd(&g_segStats[4], ss.tris); atomicAdd(&g_segStats[5], ss.entered);
        atomicAdd(&g_segStats[6], ss.cycWait); atomicAdd(&g_segStats[7], ss.cycLeaf);
#endif
    }
}

/* Cooperative drain with partner waves (k_tail_pair): workgroups of two waves,
 * each wave running paths from the drain's queue (Counters::rowNext) one at a
 * time with k_tail_coop's per-segment code.  When the queue is empty and a
 * wave's path ends while its sibling still runs one, the idle wave becomes the
 * sibling's shadow tracer: the sibling posts segment i's shadow ray to an LDS
 * mailbox and extends segment i+1 while the partner runs the any-hit walk; the
 * answer is collected after that extension, before segment i+1 is shaded, so
 * the path's radiance is added in the reference's order (renderer.cpp:415-444:
 * NEE contribution of bounce i, then whatever bounce i+1 adds).  The last
 * paths of a drain -- its latency floor -- then pay max(extend, any-hit) +
 * shade per segment instead of the sum.  Same device functions, same results. */
struct PairBox {
    uint32_t run[2];      /* wave w is in its path loop */
    uint32_t help[2];     /* help[w]: the sibling traces wave w's shadow rays */
    uint32_t post[2];     /* shadow rays wave w has posted */
    uint32_t done[2];     /* ... of which the sibling has answered */
    uint32_t occ[2];      /* the last answer */
    float4 so[2], sd[2];  /* the posted ray: (origin, tmax), (dir, sid) */
    float4 sc[2];         /* its contribution T*Ld if unoccluded (read back by the poster) */
};

__device__ __forceinline__ uint32_t ldsLoadAcq(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ldsStoreRel(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* Every wave counts its paths' events and adds them once at exit. */
struct PairCounts { uint32_t ext, hit, cont, sh, acc, un, paths, samples; };   /* paths: taken from the queue; samples: finished */

/* One path of the queue on the calling wave (w); its shadow rays go to the
 * sibling while box.help[w] is set. */
template <bool W2>
__device__ __forceinline__ void pairPath(const DevScene& S, const TraceTables& Tt, const ShadeTables& Tb, PairBox& box, uint32_t w,
                                         float4 o4, float4 d4, float4 T4, float4* __restrict__ rad, uint32_t* __restrict__ frameDone,
                                         uint32_t npx, uint32_t window, Counters* C, float* rstk, float4* pro, bool lead,
                                         uint32_t& posted, PairCounts& pc, const DevCamera& cam, const StreamGeom& G) {
    const uint32_t maxSeg = C->maxSeg, zeroCutoff = C->zeroCutoff, spp = C->spp;
    uint32_t slot = f2u(o4.w) / npx;
    bool pend = false;                     /* a posted shadow ray awaits its answer */
    V3 E = loadRadiance(rad, __builtin_amdgcn_readfirstlane(f2u(o4.w)));   /* the running sample's radiance */
#if SURF_DRAIN_TRACE
    const unsigned long long tStart = wall_clock64();
    const uint32_t state0 = drainState(d4, T4), ext0 = pc.ext;
#endif
    for (;;) {
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
        const bool hit = traceWave<false, W2>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, rstk, pro);
        ++pc.ext;
        if (pend) {
            while (ldsLoadAcq(&box.done[w]) != posted) __builtin_amdgcn_s_sleep(1);
            if (!box.occ[w]) {
                E = addU(E, xyz(box.sc[w]));
                ++pc.un; ++pc.acc;
            }
            pend = false;
        }
        ShadeOut r;
        shadePath<true>(S, Tb, o4, d4, T4, make_float4(depth, u, v, u2f(prim)), hit ? inst : kUnset, maxSeg, zeroCutoff, r);
        if (r.addRad) E = addU(E, r.radd);
        pc.hit += r.hitGeom; pc.acc += r.accd;
        if (r.shadow) {
            ++pc.sh;
            if (ldsLoadAcq(&box.help[w])) {
                ++posted;
                if (lead) {
                    box.so[w] = r.so; box.sd[w] = r.sd; box.sc[w] = r.sc;
                    ldsStoreRel(&box.post[w], posted);
                }
                pend = true;
            } else {
                float sdep = r.so.w, su = 0.0f, sv = 0.0f;
                uint32_t si = kUnset, sp = kUnset;
                if (!traceWave<true, W2>(S, Tt, xyz(r.so), xyz(r.sd), sdep, su, sv, si, sp, rstk, pro)) {
                    E = addU(E, xyz(r.sc));
                    ++pc.un; ++pc.acc;
                }
            }
        }
        if (lead && r.capped) noteCapped(C, f2u(o4.w));
        if (!r.cont) {
            if (lead) atomicMax(&C->segMax, r.seg);
            if (pend) {                    /* the sample's last shadow ray */
                while (ldsLoadAcq(&box.done[w]) != posted) __builtin_amdgcn_s_sleep(1);
                if (!box.occ[w]) {
                    E = addU(E, xyz(box.sc[w]));
                    ++pc.un; ++pc.acc;
                }
                pend = false;
            }
            ++pc.samples;
            if (lead) {
                storeRadiance(rad, __builtin_amdgcn_readfirstlane(f2u(o4.w)), E);   /* (uniform: an SGPR address) */
                __threadfence();           /* radiance before completion */
                atomicAdd(&frameDone[(blockIdx.x % kStripes) * window + slot], 1u);
            }
            /* the frame's next sample of this pixel continues on this wave */
            if (chainNext(cam, G, spp, f2u(o4.w), slot, r.seedOut, o4, d4, T4)) { ++slot; E = mk3(0.0f, 0.0f, 0.0f); continue; }
            break;
        }
        ++pc.cont;
        o4 = r.o; d4 = r.d; T4 = r.T;
    }
#if SURF_DRAIN_TRACE
    if (lead) drainTraceEnd(tStart, pc.ext - ext0, state0);
#endif
    ++pc.paths;
}

template <bool LDS, bool W2 = false>
__global__ __launch_bounds__(128, SURF_COOP_WAVES) void k_tail_pair(DevScene S, Pool cur, uint32_t n, float4* __restrict__ rad,
                                                   uint32_t* __restrict__ frameDone, uint32_t npx, uint32_t window, Counters* C,
                                                   uint32_t stackWords, uint32_t firstCounted, DevCamera cam, StreamGeom G) {
    extern __shared__ uint32_t lds[];
    __shared__ PairBox box;
    /* LDS: [record stack | prologue table] per wave, then the trace tables and the shading tables */
    const uint32_t per = stackWords + proWords(S);
    if (threadIdx.x < 2u) {
        box.run[threadIdx.x] = 1u; box.help[threadIdx.x] = 0u;
        box.post[threadIdx.x] = 0u; box.done[threadIdx.x] = 0u; box.occ[threadIdx.x] = 0u;
    }
    const TraceTables Tt = coopTrace<LDS>(S, lds, 2u * per);
    const ShadeTables Tb = coopShade<LDS>(S, lds, (2u * per + S.nInst * (uint32_t)((sizeof(TraceInst) + 4u) / 4u) + 3u) & ~3u);
    __syncthreads();                                  /* the mailboxes are initialised (global tables: no staging barrier) */
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   /* wave-uniform: the walk's LDS bases are scalar */
    const bool lead = (threadIdx.x & 63u) == 0u;
    float* rstk = reinterpret_cast<float*>(lds + w * per);
    float4* pro = reinterpret_cast<float4*>(lds + w * per + stackWords);
    PairCounts pc{0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t posted = 0u;                             /* == box.post[w] */
    for (;;) {
        uint32_t i = 0u;
        if (lead) i = atomicAdd(&C->rowNext, 1u);
        i = __builtin_amdgcn_readfirstlane(i);
        if (i >= n) break;
        pairPath<W2>(S, Tt, Tb, box, w, cur.od[2u * i], cur.od[2u * i + 1u], cur.T[i], rad, frameDone, npx, window, C, rstk, pro,
                 lead, posted, pc, cam, G);
    }
    /* queue empty: leave the path loop, then serve the sibling's shadow rays
     * while it still runs a path (one of the two always sees the other's 0) */
    const uint32_t m = w ^ 1u;
    __hip_atomic_store(&box.run[w], 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__hip_atomic_load(&box.run[m], __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP)) {
        ldsStoreRel(&box.help[m], 1u);
        uint32_t served = ldsLoadAcq(&box.done[m]);
        for (;;) {
            const uint32_t p = ldsLoadAcq(&box.post[m]);
            if (p != served) {
                const float4 so = box.so[m], sd = box.sd[m];
                float sdep = so.w, su = 0.0f, sv = 0.0f;
                uint32_t si = kUnset, sp = kUnset;
                const bool occ = traceWave<true, W2>(S, Tt, xyz(so), xyz(sd), sdep, su, sv, si, sp, rstk, pro);
                if (lead) {
                    box.occ[m] = occ ? 1u : 0u;
                    ldsStoreRel(&box.done[m], p);
                }
                served = p;
                continue;
            }
            if (!ldsLoadAcq(&box.run[m])) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lead && pc.paths) {
        unsigned long long* ev = C->evS[blockIdx.x % kStripes];
        atomicAdd(&ev[0], (unsigned long long)(pc.ext - pc.paths * firstCounted)); atomicAdd(&ev[1], (unsigned long long)pc.hit);
        atomicAdd(&ev[2], (unsigned long long)pc.cont); atomicAdd(&ev[3], (unsigned long long)pc.sh);
        atomicAdd(&ev[4], (unsigned long long)pc.acc); atomicAdd(&ev[5], (unsigned long long)pc.un);
        atomicAdd(&ev[6], (unsigned long long)pc.samples);
    }
}

/* acc[p] += (radiance, 1) for frames [f0, f0+count) of the stream, in frame
 * order (renderer.cpp:180); frame f's radiance lives in slot f % window. */
__global__ __launch_bounds__(kBlock) void k_accumulate(const float4* __restrict__ rad, float4* __restrict__ acc,
                                                       uint32_t npx, unsigned long long f0, uint32_t count, uint32_t window,
                                                       uint32_t* __restrict__ frameDone) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    /* the accumulated frames' slots are free again: reset their completion
     * stripes here, on the render stream (the escape worker may be updating
     * other slots concurrently, so the host never rewrites the whole array) */
    if (p < count * kStripes) frameDone[(p % kStripes) * window + (uint32_t)((f0 + p / kStripes) % window)] = 0u;
    if (p >= npx) return;
    float4 a = acc[p];
    for (uint32_t k = 0; k < count; ++k) {
        const uint32_t slot = (uint32_t)((f0 + k) % window);
        const float4 r = rad[(size_t)slot * npx + p];
        a.x = a.x + r.x; a.y = a.y + r.y; a.z = a.z + r.z; a.w = a.w + 1.0f;
    }
    acc[p] = a;
}

/* wavefront_finalize.comp + RgbaToU32 (cvtps2dq round-to-even, packus saturation) */
SURF_HD uint32_t packChannel(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return 0u;
    const float r = rintf(v);
    return r < 0.0f ? 0u : (r > 255.0f ? 255u : (uint32_t)r);
}
__global__ __launch_bounds__(kBlock) void k_finalize(const float4* __restrict__ acc, uint32_t* __restrict__ out,
                                                     uint32_t npx, float inv) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const float4 a = acc[p];
    out[p] = packChannel((a.x * inv) * 255.0f) | (packChannel((a.y * inv) * 255.0f) << 8) |
             (packChannel((a.z * inv) * 255.0f) << 16) | (packChannel((a.w * inv) * 255.0f) << 24);
}

/* Display step (row f2): fs_quad.frag:22-24 samples the RGBA8 finalize image
 * (UNORM: c/255) and writes sqrt(c/255) to an 8-bit UNORM target; the target's
 * float->UNORM8 conversion is taken as round-to-nearest-even with saturation
 * (packChannel).  Fused with k_finalize's packing. */
SURF_HD uint32_t displayChannel(uint32_t c8) {
    return packChannel(sqrtf((float)c8 / 255.0f) * 255.0f);
}
__global__ __launch_bounds__(kBlock) void k_display(const float4* __restrict__ acc, uint32_t* __restrict__ out,
                                                    uint32_t npx, float inv) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const float4 a = acc[p];
    out[p] = displayChannel(packChannel((a.x * inv) * 255.0f)) | (displayChannel(packChannel((a.y * inv) * 255.0f)) << 8) |
             (displayChannel(packChannel((a.z * inv) * 255.0f)) << 16) | (displayChannel(packChannel((a.w * inv) * 255.0f)) << 24);
}

/* Per-pixel term of the Lumen energy (renderer.cpp:191-201): (r/N + g/N) + b/N.
 * The sum over pixels is the reference's serial float sum, done on the host
 * in pixel order from these terms (a parallel float sum would round differently). */
__global__ __launch_bounds__(kBlock) void k_energy_terms(const float4* __restrict__ acc, float* __restrict__ out,
                                                         uint32_t npx, float inv) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const float4 a = acc[p];
    out[p] = ((a.x * inv) + (a.y * inv)) + (a.z * inv);
}

/* Traversal entry points for kernel-level parity tests. */
template <bool LDS, bool LW = false>
__global__ __launch_bounds__(kBlock) void k_trace_closest(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                          uint32_t n, float4* __restrict__ tuv, uint2* __restrict__ ip,
                                                          uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = traceTables<LDS>(S, lds, stackWords);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float depth = kFarAway, u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    const bool hit = traceScene<false, LW>(S, Tt, mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                                       depth, u, v, inst, prim, lds + threadIdx.x, blockDim.x);
    tuv[i] = make_float4(depth, hit ? u : 0.0f, hit ? v : 0.0f, 0.0f);
    ip[i] = make_uint2(hit ? inst : kUnset, hit ? prim : kUnset);
}
template <bool LDS, bool LW = false>
__global__ __launch_bounds__(kBlock) void k_trace_any(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                      const float* __restrict__ tmaxv, uint32_t n, uint8_t* __restrict__ occ,
                                                      uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = traceTables<LDS>(S, lds, stackWords);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float depth = tmaxv[i], u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    occ[i] = traceScene<true, LW>(S, Tt, mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                              depth, u, v, inst, prim, lds + threadIdx.x, blockDim.x) ? 1 : 0;
}

/* Cooperative traversal entry points (one ray per 64-lane block, the
 * lanes-as-planes traversal of the cooperative tail): the same results as
 * k_trace_closest / k_trace_any, for parity tests and latency measurements. */
template <bool LDS, bool W2 = false>
__global__ __launch_bounds__(64) void k_trace_closest_coop(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                           uint32_t n, float4* __restrict__ tuv, uint2* __restrict__ ip,
                                                           uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = coopTrace<LDS>(S, lds, stackWords + proWords(S));
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    float depth = kFarAway, u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    const V3 ro = mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), rdir = mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    const bool hit = traceWave<false, W2>(S, Tt, ro, rdir, depth, u, v, inst, prim, reinterpret_cast<float*>(lds),
                                      reinterpret_cast<float4*>(lds + stackWords));
    if (threadIdx.x == 0) {
        tuv[i] = make_float4(depth, hit ? u : 0.0f, hit ? v : 0.0f, 0.0f);
        ip[i] = make_uint2(hit ? inst : kUnset, hit ? prim : kUnset);
    }
}
template <bool LDS, bool W2 = false>
__global__ __launch_bounds__(64) void k_trace_any_coop(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                       const float* __restrict__ tmaxv, uint32_t n, uint8_t* __restrict__ occ,
                                                       uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = coopTrace<LDS>(S, lds, stackWords + proWords(S));
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const V3 ro = mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), rdir = mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    float depth = tmaxv[i], u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    const bool oc = traceWave<true, W2>(S, Tt, ro, rdir, depth, u, v, inst, prim, reinterpret_cast<float*>(lds),
                                    reinterpret_cast<float4*>(lds + stackWords));
    if (threadIdx.x == 0) occ[i] = oc ? 1 : 0;
}

/* Diagnostics (surf_debug_segment_cycles): the latency of one drain segment's
 * pieces on a lone wave, each repeated `reps` times on the same inputs (the
 * cooperative drain's device functions): cyc[0] the closest-hit wave walk
 * (instance prologue included), cyc[1] shadePath, cyc[2] the shadow ray's
 * any-hit walk, cyc[3] the cosine sample alone, cyc[4] the light sample
 * alone, cyc[5] the hit-normal fetch + normalization alone; shader clock
 * cycles (s_memtime) summed over the repetitions. */
__device__ __forceinline__ unsigned long long clockNow() {
    __builtin_amdgcn_s_waitcnt(0);                   /* every memory operation in flight has landed */
    unsigned long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    uint32_t lo = (uint32_t)t, hi = (uint32_t)(t >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));           /* a VGPR value: no scalar value crosses the branches */
    return ((unsigned long long)hi << 32) | lo;
}
template <bool LDS, bool W2>
__global__ __launch_bounds__(64) void k_segment_cycles(DevScene S, float4 o4, float4 d4, float4 T4, uint32_t reps,
                                                       unsigned long long* __restrict__ cyc, uint32_t stackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = coopTrace<LDS>(S, lds, stackWords + proWords(S));
    const ShadeTables Tb = coopShade<LDS>(S, lds, (stackWords + proWords(S) + S.nInst * (uint32_t)((sizeof(TraceInst) + 4u) / 4u) + 3u) & ~3u);
    float* rstk = reinterpret_cast<float*>(lds);
    float4* pro = reinterpret_cast<float4*>(lds + stackWords);
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    uint32_t sink = 0;
    if (reps & 0x80000000u) {
        /* the closest-hit wave walk alone (for PMC counters of just the walk) */
        for (uint32_t k = 0; k < (reps & 0x7FFFFFFFu); ++k) {
            float depth = kFarAway, u = 0.0f, v = 0.0f;
            uint32_t inst = kUnset, prim = kUnset;
            sink += traceWave<false, W2>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, rstk, pro) ? prim : 0u;
        }
        reps = 0;
    }
    for (uint32_t k = 0; k < reps; ++k) {
        const unsigned long long t0 = clockNow();
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
        const bool hit = traceWave<false, W2>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, rstk, pro);
        const unsigned long long t1 = clockNow();
        ShadeOut r;
        shadePath<true>(S, Tb, o4, d4, T4, make_float4(depth, u, v, u2f(prim)), hit ? inst : kUnset, 0u, 1u, r);
        const unsigned long long t2 = clockNow();
        bool occ = false;
        if (r.shadow) {
            float sdep = r.so.w, su = 0.0f, sv = 0.0f;
            uint32_t si = kUnset, sp = kUnset;
            occ = traceWave<true, W2>(S, Tt, xyz(r.so), xyz(r.sd), sdep, su, sv, si, sp, rstk, pro);
        }
        const unsigned long long t3 = clockNow();
        c[0] += t1 - t0; c[1] += t2 - t1; c[2] += t3 - t2;
        sink += (occ ? 1u : 0u) + f2u(r.o.x);
        /* the pieces alone, on this segment's inputs */
        if (hit) {
            const DevInstance& I = Tb.inst[inst];
            const uint32_t seed0 = f2u(T4.w);
            V3 N;
            {
                const unsigned long long a = clockNow();
                const float4* nr = S.normals + 3u * (I.triOffset + prim);
                const float4 n0 = nr[0], n1 = nr[1], n2 = nr[2];
                const float w = (1.0f - u) - v;
                const V3 no = add(add(lscl(u, xyz(n0)), lscl(v, xyz(n2))), lscl(w, xyz(n1)));
                const float* M = I.M;
                const float nx4 = mrow(M, 0, no.x, no.y, no.z, 0.0f), ny4 = mrow(M, 1, no.x, no.y, no.z, 0.0f);
                const float nz4 = mrow(M, 2, no.x, no.y, no.z, 0.0f), nw4 = mrow(M, 3, no.x, no.y, no.z, 0.0f);
                const float nn = (nx4 * nx4 + ny4 * ny4) + (nz4 * nz4 + nw4 * nw4);
                const float ninv = 1.0f / sqrtf(nn);
                N = mk3(nx4 * ninv, ny4 * ninv, nz4 * ninv);
                asm volatile("" : "+v"(N.x), "+v"(N.y), "+v"(N.z));
                c[5] += clockNow() - a;
            }
            {
                uint32_t sd = seed0;
                V3 R1;
                const unsigned long long a = clockNow();
                const bool ok = cosineTry(sd, N, R1);
                asm volatile("" : "+v"(R1.x), "+v"(R1.y), "+v"(R1.z));
                c[3] += clockNow() - a;
                sink += ok ? 1u : 0u;
            }
            {
                uint32_t sd = seed0;
                ShadeOut q;
                q.shadow = false;
                const V3 P = add(xyz(o4), lscl(depth, xyz(d4)));
                const unsigned long long a = clockNow();
                sampleNEE(S, Tb, sd, P, N, mk3(1.0f, 0.0f, 0.0f), mk3(0.3f, 0.0f, 0.0f), 0u, q);
                asm volatile("" : "+v"(q.so.x), "+v"(q.sc.x));
                c[4] += clockNow() - a;
                sink += q.shadow ? 1u : 0u;
            }
        }
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < 6; ++k) cyc[k] = c[k];
        cyc[6] = sink;
        for (int k = 0; k < 8; ++k) { cyc[7 + k] = g_walkProf[k]; g_walkProf[k] = 0ull; }
    }
}

}  // namespace surfdev
