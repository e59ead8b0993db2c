/*
 * rows_tail.h -- the drain engine for long Russian-roulette paths: four paths
 * per 64-lane wave, one per 16-lane row, each row walking the reference's
 * DFS with the lanes-as-planes node test.
 *
 * Why: at the end of a sample stream ~60-90 k paths are left with ~27 M
 * segments between them (C3; paths trapped in the glass Suzanne / lens or
 * bouncing on albedo-1 red walls, renderer.cpp:424-431 never kills them).
 * One path per wave (k_tail_coop) spends ~3.6 k VALU instructions per
 * segment for 12-14 useful lanes per node visit, and the drain is bound by
 * the VALU issue rate of the chip.  Four rows share every instruction: the
 * node test (12 slab planes + leftFirst/count in lanes 0..13 of a row), the
 * instance prologue (instance k in lane k of the row, <= 16 instances), the
 * triangle tests of a leaf (one triangle per lane) and the shading.  Rows
 * diverge only where their paths do (leaf vs interior vs next instance,
 * material branches); every decision is made in the vector unit and shared
 * in the row with DPP row_newbcast, so no decision leaves the VALU.
 *
 * A work queue (Counters::rowNext) hands each row a new path when its path
 * ends, so long paths never hold three idle rows.  Same DFS decisions as
 * blasTrace / traceWave (bvh.cpp:129-253, 654-778): bit-identical results.
 */
#pragma once
#include "wavefront_kernels.h"

namespace surfdev {

#ifndef SURF_ROWS_WAVES
#define SURF_ROWS_WAVES 3          /* k_tail_rows waves per SIMD (launch bounds: 168 VGPRs, no spills; 4 spills 37) */
#endif
constexpr uint32_t kRowInst = 16;  /* instances a row's prologue holds (one per lane) */
constexpr uint32_t kRowProWords = 64u * 16u;   /* LDS prologue table: 16 floats per lane */

/* DPP row_newbcast:L (gfx90a+): every lane of a 16-lane row reads lane L of its row. */
template <int L>
__device__ __forceinline__ uint32_t rowB(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + L, 0xF, 0xF, false);
}
template <int L>
__device__ __forceinline__ float rowBf(float v) { return __uint_as_float(rowB<L>(__float_as_uint(v))); }

/* min over the 16 lanes of a row, in every lane of the row */
__device__ __forceinline__ float rowMin(float x) {
    x = fminf(x, dppMov<0xB1>(x));      /* quad_perm [1,0,3,2] */
    x = fminf(x, dppMov<0x4E>(x));      /* quad_perm [2,3,0,1] */
    x = fminf(x, dppMov<0x124>(x));     /* row_ror:4 */
    x = fminf(x, dppMov<0x128>(x));     /* row_ror:8 */
    return x;
}
__device__ __forceinline__ float bperm(float v, int addr) { return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v))); }
__device__ __forceinline__ uint32_t bpermU(uint32_t v, int addr) { return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v); }
/* this row's 16 bits of a wave ballot */
__device__ __forceinline__ uint32_t rowBits(unsigned long long m) { return (uint32_t)(m >> (__lane_id() & 48u)) & 0xffffu; }

/* slabDecide per row: the same slab values and choices, the bits (0: the
 * right child is nearer, 1: nearer child hit, 2: farther child hit) shared in
 * the row by row_newbcast instead of leaving the vector unit. */
template <bool FIN>
__device__ __forceinline__ uint32_t slabBitsRow(float v, float oA, float rdA, float depth) {
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
    const float dist = (m1 >= m0 && m0 < depth && m1 > 0.0f) ? m0 : kFarAway;   /* lanes 4 / 10: box 0 / box 1 */
    const float d0 = dppMov<kDppShr6>(dist);          /* lane 10 <- lane 4 */
    const bool sw = d0 > dist;                          /* if (dn > df) swap */
    const float nearD = sw ? dist : d0, farD = sw ? d0 : dist;
    const uint32_t bits = (sw ? 1u : 0u) | (nearD != kFarAway ? 2u : 0u) | (farD != kFarAway ? 4u : 0u);
    return rowB<10>(bits);
}

/* Triangles [lf, lf + cnt) of a BLAS leaf, one per lane of the row; the
 * reference tests them in index order against a shrinking depth, which
 * accepts the smallest t (the first index among equal t): a row minimum and
 * the lowest lane holding it. */
template <bool ANY>
__device__ __forceinline__ bool leafRows(const float4* tri, uint32_t lf, uint32_t cnt, V3 o, V3 d, float& depth,
                                         float& hu, float& hv, uint32_t& hprim) {
    const uint32_t l16 = __lane_id() & 15u, rbase = __lane_id() & 48u;
    bool any = false;
    for (uint32_t b = 0; b < cnt; b += 16u) {
        const uint32_t k = b + l16;
        float t = depth, u = 0.0f, v = 0.0f;
        uint32_t prim = 0;
        bool h = false;
        if (k < cnt) {
            const float4* tp = tri + 3u * (lf + k);
            const float4 a = tp[0], e1 = tp[1], e2 = tp[2];
            prim = f2u(a.w);
            h = triHitFlat(xyz(a), xyz(e1), xyz(e2), o, d, depth, t, u, v);
        }
        const uint32_t m16 = rowBits(__ballot(h));
        if (ANY) {
            if (m16) return true;
            continue;
        }
        if (m16) {
            const float tm = rowMin(h ? t : __builtin_inff());
            const uint32_t w16 = rowBits(__ballot(h && t == tm));
            const int src = (int)((rbase + (uint32_t)__builtin_ctz(w16)) << 2);
            depth = tm;
            hu = bperm(u, src);
            hv = bperm(v, src);
            hprim = bpermU(prim, src);
            any = true;
        }
    }
    return any;
}

/* BvhTLAS::intersect / intersectAny over a single-leaf TLAS of <= 16 instances
 * (bvh.cpp:654-778), one ray per row.  Prologue as traceWave: lane k of the
 * row forms instance k's object-space ray, 1/d and its root children's slab
 * ranges; instances whose root children miss at the entry depth are dropped
 * (a miss stays a miss at every smaller depth).  Then each row runs a small
 * state machine -- pick the next instance in TLAS order, or visit the node
 * whose record `cur` holds (lane l holds word planeDword(l)) -- so rows at
 * different stages of their walks share the loop.  rs: this row's stack of
 * far-child records (16 words per entry, lane-indexed); pro: the wave's
 * prologue table in LDS (16 floats per lane), so the per-instance rays do not
 * hold registers through the walk. */
template <bool ANY>
__device__ __forceinline__ bool traceRows(const DevScene& S, const TraceTables& Tt, V3 o, V3 d, float& depth, float& hu,
                                          float& hv, uint32_t& hinst, uint32_t& hprim, float* rs, float4* pro) {
    constexpr uint32_t kPick = 0, kVisit = 1, kDone = 2;
    const uint32_t lane = __lane_id(), l16 = lane & 15u, rbase = lane & 48u;
    const uint32_t nI = S.tlasLeafCount;
    const uint32_t dw = planeDword(l16), ax = l16 < 12u ? (l16 % 6u) >> 1 : 0u;
    const float* nodesF = reinterpret_cast<const float*>(S.nodes);
    bool keep = false;
    if (l16 < nI) {
        const TraceInst& I = Tt.inst[Tt.order[l16]];
        V3 oo = mk3(rowDot(I.m0, o.x, o.y, o.z, 1.0f), rowDot(I.m1, o.x, o.y, o.z, 1.0f), rowDot(I.m2, o.x, o.y, o.z, 1.0f));
        if (!I.meta.z) oo = divs(oo, rowDot(I.m3, o.x, o.y, o.z, 1.0f));
        const V3 dd = mk3(rowDot(I.m0, d.x, d.y, d.z, 0.0f), rowDot(I.m1, d.x, d.y, d.z, 0.0f), rowDot(I.m2, d.x, d.y, d.z, 0.0f));
        const V3 rd = mk3(1.0f / dd.x, 1.0f / dd.y, 1.0f / dd.z);
        float a0, a1, b0, b1;
        slabRange(I.r0, I.r1, oo, rd, a0, a1);
        slabRange(I.r2, I.r3, oo, rd, b0, b1);
        keep = f2u(I.r1.w) != 0u || slabHit(a0, a1, depth) != kFarAway || slabHit(b0, b1, depth) != kFarAway;
        float4* p = pro + 4u * lane;
        p[0] = make_float4(oo.x, oo.y, oo.z, a0);
        p[1] = make_float4(dd.x, dd.y, dd.z, a1);
        p[2] = make_float4(rd.x, rd.y, rd.z, b0);
        p[3] = make_float4(b1, 0.0f, 0.0f, 0.0f);
    }
    uint32_t cand = rowBits(__ballot(keep));
    uint32_t mode = kPick, sp = 0, nodeOff = 0, triBase = 0, ii = 0;
    float cur = 0.0f, oA = 0.0f, rdA = 0.0f;
    V3 ok = mk3(0.0f, 0.0f, 0.0f), dk = ok;
    bool fin = true, any = false;
    for (;;) {
        if (mode == kPick) {
            if (cand == 0u) {
                mode = kDone;
            } else {
                const uint32_t k = (uint32_t)__builtin_ctz(cand);
                cand &= cand - 1u;
                const float4* p = pro + 4u * (rbase + k);      /* one address per row: an LDS broadcast */
                const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
                ok = xyz(q0);
                dk = xyz(q1);
                const V3 rk = xyz(q2);
                const float ka0 = q0.w, ka1 = q1.w, kb0 = q2.w, kb1 = q3.x;
                ii = Tt.order[k];
                const TraceInst& I = Tt.inst[ii];
                nodeOff = I.meta.x;
                triBase = I.meta.y;
                const uint32_t rlf = f2u(I.r0.w), rcnt = f2u(I.r1.w);
                oA = pick3(ok, ax);
                rdA = pick3(rk, ax);
                fin = S.finiteBoxes && finite3(ok) && finite3(rk);
                sp = 0;
                if (rcnt != 0u) {
                    /* root leaf: a record whose lanes 12 / 13 say (leftFirst, count) */
                    cur = u2f(l16 == 12u ? rlf : rcnt);
                    mode = kVisit;
                } else {
                    /* root: never box-tested (bvh.cpp:131); its children's ranges are the prologue's */
                    float dn = slabHit(ka0, ka1, depth), df = slabHit(kb0, kb1, depth);
                    uint32_t cn = nodeOff + rlf, cf = cn + 1u;
                    if (dn > df) { const float t = dn; dn = df; df = t; const uint32_t c = cn; cn = cf; cf = c; }
                    if (dn != kFarAway) {
                        const uint32_t cmin = cn < cf ? cn : cf;
                        const float rA = nodesF[16u * cmin + dw], rB = nodesF[16u * (cmin + 1u) + dw];
                        const bool nb = cn != cmin;
                        cur = nb ? rB : rA;
                        if (df != kFarAway) { rs[l16] = nb ? rA : rB; sp = 1; }
                        mode = kVisit;
                    }
                }
            }
        }
        if (__ballot(mode != kDone) == 0ull) break;
        if (mode == kVisit) {
            const uint32_t lf = rowB<12>(f2u(cur)), cnt = rowB<13>(f2u(cur));
            if (cnt != 0u) {
                if (leafRows<ANY>(S.tris + 3u * triBase, lf, cnt, ok, dk, depth, hu, hv, hprim)) {
                    any = true;
                    hinst = ii;
                    if (ANY) mode = kDone;
                }
                if (mode == kVisit) {
                    if (sp == 0u) mode = kPick;
                    else { --sp; cur = rs[16u * sp + l16]; }
                }
            } else {
                /* both children's records in flight while this node's boxes are tested */
                const uint32_t c0 = nodeOff + lf;
                const float rA = nodesF[16u * c0 + dw], rB = nodesF[16u * (c0 + 1u) + dw];
                const uint32_t bits = fin ? slabBitsRow<true>(cur, oA, rdA, depth) : slabBitsRow<false>(cur, oA, rdA, depth);
                if (!(bits & 2u)) {
                    if (sp == 0u) mode = kPick;
                    else { --sp; cur = rs[16u * sp + l16]; }
                } else {
                    const bool nb = (bits & 1u) != 0u;
                    if (bits & 4u) { rs[16u * sp + l16] = nb ? rA : rB; ++sp; }
                    cur = nb ? rB : rA;
                }
            }
        }
    }
    return any;
}

/* A row's next path from the drain's queue (Counters::rowNext). */
__device__ __forceinline__ uint32_t takePath(Counters* C) {
    uint32_t k = 0;
    if ((__lane_id() & 15u) == 0u) k = atomicAdd(&C->rowNext, 1u);
    return rowB<0>(k);
}

/* The drain: every path of `cur` run to its end, four rows per wave, each row
 * taking the next queued path when its own ends.  Per segment exactly the
 * device functions of the wavefront kernels (traceRows = traceScene's
 * decisions, shadePath, any-hit shadow ray), radiance added by lane 0 of the
 * row in the path's order.  firstCounted: regen already counted the first
 * extension ray of each input path.  LDS: four row stacks of rowStackWords
 * floats, the prologue table (64 lanes x 16 floats), then the trace tables. */
__global__ __launch_bounds__(64, SURF_ROWS_WAVES) void k_tail_rows(DevScene S, Pool cur, uint32_t n, float4* __restrict__ rad,
                                                  uint32_t* __restrict__ frameDone, uint32_t npx, uint32_t window, Counters* C,
                                                  uint32_t rowStackWords, uint32_t firstCounted) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = stageTrace(S, lds, 4u * rowStackWords + kRowProWords);
    const ShadeTables Tb{S.inst, S.mats, S.lights};
    float4* pro = reinterpret_cast<float4*>(lds + 4u * rowStackWords);
    const uint32_t lane = __lane_id(), row = lane >> 4;
    const bool lead = (lane & 15u) == 0u;
    float* rs = reinterpret_cast<float*>(lds) + row * rowStackWords;
    const uint32_t maxSeg = C->maxSeg, zeroCutoff = C->zeroCutoff;
    const uint32_t st = blockIdx.x % kStripes;
    uint32_t idx = takePath(C);
    float4 o4 = make_float4(0, 0, 0, 0), d4 = o4, T4 = o4;
    if (idx < n) { o4 = cur.od[2u * (idx)]; d4 = cur.od[2u * (idx) + 1u]; T4 = cur.T[idx]; }
    uint32_t nExt = 0, nHit = 0, nCont = 0, nSh = 0, nAcc = 0, nUn = 0, nPaths = 0;
#if SURF_DRAIN_TRACE
    unsigned long long tStart = wall_clock64();
    uint32_t extStart = 0, state0 = drainState(d4, T4);
#endif
    for (;;) {
        const bool act = idx < n;
        if (__ballot(act) == 0ull) break;
        if (!act) continue;
        float depth = kFarAway, u = 0.0f, v = 0.0f;
        uint32_t inst = kUnset, prim = kUnset;
        const bool hit = traceRows<false>(S, Tt, xyz(o4), xyz(d4), depth, u, v, inst, prim, rs, pro);
        ++nExt;
        ShadeOut r;
        shadePath(S, Tb, o4, d4, T4, make_float4(depth, u, v, u2f(prim)), hit ? inst : kUnset, maxSeg, zeroCutoff, r);
        if (lead && r.addRad) addRadiance(rad, f2u(o4.w), r.radd);
        nHit += r.hitGeom;
        nAcc += r.accd;
        if (r.shadow) {
            ++nSh;
            float sdep = r.so.w, su = 0.0f, sv = 0.0f;
            uint32_t si = kUnset, sp = kUnset;
            if (!traceRows<true>(S, Tt, xyz(r.so), xyz(r.sd), sdep, su, sv, si, sp, rs, pro)) {
                if (lead) addRadiance(rad, f2u(r.sd.w), xyz(r.sc));
                ++nUn;
                ++nAcc;
            }
        }
        if (lead && r.capped) {
            noteCapped(C, f2u(o4.w));
        }
        if (r.cont) {
            ++nCont;
            o4 = r.o; d4 = r.d; T4 = r.T;
            continue;
        }
        if (lead) {
            atomicMax(&C->segMax, r.seg);
            __threadfence();          /* radiance before completion */
            atomicAdd(&frameDone[st * window + f2u(o4.w) / npx], 1u);
#if SURF_DRAIN_TRACE
            drainTraceEnd(tStart, nExt - extStart, state0);
#endif
        }
        ++nPaths;
        idx = takePath(C);
        if (idx < n) { o4 = cur.od[2u * (idx)]; d4 = cur.od[2u * (idx) + 1u]; T4 = cur.T[idx]; }
#if SURF_DRAIN_TRACE
        tStart = wall_clock64();
        extStart = nExt;
        state0 = drainState(d4, T4);
#endif
    }
    if (lead && nPaths) {
        unsigned long long* ev = C->evS[st];
        atomicAdd(&ev[0], (unsigned long long)nExt - (unsigned long long)firstCounted * nPaths);
        atomicAdd(&ev[1], (unsigned long long)nHit); atomicAdd(&ev[2], (unsigned long long)nCont);
        atomicAdd(&ev[3], (unsigned long long)nSh); atomicAdd(&ev[4], (unsigned long long)nAcc);
        atomicAdd(&ev[5], (unsigned long long)nUn); atomicAdd(&ev[6], (unsigned long long)nPaths);
    }
}

/* Row traversal entry points (four rays per 64-lane block): the same results
 * as k_trace_closest / k_trace_any, for parity tests. */
__global__ __launch_bounds__(64) void k_trace_closest_rows(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                           uint32_t n, float4* __restrict__ tuv, uint2* __restrict__ ip,
                                                           uint32_t rowStackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = stageTrace(S, lds, 4u * rowStackWords + kRowProWords);
    float4* pro = reinterpret_cast<float4*>(lds + 4u * rowStackWords);
    const uint32_t row = __lane_id() >> 4, i = blockIdx.x * 4u + row;
    if (i >= n) return;
    float depth = kFarAway, u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    const V3 ro = mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), rdir = mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    const bool hit = traceRows<false>(S, Tt, ro, rdir, depth, u, v, inst, prim, reinterpret_cast<float*>(lds) + row * rowStackWords, pro);
    if ((__lane_id() & 15u) == 0u) {
        tuv[i] = make_float4(depth, hit ? u : 0.0f, hit ? v : 0.0f, 0.0f);
        ip[i] = make_uint2(hit ? inst : kUnset, hit ? prim : kUnset);
    }
}
__global__ __launch_bounds__(64) void k_trace_any_rows(DevScene S, const float* __restrict__ o, const float* __restrict__ d,
                                                       const float* __restrict__ tmaxv, uint32_t n, uint8_t* __restrict__ occ,
                                                       uint32_t rowStackWords) {
    extern __shared__ uint32_t lds[];
    const TraceTables Tt = stageTrace(S, lds, 4u * rowStackWords + kRowProWords);
    float4* pro = reinterpret_cast<float4*>(lds + 4u * rowStackWords);
    const uint32_t row = __lane_id() >> 4, i = blockIdx.x * 4u + row;
    if (i >= n) return;
    const V3 ro = mk3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), rdir = mk3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    float depth = tmaxv[i], u = 0.0f, v = 0.0f;
    uint32_t inst = kUnset, prim = kUnset;
    const bool oc = traceRows<true>(S, Tt, ro, rdir, depth, u, v, inst, prim, reinterpret_cast<float*>(lds) + row * rowStackWords, pro);
    if ((__lane_id() & 15u) == 0u) occ[i] = oc ? 1 : 0;
}

}  // namespace surfdev
