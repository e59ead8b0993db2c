// Lock-step traversal model of k_extend's lane kernel (tools/lockstep_sim.py runs it).
// Rays (file: u32 n, then n x (o.xyz, d.xyz) f32, in the order the GPU would trace
// them) are taken 64 at a time; for each instance of the single-leaf TLAS in order,
// the lanes whose ray reaches its world box walk its BLAS in lock step (one node per
// step, as the reference's DFS).  Prints visit steps per 64 rays, active lanes and
// distinct node records per step.  Modes:
//   lockstep_sim RAYS                 the wave-uniform instance loop (today's kernel)
//   lockstep_sim RAYS 1 B             per-instance compacted passes, groups within blocks of B rays
//   lockstep_sim RAYS mask OUT        writes each ray's instance world-box mask (u32) to OUT
// A probe only: links the oracle's restatement as its traversal model.
#include "../oracle/cpu_ref.cpp"
#include <set>
#include <map>
struct Lane { V3 oo, dd; uint32_t node; std::vector<uint32_t> st; bool act; };
int main(int argc, char** argv) {
    orc_scene* h = orc_scene_create(getenv("SURF_ASSETS") ? getenv("SURF_ASSETS") : "assets", getenv("SCENE_VARIANT") ? atoi(getenv("SCENE_VARIANT")) : 0);
    Scene& S = *h->s;
    FILE* f = fopen(argv[1], "rb"); uint32_t n = 0;
    if (!f || fread(&n, 4, 1, f) != 1) return 1;
    const bool ANY = getenv("LOCKSTEP_ANY") != nullptr;     /* shadow rays: 7 floats (o, d, tmax), any-hit */
    const int RS = ANY ? 7 : 6;
    std::vector<float> raw((size_t)RS * n);
    if (fread(raw.data(), 4, raw.size(), f) != raw.size()) return 1;
    fclose(f);
    std::vector<float> od(6 * (size_t)n), tmx(n, kFarAway);
    for (uint32_t i = 0; i < n; ++i) {
        for (int q = 0; q < 6; ++q) od[6 * i + q] = raw[(size_t)RS * i + q];
        if (ANY) tmx[i] = raw[(size_t)RS * i + 6];
    }
    if (argc > 2 && std::string(argv[2]) == "mask") {
        // membership of every ray: bit k = instance k's world box is hit within [0, inf)
        const Bvh& T = S.tlas; const Node& root = T.nodes[0];
        std::vector<uint32_t> m(n, 0);
        for (uint32_t i = 0; i < n; ++i) {
            V3 o = mk(od[6*i], od[6*i+1], od[6*i+2]), d = mk(od[6*i+3], od[6*i+4], od[6*i+5]);
            for (uint32_t k = 0; k < root.cnt; ++k) {
                uint32_t ii = T.idx[root.lf + k];
                if (slab(S.inst[ii].bounds, o, d, kFarAway) != kFarAway) m[i] |= 1u << ii;
            }
        }
        FILE* g = fopen(argv[3], "wb"); fwrite(m.data(), 4, n, g); fclose(g);
        return 0;
    }
    double iters = 0, active = 0, distinct = 0, uniform = 0, leafIters = 0, triDistinct = 0, triLoads = 0, nodeLoads = 0;
    double uniAct = 0;
    std::map<int,double> hist;
    std::map<uint32_t, double> instIters, instLanes, instTri;   /* per TLAS instance: wave steps, lane-steps, triangle tests */
    /* node loads by breadth-first rank of the node in its BLAS (LOCKSTEP_BFS=1): how many a staged top-K prefix would serve */
    std::map<const Bvh*, std::vector<uint32_t>> bfsRank;
    std::vector<double> rankLoads(1 << 16, 0.0);
    double allLoads = 0;
    auto rankOf = [&](const Bvh& b) -> const std::vector<uint32_t>& {
        auto it = bfsRank.find(&b);
        if (it != bfsRank.end()) return it->second;
        std::vector<uint32_t> r(b.nodes.size(), 0xffffffffu);
        std::vector<uint32_t> q{0u}; r[0] = 0; uint32_t next = 1;
        for (size_t h = 0; h < q.size(); ++h) {
            const Node& nd = b.nodes[q[h]];
            if (nd.cnt) continue;
            for (uint32_t c = nd.lf; c <= nd.lf + 1; ++c) { r[c] = next++; q.push_back(c); }
        }
        return bfsRank.emplace(&b, std::move(r)).first->second;
    };
    for (uint32_t g = 0; g + 64 <= n; g += 64) {
        V3 o[64], d[64]; float depth[64];
        bool occ[64];
        for (int l = 0; l < 64; ++l) { o[l] = mk(od[6*(g+l)], od[6*(g+l)+1], od[6*(g+l)+2]); d[l] = mk(od[6*(g+l)+3], od[6*(g+l)+4], od[6*(g+l)+5]); depth[l] = tmx[g + l]; occ[l] = false; }
        const Bvh& T = S.tlas;
        const Node& root = T.nodes[0];
        for (uint32_t k = 0; k < root.cnt; ++k) {
            const Instance& in = S.inst[T.idx[root.lf + k]];
            const Bvh& b = in.blas->bvh;
            V3 oo[64], dd[64]; uint32_t node[64]; std::vector<uint32_t> st[64]; bool act[64];
            for (int l = 0; l < 64; ++l) {
                act[l] = false;
                if (occ[l] || slab(in.bounds, o[l], d[l], depth[l]) == kFarAway) continue;
                V4 tp = mul(in.Minv, v4(o[l], 1.0f)), td = mul(in.Minv, v4(d[l], 0.0f));
                oo[l] = xyz(tp) / tp.w; dd[l] = xyz(td);
                const Node& r = b.nodes[0];
                if (r.cnt) { // root leaf: uniform scalar path on GPU; test here
                    for (uint32_t i = 0; i < r.cnt; ++i) { float u, v; if (hitTri(in.blas->mesh->tris[b.idx[r.lf + i]], oo[l], dd[l], depth[l], u, v) && ANY) { occ[l] = true; break; } }
                    continue;
                }
                uint32_t cn = r.lf, cf = r.lf + 1;
                float dn = slab(b.nodes[cn].box, oo[l], dd[l], depth[l]), df = slab(b.nodes[cf].box, oo[l], dd[l], depth[l]);
                if (ANY) {
                    if (dn == kFarAway && df == kFarAway) continue;
                    node[l] = dn != kFarAway ? cn : cf; st[l].clear(); if (dn != kFarAway && df != kFarAway) st[l].push_back(cf);
                    act[l] = true;
                    continue;
                }
                if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
                if (dn == kFarAway) continue;
                node[l] = cn; st[l].clear(); if (df != kFarAway) st[l].push_back(cf);
                act[l] = true;
            }
            for (;;) {
                std::set<uint32_t> ns, ts; int na = 0; bool anyLeaf = false;
                for (int l = 0; l < 64; ++l) if (act[l]) { ++na; ns.insert(node[l]); }
                if (!na) break;
                iters++; active += na; distinct += ns.size(); nodeLoads += na; if (ns.size() == 1) { uniform++; uniAct += na; }
                instIters[T.idx[root.lf + k]] += 1; instLanes[T.idx[root.lf + k]] += na;
                hist[std::min<int>(ns.size(), 64)]++;
                for (int l = 0; l < 64; ++l) if (act[l]) {
                    const Node& nd = b.nodes[node[l]];
                    { const uint32_t rk = rankOf(b)[node[l]]; allLoads += 1; if (rk < rankLoads.size()) rankLoads[rk] += 1; }
                    bool pop = false;
                    if (nd.cnt) {
                        anyLeaf = true;
                        bool h = false;
                        for (uint32_t i = 0; i < nd.cnt; ++i) { ts.insert(nd.lf + i); triLoads++; instTri[T.idx[root.lf + k]] += 1; float u, v; if (hitTri(in.blas->mesh->tris[b.idx[nd.lf + i]], oo[l], dd[l], depth[l], u, v) && ANY) { h = true; break; } }
                        if (h) { occ[l] = true; act[l] = false; continue; }
                        pop = true;
                    } else {
                        uint32_t cn = nd.lf, cf = nd.lf + 1;
                        float dn = slab(b.nodes[cn].box, oo[l], dd[l], depth[l]), df = slab(b.nodes[cf].box, oo[l], dd[l], depth[l]);
                        if (ANY) {
                            if (dn == kFarAway && df == kFarAway) pop = true;
                            else { node[l] = dn != kFarAway ? cn : cf; if (dn != kFarAway && df != kFarAway) st[l].push_back(cf); }
                        } else {
                            if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
                            if (dn == kFarAway) pop = true; else { node[l] = cn; if (df != kFarAway) st[l].push_back(cf); }
                        }
                    }
                    if (pop) { if (st[l].empty()) act[l] = false; else { node[l] = st[l].back(); st[l].pop_back(); } }
                }
                if (anyLeaf) { leafIters++; triDistinct += ts.size(); }
            }
        }
    }
    if (argc > 2) {
        // per-instance passes: every ray that reaches instance k (not culled at its current depth), compacted, in ray order
        std::vector<float> dep(n, kFarAway);
        double it2 = 0, act2 = 0;
        const Bvh& T = S.tlas; const Node& root = T.nodes[0];
        for (uint32_t k = 0; k < root.cnt; ++k) {
            const Instance& in = S.inst[T.idx[root.lf + k]];
            const Bvh& b = in.blas->bvh;
            std::vector<uint32_t> part;
            for (uint32_t i = 0; i < n; ++i) {
                V3 o = mk(od[6*i], od[6*i+1], od[6*i+2]), d = mk(od[6*i+3], od[6*i+4], od[6*i+5]);
                if (slab(in.bounds, o, d, dep[i]) == kFarAway) continue;
                part.push_back(i);
            }
            const uint32_t B = argc > 3 ? atoi(argv[3]) : 0;   // in-block compaction: groups never span blocks of B rays
            std::vector<size_t> starts;
            for (size_t g = 0; g < part.size();) {
                starts.push_back(g);
                size_t e = std::min(part.size(), g + 64);
                if (B) { uint32_t blk = part[g] / B; size_t q = g; while (q < e && part[q] / B == blk) ++q; e = q; }
                g = e;
            }
            starts.push_back(part.size());
            for (size_t si = 0; si + 1 < starts.size(); ++si) {
                size_t g = starts[si];
                Lane L[64]; int m = (int)(starts[si + 1] - g);
                for (int l = 0; l < m; ++l) {
                    uint32_t i = part[g + l]; L[l].act = false;
                    V3 o = mk(od[6*i], od[6*i+1], od[6*i+2]), d = mk(od[6*i+3], od[6*i+4], od[6*i+5]);
                    V4 tp = mul(in.Minv, v4(o, 1.0f)), td = mul(in.Minv, v4(d, 0.0f));
                    L[l].oo = xyz(tp) / tp.w; L[l].dd = xyz(td);
                    const Node& r = b.nodes[0];
                    if (r.cnt) { for (uint32_t q = 0; q < r.cnt; ++q) { float u, v; hitTri(in.blas->mesh->tris[b.idx[r.lf + q]], L[l].oo, L[l].dd, dep[i], u, v); } continue; }
                    uint32_t cn = r.lf, cf = r.lf + 1;
                    float dn = slab(b.nodes[cn].box, L[l].oo, L[l].dd, dep[i]), df = slab(b.nodes[cf].box, L[l].oo, L[l].dd, dep[i]);
                    if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
                    if (dn == kFarAway) continue;
                    L[l].node = cn; L[l].st.clear(); if (df != kFarAway) L[l].st.push_back(cf); L[l].act = true;
                }
                for (;;) {
                    int na = 0; for (int l = 0; l < m; ++l) na += L[l].act;
                    if (!na) break;
                    it2++; act2 += na;
                    for (int l = 0; l < m; ++l) if (L[l].act) {
                        uint32_t i = part[g + l];
                        const Node& nd = b.nodes[L[l].node]; bool pop = false;
                        if (nd.cnt) { for (uint32_t q = 0; q < nd.cnt; ++q) { float u, v; hitTri(in.blas->mesh->tris[b.idx[nd.lf + q]], L[l].oo, L[l].dd, dep[i], u, v); } pop = true; }
                        else {
                            uint32_t cn = nd.lf, cf = nd.lf + 1;
                            float dn = slab(b.nodes[cn].box, L[l].oo, L[l].dd, dep[i]), df = slab(b.nodes[cf].box, L[l].oo, L[l].dd, dep[i]);
                            if (dn > df) { std::swap(dn, df); std::swap(cn, cf); }
                            if (dn == kFarAway) pop = true; else { L[l].node = cn; if (df != kFarAway) L[l].st.push_back(cf); }
                        }
                        if (pop) { if (L[l].st.empty()) L[l].act = false; else { L[l].node = L[l].st.back(); L[l].st.pop_back(); } }
                    }
                }
            }
            printf("  after instance %u: passes' iterations %.0f (participants %zu)\n", k, it2, part.size());
        }
        printf("per-instance passes: iterations %.0f (%.1f per 64 rays) active/iter %.1f\n", it2, it2 / (n / 64), act2 / it2);
    }
    for (auto& [ii, v] : instIters)
        printf("  instance %u (blas %zu nodes): wave steps per 64 rays %.2f, lanes per step %.1f, triangle tests per ray %.2f\n", ii,
               S.inst[ii].blas->bvh.nodes.size(), v / (n / 64), instLanes[ii] / v, instTri[ii] / n);
    if (getenv("LOCKSTEP_BFS")) {
        double cum = 0; size_t k = 0;
        for (size_t K : {15, 31, 63, 127, 255, 511, 1023}) {
            for (; k < K && k < rankLoads.size(); ++k) cum += rankLoads[k];
            printf("  node loads at BFS rank < %zu: %.3f\n", K, cum / allLoads);
        }
    }
    printf("groups %u iters/group %.1f active/iter %.1f distinct nodes/iter %.2f uniform iters %.3f (lanes in uniform iters %.3f of node loads)\n",
           n / 64, iters / (n / 64), active / iters, distinct / iters, uniform / iters, uniAct / nodeLoads);
    printf("leaf iters %.3f tri loads/iter-with-leaf %.1f distinct tris %.1f\n", leafIters / iters, triLoads / leafIters, triDistinct / leafIters);
    for (auto& [k, v] : hist) if (k <= 8 || k % 8 == 0) printf("  distinct %d: %.3f\n", k, v / iters);
}
